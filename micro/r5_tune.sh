#!/bin/bash
# segment-limit A/B on the default build, then a kernel trace of the driver's 20-step run (per-frame breakdown)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
STEPS="20" bash micro/r5_env_ab.sh "base:ALOAM_X=0" "voxseg4096:ALOAM_VOX_SEG=4096" "cubeseg8192:ALOAM_CUBE_SEG=8192" || exit 1
NAME=r5t20 STEPS=20 bash micro/r4_prof.sh || exit 1
f=$(find gpurun_out/r5t20 -name "*kernel_trace.csv" | head -1)
python micro/frames.py $f 6 24 > gpurun_out/r5t20_frames.txt && python micro/frames.py $f 182 219 >> gpurun_out/r5t20_frames.txt
cat gpurun_out/r5t20_frames.txt
