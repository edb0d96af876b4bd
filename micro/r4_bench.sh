#!/bin/bash
# default bench line (as the driver runs it) + the pipeline stage occupancy (ALOAM_PIPE_TIMING)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/r4_bench.json 2> gpurun_out/r4_bench.err || { tail -20 gpurun_out/r4_bench.err; exit 1; }
STEPS=300 bash micro/phases.sh "def:ALOAM_PIPE_TIMING=1" > gpurun_out/r4_phases.txt 2>&1 || exit 1
grep -a "aloam" gpurun_out/ph_def.err | tail -6 >> gpurun_out/r4_phases.txt
