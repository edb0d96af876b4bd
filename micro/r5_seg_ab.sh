#!/bin/bash
# map filter: segment size of the split cubes' parallel sorts (ALOAM_CUBE_SEG) with the 2048-point in-LDS limit
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
STEPS="20 50" bash micro/r5_env_ab.sh "base:ALOAM_X=0" "seg3072:ALOAM_CUBE_SEG=3072" "seg6144:ALOAM_CUBE_SEG=6144" "seg8192:ALOAM_CUBE_SEG=8192" || exit 1
