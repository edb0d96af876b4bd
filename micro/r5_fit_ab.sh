#!/bin/bash
# map-filter in-LDS cube limit (ALOAM_CUBE_FIT): the slowest cubes sit just below 4096 points
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
STEPS="20 50" bash micro/r5_env_ab.sh "base:ALOAM_X=0" "fit3072:ALOAM_CUBE_FIT=3072" "fit2048:ALOAM_CUBE_FIT=2048" "fit2048seg2048:ALOAM_CUBE_FIT=2048 ALOAM_CUBE_SEG=2048" || exit 1
