#!/bin/bash
# map-filter in-LDS cube limit (ALOAM_CUBE_FIT), second sweep: below 2048
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
STEPS="20 50" bash micro/r5_env_ab.sh "fit2048:ALOAM_CUBE_FIT=2048" "fit1536:ALOAM_CUBE_FIT=1536" "fit1024:ALOAM_CUBE_FIT=1024" || exit 1
