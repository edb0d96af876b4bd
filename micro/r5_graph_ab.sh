#!/bin/bash
# round graphs vs eager round launches (ALOAM_NO_GRAPHS), driver config, interleaved
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
STEPS="20 50" bash micro/r5_env_ab.sh "base:ALOAM_X=0" "nographs:ALOAM_NO_GRAPHS=1" || exit 1
