#!/bin/bash
# stack VoxelGrid: clouds sorted whole in one workgroup up to ALOAM_VOX_FIT points (the ~6000-point corner stack
# today), and the mapping association's grid size
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
STEPS="20 50" bash micro/r5_env_ab.sh "base:ALOAM_X=0" "vfit4096:ALOAM_VOX_FIT=4096" "vfit3072seg3072:ALOAM_VOX_FIT=3072 ALOAM_VOX_SEG=3072" "ab1024:ALOAM_ASSOC_BLOCKS=1024" || exit 1
