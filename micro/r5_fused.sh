#!/bin/bash
# fused map filter (k_rb_filter): one mapping test first, then mapping / pipeline / sort GPU tests, then A/B
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 120 python -u -m pytest tests/test_gpu_mapping.py -m gpu -x -v --timeout 100 --timeout-method thread -k "publication_surface" > gpurun_out/r5_fused_t1.txt 2>&1 || { tail -30 gpurun_out/r5_fused_t1.txt; exit 1; }
tail -1 gpurun_out/r5_fused_t1.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "map or pipeline or sort or vox or bench" > gpurun_out/r5_fused_tests.txt 2>&1 || { tail -40 gpurun_out/r5_fused_tests.txt; exit 1; }
tail -2 gpurun_out/r5_fused_tests.txt
STEPS="20" bash micro/r5_env_ab.sh "fused:ALOAM_RB_FUSED=1" "three:ALOAM_RB_FUSED=0"
