#!/bin/bash
# filter fork A/B (ALOAM_RB_FORK), mapping / sort GPU tests, heap micro-benchmark (walk on 32-bit flag words)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "map or vox or sort or pipeline" > gpurun_out/r5_fork_tests.txt 2>&1 || { tail -40 gpurun_out/r5_fork_tests.txt; exit 1; }
tail -2 gpurun_out/r5_fork_tests.txt
timeout -k 10 120 python micro/heap_bench.py 300 1000 3000 > gpurun_out/r5_heap_bfe.txt 2>&1 || { cat gpurun_out/r5_heap_bfe.txt; exit 1; }
cat gpurun_out/r5_heap_bfe.txt
STEPS="20" bash micro/r5_env_ab.sh "fork:ALOAM_RB_FORK=1" "nofork:ALOAM_RB_FORK=0" "cubeseg2048:ALOAM_CUBE_SEG=2048" "voxseg4096:ALOAM_VOX_SEG=4096"
