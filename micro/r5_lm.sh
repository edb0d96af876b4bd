#!/bin/bash
# split micro-benchmark (committed split vs contiguous-run flags + one-trip median), sort / map GPU tests, then
# LM workgroup count A/B
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 60 python micro/split_bench.py micro/split_bench_base.so base > gpurun_out/r5_split2.txt 2>&1 || { cat gpurun_out/r5_split2.txt; exit 1; }
timeout -k 10 60 python micro/split_bench.py micro/split_bench.so new base >> gpurun_out/r5_split2.txt 2>&1 || { cat gpurun_out/r5_split2.txt; exit 1; }
grep -v "per level" gpurun_out/r5_split2.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "map or vox or sort" > gpurun_out/r5_lm_tests.txt 2>&1 || { tail -40 gpurun_out/r5_lm_tests.txt; exit 1; }
tail -2 gpurun_out/r5_lm_tests.txt
STEPS="20" bash micro/r5_env_ab.sh "base:ALOAM_X=0" "gmax32:ALOAM_LM_GMAX=32" "gmax16:ALOAM_LM_GMAX=16" "cubeseg6144:ALOAM_CUBE_SEG=6144"
