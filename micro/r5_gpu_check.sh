#!/bin/bash
# full GPU suite, then the A/B bench (default vs listed variant libraries) — round-5 checkpoint
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r5_gpu_tests.txt 2>&1 || { tail -40 gpurun_out/r5_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/r5_gpu_tests.txt
timeout -k 10 60 python micro/lm_tail_bench.py || exit 1
STEPS="20 50" bash micro/r5_var_ab.sh "$@"
