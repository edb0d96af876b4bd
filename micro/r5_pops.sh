#!/bin/bash
# heap pops with the top bits in registers (vs HEAD's), split with the one-trip median (vs HEAD's), sort / map
# GPU tests, A/B bench vs the listed library
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
HEAP_SO=micro/heap_bench_head.so timeout -k 10 120 python micro/heap_bench.py 300 1000 3000 > gpurun_out/r5_pops.txt 2>&1 || { cat gpurun_out/r5_pops.txt; exit 1; }
timeout -k 10 120 python micro/heap_bench.py 300 1000 3000 >> gpurun_out/r5_pops.txt 2>&1 || { cat gpurun_out/r5_pops.txt; exit 1; }
grep "^n " gpurun_out/r5_pops.txt
timeout -k 10 60 python micro/split_bench.py micro/split_bench_base.so base > gpurun_out/r5_split3.txt 2>&1 || { cat gpurun_out/r5_split3.txt; exit 1; }
timeout -k 10 60 python micro/split_bench.py micro/split_bench.so new base >> gpurun_out/r5_split3.txt 2>&1 || { cat gpurun_out/r5_split3.txt; exit 1; }
grep -v "per level" gpurun_out/r5_split3.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "map or vox or sort" > gpurun_out/r5_pops_tests.txt 2>&1 || { tail -40 gpurun_out/r5_pops_tests.txt; exit 1; }
tail -2 gpurun_out/r5_pops_tests.txt
STEPS="20" bash micro/r5_var_ab.sh "$@"
