#!/bin/bash
# split rewrite check: split micro-benchmark (round-4 split vs the new one, outputs identical), mapping / VoxelGrid /
# sort GPU tests, A/B bench vs the listed library, then stack VoxelGrid and filter phase stamps (profiling builds)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 60 python micro/split_bench.py micro/split_bench_base.so base > gpurun_out/r5_split.txt 2>&1 || { cat gpurun_out/r5_split.txt; exit 1; }
timeout -k 10 60 python micro/split_bench.py micro/split_bench.so new base >> gpurun_out/r5_split.txt 2>&1 || { cat gpurun_out/r5_split.txt; exit 1; }
cat gpurun_out/r5_split.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "map or vox or sort or pipeline or bench" > gpurun_out/r5_split_tests.txt 2>&1 || { tail -40 gpurun_out/r5_split_tests.txt; exit 1; }
tail -2 gpurun_out/r5_split_tests.txt
STEPS="20 50" bash micro/r5_var_ab.sh "$@" || exit 1
ALOAM_LIB_PATH=micro/_var_vxts2/libaloam_hip.so timeout -k 10 180 python micro/vx_stamps.py 30 > gpurun_out/r5_vx_phases.txt 2>&1 || { tail gpurun_out/r5_vx_phases.txt; exit 1; }
cat gpurun_out/r5_vx_phases.txt
ALOAM_LIB_PATH=micro/_var_rbst3/libaloam_hip.so timeout -k 10 300 python micro/rb_stamps.py 120 > gpurun_out/r5_rbst3.txt 2>&1 || { tail gpurun_out/r5_rbst3.txt; exit 1; }
cat gpurun_out/r5_rbst3.txt
