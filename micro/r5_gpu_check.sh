#!/bin/bash
# round-5 checkpoint: full GPU suite, LM tail micro-benchmark, workgroup split micro-benchmark, filter / stack
# VoxelGrid phase stamps (profiling builds), C4 U / GS sweep, then the A/B bench (default vs the listed variant)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r5_gpu_tests.txt 2>&1 || { tail -40 gpurun_out/r5_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/r5_gpu_tests.txt
timeout -k 10 60 python micro/lm_tail_bench.py || exit 1
timeout -k 10 60 python micro/split_bench.py micro/split_bench.so base > gpurun_out/r5_split_base.txt 2>&1 || { cat gpurun_out/r5_split_base.txt; exit 1; }
cat gpurun_out/r5_split_base.txt
ALOAM_LIB_PATH=micro/_var_rbst2/libaloam_hip.so timeout -k 10 300 python micro/rb_stamps.py 120 > gpurun_out/r5_rbst2.txt 2>&1 || { tail gpurun_out/r5_rbst2.txt; exit 1; }
ALOAM_LIB_PATH=micro/_var_vxts2/libaloam_hip.so timeout -k 10 180 python micro/vx_stamps.py 30 > gpurun_out/r5_vx_phases.txt 2>&1 || { tail gpurun_out/r5_vx_phases.txt; exit 1; }
cat gpurun_out/r5_rbst2.txt gpurun_out/r5_vx_phases.txt
bash micro/r5_c4u.sh || exit 1
STEPS="20 50" bash micro/r5_var_ab.sh "$@"
