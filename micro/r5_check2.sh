#!/bin/bash
# full GPU suite, A/B bench vs the listed library, C4 U / GS sweep, filter / stack VoxelGrid phase stamps
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r5_gpu_tests.txt 2>&1 || { tail -40 gpurun_out/r5_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/r5_gpu_tests.txt
STEPS="20 50" bash micro/r5_var_ab.sh "$@" || exit 1
bash micro/r5_c4u.sh || exit 1
ALOAM_LIB_PATH=micro/_var_vxts3/libaloam_hip.so timeout -k 10 180 python micro/vx_stamps.py 30 > gpurun_out/r5_vx_phases.txt 2>&1 || { tail gpurun_out/r5_vx_phases.txt; exit 1; }
tail -3 gpurun_out/r5_vx_phases.txt
ALOAM_LIB_PATH=micro/_var_rbst4/libaloam_hip.so timeout -k 10 300 python micro/rb_stamps.py 120 > gpurun_out/r5_rbst4.txt 2>&1 || { tail gpurun_out/r5_rbst4.txt; exit 1; }
cat gpurun_out/r5_rbst4.txt
