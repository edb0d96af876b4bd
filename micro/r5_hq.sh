#!/bin/bash
# dynamic heap queue in ls_sort: the mapping / sort parity GPU tests, then A/B against the previous library
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "map or sort or voxel or vox or line" > gpurun_out/r5_hq_tests.txt 2>&1 || { tail -30 gpurun_out/r5_hq_tests.txt; exit 1; }
tail -1 gpurun_out/r5_hq_tests.txt
STEPS="20 50" bash micro/r5_var_ab.sh micro/_var_hq0/libaloam_hip.so || exit 1
cat gpurun_out/r5_var_ab.txt
