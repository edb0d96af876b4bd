#!/bin/bash
# filter phase stamps (rb_stamps, 200 frames) and mapping LM pass stamps (lm_stamps, round 4) on profiling builds
set -o pipefail
mkdir -p gpurun_out
ALOAM_LIB_PATH=micro/_var_rbst/libaloam_hip.so timeout -k 10 300 python micro/rb_stamps.py 200 > gpurun_out/r5_rbst.txt 2>&1 || { tail gpurun_out/r5_rbst.txt; exit 1; }
ALOAM_LIB_PATH=micro/_var_lm20/libaloam_hip.so timeout -k 10 200 python micro/lm_stamps.py 60 > gpurun_out/r5_lm20.txt 2>&1 || { tail gpurun_out/r5_lm20.txt; exit 1; }
cat gpurun_out/r5_rbst.txt gpurun_out/r5_lm20.txt
