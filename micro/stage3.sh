#!/bin/bash
# 2- vs 3-stage pipeline with CU partitions (profiling aid)
set -e
mkdir -p gpurun_out
: > gpurun_out/st3_summary.txt
run() { local name=$1; shift; env "$@" timeout -k 10 150 python bench.py --no-cpu --c4-launches 0 --c4-reg-steps 0 --steps 100 $ARGS > gpurun_out/st3.log 2>&1; python -c "
import json;d=json.loads(open('gpurun_out/st3.log').read().strip().splitlines()[-1]);print('$name',d['value'],d['ms_per_step'])" >> gpurun_out/st3_summary.txt; }
ARGS="" run s2 X=1
ARGS="--stages 3" run s3_128_shared ALOAM_PIPE_CU_SPLIT=128 ALOAM_PIPE_CU_SPLIT3=128
ARGS="--stages 3" run s3_128_64 ALOAM_PIPE_CU_SPLIT=128 ALOAM_PIPE_CU_SPLIT3=64
ARGS="--stages 3" run s3_144_shared ALOAM_PIPE_CU_SPLIT=144 ALOAM_PIPE_CU_SPLIT3=144
ARGS="" run s2b X=1
