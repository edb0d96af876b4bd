#!/bin/bash
# experiment matrix for the C3 pipeline (profiling aid, not part of the product): one bench line per setting
set -e
mkdir -p gpurun_out
B="timeout -k 10 150 python bench.py --no-cpu --c4-launches 0 --c4-reg-steps 0 --steps 100"
run() { local name=$1; shift; env "$@" $B $EXTRA > gpurun_out/mx_$name.log 2>&1; python -c "
import json;d=json.loads(open('gpurun_out/mx_$name.log').read().strip().splitlines()[-1]);print('$name',d['value'],d['ms_per_step'])" | tee -a gpurun_out/mx_summary.txt; }
: > gpurun_out/mx_summary.txt
run q4 GPU_MAX_HW_QUEUES=4
run q8 GPU_MAX_HW_QUEUES=8
run q16 GPU_MAX_HW_QUEUES=16
EXTRA="--stages 3" run q8s3 GPU_MAX_HW_QUEUES=8
run q4b GPU_MAX_HW_QUEUES=4
