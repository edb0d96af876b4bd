#!/bin/bash
# pipeline throughput vs per-stage CU partition (profiling aid)
set -e
mkdir -p gpurun_out
: > gpurun_out/cu_summary.txt
for K in 0 128 96 112 144 160 128; do
  ALOAM_PIPE_CU_SPLIT=$K timeout -k 10 150 python bench.py --no-cpu --c4-launches 0 --c4-reg-steps 0 --steps 100 > gpurun_out/cu.log 2>&1
  python -c "
import json;d=json.loads(open('gpurun_out/cu.log').read().strip().splitlines()[-1]);print('K=$K',d['value'],d['ms_per_step'])" >> gpurun_out/cu_summary.txt
done
