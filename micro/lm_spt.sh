#!/bin/bash
# pipeline throughput vs LM slots-per-thread grid sizing (profiling aid)
set -e
mkdir -p gpurun_out
: > gpurun_out/spt_summary.txt
for v in 1 2 4 8 1; do
  ALOAM_LM_SPT=$v timeout -k 10 150 python bench.py --no-cpu --c4-launches 0 --c4-reg-steps 0 --steps 100 > gpurun_out/spt.log 2>&1
  python -c "
import json;d=json.loads(open('gpurun_out/spt.log').read().strip().splitlines()[-1]);print('spt=$v',d['value'],d['ms_per_step'],d['config']['stage_ms'])" >> gpurun_out/spt_summary.txt
done
