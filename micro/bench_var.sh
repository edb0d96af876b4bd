#!/bin/bash
# bench variance across timed-region lengths (profiling aid)
set -e
mkdir -p gpurun_out
: > gpurun_out/var_summary.txt
for steps in 50 100 200 50 100 200; do
  timeout -k 10 150 python bench.py --no-cpu --c4-launches 0 --c4-reg-steps 0 --steps $steps > gpurun_out/var.log 2>&1
  python -c "
import json;d=json.loads(open('gpurun_out/var.log').read().strip().splitlines()[-1]);print($steps,d['value'],d['ms_per_step'])" >> gpurun_out/var_summary.txt
done
