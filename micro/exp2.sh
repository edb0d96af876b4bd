#!/bin/bash
# pipeline A/B (profiling aid): bench lines + ALOAM_PIPE_TIMING stage occupancy per env setting, 2 runs each
mkdir -p gpurun_out
: > gpurun_out/ex2_summary.txt
for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}
  for r in 1 2; do
    env ALOAM_PIPE_TIMING=1 $envs timeout -k 10 150 python bench.py --no-cpu --c4-launches 0 --c4-reg-steps 0 --steps ${STEPS:-300} > gpurun_out/ex2_$name.log 2>gpurun_out/ex2_$name.err || exit 1
    python -c "
import json;d=json.loads(open('gpurun_out/ex2_$name.log').read().strip().splitlines()[-1]);print('$name',d['value'],d['ms_per_step'])" | tr '\n' ' ' >> gpurun_out/ex2_summary.txt
    grep "aloam pipe" gpurun_out/ex2_$name.err | sed 's/.aloam pipe. per scan (us)://' >> gpurun_out/ex2_summary.txt
  done
done
cat gpurun_out/ex2_summary.txt
