#!/bin/bash
# C3 pipeline experiment matrix (profiling aid): one bench line per env setting; ALOAM_EXP/ALOAM_ODOM_EXP
# settings skip work (results invalid) and only bound what a stage costs.
set -e
mkdir -p gpurun_out
B="timeout -k 10 150 python bench.py --no-cpu --c4-launches 0 --c4-reg-steps 0 --steps 100"
run() { local name=$1; shift; env "$@" $B $EXTRA > gpurun_out/ex_$name.log 2>&1; python -c "
import json;d=json.loads(open('gpurun_out/ex_$name.log').read().strip().splitlines()[-1]);print('$name',d['value'],d['ms_per_step'],d['config']['stage_ms'])" | tee -a gpurun_out/ex_summary.txt; }
: > gpurun_out/ex_summary.txt
for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}
  run $name $envs
done
