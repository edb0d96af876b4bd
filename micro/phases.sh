#!/bin/bash
# mapping phase times (ALOAM_MAP_PHASES) + bench value per env setting (profiling aid)
mkdir -p gpurun_out
for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}
  env ALOAM_MAP_PHASES=1 ALOAM_FRONT_PHASES=1 $envs timeout -k 10 150 python bench.py --no-cpu --c4-launches 0 --c4-reg-steps 0 --steps ${STEPS:-450} > gpurun_out/ph_$name.log 2> gpurun_out/ph_$name.err || exit 1
  echo "$name $(grep -a "front phases" gpurun_out/ph_$name.err | tail -1 | sed "s/.aloam front phases. us per scan://") || $(grep -a "map phases" gpurun_out/ph_$name.err | tail -1 | sed "s/.aloam map phases. us per frame://") | $(python -c "import json;d=json.loads(open('gpurun_out/ph_$name.log').read().strip().splitlines()[-1]);print('bench',d['value'])")"
done
