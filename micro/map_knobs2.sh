#!/bin/bash
# C3 pipeline throughput: LM grid sizing and association knobs, interleaved with the default (noise)
set -e
run() { echo "$1 $(env $1 timeout -k 10 200 python bench.py --steps 400 --no-cpu --c4-launches 0 --c4-reg-steps 0 2>/dev/null | grep -o '"value": [0-9.]*')"; }
for i in 1 2; do
  run ALOAM_NONE=0
  run ALOAM_LM_SPT=4
  run ALOAM_ASSOC_BLOCKS=1024
  run ALOAM_MAP_U=2
done
