#!/bin/bash
# C3 pipeline throughput vs the LM workgroup cap (mapping solves want ~100 workgroups)
set -e
run() { echo "$1 $(env $1 timeout -k 10 200 python bench.py --steps 400 --no-cpu --c4-launches 0 --c4-reg-steps 0 2>/dev/null | grep -o '"value": [0-9.]*')"; }
for i in 1 2; do
  run ALOAM_LM_GMAX=64
  run ALOAM_LM_GMAX=128
done
