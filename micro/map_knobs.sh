#!/bin/bash
# C3 pipeline throughput under mapping-stage knobs (one 400-scan run each)
set -e
run() { echo "$1 $(env $1 timeout -k 10 200 python bench.py --steps 400 --no-cpu --c4-launches 0 --c4-reg-steps 0 2>/dev/null | grep -o '"value": [0-9.]*')"; }
run ALOAM_NONE=0
run ALOAM_ASSOC_BLOCKS=256
run ALOAM_ASSOC_BLOCKS=1024
run ALOAM_MAP_U=2
run ALOAM_MAP_U=8
run ALOAM_LM_SPT=2
run ALOAM_NONE=0
