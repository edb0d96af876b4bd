#!/bin/bash
# C4 registration: association batch (points per wave pass = 8 NB) sweep
set -e
for nb in 2 4 8 2; do
  echo "nb=$nb $(ALOAM_S2M_NB=$nb timeout -k 10 120 python bench.py --c4-reg-only --c4-reg-steps 30 2>/dev/null)"
done
