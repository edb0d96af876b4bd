#!/bin/bash
# C4 registration: fused vs split association (5-NN kernel + one-fit-per-lane kernel)
set -e
for sp in 0 1 0 1; do
  echo "split=$sp $(ALOAM_S2M_SPLIT=$sp timeout -k 10 120 python bench.py --c4-reg-only --c4-reg-steps 30 2>/dev/null | grep -o '"ms_per_registration": [0-9.]*')"
done
