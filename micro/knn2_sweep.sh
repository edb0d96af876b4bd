#!/bin/bash
# C4 search sweep: fine-cell fraction x lanes per query of the two-phase k-NN (bench.py --c4-only lines,
# 100 timed launches each so the clocks have ramped)
set -e
mkdir -p gpurun_out
for gs in 8 4 16; do
  echo "single gs=$gs $(ALOAM_KNN_GS=$gs ALOAM_KNN_FINE=0 timeout -k 10 120 python bench.py --c4-only --c4-launches 100)"
done
for gs in 2 4 8 16; do
  for f in 0.25 0.3 0.4; do
    echo "gs=$gs fine=$f $(ALOAM_KNN_GS2=$gs ALOAM_KNN_FINE=$f timeout -k 10 120 python bench.py --c4-only --c4-launches 100)"
  done
done
