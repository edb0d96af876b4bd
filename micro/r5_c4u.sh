#!/bin/bash
# C4 search: loads in flight per lane (ALOAM_KNN_U 4 / 8) x lanes per query (ALOAM_KNN_GS2 8 / 16), 50 launches each
set -o pipefail
for u in 4 8; do for gs in 8 16; do
  ALOAM_KNN_U=$u ALOAM_KNN_GS2=$gs timeout -k 10 120 python bench.py --c4-only --c4-launches 50 2>&1 | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['c4']; print('U=$u GS2=$gs', c['kernel'], round(c['ms']*1e3,2), 'us', round(c['streamed']/(c['ms']*1e-3)/16.8e12,4))" || exit 1
done; done
