#!/bin/bash
# C4 registration time vs association regime (profiling aid)
set -e
mkdir -p gpurun_out
: > gpurun_out/nb_summary.txt
for v in "ALOAM_S2M_BATCH_MIN=1000000000" "ALOAM_S2M_NB=2" "ALOAM_S2M_NB=4" "ALOAM_S2M_NB=8"; do
  env $v timeout -k 10 150 python bench.py --c4-reg-only --c4-reg-steps 20 > gpurun_out/nb.log 2>&1
  python -c "
import json;d=json.loads(open('gpurun_out/nb.log').read().strip().splitlines()[-1])['c4_registration'];print('$v',d['ms_per_registration'],d['pose_err_m'])" >> gpurun_out/nb_summary.txt
done
