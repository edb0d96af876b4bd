#!/bin/bash
# one-launch s2m Solve at world 1: s2m GPU tests, then the C4 registration rate: one-launch Solve with 256 / 128
# workgroups vs the pass launches
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_s2m.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r5_s2m_tests.txt 2>&1 || { tail -40 gpurun_out/r5_s2m_tests.txt; exit 1; }
tail -1 gpurun_out/r5_s2m_tests.txt
for rep in 1 2; do for v in "1 256" "1 128" "0 256"; do
  set -- $v
  ALOAM_S2M_PERSIST=$1 ALOAM_S2M_SOLVE_G=$2 timeout -k 10 200 python bench.py --c4-reg-only --c4-reg-steps 10 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read())['c4_registration']; print('persist=$1 G=$2', d['value'], 'reg/s', d['ms_per_registration'], 'ms', d['pose_err_m'])" || exit 1
done; done
