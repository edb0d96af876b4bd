#!/bin/bash
# C4 registration per setting: pass launches (default) vs the one-launch Solve (ALOAM_S2M_PERSIST=1), then the
# group-mode exchanges (micro/s2m_xchg.py: host-ordered copies vs device exchange)
set -o pipefail
for v in 0 1 0 1; do
  ALOAM_S2M_PERSIST=$v timeout -k 10 200 python bench.py --c4-reg-only --c4-reg-steps 20 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1])['c4_registration']; print('persist', $v, d['ms_per_registration'], 'ms', d['pose_err_m'])" || exit 1
done
export GPU_MAX_HW_QUEUES=16
timeout -k 10 200 python -u micro/s2m_xchg.py host 2>/dev/null | tail -1 || exit 1
ALOAM_S2M_PEER=1 timeout -k 10 200 python -u micro/s2m_xchg.py device 2>/dev/null | tail -1 || exit 1
