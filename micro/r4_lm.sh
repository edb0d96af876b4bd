#!/bin/bash
# LM exchange check: LM / odometry / mapping parity tests, solve-16 pass stamps, then the C3 bench (STEPS)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_mapping.py -k "lm or solve or odom or mapping or c5 or pipeline_sequence or cpp_host or cu_mask or knn" > gpurun_out/r4_lm_tests.txt 2>&1 || { tail -30 gpurun_out/r4_lm_tests.txt; exit 1; }
tail -2 gpurun_out/r4_lm_tests.txt
ALOAM_LIB_PATH=/root/repo/micro/_var_lm16/libaloam_hip.so timeout -k 10 200 python micro/lm_stamps.py 60 > gpurun_out/lm16.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/lm16.txt
B="--no-cpu --c4-launches 0 --c4-reg-steps 0 --no-traffic"
for st in ${STEPS:-200}; do
  timeout -k 10 240 python bench.py --steps $st $B > gpurun_out/r4_b.json 2>gpurun_out/r4_b.err || exit 1
  python - <<'PY' | tee -a gpurun_out/r4_run.txt
import json
d = json.loads(open("gpurun_out/r4_b.json").read().strip().splitlines()[-1])
c = d["config"]
print(d["steps"], d["value"], {k: c.get("tictoc_ms", {}).get(k) for k in ("filter time", "mapping optimization time", "optimization twice time", "whole laserOdometry time", "whole mapping time")})
PY
done
# C4 search: tile kernel (default) vs ALOAM_KNN_TILE=0
for t in 1 0; do
  ALOAM_KNN_TILE=$t timeout -k 10 240 python bench.py --c4-only --c4-launches 20 --no-traffic --no-cpu > gpurun_out/r4_c4_$t.json 2>gpurun_out/r4_c4_$t.err || exit 1
  python -c "import json,sys; d=json.loads(open('gpurun_out/r4_c4_$t.json').read().strip().splitlines()[-1]); print('tile $t', d.get('roofline'))" | tee -a gpurun_out/r4_run.txt
done
