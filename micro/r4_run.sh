#!/bin/bash
# round-4 check: mapping parity tests, then the C3 pipeline at 50 / 200 steps (filter / mapping TicToc)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T=${TESTS:-"tests/test_gpu_mapping.py tests/test_gpu_parity.py -k mapping or cube or c5 or voxel"}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_mapping.py tests/test_gpu_parity.py -k "mapping or cube or c5 or voxel or pipeline_sequence" > gpurun_out/r4_tests.txt 2>&1 || { tail -30 gpurun_out/r4_tests.txt; exit 1; }
tail -3 gpurun_out/r4_tests.txt
B="--no-cpu --c4-launches 0 --c4-reg-steps 0 --no-traffic"
for st in ${STEPS:-50 200}; do
  timeout -k 10 240 python bench.py --steps $st $B > gpurun_out/r4_b.json 2>gpurun_out/r4_b.err || exit 1
  python - <<'PY' | tee -a gpurun_out/r4_run.txt
import json
d = json.loads(open("gpurun_out/r4_b.json").read().strip().splitlines()[-1])
c = d["config"]
print(d["steps"], d["value"], {k: c.get("tictoc_ms", {}).get(k) for k in ("filter time", "mapping optimization time", "map prepare time", "seperate points time", "whole mapping time")}, "ate_pcl", d.get("ate_delta_vs_pcl_order_m"))
PY
done
