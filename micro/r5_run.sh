#!/bin/bash
# round-5 check: heap micro-benchmark, mapping / sort parity GPU tests, then the C3 pipeline at the driver's
# 20-step config and 50 steps with the default library and the listed variant libraries (ALOAM_LIB_PATH)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
O=gpurun_out/r5_run.txt
: > $O
timeout -k 10 200 python micro/heap_bench.py 64 300 1000 3000 >> $O 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_mapping.py tests/test_gpu_parity.py \
  -k "mapping or cube or c5 or voxel or pipeline_sequence or scan_registration or tied" > gpurun_out/r5_tests.txt 2>&1 || { tail -30 gpurun_out/r5_tests.txt; exit 1; }
tail -2 gpurun_out/r5_tests.txt >> $O
B="--no-cpu --c4-launches 0 --c4-reg-steps 0 --no-traffic"
for st in ${STEPS:-20 50}; do
  for v in "" "$@"; do
    ALOAM_LIB_PATH=$v timeout -k 10 240 python bench.py --steps $st --warmup 5 $B > gpurun_out/r5_v.json 2>gpurun_out/r5_v.err || { tail -5 gpurun_out/r5_v.err; exit 1; }
    python - "$st" "$v" <<'PY' >> $O
import json, sys
d = json.loads(open("gpurun_out/r5_v.json").read().strip().splitlines()[-1])
c = d["config"]; ss = d.get("steady_state") or {}
keys = ("filter time", "mapping optimization time", "map prepare time", "seperate points time", "solver time", "mapping solver time", "whole mapping time")
print(sys.argv[1], sys.argv[2] or "default", d["value"], {k: c.get("tictoc_ms", {}).get(k) for k in keys}, "| steady", ss.get("scans_per_s"),
      {k: (ss.get("tictoc_ms") or {}).get(k) for k in keys})
PY
  done
done
cat $O
