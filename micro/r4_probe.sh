#!/bin/bash
# round-4 probe: ls_sort phase costs, and the C3 pipeline with / without the heap sorts (timing only)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
#timeout -k 10 120 python micro/ls_bench.py 1300 2000 4000 6000 10000 > gpurun_out/r4_lsbench.txt 2>&1 || exit 1
B="--no-cpu --c4-launches 0 --c4-reg-steps 0 --no-traffic"
for st in 50 200; do
  for v in "" micro/_var_noheap/libaloam_hip.so; do
    echo "steps $st lib=$v" >> gpurun_out/r4_probe.txt
    ALOAM_LIB_PATH=$v timeout -k 10 240 python bench.py --steps $st $B > gpurun_out/r4_b.json 2>gpurun_out/r4_b.err || exit 1
    python - >> gpurun_out/r4_probe.txt <<'PY'
import json
d = json.loads(open("gpurun_out/r4_b.json").read().strip().splitlines()[-1])
c = d["config"]
print(d["value"], {k: c.get("tictoc_ms", {}).get(k) for k in ("filter time", "mapping optimization time", "map prepare time", "seperate points time", "whole mapping time")})
PY
  done
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_mapping.py "tests/test_gpu_parity.py::test_mapping_frames_teacher_forced" > gpurun_out/r4_maptests.txt 2>&1
