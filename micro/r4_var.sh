#!/bin/bash
# C3 pipeline (STEPS) with the default library and the listed variant libraries (timing experiments)
set -o pipefail
mkdir -p gpurun_out
B="--no-cpu --c4-launches 0 --c4-reg-steps 0 --no-traffic"
for st in ${STEPS:-50 200}; do
  for v in "" "$@"; do
    ALOAM_LIB_PATH=$v timeout -k 10 240 python bench.py --steps $st $B > gpurun_out/r4_v.json 2>gpurun_out/r4_v.err || exit 1
    python - "$st" "$v" <<'PY' | tee -a gpurun_out/r4_var.txt
import json, sys
d = json.loads(open("gpurun_out/r4_v.json").read().strip().splitlines()[-1])
c = d["config"]
print(sys.argv[1], sys.argv[2] or "default", d["value"], {k: c.get("tictoc_ms", {}).get(k) for k in ("filter time", "mapping optimization time", "map prepare time", "seperate points time")})
PY
  done
done
