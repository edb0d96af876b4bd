#!/bin/bash
# C3 pipeline at STEPS (driver config: warmup 5), default library and the listed variant libraries, twice interleaved
set -o pipefail
O=gpurun_out/r5_var_ab.txt
: > $O
B="--no-cpu --c4-launches 0 --c4-reg-steps 0 --no-traffic"
for rep in 1 2; do
for st in ${STEPS:-20 50}; do
  for v in "" "$@"; do
    ALOAM_LIB_PATH=$v timeout -k 10 240 python bench.py --steps $st --warmup 5 $B > gpurun_out/r5_v.json 2>gpurun_out/r5_v.err || { tail -5 gpurun_out/r5_v.err; exit 1; }
    python - "$st" "$v" <<'PY' >> $O
import json, sys
d = json.loads(open("gpurun_out/r5_v.json").read().strip().splitlines()[-1])
c = d["config"]; ss = d.get("steady_state") or {}
keys = ("filter time", "mapping optimization time", "mapping solver time", "solver time", "map prepare time", "whole mapping time")
print(sys.argv[1], sys.argv[2] or "default", d["value"], {k: c.get("tictoc_ms", {}).get(k) for k in keys}, "| steady", ss.get("scans_per_s"),
      {k: (ss.get("tictoc_ms") or {}).get(k) for k in keys[:3]})
PY
  done
done
done
cat $O
