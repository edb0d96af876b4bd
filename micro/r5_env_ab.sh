#!/bin/bash
# C3 pipeline at 20 / 50 steps (the driver's config: warmup 5) for each "name:ENV=VAL ..." spec, twice, interleaved
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r5_env_ab.txt
: > $O
B="--no-cpu --c4-launches 0 --c4-reg-steps 0 --no-traffic"
for rep in 1 2; do
for st in ${STEPS:-20 50}; do
  for spec in "$@"; do
    name=${spec%%:*}; envs=${spec#*:}
    env $envs timeout -k 10 240 python bench.py --steps $st --warmup 5 $B > gpurun_out/r5_e.json 2>gpurun_out/r5_e.err || { tail -5 gpurun_out/r5_e.err; exit 1; }
    python - "$st" "$name" <<'PY' >> $O
import json, sys
d = json.loads(open("gpurun_out/r5_e.json").read().strip().splitlines()[-1])
c = d["config"]; ss = d.get("steady_state") or {}
keys = ("filter time", "mapping optimization time", "map prepare time", "seperate points time", "whole mapping time")
print(sys.argv[1], sys.argv[2], d["value"], {k: c.get("tictoc_ms", {}).get(k) for k in keys}, "| steady", ss.get("scans_per_s"),
      {k: (ss.get("tictoc_ms") or {}).get(k) for k in keys[:3]})
PY
  done
done
done
cat $O
