#!/bin/bash
# round-5 A/B on one box: C4 search (tile vs two-phase), C3 pipeline of this tree vs the round-3 tree
# (micro/_var_r3tree: `git archive 05beba1`, built in place) at the driver's 20-step config and 50 steps.
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r5_ab.txt
: > $O
for t in 0 1; do
  ALOAM_KNN_TILE=$t timeout -k 10 120 python bench.py --c4-only --c4-launches 50 > gpurun_out/r5_c4_$t.json 2>&1 || exit 1
  echo "c4 tile=$t $(tail -1 gpurun_out/r5_c4_$t.json)" >> $O
done
B="--no-cpu --c4-launches 0 --c4-reg-steps 0 --no-traffic"
summ() {
python - "$1" "$2" <<'PY' >> gpurun_out/r5_ab.txt
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = d["config"]; ss = d.get("steady_state") or {}
print(sys.argv[2], d["steps"], d["value"], json.dumps(c.get("tictoc_ms")), "steady", ss.get("scans_per_s"), json.dumps(ss.get("tictoc_ms")))
PY
}
for rep in 1 2; do
  for tree in . micro/_var_r3tree; do
    for st in 20 50; do
      (cd $tree && timeout -k 10 240 python bench.py --steps $st --warmup 5 $B) > gpurun_out/r5_b.json 2>gpurun_out/r5_b.err || { tail -5 gpurun_out/r5_b.err; exit 1; }
      summ gpurun_out/r5_b.json "$tree"
    done
  done
done
cat $O
