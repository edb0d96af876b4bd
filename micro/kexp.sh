#!/bin/bash
# kernel-time experiments (profiling aid): rocprofv3 kernel-trace of a short serial bench per env setting,
# prints avg duration of the named kernels. Experiments that skip work give invalid results by design.
set -e
R=$PWD
mkdir -p $R/gpurun_out
: > $R/gpurun_out/kexp_summary.txt
for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}
  cd /tmp && export TMPDIR=/tmp
  env $envs timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/kexp_$name -o run --output-format csv -- python3 $R/bench.py --mode ${KEXP_MODE:-serial} --steps 20 --no-cpu --c4-launches 0 --c4-reg-steps 0 --no-traffic > $R/gpurun_out/kexp_$name.log 2>&1
  cd $R
  python3 - $name >> gpurun_out/kexp_summary.txt <<'PY'
import csv, sys
n = sys.argv[1]
rows = list(csv.DictReader(open(f"gpurun_out/kexp_{n}/run_kernel_stats.csv")))
for r in rows:
    k = r["Name"]
    if any(s in k for s in ("k_odom_search", "k_map_assoc", "k_lm_coop", "k_line_features")):
        print(n, k.split("(")[0][:40], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2))
PY
done
cat gpurun_out/kexp_summary.txt
