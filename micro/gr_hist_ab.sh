#!/bin/bash
# k_gr_hist A/B (ALOAM_GR_PLAIN bits: pass 1 / pass 2 with plain LDS atomics): kernel trace of the C4 build per setting
set -o pipefail
R=$PWD
for v in 0 2 4 6; do
  ( cd /tmp && export TMPDIR=/tmp && ALOAM_GR_PLAIN=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/grh_$v -o run --output-format csv -- python3 $R/bench.py --c4-only --c4-launches 3 ) > gpurun_out/grh_$v.log 2>&1 || { tail -5 gpurun_out/grh_$v.log; exit 1; }
  python3 - $v <<'PY'
import csv, sys
rows = list(csv.DictReader(open(f"gpurun_out/grh_{sys.argv[1]}/run_kernel_stats.csv")))
print(sys.argv[1], {r["Name"][7:25]: round(float(r["AverageNs"]) / 1e3, 1) for r in rows if "k_gr_hist" in r["Name"] or "k_gr_scatter" in r["Name"]})
PY
done
