#!/bin/bash
# kernel durations of the PCL-order sort sites (micro/sort_probe.py) -> gpurun_out/sp/*
set -e
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/sp -o run --output-format csv -- python3 $R/micro/sort_probe.py > $R/gpurun_out/sp.log 2>&1
cd $R && python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/sp/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
by = collections.defaultdict(list)
for r in rows:
    n = r["Kernel_Name"]
    if any(k in n for k in ("k_line_features", "k_vox_pcl", "k_rb_cubevox")):
        by[n.split("(")[0]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
for n, v in by.items():
    print(n, len(v), " ".join(f"{x:.0f}" for x in v[:40]))
PY
