"""Per-queue kernel time per frame of a rocprofv3 kernel trace of bench.py (profiling aid).
usage: queue_stats.py trace.csv [first_frame last_frame]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
lf = [i for i, r in enumerate(rows) if "k_line_features" in r["Kernel_Name"]]
f0, f1 = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (10, min(34, len(lf) - 1))
a, b, nf = lf[f0], lf[f1], f1 - f0
byq = collections.defaultdict(lambda: collections.defaultdict(lambda: [0, 0.0]))
busy = collections.defaultdict(float)
for r in rows[a:b]:
    q = r["Queue_Id"]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    n = r["Kernel_Name"].split("(")[0].replace("void ", "")[:50]
    if "rocprim" in n:
        n = "rocprim"
    byq[q][n][0] += 1
    byq[q][n][1] += d
    busy[q] += d
print("wall per frame us", round((int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1e3 / nf, 1))
for q in byq:
    print("QUEUE", q, "busy us/frame", round(busy[q] / nf, 1), "launches/frame", round(sum(v[0] for v in byq[q].values()) / nf, 1))
    for n, (c, d) in sorted(byq[q].items(), key=lambda x: -x[1][1])[:16]:
        print(f"   {n:50s} {c / nf:6.1f} {d / c:8.2f}us {d / nf:8.1f}us/f")
