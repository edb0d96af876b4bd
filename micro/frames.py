"""Per-frame breakdown of the mapping queue from a rocprofv3 kernel trace (profiles/prof.sh output): frames are cut
at each k_map_prepare launch; for the frames in [a, b) prints the mean frame span (prepare to next prepare), the
busy time, the idle gaps, and the mean time per kernel name; then the same for the front queue over the same wall
window. Profiling aid only.

usage: python micro/frames.py gpurun_out/NAME/run_kernel_trace.csv a b [top]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
a, b = int(sys.argv[2]), int(sys.argv[3])
top = int(sys.argv[4]) if len(sys.argv) > 4 else 14
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"], r["Kernel_Name"].split("(")[0].replace("aloam::", ""))
            for r in rows)
mq = next(e[2] for e in ev if "k_map_prepare" in e[3])
m = [e for e in ev if e[2] == mq]
starts = [i for i, e in enumerate(m) if "k_map_prepare" in e[3]]
b = min(b, len(starts) - 1)
span = busy = 0
per = collections.Counter()
for f in range(a, b):
    seg = m[starts[f]:starts[f + 1]]
    t0, t1 = seg[0][0], m[starts[f + 1]][0]
    span += t1 - t0
    end = t0
    for s, e, _, n in seg:
        if e > end:
            busy += e - max(s, end)
            end = e
        per[n] += e - s
nf = b - a
w0, w1 = m[starts[a]][0], m[starts[b]][0]
print(f"mapping queue {mq}: frames {a}..{b - 1}: span {span / nf / 1e3:.1f} us/frame, busy {busy / nf / 1e3:.1f}, idle {(span - busy) / nf / 1e3:.1f}")
for n, t in per.most_common(top):
    print(f"   {t / nf / 1e3:8.1f} us  {n[:70]}")
byq = collections.defaultdict(collections.Counter)
for s, e, q, n in ev:
    if q != mq and s >= w0 and e <= w1:
        byq[q][n] += e - s
for q, c in byq.items():
    tot = sum(c.values())
    print(f"queue {q}: {tot / nf / 1e3:.1f} us/frame of kernels in the same window")
    for n, t in c.most_common(8):
        print(f"   {t / nf / 1e3:8.1f} us  {n[:70]}")
