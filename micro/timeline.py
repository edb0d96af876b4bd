"""Queue occupancy from a rocprofv3 kernel trace (profiles/prof.sh output): per hardware queue, the share
of the steady window (the middle of the run) covered by its kernels, and the kernels that fill it, so the
pipeline stage that bounds the step shows up as the queue near 100 %. Profiling aid only.

usage: python micro/timeline.py gpurun_out/NAME/run_kernel_trace.csv [top]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 8
ev = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"], r["Kernel_Name"].split("(")[0]) for r in rows))
t0, t1 = ev[0][0], ev[-1][1]
w0, w1 = t0 + (t1 - t0) * 0.3, t0 + (t1 - t0) * 0.7     # steady window
byq = collections.defaultdict(list)
for s, e, q, n in ev:
    if e > w0 and s < w1:
        byq[q].append((max(s, w0), min(e, w1), n))
span = w1 - w0
print(f"window {span / 1e6:.2f} ms")
for q, v in sorted(byq.items(), key=lambda kv: -sum(e - s for s, e, _ in kv[1])):
    busy, end = 0, 0
    for s, e, _ in v:                    # union of intervals (kernels of one queue may overlap)
        if e > end:
            busy += e - max(s, end)
            end = e
    tot = collections.Counter()
    for s, e, n in v:
        tot[n] += e - s
    print(f"queue {q}: busy {100 * busy / span:.1f} %  ({len(v)} kernels)")
    for n, t in tot.most_common(top):
        print(f"    {100 * t / span:5.1f} %  {n}")
