"""Per-stream timeline of a rocprofv3 kernel trace: usage  timeline.py trace.csv [t0_frac] [window_us]
Prints kernels (stream, start offset us, duration us, name) in a window, then busy time per stream."""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
t_first, t_last = int(rows[0]["Start_Timestamp"]), int(rows[-1]["End_Timestamp"])
t0 = t_first + int(float(sys.argv[2] if len(sys.argv) > 2 else 0.5) * (t_last - t_first))
win = float(sys.argv[3] if len(sys.argv) > 3 else 3000) * 1e3
busy = {}
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if s < t0 or s > t0 + win:
        continue
    q = r["Queue_Id"]
    busy[q] = busy.get(q, 0) + (e - s)
    print(f"q{q:>3} +{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f}  {r['Kernel_Name'][:70]}")
print({k: round(v / 1e3, 1) for k, v in busy.items()}, "window us", win / 1e3)
