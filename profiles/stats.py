import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
nf = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
tot = sum(float(r['TotalDurationNs']) for r in rows)
for r in rows[:int(sys.argv[3]) if len(sys.argv) > 3 else 30]:
    print(f"{r['Name'][:58]:58s} calls/f={int(r['Calls'])/nf:7.1f} avg_us={float(r['AverageNs'])/1e3:8.1f} us/frame={float(r['TotalDurationNs'])/1e3/nf:8.1f} {float(r['Percentage']):5.1f}%")
print("total us/frame", tot / 1e3 / nf)
