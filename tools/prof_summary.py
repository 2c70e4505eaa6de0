"""Summarise a rocprofv3 kernel_stats.csv: top kernels by total time."""
import csv
import sys

path = sys.argv[1]
n_upd = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:30]:
    print(f"{float(r['TotalDurationNs'])/1e6/n_upd:9.3f}ms/upd {int(r['Calls']):6d} calls "
          f"avg {float(r['AverageNs'])/1e3:9.2f}us {float(r['TotalDurationNs'])/tot*100:5.1f}%  "
          f"{r['Name'][:100]}")
print("total ms/upd", tot / 1e6 / n_upd)
