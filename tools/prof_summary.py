"""Summarise a rocprofv3 kernel_stats.csv: top kernels by total time.
usage: prof_summary.py kernel_stats.csv [num_updates]  (totals divided by
num_updates; the default 1 prints whole-run totals)."""
import csv
import sys

path = sys.argv[1]
n_upd = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:30]:
    print(f"{float(r['TotalDurationNs'])/1e6/n_upd:9.3f}ms {int(r['Calls']):6d} calls "
          f"avg {float(r['AverageNs'])/1e3:9.2f}us {float(r['TotalDurationNs'])/tot*100:5.1f}%  "
          f"{r['Name'][:100]}")
print("total ms", tot / 1e6 / n_upd, "(per update)" if n_upd != 1.0 else "(whole run)")
