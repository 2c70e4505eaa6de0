"""Per-dispatch durations of one kernel from a rocprofv3 kernel_trace.csv,
split by dispatch parity (the ML_PROBE_WG_TWICE variant launches the
weight-gradient kernel twice back to back: even = first, odd = second).
usage: wg_pairs.py kernel_trace.csv [name_substring]"""
import csv
import statistics
import sys

path = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else "wgrad_kernel"
rows = list(csv.DictReader(open(path)))
nk = "Kernel_Name" if "Kernel_Name" in rows[0] else "Name"
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
     for r in sorted(rows, key=lambda r: int(r["Start_Timestamp"])) if pat in r[nk]]
ev, od = d[0::2], d[1::2]
print(f"{pat}: {len(d)} dispatches; first of pair median {statistics.median(ev):.2f} us "
      f"mean {statistics.mean(ev):.2f}; second median {statistics.median(od):.2f} us "
      f"mean {statistics.mean(od):.2f}")
