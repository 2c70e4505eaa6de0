"""Average PMC counter values per kernel over the passes under a pmc dir."""
import collections
import csv
import glob
import re
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{root}/p*/*counter_collection.csv")):
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"]
        m = re.search(r"ml(?:::|\d+)(\w+?_kernel)", k)
        name = m.group(1) if m else k[:40]
        if "IDF16b" in k:
            name += "<bf16" + ("," + ",".join(re.findall(r"Li(\d+)E", k)) if "Li" in k else "") + ">"
        vals[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
for name, cs in vals.items():
    print(name)
    for c, v in sorted(cs.items()):
        print(f"   {c:24s} {sum(v)/len(v):16.1f}  (n={len(v)})")
