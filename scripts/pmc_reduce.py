"""Reduce a rocprofv3 counter_collection.csv to per-kernel (dispatches, mean, min, max) of one counter."""
import csv
import sys
from collections import defaultdict

path, counter = sys.argv[1], sys.argv[2]
vals = defaultdict(list)
with open(path) as f:
    for row in csv.DictReader(f):
        if row.get("Counter_Name") != counter:
            continue
        grid = row.get("Grid_Size") or "x".join(row.get(k, "") for k in ("Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z"))
        vals[row["Kernel_Name"]].append(float(row["Counter_Value"]))
        if grid:
            vals[row["Kernel_Name"].split("(")[0] + "@" + grid].append(float(row["Counter_Value"]))
w = csv.writer(sys.stdout)
w.writerow(["kernel", "counter", "dispatches", "mean", "min", "max"])
for k, v in sorted(vals.items(), key=lambda kv: -sum(kv[1])):
    w.writerow([k[:160], counter, len(v), sum(v) / len(v), min(v), max(v)])
