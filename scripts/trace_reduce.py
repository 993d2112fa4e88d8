"""Per (kernel, grid) mean duration from a rocprofv3 --kernel-trace CSV (distinguishes the GEMMs of the
update by their grid).  ``tail_mean_us`` averages only each kernel's last TAIL launches (env TAIL, default 120 =
bench.py's 5 timed iterations x 24 env steps), i.e. the launches of bench.py's timed region, which is what its
HIP-event ``env_step_kernel_ms`` averages.  usage: python scripts/trace_reduce.py <kernel_trace.csv> [name-filter]"""
import os
import csv
import sys
from collections import defaultdict

path = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else "lrl::"
agg = defaultdict(list)
with open(path) as f:
    for r in csv.DictReader(f):
        name = r["Kernel_Name"]
        if filt not in name:
            continue
        grid = tuple(r.get(k, "") for k in ("Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z"))
        if grid == ("", "", ""):
            grid = (r.get("Grid_Size", ""),)
        agg[(name[:70], grid)].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
tail = int(os.environ.get("TAIL", "120"))
rows = sorted(((k, [d for _, d in sorted(v)]) for k, v in agg.items()), key=lambda kv: -sum(kv[1]))
print("kernel,grid,calls,mean_us,total_ms,tail_mean_us")
for (name, grid), v in rows:
    t = v[-tail:]
    print(f'"{name}","{"x".join(grid)}",{len(v)},{sum(v) / len(v) / 1e3:.1f},{sum(v) / 1e6:.2f},'
          f'{sum(t) / len(t) / 1e3:.1f}')
