"""Per-kernel means of the SQ pass of scripts/gpu_profile.sh (gpurun_out/<tag>/sq_*.csv, one file per counter) as
one JSON: {kernel: {counter: mean per dispatch, "dispatches": n}}.
usage: python scripts/sq_summary.py gpurun_out/<tag> > profiles/<tag>_sq.json"""
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
out = {}
for path in sorted(glob.glob(os.path.join(d, "sq_*.csv"))):
    with open(path) as f:
        for row in csv.DictReader(f):
            k = out.setdefault(row["kernel"], {})
            k[row["counter"]] = float(row["mean"])
            k["dispatches"] = int(row["dispatches"])
print(json.dumps({"units": "per-launch means; SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_* / SQ_BUSY_CYCLES in quad-cycles "
                           "summed over waves (MI355X_MICROARCH.md)", "kernels": out}, indent=1))
