"""Turn the per-kernel PMC means of scripts/gpu_profile.sh into HBM bytes per launch.

Corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE and WRITE_SIZE are KiB; on gfx950 FETCH_SIZE
counts half the bytes of wide streaming reads, so it is doubled.  The calibration copy (512 MiB read +
512 MiB written, scripts/pmc_calibrate.py) is kept next to the numbers to show both corrections hold.
usage: python scripts/pmc_summary.py gpurun_out/<tag> > profiles/<tag>_pmc.json
"""
import csv
import json
import os
import sys

d = sys.argv[1]


def load(name):
    out = {}
    with open(os.path.join(d, name)) as f:
        for r in csv.DictReader(f):
            out[r["kernel"]] = (int(r["dispatches"]), float(r["mean"]))
    return out


fetch, write = load("pmc_FETCH_SIZE.csv"), load("pmc_WRITE_SIZE.csv")
cf, cw = load("cal_FETCH_SIZE.csv"), load("cal_WRITE_SIZE.csv")
cal_f = [v for k, v in cf.items() if "copyBuffer" in k or "copy" in k]
cal_w = [v for k, v in cw.items() if "copyBuffer" in k or "copy" in k]
res = {"units": "bytes per launch (FETCH_SIZE KiB x 1024 x 2 + WRITE_SIZE KiB x 1024)",
       "calibration": {"expected_bytes": 512 * 2 ** 20,
                       "fetch_bytes_corrected": cal_f[0][1] * 1024 * 2 if cal_f else None,
                       "write_bytes": cal_w[0][1] * 1024 if cal_w else None},
       "kernels": {}}
for k in fetch:
    if "lrl::" not in k:
        continue
    short = k.split("(")[0].replace("void ", "")
    fb = fetch[k][1] * 1024 * 2
    wb = write.get(k, (0, 0.0))[1] * 1024
    res["kernels"][short] = {"dispatches": fetch[k][0], "fetch_bytes": fb, "write_bytes": wb,
                             "traffic_bytes": fb + wb}
json.dump(res, sys.stdout, indent=1)
print()
