"""Every kernel (torch's too) of a rocprofv3 kernel trace in a window after the N-th launch of a named kernel:
start offset, duration, stream, name.  usage: python scripts/trace_window.py <kernel_trace.csv> <name> [n] [ms]"""
import csv
import sys

path, key = sys.argv[1], sys.argv[2]
nth = int(sys.argv[3]) if len(sys.argv) > 3 else 20
span = float(sys.argv[4]) if len(sys.argv) > 4 else 2.0
rows = []
with open(path) as f:
    for r in csv.DictReader(f):
        q = r.get("Stream_Id") or r.get("Queue_Id") or "0"
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), q, r["Kernel_Name"][:90]))
rows.sort()
hits = [r for r in rows if key in r[3]]
t0 = hits[min(nth, len(hits) - 1)][0]
for s, e, q, n in rows:
    if t0 <= s < t0 + span * 1e6:
        print(f"{(s - t0) / 1e3:9.1f},{(e - s) / 1e3:7.1f},{q},{n}")
