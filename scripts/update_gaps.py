"""Idle gaps of the update's main stream (development helper): from a rocprofv3 --kernel-trace CSV of bench.py, take
the last complete update (ppo_head_kernel launches up to the next env-step launch), find the stream that ran the
heads, and list every gap over 3 us on it with the kernels either side and what the other streams ran meanwhile;
then the gap total by (before -> after) pair.
usage: python scripts/update_gaps.py <kernel_trace.csv> [min_gap_us]"""
import csv
import sys
from collections import defaultdict

min_gap = float(sys.argv[2]) if len(sys.argv) > 2 else 3.0
rows = []
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        q = r.get("Stream_Id") or r.get("Queue_Id") or "0"
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][:70], q))
rows.sort()
heads = [i for i, k in enumerate(rows) if "ppo_head_kernel" in k[2]]
envs = [i for i, k in enumerate(rows) if "env_step_kernel" in k[2]]
if not heads:
    sys.exit("no ppo_head_kernel launches in the trace")
last_head = heads[-1]
# start of that update: the first head after the last env step before it
prev_env = max([e for e in envs if e < last_head], default=-1)
first = min(h for h in heads if h > prev_env)
nxt_env = min([e for e in envs if e > last_head], default=len(rows))
upd = rows[first:nxt_env]
main = rows[first][3]
t0 = upd[0][0]
ms = [k for k in upd if k[3] == main]
others = [k for k in upd if k[3] != main]
print(f"update: {len(upd)} kernels, {(upd[-1][1] - t0) / 1e3:.3f} ms; main stream {main}: {len(ms)} kernels, "
      f"busy {sum(k[1] - k[0] for k in ms) / 1e3:.3f} ms")
for q in sorted({k[3] for k in others}):
    sel = [k for k in others if k[3] == q]
    print(f"  stream {q}: {len(sel)} kernels, busy {sum(k[1] - k[0] for k in sel) / 1e3:.3f} ms")
pairs = defaultdict(lambda: [0, 0.0])
print("gaps on the main stream (start_us rel. to update, gap_us, before -> after | other streams running):")
total = 0.0
for a, b in zip(ms, ms[1:]):
    gap = (b[0] - a[1]) / 1e3
    if gap < min_gap:
        continue
    total += gap
    over = [k for k in others if k[0] < b[0] and k[1] > a[1]]
    cov = sum(min(k[1], b[0]) - max(k[0], a[1]) for k in over) / 1e3
    key = (a[2], b[2])
    pairs[key][0] += 1
    pairs[key][1] += gap
    names = ", ".join(sorted({k[2].replace("void lrl::", "").replace("lrl::", "")[:40] for k in over}))
    print(f"{(a[1] - t0) / 1e3:9.1f} {gap:7.1f}  {a[2][-45:]} -> {b[2][-45:]} | {cov:.1f} us: {names}")
print(f"total main-stream gaps >= {min_gap} us: {total:.1f} us")
for (a, b), (n, g) in sorted(pairs.items(), key=lambda kv: -kv[1][1])[:12]:
    print(f"{g:8.1f} us over {n:3d}: {a[-50:]} -> {b[-50:]}")
