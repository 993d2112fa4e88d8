"""Where an iteration's wall time goes, from a rocprofv3 --kernel-trace CSV of bench.py: per PPO iteration (split at
the first env-step launch after an update), the wall span, the time at least one kernel runs (union over streams),
the idle gaps, and the rollout / update spans; then the update's busy time per stream.
usage: python scripts/timeline.py <kernel_trace.csv>"""
import csv
import sys
from collections import defaultdict

rows = []
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        if "lrl::" not in r["Kernel_Name"]:
            continue
        q = r.get("Stream_Id") or r.get("Queue_Id") or "0"
        grid = r.get("Grid_Size_X") or r.get("Grid_Size") or ""
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60] + "@" + grid, q))
rows.sort()
# iterations: an env-step launch that follows a non-env, non-act kernel of the update starts one
iters, cur, in_update = [], [], False
for k in rows:
    is_env = "env_step_kernel" in k[2] or "shift_history" in k[2]
    if is_env and in_update and cur:
        iters.append(cur)
        cur = []
    if "ppo_head_kernel" in k[2]:
        in_update = True
    if is_env:
        in_update = False
    cur.append(k)
if cur:
    iters.append(cur)


def union(ks):
    busy, end = 0, None
    for s, e, _, _ in sorted(ks):
        if end is None or s > end:
            busy += e - s
            end = e
        elif e > end:
            busy += e - end
            end = e
    return busy


print("iter,wall_ms,busy_ms,idle_ms,rollout_ms,rollout_idle_ms,update_ms,update_idle_ms,kernels,gaps_over_5us_ms")
for i, it in enumerate(iters):
    t0, t1 = it[0][0], max(e for _, e, _, _ in it)
    busy = union(it)
    first_upd = next((s for s, _, n, _ in it if "ppo_head_kernel" in n), t1)
    # rollout: up to the last act / GAE launch before the first PPO head
    roll = [k for k in it if k[0] < first_upd]
    upd = [k for k in it if k[0] >= first_upd]
    # gaps
    gaps, end = 0, None
    for s, e, _, _ in sorted(it):
        if end is not None and s - end > 5000:
            gaps += s - end
        end = e if end is None else max(end, e)
    r_idle = (first_upd - t0) - union([(s, min(e, first_upd), n, q) for s, e, n, q in roll])
    u_idle = (t1 - first_upd) - union(upd) if upd else 0
    print(f"{i},{(t1 - t0) / 1e6:.3f},{busy / 1e6:.3f},{(t1 - t0 - busy) / 1e6:.3f},"
          f"{(first_upd - t0) / 1e6:.3f},{r_idle / 1e6:.3f},{(t1 - first_upd) / 1e6:.3f},{u_idle / 1e6:.3f},{len(it)},"
          f"{gaps / 1e6:.3f}")
# per-stream busy inside the updates of the last iterations
per = defaultdict(int)
for it in iters[-5:]:
    first_upd = next((s for s, _, n, _ in it if "ppo_head_kernel" in n), None)
    if first_upd is None:
        continue
    for q in set(k[3] for k in it):
        per[q] += union([k for k in it if k[3] == q and k[0] >= first_upd])
print("update busy per stream over the last 5 iterations (ms):", {q: round(v / 1e6 / 5, 3) for q, v in per.items()})
# one minibatch of the last full iteration's update, in launch order (stream, start offset, duration)
if len(iters) >= 2:
    it = iters[-2]
    heads = [k for k in it if "ppo_head_kernel" in k[2]]
    if len(heads) >= 3:
        t0, t1 = heads[1][0], heads[2][0]
        # from the end of the previous head's launch group to the next: the phase-1 tail, phase 2, phase 3/4 and
        # the next phase-1 head
        sel = [k for k in it if t0 - 2_000_000 <= k[0] < t1]
        base = sel[0][0]
        print("minibatch sequence: start_us,dur_us,stream,kernel")
        for s, e, n, q in sel:
            print(f"{(s - base) / 1e3:9.1f},{(e - s) / 1e3:7.1f},{q},{n}")
# the largest idle gaps inside the last full iteration's rollout (what ran before / after each)
if len(iters) >= 2:
    it = sorted(iters[-2])
    first_upd = next((s for s, _, n, _ in it if "ppo_head_kernel" in n), it[-1][1])
    roll = [k for k in it if k[0] < first_upd]
    gaps, end, prev = [], None, None
    for k in roll:
        if end is not None and k[0] > end:
            gaps.append((k[0] - end, prev[2].split("(")[0][-40:], k[2].split("(")[0][-40:]))
        if end is None or k[1] > end:
            end, prev = k[1], k
    gaps.sort(reverse=True)
    print("rollout gaps: count", len(gaps), "total_us", round(sum(g[0] for g in gaps) / 1e3, 1))
    agg = defaultdict(lambda: [0, 0])
    for d, a, b in gaps:
        agg[(a, b)][0] += d
        agg[(a, b)][1] += 1
    for (a, b), (d, c) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:12]:
        print(f"  {d / 1e3:8.1f} us over {c:3d} gaps: after {a} -> before {b}")
