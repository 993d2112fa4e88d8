"""Summarise a $LRL_PARITY_STATS file (tests/helpers.py record_errors): per physics field, the largest kernel-vs-oracle
error over every compared step (non-excluded envs), its p99, and the fp64 oracle's own spread under fp32-size input
noise.  usage: python scripts/parity_stats_summary.py profiles/r4b_parity_stats.jsonl"""
import json
import sys

recs = [json.loads(l) for l in open(sys.argv[1])]
fields = ["pos", "quat", "dof_pos", "dof_vel", "lin_vel", "ang_vel", "contact"]
print(f"{len(recs)} compared steps, {sum(r['n'] for r in recs)} env-steps, {sum(r['excluded'] for r in recs)} excluded "
      f"(worst step {max(r['excluded'] / r['n'] for r in recs) * 100:.1f} %)")
print(f"{'field':8s} {'k-o abs max':>12s} {'k-o abs p99*':>12s} {'k-o scaled max':>14s} {'oracle abs max':>14s} "
      f"{'oracle scaled max':>17s}  worst step")
for f in fields:
    ko = [(r["kernel_vs_oracle"][f], r["tag"]) for r in recs if f in r["kernel_vs_oracle"]]
    osp = [r["oracle_spread"][f] for r in recs if "oracle_spread" in r and f in r["oracle_spread"]]
    worst = max(ko, key=lambda x: x[0]["abs_max"])
    print(f"{f:8s} {worst[0]['abs_max']:12.3e} {max(k['abs_p99'] for k, _ in ko):12.3e} "
          f"{max(k['scaled_max'] for k, _ in ko):14.3e} {max(o['abs_max'] for o in osp):14.3e} "
          f"{max(o['scaled_max'] for o in osp):17.3e}  {worst[1]}")
