#!/bin/bash
# Quick kernel-trace pass of a short bench run (no PMC): per-kernel / per-grid means into gpurun_out/<tag>/.
# usage: bash scripts/kernel_trace.sh <tag>
set -euo pipefail
TAG=${1:-quick}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
rm -rf /tmp/lrlq && mkdir -p /tmp/lrlq
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/lrlq -o run -- \
  python3 "$ROOT/bench.py" --steps 3 --warmup 2 --no-cpu-baseline --no-secondary > "$OUT/trace.log" 2>&1
find /tmp/lrlq -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
KT=$(find /tmp/lrlq -name "*kernel_trace.csv" | head -n 1)
python3 "$ROOT/scripts/trace_reduce.py" "$KT" > "$OUT/kernel_by_grid.csv"
