#!/bin/bash
# SQ stall breakdown of the GEMM micro-benchmark shapes (development tool): one rocprofv3 PMC pass
# (no traces), reduced per kernel@grid.  usage: bash scripts/sq_counters.sh <tag> [shape filter]
set -euo pipefail
TAG=${1:-sq}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
rm -rf /tmp/lrlsq
CS="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
GEMM_BENCH_FILTER="${2:-}" timeout -k 10 300 rocprofv3 --pmc $CS --output-format csv -d /tmp/lrlsq -o run -- \
  python3 "$ROOT/scripts/gemm_bench.py" > "$OUT/sq.log" 2>&1
F=$(find /tmp/lrlsq -name "*counter_collection.csv" | head -n 1)
for C in $CS; do python3 "$ROOT/scripts/pmc_reduce.py" "$F" "$C" | grep "@" > "$OUT/$C.csv" || true; done
ls "$OUT"
