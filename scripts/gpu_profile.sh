#!/bin/bash
# Round profile on the GPU box: kernel-trace stats + two separate PMC passes (FETCH_SIZE, WRITE_SIZE; the
# guide forbids combining them with traces and they do not fit one TCC pass). Only small CSVs are kept.
# usage: bash scripts/gpu_profile.sh <tag>
set -euo pipefail
TAG=${1:-r1}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
rm -rf /tmp/lrlprof && mkdir -p /tmp/lrlprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/lrlprof/trace -o run -- \
  python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-secondary > "$OUT/trace.log" 2>&1
find /tmp/lrlprof/trace -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
KT=$(find /tmp/lrlprof/trace -name "*kernel_trace.csv" | head -n 1)
python3 "$ROOT/scripts/trace_reduce.py" "$KT" > "$OUT/kernel_by_grid.csv"
python3 "$ROOT/scripts/timeline.py" "$KT" > "$OUT/timeline.csv"
[ "${NO_PMC:-0}" = 1 ] && exit 0
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d /tmp/lrlprof/$C -o run -- \
    python3 "$ROOT/bench.py" --steps 1 --warmup 1 --no-cpu-baseline --no-secondary > "$OUT/pmc_$C.log" 2>&1
  F=$(find /tmp/lrlprof/$C -name "*counter_collection.csv" | head -n 1)
  python3 "$ROOT/scripts/pmc_reduce.py" "$F" "$C" > "$OUT/pmc_$C.csv"
  timeout -k 10 120 rocprofv3 --pmc $C --output-format csv -d /tmp/lrlprof/cal_$C -o run -- \
    python3 "$ROOT/scripts/pmc_calibrate.py" > "$OUT/cal_$C.log" 2>&1
  F=$(find /tmp/lrlprof/cal_$C -name "*counter_collection.csv" | head -n 1)
  python3 "$ROOT/scripts/pmc_reduce.py" "$F" "$C" > "$OUT/cal_$C.csv"
done
# SQ pass (one run, 8 SQ counters): wave cycles split into issue / wait / active, VALU instructions, for the
# env kernel's latency-bound diagnosis (SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_* count quad-cycles)
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
timeout -s KILL 120 rocprofv3 --pmc $SQ --output-format csv -d /tmp/lrlprof/sq -o run -- \
  python3 "$ROOT/bench.py" --steps 1 --warmup 1 --no-cpu-baseline --no-secondary > "$OUT/pmc_sq.log" 2>&1
F=$(find /tmp/lrlprof/sq -name "*counter_collection.csv" | head -n 1)
for C in $SQ; do python3 "$ROOT/scripts/pmc_reduce.py" "$F" "$C" > "$OUT/sq_$C.csv"; done
ls -la "$OUT"
