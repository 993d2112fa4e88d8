#!/bin/bash
# SQ counters of the update GEMM shapes (scripts/gemm_bench.py), one rocprofv3 --pmc pass per counter group.
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/gemm_pmc
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for CS in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES" \
          "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_INSTS_MFMA"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $CS --output-format csv -d /tmp/gpmc$i -o run -- \
    python3 "$ROOT/scripts/gemm_bench.py" > "$OUT/pass$i.log" 2>&1
  F=$(find /tmp/gpmc$i -name "*counter_collection.csv" | head -n 1)
  for C in $CS; do python3 "$ROOT/scripts/pmc_reduce.py" "$F" "$C" | grep -E "gemm_kernel|kernel,counter" >> "$OUT/counters.csv" || true; done
done
