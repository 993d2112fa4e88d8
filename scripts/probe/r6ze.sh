#!/bin/bash
# the N = 1 bench line with the update's collectives issued through a one-rank RCCL group, beside the plain line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary >> gpurun_out/r6ze_bench.jsonl 2>>gpurun_out/r6ze_bench.err || exit 1
  LRL_FORCE_COLLECTIVES=1 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary >> gpurun_out/r6ze_bench.jsonl 2>>gpurun_out/r6ze_bench.err || exit 1
done
echo done
