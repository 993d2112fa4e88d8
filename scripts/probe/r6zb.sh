#!/bin/bash
# tile of the short-k (k <= 32) products: E1 (NT 18 -> 256, gathered) and dHe2 (NN 18 -> 128, DELU), 24,576 rows
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
L=$PWD/rapid-locomotion-rl_amd/csrc/liblrl.so
for t in 0 128 12864 64128; do
  for f in E1 dHe2; do
    echo "tile=$t filter=$f" >> gpurun_out/r6zb_shortk.txt
    LRL_SHORTK_TILE=$t GEMM_BENCH_FILTER=$f timeout -k 10 100 python scripts/gemm_bench.py $L >> gpurun_out/r6zb_shortk.txt 2>&1 || exit 1
  done
done
echo done
