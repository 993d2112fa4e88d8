#!/bin/bash
# final tree: the 1 x 4096 / 2 x 2048 sharding case repeated (TGS, all round-6 kernels)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export PYTHONPATH=$PWD/rapid-locomotion-rl_amd
timeout -k 10 900 python -u scripts/sharding_repeat.py 6 1 4096 > gpurun_out/r6zg_sharding_repeat.txt 2>&1
echo "rc=$?"
