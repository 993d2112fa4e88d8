#!/bin/bash
# train from scratch under the presets' TGS solver, then play the learned student policy
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export PYTHONPATH=$PWD/rapid-locomotion-rl_amd
timeout -k 10 500 python -u scripts/train_eval.py --iterations 1500 --out /tmp/te > gpurun_out/r6za_train_eval.txt 2>&1
echo "rc=$?"
