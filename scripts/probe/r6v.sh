#!/bin/bash
# PPO head kernel with float4 LDS rows: the update's GPU tests, then whole-iteration A/B against the r6u tree's library
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export PYTHONPATH=$PWD/rapid-locomotion-rl_amd
timeout -k 10 600 python -u -m pytest tests/test_ppo_gpu.py tests/test_checkpoint.py -x -v --timeout 300 --timeout-method thread \
  -m gpu > gpurun_out/r6v_tests.log 2>&1 || { echo "tests failed"; exit 1; }
B=$PWD/ab/r6base/rapid-locomotion-rl_amd/csrc/liblrl.so
for r in 1 2 3; do
  LRL_LIB=$B timeout -k 10 100 python scripts/ab_iter.py 12 base >> gpurun_out/r6v_ab.jsonl 2>/dev/null || exit 1
  timeout -k 10 100 python scripts/ab_iter.py 12 head4 >> gpurun_out/r6v_ab.jsonl 2>/dev/null || exit 1
done
echo done
