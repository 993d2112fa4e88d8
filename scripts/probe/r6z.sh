#!/bin/bash
# episode / command sum rows preloaded ahead of the reward terms: env GPU tests, bit-identity of the state after two
# PPO iterations against the previous library, then whole-iteration A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export PYTHONPATH=$PWD/rapid-locomotion-rl_amd
B=$PWD/ab/r6base/rapid-locomotion-rl_amd/csrc/liblrl.so
timeout -k 10 600 python -u -m pytest tests/test_env_gpu.py -x -v --timeout 300 --timeout-method thread -m gpu \
  > gpurun_out/r6z_tests.log 2>&1 || { echo "tests failed"; exit 1; }
LRL_LIB=$B timeout -k 10 200 python scripts/ab_state.py run /tmp/a.npz 2 > gpurun_out/r6z_state.txt 2>&1 || exit 1
timeout -k 10 200 python scripts/ab_state.py run /tmp/b.npz 2 >> gpurun_out/r6z_state.txt 2>&1 || exit 1
python scripts/ab_state.py compare /tmp/a.npz /tmp/b.npz >> gpurun_out/r6z_state.txt 2>&1
for r in 1 2 3; do
  LRL_LIB=$B timeout -k 10 100 python scripts/ab_iter.py 12 base >> gpurun_out/r6z_ab.jsonl 2>/dev/null || exit 1
  timeout -k 10 100 python scripts/ab_iter.py 12 sums >> gpurun_out/r6z_ab.jsonl 2>/dev/null || exit 1
done
echo done
