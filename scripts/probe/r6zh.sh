#!/bin/bash
# the plane env kernel under other machine-scheduler strategies (scripts/ab_flags.sh builds): whole-iteration A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export PYTHONPATH=$PWD/rapid-locomotion-rl_amd
for r in 1 2; do
  timeout -k 10 100 python scripts/ab_iter.py 12 base >> gpurun_out/r6zh_ab.jsonl 2>/dev/null || exit 1
  for v in ilp bias memclause; do
    LRL_LIB=$PWD/ab/$v/rapid-locomotion-rl_amd/csrc/liblrl.so timeout -k 10 100 python scripts/ab_iter.py 12 $v >> gpurun_out/r6zh_ab.jsonl 2>/dev/null || exit 1
  done
done
echo done
