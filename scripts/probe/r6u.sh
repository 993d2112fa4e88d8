#!/bin/bash
# Final-tree evidence after TGS: parity exclusion statistics (kernel vs oracle, every physics test) and the profile set
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export PYTHONPATH=$PWD/rapid-locomotion-rl_amd
LRL_PARITY_STATS=$PWD/gpurun_out/r6u_parity_stats.jsonl timeout -k 10 600 python -u -m pytest tests/test_env_gpu.py tests/test_terrain_gpu.py \
  -k "physics or pgs or joint_limits or self_collision or control_types" -v --timeout 300 --timeout-method thread \
  > gpurun_out/r6u_parity.log 2>&1 && \
bash scripts/gpu_profile.sh r6u > gpurun_out/r6u_profile.log 2>&1
echo "rc=$?"
