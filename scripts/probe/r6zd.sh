#!/bin/bash
# the update's collectives through RCCL in a one-rank group, and the multi-process / update GPU tests around it
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_rccl_world1_gpu.py tests/test_dist_gpu.py tests/test_ppo_gpu.py -x -v \
  --timeout 300 --timeout-method thread -m gpu > gpurun_out/r6zd_tests.log 2>&1
echo "rc=$?"
