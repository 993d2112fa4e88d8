#!/bin/bash
# TGS outlier probe + the physics parity tests without -x
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export PYTHONPATH=$PWD/rapid-locomotion-rl_amd
timeout -k 10 300 python -u scripts/tgs_probe.py mc 4096 10 > gpurun_out/r6r_probe.log 2>&1 || echo "probe rc=$?"
timeout -k 10 600 python -u -m pytest tests/test_env_gpu.py -k "physics_matches or pgs or joint_limits or self_collision or control_types" -v --timeout 300 --timeout-method thread > gpurun_out/r6r_tests.log 2>&1
echo "tests rc=$?"
