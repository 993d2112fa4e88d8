#!/bin/bash
# 16-row thin-product tiles (the latent gradient) and the fused encoder launch of the rollout act: GEMM / update / act
# GPU tests, then whole-iteration A/B of the two switches in the same library, and a kernel trace of each arm
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export PYTHONPATH=$PWD/rapid-locomotion-rl_amd
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_ppo_gpu.py tests/test_checkpoint.py -x -v \
  --timeout 300 --timeout-method thread -m gpu > gpurun_out/r6w_tests.log 2>&1 || { echo "tests failed"; exit 1; }
for r in 1 2 3; do
  LRL_THIN16=0 LRL_ACT_ENC_FUSED=0 timeout -k 10 100 python scripts/ab_iter.py 12 base >> gpurun_out/r6w_ab.jsonl 2>/dev/null || exit 1
  LRL_THIN16=1 LRL_ACT_ENC_FUSED=0 timeout -k 10 100 python scripts/ab_iter.py 12 thin16 >> gpurun_out/r6w_ab.jsonl 2>/dev/null || exit 1
  LRL_THIN16=0 LRL_ACT_ENC_FUSED=1 timeout -k 10 100 python scripts/ab_iter.py 12 encf >> gpurun_out/r6w_ab.jsonl 2>/dev/null || exit 1
  LRL_THIN16=1 LRL_ACT_ENC_FUSED=1 timeout -k 10 100 python scripts/ab_iter.py 12 both >> gpurun_out/r6w_ab.jsonl 2>/dev/null || exit 1
done
cd /tmp && export TMPDIR=/tmp
for v in 0 1; do
  export LRL_THIN16=$v LRL_ACT_ENC_FUSED=$v
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r6w_t$v -o run -- \
    python3 "$GRAFT_REPO_ROOT/scripts/ab_iter.py" 4 t$v > /dev/null 2>&1 || exit 1
  f=$(find /tmp/r6w_t$v -name "*kernel_stats.csv" | head -n 1)
  cp "$f" "$GRAFT_REPO_ROOT/gpurun_out/r6w_kernel_stats_$v.csv"
done
echo done
