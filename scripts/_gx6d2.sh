set -e
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_gpu.py > gpurun_out/r4o_gemm_tests.log 2>&1
for r in 1 2; do
  for v in 1 0; do
    LRL_GEMM_X6D=$v timeout -k 10 120 python scripts/ab_iter.py 15 x6dnn$v >> gpurun_out/r4o_ab.jsonl
  done
done
NO_PMC=1 bash scripts/gpu_profile.sh r4o > gpurun_out/r4o_profile.log 2>&1
