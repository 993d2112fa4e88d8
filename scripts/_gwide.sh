set -e
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_gpu.py > gpurun_out/r4p_gemm_tests.log 2>&1
for r in 1 2; do
  for v in 1 0; do
    LRL_X6_WIDE=$v timeout -k 10 120 python scripts/ab_iter.py 15 wide$v >> gpurun_out/r4p_ab.jsonl
  done
done
GEMM_BENCH_FILTER=fwd timeout -k 10 120 python scripts/gemm_bench.py > gpurun_out/r4p_gemm_wide1.txt 2>&1
LRL_X6_WIDE=0 GEMM_BENCH_FILTER=fwd timeout -k 10 120 python scripts/gemm_bench.py > gpurun_out/r4p_gemm_wide0.txt 2>&1
