set -e
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_env_gpu.py -k "extras" > gpurun_out/r4n_extras.log 2>&1
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_gpu.py > gpurun_out/r4n_gemm_tests.log 2>&1
timeout -k 10 180 python scripts/x6d_bench.py > gpurun_out/r4n_x6d.jsonl 2> gpurun_out/r4n_x6d.err
for r in 1 2; do
  for v in 1 0; do
    LRL_GEMM_X6D=$v timeout -k 10 120 python scripts/ab_iter.py 15 x6d$v >> gpurun_out/r4n_ab.jsonl
  done
done
