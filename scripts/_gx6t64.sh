set -e
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_gpu.py > gpurun_out/r4r_gemm_tests.log 2>&1
timeout -k 10 120 python scripts/x6t_bench.py > gpurun_out/r4r_x6t.jsonl 2> gpurun_out/r4r_x6t.err
rm -f gpurun_out/ab.jsonl
bash scripts/ab_run.sh
cp gpurun_out/ab.jsonl gpurun_out/r4r_ab.jsonl
