set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r4x_gputest.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4x_smoke.log 2>&1 && \
timeout -k 10 400 python bench.py > gpurun_out/r4x_bench.jsonl 2> gpurun_out/r4x_bench.err && \
bash scripts/gpu_profile.sh r4x > gpurun_out/r4x_profile.log 2>&1
