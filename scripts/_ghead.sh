set -e
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ppo_gpu.py tests/test_configs_gpu.py -k "act or rollout or sampling" > gpurun_out/r4q_tests.log 2>&1
rm -f gpurun_out/ab.jsonl
bash scripts/ab_run.sh
cp gpurun_out/ab.jsonl gpurun_out/r4q_head_ab.jsonl
