set -e
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_env_gpu.py -k "device_reset or curriculum" > gpurun_out/r4z_cd_test.log 2>&1
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_configs_gpu.py -k "configs2 or rough or upstream" > gpurun_out/r4z_cd_test2.log 2>&1 || true
DEVR=1 bash scripts/_gsectr.sh
export PYTHONPATH=$GRAFT_REPO_ROOT/rapid-locomotion-rl_amd
rm -f gpurun_out/r4z_sec_ab.jsonl
for r in 1 2; do
  timeout -k 10 200 python scripts/ab_secondary.py dev1 8 >> gpurun_out/r4z_sec_ab.jsonl
done
