set -e
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_env_gpu.py -k "device_reset" > gpurun_out/r4u_devtest.log 2>&1
DEVR=1 bash scripts/_gsectr.sh
export PYTHONPATH=$GRAFT_REPO_ROOT/rapid-locomotion-rl_amd
rm -f gpurun_out/r4u_sec_ab.jsonl
for r in 1 2 3; do
  for v in 1 0; do
    LRL_DEVICE_RESETS=$v timeout -k 10 200 python scripts/ab_secondary.py dev$v 8 >> gpurun_out/r4u_sec_ab.jsonl
  done
done
