set -o pipefail
B=$PWD/ab/base6/rapid-locomotion-rl_amd/csrc/liblrl.so
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6n_gputest.log 2>&1 || exit 1
for r in 1 2 3; do
  LRL_LIB=$B timeout -k 10 100 python scripts/ab_iter.py 12 base >> gpurun_out/r6n_ab.jsonl 2>/dev/null || exit 1
  timeout -k 10 100 python scripts/ab_iter.py 12 new >> gpurun_out/r6n_ab.jsonl 2>/dev/null || exit 1
done
for r in 1 2; do
  LRL_LIB=$B timeout -k 10 150 python scripts/ab_secondary.py base 6 >> gpurun_out/r6n_sec.jsonl 2>/dev/null || exit 1
  timeout -k 10 150 python scripts/ab_secondary.py new 6 >> gpurun_out/r6n_sec.jsonl 2>/dev/null || exit 1
done
bash scripts/kernel_trace.sh r6n_trace > /dev/null 2>&1 || exit 1
