set -o pipefail
B=$PWD/ab/base6/rapid-locomotion-rl_amd/csrc/liblrl.so
export PYTHONPATH=$PWD/rapid-locomotion-rl_amd
for r in 1 2 3 4; do
  LRL_LIB=$B timeout -k 10 100 python scripts/ab_iter.py 12 base >> gpurun_out/r6p_ab.jsonl 2>/dev/null || exit 1
  timeout -k 10 100 python scripts/ab_iter.py 12 epi >> gpurun_out/r6p_ab.jsonl 2>/dev/null || exit 1
done
for r in 1 2; do
  LRL_LIB=$B timeout -k 10 150 python scripts/ab_secondary.py base 6 >> gpurun_out/r6p_sec.jsonl 2>>gpurun_out/r6p_sec.err || exit 1
  timeout -k 10 150 python scripts/ab_secondary.py epi 6 >> gpurun_out/r6p_sec.jsonl 2>>gpurun_out/r6p_sec.err || exit 1
done
