L=$PWD/rapid-locomotion-rl_amd/csrc
for r in 1 2 3; do
  timeout -k 10 100 python -u scripts/ab_iter.py 12 base >> gpurun_out/r6j_ab.jsonl 2>/dev/null || exit 1
  LRL_LIB=$L/liblrl_nopk.so timeout -k 10 100 python -u scripts/ab_iter.py 12 nopk >> gpurun_out/r6j_ab.jsonl 2>/dev/null || exit 1
done
LRL_LIB=$L/liblrl_nopk.so timeout -k 10 400 python -u scripts/sharding_replay.py 12 > gpurun_out/r6j_nopk.log 2>&1
