L=$PWD/rapid-locomotion-rl_amd/csrc
for r in 1 2 3; do
  LRL_LIB=$L/liblrl_nopk.so timeout -k 10 100 python -u scripts/ab_iter.py 12 nopk_env >> gpurun_out/r6k_ab.jsonl 2>/dev/null || exit 1
  LRL_LIB=$L/liblrl_nopkall.so timeout -k 10 100 python -u scripts/ab_iter.py 12 nopk_all >> gpurun_out/r6k_ab.jsonl 2>/dev/null || exit 1
done
