set -e
A=ab/A/rapid-locomotion-rl_amd/csrc/liblrl.so
B=ab/B/rapid-locomotion-rl_amd/csrc/liblrl.so
for r in 1 2; do
  for v in A B; do
    L=$A; [ $v = B ] && L=$B
    LRL_LIB=$L timeout -k 10 120 python scripts/ab_iter.py 15 $v >> gpurun_out/ab.jsonl
  done
done
