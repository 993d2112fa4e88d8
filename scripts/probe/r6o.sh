set -o pipefail
B=$PWD/ab/base6/rapid-locomotion-rl_amd/csrc/liblrl.so
N=$PWD/rapid-locomotion-rl_amd/csrc/liblrl.so
export PYTHONPATH=$PWD/rapid-locomotion-rl_amd
timeout -k 10 200 python scripts/gemm_bench.py $B $N > gpurun_out/r6o_gemm.txt 2>&1 || exit 1
GEMM_BENCH_B=4096 timeout -k 10 200 python scripts/gemm_bench.py $B $N > gpurun_out/r6o_gemm4096.txt 2>&1 || exit 1
for r in 1 2; do
  LRL_LIB=$B timeout -k 10 150 python scripts/ab_secondary.py base 6 >> gpurun_out/r6o_sec.jsonl 2>>gpurun_out/r6o_sec.err || exit 1
  timeout -k 10 150 python scripts/ab_secondary.py new 6 >> gpurun_out/r6o_sec.jsonl 2>>gpurun_out/r6o_sec.err || exit 1
done
