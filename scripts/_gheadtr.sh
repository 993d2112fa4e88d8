set -e
cd /tmp && export TMPDIR=/tmp
for v in A B; do
  LRL_LIB=$GRAFT_REPO_ROOT/ab/$v/rapid-locomotion-rl_amd/csrc/liblrl.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/tr$v -o run -- python3 $GRAFT_REPO_ROOT/scripts/ab_iter.py 4 $v > /dev/null 2>&1
  find /tmp/tr$v -name "*kernel_stats.csv" -exec cp {} $GRAFT_REPO_ROOT/gpurun_out/r4q_stats_$v.csv \;
done
