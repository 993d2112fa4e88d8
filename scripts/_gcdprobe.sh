set -e
cd /tmp && export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT/rapid-locomotion-rl_amd
for v in W B; do
  L=$GRAFT_REPO_ROOT/rapid-locomotion-rl_amd/csrc/liblrl.so; [ $v = B ] && L=$GRAFT_REPO_ROOT/ab/B/rapid-locomotion-rl_amd/csrc/liblrl.so
  LRL_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/cd$v -o run -- python3 $GRAFT_REPO_ROOT/scripts/ab_secondary.py $v 3 > /dev/null 2>&1
  find /tmp/cd$v -name "*kernel_stats.csv" -exec cp {} $GRAFT_REPO_ROOT/gpurun_out/r4z_cd_$v.csv \;
done
