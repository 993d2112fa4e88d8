set -e
cd /tmp && export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT/rapid-locomotion-rl_amd
export LRL_DEVICE_RESETS=${DEVR:-0}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/trsec -o run -- python3 $GRAFT_REPO_ROOT/scripts/ab_secondary.py sec 4 > $GRAFT_REPO_ROOT/gpurun_out/r4t${DEVR:-0}_sec.log 2>&1
find /tmp/trsec -name "*kernel_stats.csv" -exec cp {} $GRAFT_REPO_ROOT/gpurun_out/r4t${DEVR:-0}_sec_stats.csv \;
KT=$(find /tmp/trsec -name "*kernel_trace.csv" | head -n 1)
python3 $GRAFT_REPO_ROOT/scripts/timeline.py "$KT" > $GRAFT_REPO_ROOT/gpurun_out/r4t${DEVR:-0}_sec_timeline.csv
