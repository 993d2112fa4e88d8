#!/bin/bash
# The reference's trained policy in this physics under TGS (and PGS), and the env kernel's phase breakdown with the
# post-physics sub-phases (bench workload)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export PYTHONPATH=$PWD/rapid-locomotion-rl_amd
timeout -k 10 200 python scripts/play.py --envs 64 --steps 500 > gpurun_out/r6y_play_tgs.txt 2>&1 || exit 1
LRL_SOLVER_TYPE=0 timeout -k 10 200 python scripts/play.py --envs 64 --steps 500 > gpurun_out/r6y_play_pgs.txt 2>&1 || exit 1
P=$PWD/rapid-locomotion-rl_amd/csrc/liblrl_prof.so
LRL_LIB=$P timeout -k 10 200 python scripts/bench_env_profile.py 2 > gpurun_out/r6y_envprof.txt 2>&1 || exit 1
echo done
