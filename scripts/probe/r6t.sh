#!/bin/bash
# TGS vs PGS cost on one box: whole-iteration A/B (same library, Cfg.sim.physx.solver_type 1 / 0) and the env kernel's
# phase breakdown under each
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export PYTHONPATH=$PWD/rapid-locomotion-rl_amd
for r in 1 2 3; do
  LRL_SOLVER_TYPE=0 timeout -k 10 100 python scripts/ab_iter.py 12 pgs >> gpurun_out/r6t_ab.jsonl 2>/dev/null || exit 1
  LRL_SOLVER_TYPE=1 timeout -k 10 100 python scripts/ab_iter.py 12 tgs >> gpurun_out/r6t_ab.jsonl 2>/dev/null || exit 1
done
P=$PWD/rapid-locomotion-rl_amd/csrc/liblrl_prof.so
LRL_SOLVER_TYPE=1 LRL_LIB=$P timeout -k 10 200 python scripts/bench_env_profile.py 2 > gpurun_out/r6t_envprof_tgs.txt 2>&1 || exit 1
LRL_SOLVER_TYPE=0 LRL_LIB=$P timeout -k 10 200 python scripts/bench_env_profile.py 2 > gpurun_out/r6t_envprof_pgs.txt 2>&1 || exit 1
echo done
