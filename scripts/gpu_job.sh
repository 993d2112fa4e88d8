#!/bin/bash
# One parameterised GPU-box job (replaces the one-off scripts/_g*.sh files of rounds 1-4).
# usage: bash scripts/gpu_job.sh <tag> <step>[,<step>...] [pytest args for the "tests" step]
#   steps: tests   full `pytest -m gpu` (or the given pytest args) -> gpurun_out/<tag>_gputest.log
#          smoke   __graft_entry__.smoke()                          -> gpurun_out/<tag>_smoke.log
#          bench   python bench.py (default flags)                  -> gpurun_out/<tag>_bench.jsonl
#          profile scripts/gpu_profile.sh <tag> (trace + PMC + SQ)  -> gpurun_out/<tag>/
# Every GPU step runs under its own time limit and the steps are chained: the job ends at the first failure.
set -o pipefail
TAG=${1:?tag}
STEPS=${2:-tests,smoke,bench}
shift 2 || true
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
run_step() {
  case "$1" in
    tests)
      if [ $# -gt 1 ]; then shift; ARGS=("$@"); else ARGS=(tests -m gpu); fi
      timeout -k 10 1000 python -u -m pytest "${ARGS[@]}" -x -v --timeout 300 --timeout-method thread \
        > "gpurun_out/${TAG}_gputest.log" 2>&1 ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "gpurun_out/${TAG}_smoke.log" 2>&1 ;;
    bench)
      timeout -k 10 400 python bench.py > "gpurun_out/${TAG}_bench.jsonl" 2> "gpurun_out/${TAG}_bench.err" ;;
    profile)
      bash scripts/gpu_profile.sh "$TAG" > "gpurun_out/${TAG}_profile.log" 2>&1 ;;
    *) echo "unknown step $1" >&2; return 2 ;;
  esac
}
IFS=, read -r -a LIST <<< "$STEPS"
for s in "${LIST[@]}"; do
  echo "== $TAG: $s ($(date +%T))"
  if [ "$s" = tests ]; then run_step tests "$@" || { echo "step $s failed rc=$?"; exit 1; }
  else run_step "$s" || { echo "step $s failed rc=$?"; exit 1; }; fi
done
echo "== $TAG: done"
