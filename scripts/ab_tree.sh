#!/bin/bash
# A/B trees for Python + native changes: ab/<name>/ gets the package (lrl + csrc + include) and bench.py of a git
# revision (or "WT": the working tree), with liblrl.so built there.  Run a script against it with
# PYTHONPATH=ab/<name>/rapid-locomotion-rl_amd (and LRL_LIB unset: the tree's own csrc/liblrl.so is loaded).
# usage: bash scripts/ab_tree.sh <name> <rev|WT>
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1
REV=$2
OUT=$ROOT/ab/$NAME
rm -rf "$OUT"
mkdir -p "$OUT"
if [ "$REV" = WT ]; then
  mkdir -p "$OUT/rapid-locomotion-rl_amd"
  cp -r "$ROOT/include" "$OUT/include"
  cp -r "$ROOT/rapid-locomotion-rl_amd/lrl" "$OUT/rapid-locomotion-rl_amd/lrl"
  mkdir -p "$OUT/rapid-locomotion-rl_amd/csrc"
  cp "$ROOT"/rapid-locomotion-rl_amd/csrc/*.hip "$ROOT"/rapid-locomotion-rl_amd/csrc/*.h "$ROOT"/rapid-locomotion-rl_amd/csrc/*.cpp \
     "$ROOT"/rapid-locomotion-rl_amd/csrc/Makefile "$OUT/rapid-locomotion-rl_amd/csrc/"
  cp "$ROOT/bench.py" "$OUT/"
else
  (cd "$ROOT" && git archive "$REV" include rapid-locomotion-rl_amd/csrc rapid-locomotion-rl_amd/lrl bench.py) | tar -x -C "$OUT"
fi
find "$OUT" -name "__pycache__" -prune -exec rm -rf {} +
rm -f "$OUT"/rapid-locomotion-rl_amd/csrc/liblrl.so
make -s -j8 -C "$OUT/rapid-locomotion-rl_amd/csrc" liblrl.so
echo "$OUT"
