#!/bin/bash
# A/B builds for timing experiments: exports the csrc + include trees of a git revision (or the working tree with
# "WT") into ab/<name>/ and builds liblrl.so there.  Load it with LRL_LIB=ab/<name>/rapid-locomotion-rl_amd/csrc/liblrl.so
# (scripts/ab_iter.py).  usage: bash scripts/ab_build.sh <name> <rev|WT>
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1
REV=$2
OUT=$ROOT/ab/$NAME
rm -rf "$OUT"
mkdir -p "$OUT/rapid-locomotion-rl_amd"
if [ "$REV" = WT ]; then
  cp -r "$ROOT/include" "$OUT/include"
  mkdir -p "$OUT/rapid-locomotion-rl_amd/csrc"
  cp "$ROOT"/rapid-locomotion-rl_amd/csrc/*.hip "$ROOT"/rapid-locomotion-rl_amd/csrc/*.h "$ROOT"/rapid-locomotion-rl_amd/csrc/*.cpp \
     "$ROOT"/rapid-locomotion-rl_amd/csrc/Makefile "$OUT/rapid-locomotion-rl_amd/csrc/"
else
  (cd "$ROOT" && git archive "$REV" include rapid-locomotion-rl_amd/csrc) | tar -x -C "$OUT"
fi
make -s -j8 -C "$OUT/rapid-locomotion-rl_amd/csrc" liblrl.so
echo "$OUT/rapid-locomotion-rl_amd/csrc/liblrl.so"
