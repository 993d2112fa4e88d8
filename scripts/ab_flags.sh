#!/bin/bash
# Variant libraries of the plane env kernel's translation unit built with extra compiler flags (A/B of code
# generation; the other objects are the tree's own build): ab/<tag>/rapid-locomotion-rl_amd/csrc/liblrl.so
# usage: bash scripts/ab_flags.sh <tag> "<extra flags>"
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
C=$ROOT/rapid-locomotion-rl_amd/csrc
TAG=$1; EXTRA=$2
OUT=$ROOT/ab/$TAG/rapid-locomotion-rl_amd/csrc
mkdir -p "$OUT"
cd "$C"
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=fast-honor-pragmas -Wall -Wno-unused-function -Wno-unused-variable -Xclang -target-feature -Xclang -packed-fp32-ops"
/opt/rocm/bin/hipcc $FLAGS $EXTRA -c lrl_env_flat.hip -o "$OUT/lrl_env_flat.hip.o" 2> "$OUT/err.txt" || { grep -v "not a recognized" "$OUT/err.txt"; exit 1; }
OBJS=$(ls build/*.o | grep -v lrl_env_flat.hip.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT/liblrl.so" $OBJS "$OUT/lrl_env_flat.hip.o"
rm -f "$OUT/lrl_env_flat.hip.o" "$OUT/err.txt"
echo "$OUT/liblrl.so"
