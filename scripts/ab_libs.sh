#!/bin/bash
# Alternated A/B timing of whole PPO iterations (scripts/ab_iter.py) over library builds copied to abx/<name>.so
# (scripts/ab_build.sh builds them; ab/ itself stays local, abx/ travels to the GPU box).
# usage: bash scripts/ab_libs.sh <out.jsonl> <rounds> <name> [<name> ...]
set -o pipefail
OUT=$1; ROUNDS=$2; shift 2
mkdir -p "$(dirname "$OUT")"
for r in $(seq "$ROUNDS"); do
  for v in "$@"; do
    LRL_LIB=abx/$v.so timeout -k 10 150 python scripts/ab_iter.py 15 "$v" >> "$OUT" || exit 1
  done
done
