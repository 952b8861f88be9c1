#!/bin/bash
# hot_levels confirmation on another box: 2 / 3 vs 4, alternating, at 8M and 4M
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${TAG:-r04_x}
mkdir -p "$OUT"
for T in 8000000 4000000; do
  timeout -k 10 400 python -u bench.py --topics $T --ab-opt hot_levels=2 --ab-opt hot_levels=4 --ab-opt hot_levels=2 \
    --ab-opt hot_levels=4 --ab-opt hot_levels=3 --ab-opt hot_levels=4 --steps 20 --warmup 3 --no-extras --cpu-sample 0 \
    --weak-topics 0 --check 2000 > "$OUT/ab_hot_$T.json" 2> "$OUT/ab_hot_$T.log" || exit $?
done
