#!/bin/bash
# walk order at every slice size, LDS-local radix scatter: presort 1 (word-hash
# key, 4 passes) vs 2 (tail order, 1 pass) vs 0 (arrival), in one process per size
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${TAG:-r04_o}
mkdir -p "$OUT"
for T in ${SIZES:-8000000 4000000 2000000 1000000}; do
  timeout -k 10 300 python -u bench.py --topics $T --ab-opt presort=1 --ab-opt presort=2 --ab-opt presort=0 \
    --ab-opt presort=1 --ab-opt presort=2 --ab-opt presort=0 --steps 20 --warmup 3 --no-extras --cpu-sample 0 \
    --weak-topics 0 --check 2000 > "$OUT/ab_$T.json" 2> "$OUT/ab_$T.log" || exit $?
done
