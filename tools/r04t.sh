#!/bin/bash
# range-local word-hash order (presort 5): key width A/B (sort_bits 16 / 24 / 32)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${TAG:-r04_t}
mkdir -p "$OUT"
for T in 8000000 4000000; do
  timeout -k 10 300 python -u bench.py --topics $T --ab-opt sort_bits=24 --ab-opt sort_bits=32 --ab-opt sort_bits=16 \
    --ab-opt sort_bits=24 --ab-opt sort_bits=32 --ab-opt sort_bits=16 --steps 20 --warmup 3 --no-extras --cpu-sample 0 \
    --weak-topics 0 --check 2000 > "$OUT/ab_bits5_$T.json" 2> "$OUT/ab_bits5_$T.log" || exit $?
done
