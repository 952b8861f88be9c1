#!/bin/bash
# walk-order A/B at C3: presort 1 (word-hash key, 4 radix passes) vs arrival
# order at 8M topics, and the tail order vs arrival at 2M / 4M (presort 3's
# threshold); one process per size, variants interleaved
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${TAG:-r04_h}
mkdir -p "$OUT"
timeout -k 10 300 python -u bench.py --topics 8000000 --ab-opt presort=1 --ab-opt presort=0 --ab-opt presort=1 \
  --ab-opt presort=0 --steps 20 --warmup 3 --no-extras --cpu-sample 0 --weak-topics 0 --check 2000 \
  > "$OUT/ab_p1_8000000.json" 2> "$OUT/ab_p1_8000000.log" || exit $?
for T in 2000000 4000000; do
  timeout -k 10 300 python -u bench.py --topics $T --ab-opt presort=2 --ab-opt presort=0 --ab-opt presort=2 \
    --ab-opt presort=0 --steps 40 --warmup 3 --no-extras --cpu-sample 0 --weak-topics 0 --check 2000 \
    > "$OUT/ab_tail_$T.json" 2> "$OUT/ab_tail_$T.log" || exit $?
done
