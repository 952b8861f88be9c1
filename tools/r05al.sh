#!/bin/bash
# round 5: with the lanes on their own hardware queues the drain hides
# behind the next walk -- does the range-local word-hash order (presort 5,
# locality) now beat the tail order (2, short drain) below sort_min?  A/B
# at 1M and 2M topics (the N = 8 and N = 4 slices)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_al}
mkdir -p "$OUT"
A="--steps 40 --warmup 5 --no-extras --cpu-sample 0 --weak-topics 0 --check 2000"
AB="--ab-opt presort=5 --ab-opt presort=2 --ab-opt presort=6 --ab-opt presort=5 --ab-opt presort=2"
for T in 1000000 2000000; do
  timeout -k 10 300 python -u bench.py $A --topics $T $AB > "$OUT/c3_$T.json" 2> "$OUT/c3_$T.log" || exit $?
done
