#!/bin/bash
# round 5: the light tail (presort 6) vs the range-local word-hash order (5)
# at 4M and 8M topics with the lanes on their own hardware queues
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_am}
mkdir -p "$OUT"
A="--steps 30 --warmup 4 --no-extras --cpu-sample 0 --weak-topics 0 --check 2000"
AB="--ab-opt presort=6 --ab-opt presort=5 --ab-opt presort=6 --ab-opt presort=5"
for T in 8000000 4000000; do
  timeout -k 10 400 python -u bench.py $A --topics $T $AB > "$OUT/c3_$T.json" 2> "$OUT/c3_$T.log" || exit $?
done
