#!/bin/bash
# range-keyed walk orders (presort 4, 5) against the tail order (2) and the
# word-hash order (1), per batch size, after their parity variants
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${TAG:-r04_s}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
STEPS="tests" TESTS="tests/test_gpu_parity.py -k variant" TAG=$TAG T_TESTS=300 bash tools/gpu.sh || exit $?
for T in 1000000 2000000 4000000 8000000; do
  timeout -k 10 300 python -u bench.py --topics $T --ab-opt presort=4 --ab-opt presort=5 --ab-opt presort=2 \
    --ab-opt presort=1 --ab-opt presort=4 --ab-opt presort=5 --steps 20 --warmup 3 --no-extras \
    --cpu-sample 0 --weak-topics 0 --check 2000 > "$OUT/ab_ord_$T.json" 2> "$OUT/ab_ord_$T.log" || exit $?
done
