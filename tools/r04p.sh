#!/bin/bash
# presort 1 key width A/B (sort_bits 32 / 24 / 16 = 4 / 3 / 2 radix passes) at
# 8M and 4M topics, after the parity tests (which cover 3 and 2 passes)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${TAG:-r04_p}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
STEPS="tests" TESTS="tests/test_gpu_parity.py" TAG=$TAG T_TESTS=300 bash tools/gpu.sh || exit $?
for T in 8000000 4000000; do
  timeout -k 10 300 python -u bench.py --topics $T --ab-opt sort_bits=24 --ab-opt sort_bits=16 --ab-opt sort_bits=32 \
    --ab-opt sort_bits=24 --ab-opt sort_bits=16 --steps 20 --warmup 3 --no-extras --cpu-sample 0 \
    --weak-topics 0 --check 2000 > "$OUT/ab_bits_$T.json" 2> "$OUT/ab_bits_$T.log" || exit $?
done
