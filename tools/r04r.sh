#!/bin/bash
# option tail_wave: parity variants, then A/B per batch size (one process per size)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${TAG:-r04_r}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
STEPS="tests" TESTS="tests/test_gpu_parity.py -k variant" TAG=$TAG T_TESTS=300 bash tools/gpu.sh || exit $?
for T in 1000000 2000000 8000000; do
  timeout -k 10 300 python -u bench.py --topics $T --ab-opt tail_wave=512 --ab-opt tail_wave=2048 --ab-opt tail_wave=0 \
    --ab-opt tail_wave=1024 --ab-opt tail_wave=4096 --ab-opt tail_wave=0 --steps 20 --warmup 3 --no-extras \
    --cpu-sample 0 --weak-topics 0 --check 2000 > "$OUT/ab_tw_$T.json" 2> "$OUT/ab_tw_$T.log" || exit $?
done
