#!/bin/bash
# round 5: the light tail (presort 6) vs the range-local order (5), occupancy
# (walk blocks per CU), with per-XCD walk clocks; C5 at HEAD; parity of the
# new variants
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_e}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "order6 or blocks" --timeout 120 \
  --timeout-method thread > "$OUT/pytest_variants.log" 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --ab-opt presort=6 --ab-opt presort=5 --ab-opt presort=6,light_tail=120 \
  --ab-opt presort=6,light_tail=30 --ab-opt presort=5 --ab-opt walk_bpc=5 --ab-opt walk_bpc=0 \
  --steps 20 --warmup 3 --no-extras --cpu-sample 0 --weak-topics 0 --check 2000 > "$OUT/ab_tail.json" 2> "$OUT/ab_tail.log" || exit $?
timeout -k 10 400 python -u bench.py --topics 1000000 --ab-opt presort=6 --ab-opt presort=2 --ab-opt presort=5 \
  --steps 20 --warmup 3 --no-extras --cpu-sample 0 --weak-topics 0 --check 2000 > "$OUT/ab_tail_1m.json" 2> "$OUT/ab_tail_1m.log" || exit $?
timeout -k 10 400 python -u bench.py --config 5 --cpu-sample 20000 --check 2000 --no-extras --weak-topics 0 \
  --ab-opt presort=6 --ab-opt presort=5 > "$OUT/bench_c5.json" 2> "$OUT/bench_c5.log" || exit $?
