#!/bin/bash
# round 5: option donate without scratch spills (the donee writes the piece
# records) -- parity cases, A/B at C3 1M / 8M and C2 1M
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_q}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread \
  -k "donate or c5_sample or grows" > "$OUT/tests.log" 2>&1 || exit $?
A="--steps 20 --warmup 3 --no-extras --cpu-sample 0 --weak-topics 0 --check 2000"
AB="--ab-opt donate=1,donate_busy=2 --ab-opt donate=1,donate_busy=4 --ab-opt donate=1,donate_busy=8
 --ab-opt donate=1,donate_busy=16 --ab-opt donate=1,donate_busy=32 --ab-opt donate=0
 --ab-opt donate=1,donate_busy=8,donate_min=3 --ab-opt donate=1,donate_busy=64 --ab-opt donate=0"
timeout -k 10 300 python -u bench.py $A --topics 1000000 $AB > "$OUT/c3_1m.json" 2> "$OUT/c3_1m.log" || exit $?
timeout -k 10 300 python -u bench.py $A --topics 1000000 --lib emqx_amd/variants/libtopicmatch_clocks.so \
  --ab-opt donate=1,donate_busy=8 --ab-opt donate=0 --ab-opt donate=1,donate_busy=32 \
  > "$OUT/c3_1m_clocks.json" 2> "$OUT/c3_1m_clocks.log" || exit $?
timeout -k 10 300 python -u bench.py $A --config 2 --ab-opt donate=1,donate_busy=8 --ab-opt donate=0 \
  --ab-opt donate=1,donate_busy=32 > "$OUT/c2_1m.json" 2> "$OUT/c2_1m.log" || exit $?
timeout -k 10 400 python -u bench.py $A --ab-opt donate=1,donate_busy=8 --ab-opt donate=0 \
  --ab-opt donate=1,donate_busy=32 > "$OUT/c3_8m.json" 2> "$OUT/c3_8m.log" || exit $?
