#!/bin/bash
# round 5: option donate, restricted to each wave's last walkers
# (donate_busy) -- A/B at C3 1M (the 8-GPU strong-scaling slice), parity
# by the lists-equal check against the headline pass
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_p}
mkdir -p "$OUT"
A="--steps 20 --warmup 3 --no-extras --cpu-sample 0 --weak-topics 0 --check 2000 --topics 1000000"
AB="--ab-opt donate=1,donate_busy=1 --ab-opt donate=1,donate_busy=2 --ab-opt donate=1,donate_busy=4
 --ab-opt donate=1,donate_busy=8 --ab-opt donate=1,donate_busy=16 --ab-opt donate=0
 --ab-opt donate=1,donate_busy=4,donate_min=3 --ab-opt donate=1,donate_busy=4,donate_min=1 --ab-opt donate=0"
timeout -k 10 300 python -u bench.py $A $AB > "$OUT/c3_1m.json" 2> "$OUT/c3_1m.log" || exit $?
timeout -k 10 300 python -u bench.py $A --lib emqx_amd/variants/libtopicmatch_clocks.so \
  --ab-opt donate=1,donate_busy=4 --ab-opt donate=0 --ab-opt donate=1,donate_busy=8 \
  > "$OUT/c3_1m_clocks.json" 2> "$OUT/c3_1m_clocks.log" || exit $?
timeout -k 10 300 python -u bench.py $A --config 2 --ab-opt donate=1,donate_busy=4 --ab-opt donate=0 \
  > "$OUT/c2_1m.json" 2> "$OUT/c2_1m.log" || exit $?
