#!/bin/bash
# round 5: the donating walk kernel's main phase ran out of topics earlier
# (0.74 vs 0.93 ms at C3 1M): its kernel alone (donate_busy 0: nothing
# donated), and the default walk built with the same waves-per-EU hint
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_r}
mkdir -p "$OUT"
A="--steps 20 --warmup 3 --no-extras --cpu-sample 0 --weak-topics 0 --check 2000"
timeout -k 10 300 python -u bench.py $A --topics 1000000 --lib emqx_amd/variants/libtopicmatch_clocks.so \
  --ab-opt donate=1,donate_busy=0 --ab-opt donate=0 --ab-opt donate=1,donate_busy=0 --ab-opt donate=0 \
  > "$OUT/c3_1m_clocks.json" 2> "$OUT/c3_1m_clocks.log" || exit $?
timeout -k 10 300 python -u bench.py $A --topics 1000000 --lib emqx_amd/variants/libtopicmatch_w6attr.so \
  > "$OUT/c3_1m_w6attr.json" 2> "$OUT/c3_1m_w6attr.log" || exit $?
timeout -k 10 300 python -u bench.py $A --topics 1000000 > "$OUT/c3_1m_default.json" 2> "$OUT/c3_1m_default.log" || exit $?
timeout -k 10 400 python -u bench.py $A --ab-opt donate=1,donate_busy=0 --ab-opt donate=0 \
  > "$OUT/c3_8m.json" 2> "$OUT/c3_8m.log" || exit $?
timeout -k 10 400 python -u bench.py $A --lib emqx_amd/variants/libtopicmatch_w6attr.so \
  > "$OUT/c3_8m_w6attr.json" 2> "$OUT/c3_8m_w6attr.log" || exit $?
