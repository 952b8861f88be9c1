#!/bin/bash
# round 5: per-node child blocks vs the shared edge table (in one process, the
# same trie converted back and forth), the global vs range-local walk order
# with blocks, repeated relayouts, with per-XCD walk clocks; then C2 / C5
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_d}
mkdir -p "$OUT"
timeout -k 10 600 python -u bench.py --ab-opt blocks=0 --ab-opt blocks=1 --ab-opt blocks=0 --ab-opt blocks=1 \
  --ab-opt presort=1,sort_bits=16 --ab-opt presort=3,sort_bits=24 --ab-opt relayout=1 --ab-opt relayout=1 \
  --steps 20 --warmup 3 --no-extras --cpu-sample 0 --weak-topics 0 --check 2000 > "$OUT/ab_blocks.json" 2> "$OUT/ab_blocks.log" || exit $?
for C in 2 5; do
  timeout -k 10 400 python -u bench.py --config $C --no-extras --weak-topics 0 > "$OUT/bench_c$C.json" 2> "$OUT/bench_c$C.log" || exit $?
done
