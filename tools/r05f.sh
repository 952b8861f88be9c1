#!/bin/bash
# round 5: NIF path latency under offered load with the adaptive eager rule
# (tm_batcher_config.eager_us); the walk's blocks per CU with the pipeline's
# 3 streams (a free slot per CU lets the next batch's tokenizer and the last
# one's copy-out run beside a walk, and the next walk start in its drain)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_f}
mkdir -p "$OUT"
timeout -k 10 500 python -u tools/bench_batcher_latency.py --rates 1e6,1e7 --deadlines 200 --eager 1 \
  --eager-us 1,40,60,100,150 >> "$OUT/latency.jsonl" 2>> "$OUT/latency.log" || exit $?
A="--steps 30 --warmup 3 --no-extras --cpu-sample 0 --weak-topics 0 --check 2000"
timeout -k 10 400 python -u bench.py $A --ab-opt walk_bpc=5 --ab-opt walk_bpc=0 --ab-opt walk_bpc=4 --ab-opt walk_bpc=0 \
  > "$OUT/ab_bpc_8m.json" 2> "$OUT/ab_bpc_8m.log" || exit $?
timeout -k 10 400 python -u bench.py $A --topics 1000000 --ab-opt walk_bpc=5 --ab-opt walk_bpc=0 --ab-opt walk_bpc=4 \
  --ab-opt walk_bpc=0 > "$OUT/ab_bpc_1m.json" 2> "$OUT/ab_bpc_1m.log" || exit $?
