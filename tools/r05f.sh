#!/bin/bash
# round 5: NIF path latency under offered load with the adaptive eager rule
# (tm_batcher_config.eager_us), then C4 (100M filters replicated on one GPU)
# with child blocks and the hot edge table against the default
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_f}
mkdir -p "$OUT"
timeout -k 10 500 python -u tools/bench_batcher_latency.py --rates 1e6,1e7 --deadlines 200 --eager 1 \
  --eager-us 1,40,60,100,150 >> "$OUT/latency.jsonl" 2>> "$OUT/latency.log" || exit $?
timeout -k 10 1000 python -u bench.py --config 4 --ab-opt blocks=1 --ab-opt blocks=0 --ab-opt hot_edges=4 --steps 10 \
  --warmup 2 --roof-steps 10 --no-extras --cpu-sample 0 --check 2000 --weak-topics 0 \
  > "$OUT/bench_c4_ab.json" 2> "$OUT/bench_c4_ab.log" || exit $?
