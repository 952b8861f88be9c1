#!/bin/bash
# round 5: 2 vs 4 batcher lanes -- latency at 1M / 10M publishes/s (three
# runs of 2 lanes) and the flood with each
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_ae}
mkdir -p "$OUT"
for i in 1 2 3; do
  timeout -k 10 200 python -u tools/bench_batcher_latency.py --rates 1e6,1e7 --deadlines 200 --eager 1 --eager-us 40 \
    --lanes 2 > "$OUT/lat_l2_$i.jsonl" 2>> "$OUT/latency.log" || exit $?
done
for L in 2 4; do
  timeout -k 10 300 python -u tools/bench_batcher.py --lanes $L --max-topics 262144 --eager 1 --cb-threads 8 \
    > "$OUT/flood_l$L.json" 2> "$OUT/flood_l$L.log" || exit $?
done
