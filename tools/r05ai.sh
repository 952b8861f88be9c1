#!/bin/bash
# round 5: the latency driver with a 100 ms settling phase after the flood
# warm-up -- 4 and 2 lanes, 1M and 10M publishes/s, three runs each
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_ai}
mkdir -p "$OUT"
for i in 1 2 3; do
  for L in 4 2; do
    timeout -k 10 200 python -u tools/bench_batcher_latency.py --rates 1e6,1e7 --deadlines 200 --eager 1 --eager-us 40 \
      --lanes $L > "$OUT/lat_l${L}_$i.jsonl" 2>> "$OUT/latency.log" || exit $?
  done
done
