#!/bin/bash
# round 5: where the 10M publishes/s stall sits -- the worst single batch's
# phases (tm_batcher_stats max_*), 4 lanes, three runs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_af}
mkdir -p "$OUT"
for i in 1 2 3; do
  timeout -k 10 200 python -u tools/bench_batcher_latency.py --rates 1e7 --deadlines 200 --eager 1 --eager-us 40 \
    --lanes 4 > "$OUT/lat_l4_$i.jsonl" 2>> "$OUT/latency.log" || exit $?
done
