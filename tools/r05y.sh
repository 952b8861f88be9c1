#!/bin/bash
# round 5: batcher lanes on normal- vs high-priority streams (TM_BATCHER_PRIO),
# alternating, three latency runs each (1M and 10M publishes/s), and the
# flood throughput of each
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_y}
mkdir -p "$OUT"
for i in 1 2 3; do
  for P in 0 1; do
    TM_BATCHER_PRIO=$P timeout -k 10 200 python -u tools/bench_batcher_latency.py --rates 1e6,1e7 --deadlines 200 \
      --eager 1 --eager-us 40 > "$OUT/lat_p${P}_$i.jsonl" 2>> "$OUT/latency.log" || exit $?
  done
done
for P in 0 1; do
  TM_BATCHER_PRIO=$P timeout -k 10 300 python -u tools/bench_batcher.py --lanes 4 --max-topics 262144 --eager 1 \
    > "$OUT/flood_p$P.json" 2> "$OUT/flood_p$P.log" || exit $?
done
