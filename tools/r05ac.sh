#!/bin/bash
# round 5: the 10M publishes/s stalls -- callback threads (8 / 0) and lanes
# (4 / 2), two runs each
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_ac}
mkdir -p "$OUT"
for i in 1 2; do
  for C in "--cb-threads 0" "--lanes 2" "--cb-threads 0 --lanes 2"; do
    t=$(echo $C | tr -d ' -')
    timeout -k 10 200 python -u tools/bench_batcher_latency.py --rates 1e7 --deadlines 200 --eager 1 --eager-us 40 \
      $C > "$OUT/lat_${t}_$i.jsonl" 2>> "$OUT/latency.log" || exit $?
  done
done
