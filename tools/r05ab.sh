#!/bin/bash
# round 5: the 10M publishes/s latency tail against the number of producer
# threads (16, 8, 4): host scheduling of the benchmark's own threads?
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_ab}
mkdir -p "$OUT"
for i in 1 2; do
  for P in 16 8 4; do
    timeout -k 10 200 python -u tools/bench_batcher_latency.py --rates 1e7 --deadlines 200 --eager 1 --eager-us 40 \
      --producers $P > "$OUT/lat_p${P}_$i.jsonl" 2>> "$OUT/latency.log" || exit $?
  done
done
