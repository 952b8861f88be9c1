#!/bin/bash
# round 5: the 10M publishes/s stalls with 4 lanes but not 2 -- 4 lanes over
# 4 workspace slots (engine option slots) vs the default 2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_ad}
mkdir -p "$OUT"
for i in 1 2; do
  for S in 4 2; do
    timeout -k 10 200 python -u tools/bench_batcher_latency.py --rates 1e6,1e7 --deadlines 200 --eager 1 --eager-us 40 \
      --opt slots=$S > "$OUT/lat_s${S}_$i.jsonl" 2>> "$OUT/latency.log" || exit $?
  done
done
