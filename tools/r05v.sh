#!/bin/bash
# round 5: high-priority lane streams by default (bench.py lanes and the
# batcher's lanes): the default bench line with its host and batcher legs,
# and the NIF path's latency at 1M and 10M publishes/s
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_v}
mkdir -p "$OUT"
timeout -k 10 600 python -u bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.log" || exit $?
timeout -k 10 300 python -u tools/bench_batcher_latency.py --rates 1e6,1e7 --deadlines 200 --eager 1 --eager-us 40 \
  >> "$OUT/latency.jsonl" 2>> "$OUT/latency.log" || exit $?
