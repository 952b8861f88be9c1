#!/bin/bash
# round 5: kernel + copy timeline of the 10M publishes/s latency run (4
# lanes): does the GPU stall, or a kernel / copy run long?
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_ag}
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$OUT/trace" -o run -- \
  python3 tools/bench_batcher_latency.py --rates 1e7 --deadlines 200 --eager 1 --eager-us 40 --lanes 4 \
  > "$OUT/lat.jsonl" 2> "$OUT/lat.log" || exit $?
