#!/bin/bash
# round 5: stream -> hardware queue mapping (two of bench.py's three torch
# streams shared one hardware queue in profiles/r05_s)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_t}
mkdir -p "$OUT"
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$OUT/sq" -o run -- python3 tools/stream_queues.py \
  > "$OUT/sq.log" 2>&1 || exit $?
