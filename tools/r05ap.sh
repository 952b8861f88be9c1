#!/bin/bash
# round 5: the default bench line at the final sources (weak leg on the
# lanes' stream kind, sort_min 1.5M)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_ap}
mkdir -p "$OUT"
timeout -k 10 700 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.log" || exit $?
