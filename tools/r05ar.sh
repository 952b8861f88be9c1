#!/bin/bash
# round 5: C4 (100M filters replicated on one GPU) at the final sources
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_ar}
mkdir -p "$OUT"
timeout -k 10 1100 python -u bench.py --config 4 --steps 20 --warmup 3 --no-extras --weak-topics 0 --cpu-sample 20000 \
  --check 2000 > "$OUT/bench_c4.json" 2> "$OUT/bench_c4.log" || exit $?
