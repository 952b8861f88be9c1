#!/bin/bash
# round 5: C4 (100M filters replicated on one GPU) at HEAD, with the hot edge
# table (parents of depth < 4) against the default
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_i}
mkdir -p "$OUT"
timeout -k 10 1100 python -u bench.py --config 4 --ab-opt hot_edges=4 --ab-opt hot_edges=0 --steps 10 \
  --warmup 2 --roof-steps 10 --no-extras --cpu-sample 0 --check 2000 --weak-topics 0 \
  > "$OUT/bench_c4_ab.json" 2> "$OUT/bench_c4_ab.log" || exit $?
