#!/bin/bash
# round 5: C2 and C5 lines at the final sources
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_aq}
mkdir -p "$OUT"
timeout -k 10 400 python -u bench.py --config 2 --steps 100 --warmup 5 --no-extras --weak-topics 0 \
  > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.log" || exit $?
timeout -k 10 500 python -u bench.py --config 5 --steps 10 --warmup 2 --no-extras --weak-topics 0 --cpu-sample 20000 \
  --check 2000 > "$OUT/bench_c5.json" 2> "$OUT/bench_c5.log" || exit $?
