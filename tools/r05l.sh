#!/bin/bash
# round 5: kernel timelines of the 3-stream pipeline (do a batch's walk and
# its neighbours' kernels overlap?) at 1M and 8M topics per step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_l}
mkdir -p "$OUT"
for T in 1000000 8000000; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof3_$T" -o run -- \
    python3 bench.py --topics $T --steps 20 --warmup 3 --cpu-sample 0 --check 0 --streams 3 --no-extras --weak-topics 0 \
    > "$OUT/prof3_$T.json" 2> "$OUT/prof3_$T.log" || exit $?
  python3 tools/overlap.py "$OUT/prof3_$T/run_kernel_trace.csv" 23 2 > "$OUT/overlap_$T.json" || exit $?
  python3 tools/trace_walks.py "$OUT/prof3_$T/run_kernel_trace.csv" > "$OUT/walks_$T.jsonl" || exit $?
done
