#!/bin/bash
# round 5: do the next batches' tokenize / presort and the last batch's
# copy-out co-run with a walk when the walk leaves wave slots free (option
# walk_bpc: walk blocks per CU, 0 = every slot)?  A/B at C3 8M and 1M, then
# a kernel timeline at 8M with walk_bpc 5
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_n}
mkdir -p "$OUT"
A="--steps 20 --warmup 3 --no-extras --cpu-sample 0 --weak-topics 0 --check 2000"
AB="--ab-opt walk_bpc=5 --ab-opt walk_bpc=0 --ab-opt walk_bpc=4 --ab-opt walk_bpc=0 --ab-opt walk_bpc=5"
timeout -k 10 400 python -u bench.py $A $AB > "$OUT/c3_8m.json" 2> "$OUT/c3_8m.log" || exit $?
timeout -k 10 300 python -u bench.py $A --topics 1000000 $AB > "$OUT/c3_1m.json" 2> "$OUT/c3_1m.log" || exit $?
T=8000000
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_bpc5" -o run -- \
  python3 bench.py --topics $T --steps 20 --warmup 3 --cpu-sample 0 --check 0 --no-extras --weak-topics 0 \
  --opt walk_bpc=5 > "$OUT/prof_bpc5.json" 2> "$OUT/prof_bpc5.log" || exit $?
python3 tools/overlap.py "$OUT/prof_bpc5/run_kernel_trace.csv" 23 2 > "$OUT/overlap_bpc5.json" || exit $?
