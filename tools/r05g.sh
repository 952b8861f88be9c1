#!/bin/bash
# round 5: build-variant A/Bs of the walk at C3 8M (one process per build,
# default build first and last): phase clocks, 16-id stage groups, non-temporal
# copy-out, 5 waves/SIMD, child blocks (+ its option)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_g}
mkdir -p "$OUT"
A="--steps 20 --warmup 3 --no-extras --cpu-sample 0 --weak-topics 0 --check 2000"
run() { timeout -k 10 300 python -u bench.py $A "$@"; }
run > "$OUT/default_a.json" 2> "$OUT/default_a.log" || exit $?
for v in clocks ids16 copynt w5; do
  run --lib emqx_amd/variants/libtopicmatch_$v.so > "$OUT/$v.json" 2> "$OUT/$v.log" || exit $?
done
run --lib emqx_amd/variants/libtopicmatch_blocks.so --ab-opt blocks=1 --ab-opt blocks=0 --ab-opt blocks=1 \
  > "$OUT/blocks.json" 2> "$OUT/blocks.log" || exit $?
run > "$OUT/default_b.json" 2> "$OUT/default_b.log" || exit $?
