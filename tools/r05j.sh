#!/bin/bash
# round 5: non-temporal streams (TM_NT_STREAM: tokenizer bytes and rows, the
# walk's chunk-row fill, the copy-out's stage reads) against the default
# build, alternating, one process per run
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_j}
mkdir -p "$OUT"
A="--steps 30 --warmup 3 --no-extras --cpu-sample 0 --weak-topics 0 --check 2000"
run() { timeout -k 10 300 python -u bench.py $A "$@"; }
for k in 1 2; do
  run > "$OUT/default_$k.json" 2> "$OUT/default_$k.log" || exit $?
  run --lib emqx_amd/variants/libtopicmatch_ntstream.so > "$OUT/ntstream_$k.json" 2> "$OUT/ntstream_$k.log" || exit $?
  run --lib emqx_amd/variants/libtopicmatch_copynt.so > "$OUT/copynt_$k.json" 2> "$OUT/copynt_$k.log" || exit $?
done
run --topics 1000000 > "$OUT/default_1m.json" 2> "$OUT/default_1m.log" || exit $?
run --topics 1000000 --lib emqx_amd/variants/libtopicmatch_ntstream.so > "$OUT/ntstream_1m.json" 2> "$OUT/ntstream_1m.log" || exit $?
