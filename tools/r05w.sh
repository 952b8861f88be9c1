#!/bin/bash
# round 5: the tokenizer's pipeline depth (dictionary probes of 1 / 2 / 3
# levels ahead in flight; slim 8-VGPR probes) -- tokenizer parity tests,
# then C3 8M and 1M per build (default = 2)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_w}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread \
  -k "tokenizer or kat or o1_vectors or single_topic or empty or c1_full" > "$OUT/tests.log" 2>&1 || exit $?
A="--steps 30 --warmup 3 --no-extras --cpu-sample 0 --weak-topics 0 --check 2000"
for T in 8000000 1000000; do
  timeout -k 10 300 python -u bench.py $A --topics $T > "$OUT/d2_$T.json" 2> "$OUT/d2_$T.log" || exit $?
  for v in tok1 tok3; do
    timeout -k 10 300 python -u bench.py $A --topics $T --lib emqx_amd/variants/libtopicmatch_$v.so \
      > "$OUT/${v}_$T.json" 2> "$OUT/${v}_$T.log" || exit $?
  done
  timeout -k 10 300 python -u bench.py $A --topics $T > "$OUT/d2b_$T.json" 2> "$OUT/d2b_$T.log" || exit $?
done
