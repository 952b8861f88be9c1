#!/bin/bash
# round 5: option root_split (each topic walked as two queue items: the
# root's '+' subtree / the rest) -- parity cases, then A/B against the
# default walk at C3 8M and 1M topics per step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_m}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread \
  -k "rootsplit or c5_sample or grows" > "$OUT/tests.log" 2>&1 || exit $?
A="--steps 20 --warmup 3 --no-extras --cpu-sample 0 --weak-topics 0 --check 2000"
AB="--ab-opt root_split=1 --ab-opt root_split=0 --ab-opt root_split=1 --ab-opt root_split=0"
timeout -k 10 400 python -u bench.py $A $AB > "$OUT/c3_8m.json" 2> "$OUT/c3_8m.log" || exit $?
timeout -k 10 300 python -u bench.py $A --topics 1000000 $AB > "$OUT/c3_1m.json" 2> "$OUT/c3_1m.log" || exit $?
