#!/bin/bash
# GPU call: full parity suite, then bench.py over the default build and the
# compile-time variants in VARS (emqx_amd/variants/libtopicmatch_<v>.so),
# interleaved over two rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-abn}
mkdir -p $OUT
A="--steps 20 --warmup 3 --check 2000 --cpu-sample 0 ${BENCH_ARGS}"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit 1
for round in 1 2; do
  timeout -k 10 200 python -u bench.py $A > $OUT/default_$round.json 2> $OUT/default_$round.log || exit 1
  for v in $VARS; do
    timeout -k 10 200 python -u bench.py $A --lib emqx_amd/variants/libtopicmatch_$v.so > $OUT/${v}_$round.json 2> $OUT/${v}_$round.log || exit 1
  done
done
