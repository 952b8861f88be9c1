#!/bin/bash
# A/B of compile-time variants (bench.py --lib), alternating processes:
# base, new, base, new; walk/step times from each run's JSON line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-abvar}
mkdir -p $OUT
A="--steps 30 --warmup 3 --check 2000 --cpu-sample 0 ${BENCH_ARGS}"
timeout -k 10 200 python -u bench.py $A --lib emqx_amd/variants/libtopicmatch_${VAR:-base}.so > $OUT/base1.json 2> $OUT/base1.log && \
timeout -k 10 200 python -u bench.py $A > $OUT/new1.json 2> $OUT/new1.log && \
timeout -k 10 200 python -u bench.py $A --lib emqx_amd/variants/libtopicmatch_${VAR:-base}.so > $OUT/base2.json 2> $OUT/base2.log && \
timeout -k 10 200 python -u bench.py $A > $OUT/new2.json 2> $OUT/new2.log
