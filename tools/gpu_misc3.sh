#!/bin/bash
# GPU call: full parity suite, micro-batcher end-to-end benchmark, then the
# C5 adversarial configuration through bench.py (16-level topics, fan-out ~900).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-misc3}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 300 ./tools/ubench/batcher_bench 10000000 2000000 16 > $OUT/batcher.json 2> $OUT/batcher.log && \
timeout -k 10 400 python -u bench.py --config 5 --topics 1000000 --cpu-sample 20000 --check 5000 --steps 10 > $OUT/bench_c5.json 2> $OUT/bench_c5.log
