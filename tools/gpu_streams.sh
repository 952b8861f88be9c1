#!/bin/bash
# GPU call: parity suite, then C3 bench with steps on 2 streams vs 1 stream.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-streams}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u bench.py --cpu-sample 0 --check 5000 --streams 1 > $OUT/bench_s1.json 2> $OUT/bench_s1.log && \
timeout -k 10 300 python -u bench.py --cpu-sample 0 --check 5000 --streams 2 > $OUT/bench_s2.json 2> $OUT/bench_s2.log && \
timeout -k 10 300 python -u bench.py --cpu-sample 0 --check 5000 --streams 3 > $OUT/bench_s3.json 2> $OUT/bench_s3.log
