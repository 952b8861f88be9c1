#!/bin/bash
# GPU call: parity suite, C3 headline bench, C5 bench and its kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-c5}
mkdir -p $OUT
C5ARGS="--config 5 --topics 1000000 --cpu-sample 20000 --check 5000 --steps 10"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.log && \
timeout -k 10 400 python -u bench.py $C5ARGS > $OUT/bench_c5.json 2> $OUT/bench_c5.log && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c5 -o run -- python3 bench.py --config 5 --topics 1000000 --cpu-sample 0 --check 0 --steps 5 > $OUT/prof_c5.json 2> $OUT/prof_c5.log
