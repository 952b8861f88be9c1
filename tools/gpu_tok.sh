#!/bin/bash
# GPU call: parity suite, C3 bench (tokenizer time), sharded bench path at world 1.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-tok}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 400 python -u bench.py --cpu-sample 0 > $OUT/bench.json 2> $OUT/bench.log && \
timeout -k 10 400 python -u bench.py --config 3 --mode sharded --topics 2000000 --check 20000 --steps 10 > $OUT/bench_sharded1.json 2> $OUT/bench_sharded1.log
