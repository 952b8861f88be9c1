#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-shard2}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_shard.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 400 python -u bench.py --config 3 --mode sharded --topics 2000000 --check 20000 --steps 10 > $OUT/bench_sharded1.json 2> $OUT/bench_sharded1.log
