#!/bin/bash
# GPU call: aggre / routes / batcher parity, then the C3 and C5 deliveries benches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-aggre}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_aggre.py tests/test_gpu_routes.py tests/test_gpu_batcher.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest_aggre.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_routes -o run -- python3 tools/bench_routes.py > $OUT/routes.json 2> $OUT/routes.log && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c5 -o run -- python3 tools/bench_routes.py --config 5 --topics 200000 --exact 10000 --check 2000 --steps 3 > $OUT/c5.json 2> $OUT/c5.log
