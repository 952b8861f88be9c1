#!/bin/bash
# GPU call: aggre parity tests + the full GPU suite, then the routes /
# deliveries bench under rocprofv3 (kernel trace + stats).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-aggre}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_aggre.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest_aggre.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_routes -o run -- python3 tools/bench_routes.py > $OUT/routes.json 2> $OUT/routes.log
