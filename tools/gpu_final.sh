#!/bin/bash
# GPU call: full parity suite, smoke, default bench line, rocprofv3 kernel
# trace of the bench (no PMC passes).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-final}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.log && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 10 --warmup 2 --cpu-sample 0 --check 0 --streams 1 > $OUT/prof_bench.json 2> $OUT/prof_bench.log
