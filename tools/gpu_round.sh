#!/bin/bash
# One GPU call: parity tests, smoke, default bench line, rocprofv3 kernel
# trace, PMC passes.  Every GPU step has its own time limit; steps are
# chained with &&.  TAG names the output directory under gpurun_out/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-run}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 400 python -u bench.py ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/bench.log && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 10 --warmup 2 --cpu-sample 0 --check 0 --streams 1 ${BENCH_ARGS} > $OUT/prof_bench.json 2> $OUT/prof_bench.log && \
PMC_DIR=${TAG:-run}/pmc ./tools/pmc_passes.sh && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_routes -o run -- python3 tools/bench_routes.py > $OUT/routes.json 2> $OUT/routes.log
