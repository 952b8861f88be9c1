#!/bin/bash
# HEAD check + headline evidence in one box: the small-path / batcher / parity
# GPU tests, the walk's PMC passes -> traffic (profiles/traffic_c3.json on the
# box, read by the bench after it), the default bench line, then the batcher
# latency A/B (one-launch vs CSR small batches, eager sealing on/off)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${TAG:-r04_m}
STEPS="tests" TESTS="tests/test_gpu_small.py tests/test_gpu_batcher.py tests/test_gpu_parity.py" TAG=$TAG T_TESTS=300 \
  bash tools/gpu.sh || exit $?
PMC_DIR=$TAG/pmc PASSES="fetch write tcc" T_PMC=150 bash tools/pmc_passes.sh || exit $?
STEPS="traffic bench" TAG=$TAG T_BENCH=420 bash tools/gpu.sh || exit $?
STEPS="latency" LAT_ARGS="--rates 1e6,1e7 --deadlines 200 --seconds 0.5 --eager 0,1 --csr 0,1" TAG=$TAG \
  bash tools/gpu.sh || exit $?
