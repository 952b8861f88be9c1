#!/bin/bash
# one-launch small path: GPU tests, then the batcher's latency A/B (one-launch
# vs CSR path, eager sealing on/off), then the stage-row group A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${TAG:-r04_k}
STEPS="tests" TESTS="tests/test_gpu_small.py tests/test_gpu_batcher.py tests/test_gpu_parity.py" TAG=$TAG T_TESTS=300 bash tools/gpu.sh || exit $?
STEPS="latency" LAT_ARGS="--rates 1e6,1e7 --deadlines 200 --seconds 0.5 --eager 0,1 --csr 0,1" TAG=$TAG \
  bash tools/gpu.sh || exit $?
LIBS="base s16 s4" ROUNDS=2 TAG=$TAG T_RUN=200 bash tools/ab_libs.sh || exit $?
