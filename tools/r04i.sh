#!/bin/bash
# routed/batcher/multi GPU tests, the walk-order A/Bs (tools/r04h.sh) and the
# batcher's latency at low offered load with the device-time split
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${TAG:-r04_i}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
STEPS="tests" TESTS="tests/test_gpu_routed.py tests/test_gpu_batcher.py tests/test_gpu_multi.py" TAG=$TAG T_TESTS=300 \
  bash tools/gpu.sh || exit $?
TAG=$TAG bash tools/r04h.sh || exit $?
STEPS="latency" LAT_ARGS="--rates 1e6,1e7 --deadlines 100,200 --seconds 0.5 --eager 0,1" TAG=$TAG bash tools/gpu.sh || exit $?
