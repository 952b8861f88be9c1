#!/bin/bash
# the pipelined host-buffer path: its parity test, then the bench's host-path leg
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${TAG:-r04_v}
STEPS="tests" TESTS="tests/test_gpu_parity.py -k pipelined_host" TAG=$TAG T_TESTS=300 bash tools/gpu.sh || exit $?
STEPS="bench" BENCH_ARGS="--steps 10 --warmup 2 --cpu-sample 0 --weak-topics 0 --opt host_pipeline=1" TAG=$TAG T_BENCH=400 bash tools/gpu.sh || exit $?
