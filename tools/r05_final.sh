#!/bin/bash
# Round-5 HEAD evidence, in three gpurun calls:
#   PART=1  PMC passes of the walk -> traffic (profiles/traffic_c3.json on the
#           box, read by the bench that follows) -> the default bench line ->
#           rocprofv3 kernel stats of the same bench (1 stream) and over the
#           default 3 lanes with the kernel overlap
#   PART=2  every -m gpu test but the full-size and config files, the smoke
#   PART=3  the full-size (8M-topic C3) and config (C1-C5) tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${TAG:-r05_final}
case ${PART:-1} in
  1) STEPS="pmc traffic bench prof prof3" TAG=$TAG T_BENCH=600 bash tools/gpu.sh ;;
  2) STEPS="tests smoke" TAG=$TAG T_TESTS=1000 \
       TESTS="tests --ignore=tests/test_gpu_fullsize.py --ignore=tests/test_gpu_configs.py" bash tools/gpu.sh ;;
  3) STEPS="tests" TAG=${TAG}_big T_TESTS=1100 TESTS="tests/test_gpu_fullsize.py tests/test_gpu_configs.py" \
       bash tools/gpu.sh ;;
esac
# PART=4: the per-rank slices of strong scaling (1M/2M/4M/8M, rocprofv3 stats)
# and the driver's N = 2 launch rehearsed on one GPU
if [ "${PART:-1}" = 4 ]; then
  STEPS="slices rehearse" TAG=${TAG}_slices NPROC=2 bash tools/gpu.sh
fi
