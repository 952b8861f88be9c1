#!/bin/bash
# Round-4 HEAD evidence, in two gpurun calls:
#   PART=1  PMC passes of the walk -> traffic (profiles/traffic_c3.json on the
#           box, read by the bench that follows) -> the default bench line ->
#           rocprofv3 kernel stats of the same bench
#   PART=2  every -m gpu test, the smoke
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${TAG:-r04_final}
case ${PART:-1} in
  1) STEPS="pmc traffic bench prof" TAG=$TAG T_BENCH=420 bash tools/gpu.sh ;;
  2) STEPS="tests smoke" TAG=$TAG T_TESTS=900 bash tools/gpu.sh ;;
esac
