#!/bin/bash
# the driver's N > 1 launch rehearsed on one GPU at HEAD (2 and 4 ranks sharing
# GPU 0, parity on every rank), then the batcher flood: lanes x batch size, and
# two replicas of the engine on the same GPU (the host side's share)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${TAG:-r04_q}
STEPS="rehearse" NPROC=2 TAG=$TAG bash tools/gpu.sh || exit $?
STEPS="rehearse" NPROC=4 PORT=29541 TAG=$TAG bash tools/gpu.sh || exit $?
STEPS="batcher" BATCHER_ARGS="--topics 8000000 --lanes 4,8 --max-topics 131072,262144 --cb-threads 8 --eager 0" \
  TAG=$TAG T_BATCHER=400 bash tools/gpu.sh || exit $?
STEPS="batcher" BATCHER_ARGS="--topics 8000000 --lanes 2,4 --max-topics 262144 --cb-threads 8 --eager 0 --replicas 0,0" \
  TAG=$TAG T_BATCHER=300 bash tools/gpu.sh || exit $?
