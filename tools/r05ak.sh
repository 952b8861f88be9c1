#!/bin/bash
# round 5: the batcher worst-batch stats test
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_ak}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_batcher.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -k worst > "$OUT/tests.log" 2>&1 || exit $?
