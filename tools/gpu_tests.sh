#!/bin/bash
# GPU parity suite only (one call), output under gpurun_out/$TAG.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-tests}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
