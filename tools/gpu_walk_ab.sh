#!/bin/bash
# GPU call: full parity suite, then the compile-time A/B (tools/gpu_abvar.sh).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-walkab}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
TAG=${TAG:-walkab} ./tools/gpu_abvar.sh
