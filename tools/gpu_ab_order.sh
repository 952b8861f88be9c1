#!/bin/bash
# GPU call: the walk-variant parity tests, then an interleaved A/B of image
# variants (tools/ab_image.py, VARIANTS) at C3.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-ab}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "${TESTK:-variant}" -x -v --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 500 python -u tools/ab_image.py --variants "${VARIANTS:-order=0,order=1,order=2,order=3}" > $OUT/ab.json 2> $OUT/ab.log
