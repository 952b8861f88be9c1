#!/bin/bash
# round 5: the batcher-facing GPU tests again after the stats struct grew
# (max_* fields) and the NIF's lane count settled; the smoke
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_aj}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_batcher.py tests/test_id_reuse.py tests/test_gpu_multi.py \
  tests/test_gpu_small.py -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit $?
