#!/bin/bash
# round 5: after sort_min 1.5M -- the parity file (batches of 2.4M topics
# now take order 5 on the one-shot path) and the 2M slice
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_an}
mkdir -p "$OUT"
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
  > "$OUT/tests.log" 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --topics 2000000 --steps 40 --warmup 5 --cpu-sample 0 --check 2000 --weak-topics 0 \
  --no-extras > "$OUT/slice_2m.json" 2> "$OUT/slice_2m.log" || exit $?
