#!/bin/bash
# round 5: workspaces reserved up front (tm_reserve from tm_batcher_open):
# batcher / small-batch / reserve tests, then three latency runs (1M and 10M
# publishes/s) and the flood
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_aa}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_batcher.py tests/test_gpu_small.py tests/test_gpu_parity.py -x -v \
  --timeout 120 --timeout-method thread -k "batcher or small or reserve" > "$OUT/tests.log" 2>&1 || exit $?
for i in 1 2 3; do
  timeout -k 10 200 python -u tools/bench_batcher_latency.py --rates 1e6,1e7 --deadlines 200 --eager 1 --eager-us 40 \
    > "$OUT/lat_$i.jsonl" 2>> "$OUT/latency.log" || exit $?
done
timeout -k 10 300 python -u tools/bench_batcher.py --lanes 4 --max-topics 262144 --eager 1 \
  > "$OUT/flood.json" 2> "$OUT/flood.log" || exit $?
