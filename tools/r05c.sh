#!/bin/bash
# round 5: layout experiment (three forced relayouts of the C3 image in one
# process, each measured), C2 / C5 at HEAD with rocprof kernel stats, and the
# batcher latency sweep over the eager age (tm_batcher_config.eager_us)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_c}
mkdir -p "$OUT"
timeout -k 10 500 python -u bench.py --ab-opt relayout=1 --ab-opt relayout=1 --ab-opt relayout=1 --steps 20 --warmup 3 \
  --no-extras --cpu-sample 0 --weak-topics 0 --check 2000 > "$OUT/ab_relayout.json" 2> "$OUT/ab_relayout.log" || exit $?
for C in 2 5; do
  timeout -k 10 400 python -u bench.py --config $C --no-extras --weak-topics 0 > "$OUT/bench_c$C.json" 2> "$OUT/bench_c$C.log" || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c$C" -o run -- \
    python3 bench.py --config $C --steps 10 --warmup 2 --cpu-sample 0 --check 0 --streams 1 --no-extras --weak-topics 0 \
    > "$OUT/prof_c$C.json" 2> "$OUT/prof_c$C.log" || exit $?
done
timeout -k 10 400 python -u tools/bench_batcher_latency.py --rates 1e6,1e7 --deadlines 200 --eager 1 \
  --eager-us 30,60,100,150 > "$OUT/latency.jsonl" 2> "$OUT/latency.log" || exit $?
