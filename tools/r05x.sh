#!/bin/bash
# round 5: the walk built with amdgpu_waves_per_eu(6, 8) (TM_WALK_WAVES=6)
# against the default build, interleaved, C3 8M and 1M; then the NIF path's
# latency with normal-priority batcher lanes again
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_x}
mkdir -p "$OUT"
A="--steps 30 --warmup 3 --no-extras --cpu-sample 0 --weak-topics 0 --check 2000"
W=emqx_amd/variants/libtopicmatch_w6attr.so
for i in 1 2; do
  timeout -k 10 300 python -u bench.py $A > "$OUT/def_8m_$i.json" 2> "$OUT/def_8m_$i.log" || exit $?
  timeout -k 10 300 python -u bench.py $A --lib $W > "$OUT/w6_8m_$i.json" 2> "$OUT/w6_8m_$i.log" || exit $?
done
timeout -k 10 300 python -u bench.py $A --topics 1000000 > "$OUT/def_1m.json" 2> "$OUT/def_1m.log" || exit $?
timeout -k 10 300 python -u bench.py $A --topics 1000000 --lib $W > "$OUT/w6_1m.json" 2> "$OUT/w6_1m.log" || exit $?
timeout -k 10 300 python -u tools/bench_batcher_latency.py --rates 1e6,1e7 --deadlines 200 --eager 1 --eager-us 40 \
  >> "$OUT/latency.jsonl" 2>> "$OUT/latency.log" || exit $?
