#!/bin/bash
# round 5: lane streams on distinct hardware queues -- high-priority lanes
# (a queue set of their own) vs torch's pool, 2-4 lanes, C3 1M and 8M; then
# a kernel timeline of the best at 1M
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_u}
mkdir -p "$OUT"
A="--steps 30 --warmup 3 --no-extras --cpu-sample 0 --weak-topics 0 --check 2000"
for T in 1000000 8000000; do
  for K in pool prio; do
    for S in 2 3 4; do
      timeout -k 10 300 python -u bench.py $A --topics $T --stream-kind $K --streams $S --batches $S \
        > "$OUT/c3_${T}_${K}_${S}.json" 2> "$OUT/c3_${T}_${K}_${S}.log" || exit $?
    done
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_1m_prio3" -o run -- \
  python3 bench.py --topics 1000000 --steps 20 --warmup 3 --cpu-sample 0 --check 0 --no-extras --weak-topics 0 \
  --stream-kind prio > "$OUT/prof_1m_prio3.json" 2> "$OUT/prof_1m_prio3.log" || exit $?
