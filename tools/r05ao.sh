#!/bin/bash
# round 5: engine options at the 1M slice (the N = 8 rank's batch) with the
# lanes on their own hardware queues
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_ao}
mkdir -p "$OUT"
A="--steps 60 --warmup 5 --no-extras --cpu-sample 0 --weak-topics 0 --check 2000 --topics 1000000"
AB="--ab-opt walk_bpc=5 --ab-opt walk_bpc=0 --ab-opt presort=6,light_tail=150 --ab-opt presort=6,light_tail=30
 --ab-opt presort=3 --ab-opt stage_k=64 --ab-opt stage_k=128 --ab-opt slots=3 --ab-opt slots=2 --ab-opt walk_bpc=5"
timeout -k 10 300 python -u bench.py $A $AB > "$OUT/c3_1m.json" 2> "$OUT/c3_1m.log" || exit $?
