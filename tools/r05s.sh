#!/bin/bash
# round 5: pipeline depth -- with 2 workspace slots a batch's tokenizer
# waits for the copy-out two batches back, so it lands behind the running
# walk; with 3-4 slots it can run before the walk takes the whole GPU and
# the next walk can fill the drain.  A/B of option slots at C3 1M and 8M
# (3 and 4 streams), then a kernel timeline at 1M with 3 slots
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_s}
mkdir -p "$OUT"
A="--steps 20 --warmup 3 --no-extras --cpu-sample 0 --weak-topics 0 --check 2000"
AB="--ab-opt slots=3 --ab-opt slots=2 --ab-opt slots=4 --ab-opt slots=2 --ab-opt slots=3"
timeout -k 10 300 python -u bench.py $A --topics 1000000 $AB > "$OUT/c3_1m.json" 2> "$OUT/c3_1m.log" || exit $?
timeout -k 10 300 python -u bench.py $A --topics 1000000 --streams 4 --batches 4 $AB > "$OUT/c3_1m_s4.json" 2> "$OUT/c3_1m_s4.log" || exit $?
timeout -k 10 400 python -u bench.py $A $AB > "$OUT/c3_8m.json" 2> "$OUT/c3_8m.log" || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_1m_slots3" -o run -- \
  python3 bench.py --topics 1000000 --steps 20 --warmup 3 --cpu-sample 0 --check 0 --no-extras --weak-topics 0 \
  --opt slots=3 > "$OUT/prof_1m_slots3.json" 2> "$OUT/prof_1m_slots3.log" || exit $?
