#!/bin/bash
# C4 (100M filters, replicated on one GPU) walk-order A/B in one process
# (one trie build): the default (presort 3: the word-hash order over the key's
# top 16 bits at 8M topics), arrival order, the tail order and the full 32-bit
# key, then one PMC pass (L2 + address translation counters) of the same
# variants; per-dispatch counters with tools/pmc_sequence.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04_c4}
mkdir -p "$OUT"
if [ "${SKIP_BENCH:-0}" != 1 ]; then
  timeout -k 10 ${T_BENCH:-1000} python -u bench.py --config 4 ${C4_AB:---ab-opt presort=0 --ab-opt presort=2 --ab-opt sort_bits=32} --steps 10 \
    --warmup 2 --roof-steps 10 --no-extras --cpu-sample 0 --check 2000 --weak-topics 0 \
    > "$OUT/bench_c4_ab.json" 2> "$OUT/bench_c4_ab.log" || exit $?
fi
if [ "${SKIP_PMC:-0}" != 1 ]; then
  PMC_DIR=${TAG:-r04_c4}/pmc PASSES=tcctlb T_PMC=${T_PMC:-1000} \
    BENCH_ARGS="--config 4 ${C4_AB:---ab-opt presort=0 --ab-opt presort=2 --ab-opt sort_bits=32}" bash tools/pmc_passes.sh || exit $?
  python3 tools/pmc_sequence.py "$OUT/pmc/tcctlb" tm_walk_queue --topics 8000000 > "$OUT/pmc_walk_sequence.jsonl"
fi
