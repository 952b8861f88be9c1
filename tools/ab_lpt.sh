#!/bin/bash
# Tail-order experiment: the same batch sizes walked in arrival order and
# with the predicted-heavy topics first in each XCD range (bench.py
# --presort lpt, host-ordered), interleaved; one JSON line per run in
# gpurun_out/$TAG/ab.jsonl.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-ab_lpt}
mkdir -p "$OUT"
for r in $(seq 1 ${ROUNDS:-2}); do
  for T in ${SIZES:-1000000 8000000}; do
    for mode in base lpt; do
      extra=""
      [ $mode = lpt ] && extra="--presort lpt"
      timeout -k 10 ${T_RUN:-300} python -u bench.py --topics $T $extra --steps ${STEPS_N:-40} --warmup 3 \
        --cpu-sample 0 --check 2000 --weak-topics 0 --no-extras > "$OUT/run_${r}_${T}_$mode.json" \
        2> "$OUT/run_${r}_${T}_$mode.log" || exit $?
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(json.dumps({'round':$r,'topics':$T,'mode':'$mode','value':d['value'],'ms_per_step':d['ms_per_step'],'kernel_ms':d.get('kernel_ms'),'parity':d.get('parity_check')}))" \
        "$OUT/run_${r}_${T}_$mode.json" | tee -a "$OUT/ab.jsonl"
    done
  done
done
