#!/bin/bash
# GPU call: walk time with the batch presorted on the host (untimed) by the
# word at one level, for LEVELS (and "all" = whole-topic sort), vs unsorted.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-presort}
mkdir -p $OUT
A="--steps 10 --warmup 2 --check 0 --cpu-sample 0 --streams 1 --topics 2000000"
timeout -k 10 200 python -u bench.py $A > $OUT/none.json 2> $OUT/none.log || exit 1
for lv in $LEVELS; do
  if [ "$lv" = all ]; then P="--presort"; else P="--presort-level $lv"; fi
  timeout -k 10 300 python -u bench.py $A $P > $OUT/l$lv.json 2> $OUT/l$lv.log || exit 1
done
