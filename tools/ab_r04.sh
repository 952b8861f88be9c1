#!/bin/bash
# Interleaved same-box A/B of round-4's tree (abtree_r04/: `git archive 90aaef7`,
# built in place with its own Makefile) against HEAD, VERDICT r5 item 1.
# Each round runs, in this order: HEAD with high-priority lanes (the default),
# HEAD with torch pool streams (--stream-kind pool, round 4's lanes), round 4's
# bench.py + library.  Every run reports the C3 8M strong figure and the weak
# 1M/GPU figure of the same process.  One JSON line per run in
# gpurun_out/$TAG/ab.jsonl.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/${TAG:-ab_r04}
mkdir -p "$OUT"
ARGS="--steps ${STEPS_N:-20} --warmup ${WARM_N:-5} --cpu-sample 0 --check 2000 --no-extras ${BENCH_ARGS}"
for r in $(seq 1 ${ROUNDS:-3}); do
  for v in ${VARIANTS:-head_prio head_pool r04}; do
    case $v in
      head_prio) dir=.; extra="" ;;
      head_pool) dir=.; extra="--stream-kind pool" ;;
      r04) dir=abtree_r04; extra="" ;;
      *) dir=.; extra="$(echo ${v#*:} | tr ',' ' ')" ;;
    esac
    echo "round $r $v"
    (cd $dir && timeout -k 10 ${T_RUN:-300} python -u bench.py $ARGS $extra) > "$OUT/run_${r}_${v%%:*}.json" \
      2> "$OUT/run_${r}_${v%%:*}.log"
    rc=$?
    [ $rc -eq 0 ] || { echo "run $r $v rc=$rc"; exit $rc; }
    python3 -c "
import json,sys
d=json.load(open(sys.argv[1])); w=d.get('weak') or {}
print(json.dumps({'round':$r,'variant':'$v','value':d['value'],'ms_per_step':d['ms_per_step'],
  'walk_ms':(d.get('kernel_ms') or {}).get('walk'),'weak_value':w.get('value'),'weak_ms':w.get('ms_per_step'),
  'parity':d.get('parity_check')}))" "$OUT/run_${r}_${v%%:*}.json" | tee -a "$OUT/ab.jsonl"
  done
done
