#!/bin/bash
# Interleaved A/B of compile-time variants (make variant TAG=x TMDEFS=...):
# ROUNDS rounds, each running bench.py once per library in LIBS ("base" =
# emqx_amd/libtopicmatch.so, otherwise emqx_amd/variants/libtopicmatch_<x>.so;
# "lib:name=val,name=val" adds engine options, bench.py --opt),
# one JSON line per run in gpurun_out/$TAG/ab.jsonl (value, walk ms, tag).
# e.g. gpurun -- 'LIBS="base nt6 ntst" ROUNDS=2 TAG=ab_nt bash tools/ab_libs.sh'
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-ab}
mkdir -p "$OUT"
for r in $(seq 1 ${ROUNDS:-2}); do
  for spec in ${LIBS:-base}; do
    l=${spec%%:*}
    opts=""
    if [ "$spec" != "$l" ]; then for o in $(echo ${spec#*:} | tr ',' ' '); do opts="$opts --opt $o"; done; fi
    if [ "$l" = base ]; then lib=emqx_amd/libtopicmatch.so; else lib=emqx_amd/variants/libtopicmatch_$l.so; fi
    l=$(echo "$spec" | tr ':=,' '_-_')
    echo "round $r lib $l"
    timeout -k 10 ${T_RUN:-240} python -u bench.py --lib $lib $opts --steps ${STEPS_N:-10} --warmup 3 --cpu-sample 0 \
      --check ${CHECK:-2000} --no-extras ${BENCH_ARGS} > "$OUT/run_${r}_$l.json" 2> "$OUT/run_${r}_$l.log"
    rc=$?
    [ $rc -eq 0 ] || { echo "run $r $l rc=$rc"; exit $rc; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(json.dumps({'round':$r,'lib':'$l','value':d['value'],'ms_per_step':d['ms_per_step'],'kernel_ms':d.get('kernel_ms'),'parity':d.get('parity_check')}))" \
      "$OUT/run_${r}_$l.json" | tee -a "$OUT/ab.jsonl"
  done
done
