#!/bin/bash
# Round 6, C4 (100M filters replicated on one GPU), VERDICT r5 item 3:
#   PART=1  the C4 bench with the big nodes' filters off (headline) and an
#           in-process A/B of option gfilter (on / off / on), O3 check
#   PART=2  one PMC pass (L2 hit / miss, EA read requests, UTCL1) over the
#           C4 bench: per-dispatch counters of the walk (tools/pmc_sequence.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06_c4}
mkdir -p "$OUT"
case ${PART:-1} in
  1) timeout -k 10 1100 python -u bench.py --config 4 --steps 20 --warmup 3 --no-extras --weak-topics 0 \
       --cpu-sample 0 --check 2000 --ab-opt gfilter=1 --ab-opt gfilter=0 --ab-opt gfilter=1 \
       > "$OUT/bench_c4_gf.json" 2> "$OUT/bench_c4_gf.log" ;;
  2) timeout -s KILL 1100 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCP_UTCL1_TRANSLATION_MISS_sum \
       TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_TCC_READ_REQ_sum --output-format csv \
       -d "$OUT/pmc_tcctlb" -o run -- python3 bench.py --config 4 --steps 2 --warmup 1 --roof-steps 0 --cpu-sample 0 \
       --check 0 --streams 1 --batches 1 --no-extras --weak-topics 0 \
       > "$OUT/pmc_tcctlb.log" 2>&1 ;;
esac
