#!/bin/bash
# Round 6, VERDICT r5 item 7: the routed sharded mode at C4 (100M filters) in
# one process, S = 8 routed shards on GPU 0 (each shard the filters routed to
# it by their first two levels plus the wildcard-led ones, global ids; the
# topic exchange and list return by device copies through the RCCL-group
# entry points), every shard's lists checked against O3 over all filters.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06_routed}
mkdir -p "$OUT"
timeout -k 10 ${T_RUN:-1100} python -u bench.py --mode routed --single-process --shards ${SHARDS:-8} \
  --config ${CONFIG:-4} --steps 10 --warmup 2 --depth 2 --check 2000 --check-rank 2000 \
  > "$OUT/routed_c${CONFIG:-4}_s${SHARDS:-8}.json" 2> "$OUT/routed_c${CONFIG:-4}_s${SHARDS:-8}.log"
