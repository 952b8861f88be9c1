#!/bin/bash
# Round 6, VERDICT r5 item 3: the walk's cache model (tools/sim) at C4 (100M
# filters): the per-class miss table DESIGN 5.2b has for C3, for the current
# layout, the upper bound without Bloom false positives, and node-ordered
# child blocks.  CPU only (the host mirror of a 100M-filter trie needs ~40 GB,
# more than the build container has), run on the GPU box's host.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${TAG:-r06_sim_c4}
mkdir -p "$OUT"
timeout -k 10 ${T_RUN:-1100} python3 -u tools/sim/run_sim.py --config 4 --topics 1000000 --sorted --l2 2097152 \
  --bloom-hist --layouts ${LAYOUTS:-cur,nofp,blocks+div8} > "$OUT/sim_c4.jsonl" 2> "$OUT/sim_c4.log"
