#!/bin/bash
# GPU call: C5 bench (adaptive stage rows) + its kernel trace, ACL bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-c5b}
mkdir -p $OUT
timeout -k 10 400 python -u bench.py --config 5 --topics 1000000 --cpu-sample 20000 --check 5000 --steps 10 > $OUT/bench_c5.json 2> $OUT/bench_c5.log && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c5 -o run -- python3 bench.py --config 5 --topics 1000000 --cpu-sample 0 --check 0 --steps 5 > $OUT/prof_c5.json 2> $OUT/prof_c5.log && \
timeout -k 10 300 python -u tools/bench_acl.py > $OUT/acl.json 2> $OUT/acl.log
