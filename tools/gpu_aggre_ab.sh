#!/bin/bash
# GPU call: routes / deliveries bench over the default build and aggre.hip
# experiment variants (emqx_amd/variants/libtopicmatch_<v>.so).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-aggre_ab}
mkdir -p $OUT
timeout -k 10 300 python -u tools/bench_routes.py --check 0 > $OUT/default.json 2> $OUT/default.log || exit 1
for v in $VARS; do
  timeout -k 10 300 python -u tools/bench_routes.py --check 0 --lib emqx_amd/variants/libtopicmatch_$v.so > $OUT/$v.json 2> $OUT/$v.log || exit 1
done
