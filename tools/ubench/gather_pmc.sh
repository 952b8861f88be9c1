#!/bin/bash
# PMC calibration of a random 16-B gather (tools/ubench/gather.hip): how many
# bytes FETCH_SIZE / TCC_EA0_RDREQ charge per missed 16-B load, against the
# known access count.  Output under gpurun_out/gather_pmc/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
D=gpurun_out/gather_pmc
mkdir -p $D
for cfg in "1 8 4096" "1 8 1024" "1 8 2"; do
  tag=$(echo $cfg | tr ' ' _)
  timeout -k 10 60 tools/ubench/gather $cfg > $D/rate_$tag.txt 2>&1 || exit 1
  timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/fetch_$tag -o run -- tools/ubench/gather $cfg \
    > $D/fetch_$tag.log 2>&1 || exit 1
  timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d $D/tcc_$tag -o run \
    -- tools/ubench/gather $cfg > $D/tcc_$tag.log 2>&1 || exit 1
done
echo done
