#!/bin/bash
# A/B of HW queues per process x walk blocks per CU (stream overlap of
# neighbouring batches), one bench.py run per point, 2 rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab_q
for r in 1 2; do
for cfg in "4 0" "8 0" "8 6" "8 5"; do
  set -- $cfg
  echo "round $r queues $1 bpc $2"
  GPU_MAX_HW_QUEUES=$1 timeout -k 10 240 python -u bench.py --opt walk_bpc=$2 --steps 10 --warmup 2 --cpu-sample 0 --check 2000 --no-extras > gpurun_out/ab_q/run_${r}_$1_$2.json 2> gpurun_out/ab_q/run_${r}_$1_$2.log || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(json.dumps({'round':$r,'queues':$1,'bpc':$2,'value':d['value'],'ms_per_step':d['ms_per_step'],'kernel_ms':d.get('kernel_ms')}))" gpurun_out/ab_q/run_${r}_$1_$2.json | tee -a gpurun_out/ab_q/ab.jsonl
done
done
