#!/bin/bash
# PMC passes over the C3 bench (one counter group per rocprofv3 run, per the
# gfx950 slot limits in /opt/skills/guides/MI355X_MICROARCH.md).  Output:
# gpurun_out/pmc/<pass>/...counter_collection.csv
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
ARGS="--steps 3 --warmup 1 --cpu-sample 0 --check 0 ${BENCH_ARGS}"
run() {
  name=$1; shift
  mkdir -p gpurun_out/pmc/$name
  timeout -k 10 240 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/pmc/$name -o run -- python3 bench.py $ARGS > gpurun_out/pmc/$name/log.txt 2>&1
}
run fetch FETCH_SIZE
run write WRITE_SIZE
run tcc TCC_HIT_sum TCC_MISS_sum
run sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY
run tcp TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum
