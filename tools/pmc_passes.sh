#!/bin/bash
# PMC passes over the bench (one counter group per rocprofv3 run, within the
# gfx950 per-block slot limits of /opt/skills/guides/MI355X_MICROARCH.md).
# Output: gpurun_out/${PMC_DIR:-pmc}/<pass>/run_counter_collection.csv, then a
# per-kernel summary (tools/pmc_summary.py) in gpurun_out/${PMC_DIR}/summary.json
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
D=gpurun_out/${PMC_DIR:-pmc}
ARGS="--steps 3 --warmup 1 --roof-steps 0 --cpu-sample 0 --check 0 --streams 1 --batches 1 --no-extras --weak-topics 0 ${BENCH_ARGS}"
run() {
  name=$1; shift
  mkdir -p $D/$name
  timeout -s KILL ${T_PMC:-180} rocprofv3 --pmc "$@" --output-format csv -d $D/$name -o run -- python3 bench.py $ARGS > $D/$name/log.txt 2>&1
}
pass() {
  case $1 in
    fetch) run fetch FETCH_SIZE ;;
    write) run write WRITE_SIZE ;;
    wr)    run wr WRITE_SIZE TCC_EA0_WRREQ_sum TCP_TCC_WRITE_REQ_sum ;;
    tcc)   run tcc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum ;;
    sq)    run sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES ;;
    tcp)   run tcp TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_TOTAL_READ_sum ;;
    ta)    run ta TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum ;;
    # LDS behaviour of the tokenizer and the walk: bank conflicts, unaligned
    # 64/128-bit replays, LDS issue stalls (MI355X_MICROARCH.md LDS section)
    lds)   run lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_INSTS_LDS SQ_WAIT_INST_LDS \
              SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAIT_ANY ;;
    tlb)   run tlb TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_TCC_READ_REQ_sum ;;
    # the L2 and translation groups in one pass (3 TCC + 4 TCP slots): for
    # workloads whose build dominates a pass (C4: 100M filters)
    tcctlb) run tcctlb TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCP_UTCL1_TRANSLATION_MISS_sum \
              TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_TCC_READ_REQ_sum ;;
    *)     echo "unknown pass $1"; false ;;
  esac
}
for p in ${PASSES:-fetch write tcc sq tcp ta}; do
  pass $p || exit $?
done
python3 tools/pmc_summary.py $D > $D/summary.json
