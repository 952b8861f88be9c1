#!/bin/bash
# One parameterised GPU job (run through gpurun), output under gpurun_out/$TAG.
# Steps (space-separated in STEPS, run in order, each under its own time
# limit, stopping at the first failure):
#   tests     pytest -m gpu over $TESTS (default: tests)
#   smoke     __graft_entry__.smoke()
#   bench     python bench.py $BENCH_ARGS                -> bench.json / bench.log
#   prof      rocprofv3 --kernel-trace --stats of the bench -> prof/ (kernel_stats.csv)
#   prof3     the same over 3 streams, with the kernel overlap (tools/overlap.py) -> overlap.json
#   pmc       PMC passes (tools/pmc_passes.sh)           -> pmc/summary.json
#   traffic   per-launch walk traffic from those passes  -> profiles/traffic_c3.json (read by bench)
#   cmd       an arbitrary python command in $CMD         -> cmd.log
#   latency   open-loop batcher latency sweep             -> latency.jsonl
#   slices    rocprofv3 stats of one-GPU batches of $SLICES topics (the per-rank slices of strong scaling)
#   rehearse  the driver's N > 1 launch with $NPROC ranks sharing GPU 0 (control plane over gloo)
#   routed    bench --mode routed in one process: $SHARDS routed shards on GPU 0 (device-copy exchange)
#   routed1   bench --mode routed through the driver's torchrun launch at world 1, own buckets over RCCL
#   sharded1  bench --mode sharded likewise (tm_shard_exchange over a one-rank RCCL communicator)
#   batcher   tools/bench_batcher.py $BATCHER_ARGS (flood: per-stage split, eager sealing, replicas)
# e.g. gpurun -- 'STEPS="tests bench prof" TAG=r02_head bash tools/gpu.sh'
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-job}
mkdir -p "$OUT"
for s in ${STEPS:-tests}; do
  case $s in
    tests) timeout -k 10 ${T_TESTS:-1500} python -u -m pytest ${TESTS:-tests} -m gpu -x -v --durations=20 \
             --timeout ${T_TEST1:-420} --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 ;;
    smoke) timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 ;;
    bench) timeout -k 10 ${T_BENCH:-600} python -u bench.py ${BENCH_ARGS} > "$OUT/bench.json" 2> "$OUT/bench.log" ;;
    prof)  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
             python3 bench.py --steps 10 --warmup 2 --cpu-sample 0 --check 0 --streams 1 --no-extras --weak-topics 0 ${BENCH_ARGS} \
             > "$OUT/prof_bench.json" 2> "$OUT/prof_bench.log" ;;
    pmc)   PMC_DIR=${TAG:-job}/pmc bash tools/pmc_passes.sh ;;
    prof3) timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof3" -o run -- \
             python3 bench.py --steps 20 --warmup 3 --cpu-sample 0 --check 0 --streams 3 --no-extras ${BENCH_ARGS} \
             > "$OUT/prof3_bench.json" 2> "$OUT/prof3_bench.log" && \
           python3 tools/overlap.py "$OUT/prof3/run_kernel_trace.csv" 23 2 > "$OUT/overlap.json" ;;
    prof4) timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof4" -o run -- \
             python3 bench.py --config 4 --steps 10 --warmup 2 --cpu-sample 0 --check 0 --streams 1 --no-extras \
             > "$OUT/prof4_bench.json" 2> "$OUT/prof4_bench.log" ;;
    traffic) python3 tools/traffic.py "$OUT/pmc" ${TRAFFIC_OUT:-profiles/traffic_c3.json} > "$OUT/traffic.json" ;;
    slices) for T in ${SLICES:-1000000 2000000 4000000 8000000}; do
             timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/slice_$T" -o run -- \
               python3 bench.py --topics $T --steps 40 --warmup 5 --cpu-sample 0 --check 2000 --weak-topics 0 \
               --no-extras ${BENCH_ARGS} > "$OUT/slice_$T.json" 2> "$OUT/slice_$T.log" || exit $?
           done ;;
    rehearse) TM_BENCH_SHARE_GPU=1 timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 \
               --nproc-per-node ${NPROC:-2} --master-addr 127.0.0.1 --master-port ${PORT:-29533} bench.py \
               --gpus ${NPROC:-2} --steps 20 --warmup 3 --no-extras ${BENCH_ARGS} \
               > "$OUT/rehearse_${NPROC:-2}.json" 2> "$OUT/rehearse_${NPROC:-2}.log" ;;
    routed) timeout -k 10 600 python3 -u bench.py --mode routed --single-process --shards ${SHARDS:-4} \
               --steps 20 --warmup 3 --depth ${DEPTH:-2} ${BENCH_ARGS} > "$OUT/routed_${SHARDS:-4}.json" \
               2> "$OUT/routed_${SHARDS:-4}.log" ;;
    routed1) timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
               --master-port ${PORT:-29534} bench.py --mode routed --self-rccl --steps 20 --warmup 3 \
               --depth ${DEPTH:-2} ${BENCH_ARGS} > "$OUT/routed_torchrun_w1.json" 2> "$OUT/routed_torchrun_w1.log" ;;
    sharded1) timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
               --master-port ${PORT:-29535} bench.py --mode sharded --self-rccl --steps 10 --warmup 2 \
               ${BENCH_ARGS} > "$OUT/sharded_torchrun_w1.json" 2> "$OUT/sharded_torchrun_w1.log" ;;
    batcher) timeout -k 10 ${T_BATCHER:-600} python3 -u tools/bench_batcher.py ${BATCHER_ARGS} \
               >> "$OUT/batcher.jsonl" 2>> "$OUT/batcher.log" ;;
    cmd)   timeout -k 10 ${T_CMD:-600} python -u -c "$CMD" > "$OUT/cmd.log" 2>&1 ;;
    latency) timeout -k 10 ${T_LAT:-400} python -u tools/bench_batcher_latency.py ${LAT_ARGS} \
             >> "$OUT/latency.jsonl" 2>> "$OUT/latency.log" ;;
    *)     echo "unknown step $s"; false ;;
  esac
  rc=$?
  echo "step $s rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
