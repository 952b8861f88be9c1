#!/bin/bash
# GPU call: new-feature parity tests, sharded merge timing (C3-size
# emulation under rocprofv3), subscription churn beside matching.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-misc}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_batcher.py tests/test_gpu_shard.py tests/test_gpu_routes.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_emu -o run -- python3 tools/c4_emulate.py --config 3 --filters 10000000 --topics 2000000 --check 20000 > $OUT/c4emu_c3.json 2> $OUT/c4emu_c3.log && \
timeout -k 10 400 python -u tools/bench_churn.py > $OUT/churn.json 2> $OUT/churn.log
