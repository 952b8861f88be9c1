#!/bin/bash
# One GPU call for the sharded mode: parity tests, C4 emulation at C3 size
# with a bit-exact check against a whole-set engine, then the full C4
# emulation (100M filters, 8 shards, 8M-topic batch).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-shard}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_shard.py -x -v --timeout 200 --timeout-method thread > $OUT/pytest_shard.log 2>&1 && \
timeout -k 10 300 python -u tools/c4_emulate.py --config 3 --filters 10000000 --topics 2000000 --check 20000 > $OUT/c4emu_c3.json 2> $OUT/c4emu_c3.log && \
timeout -k 10 600 python -u tools/c4_emulate.py > $OUT/c4emu.json 2> $OUT/c4emu.log
