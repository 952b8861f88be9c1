#!/bin/bash
# GPU call: micro-batcher end-to-end (single-topic submits, C3), then the
# full C4 emulation (100M filters, 8 shards) with the LDS merge kernel.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-misc2}
mkdir -p $OUT
timeout -k 10 300 ./tools/ubench/batcher_bench 10000000 2000000 16 > $OUT/batcher.json 2> $OUT/batcher.log && \
timeout -k 10 700 python -u tools/c4_emulate.py > $OUT/c4emu.json 2> $OUT/c4emu.log
