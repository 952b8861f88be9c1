#!/bin/bash
# GPU parity suite, then an interleaved A/B of image layouts (tools/ab_image.py)
# and the sharded pipeline's kernel trace at C3 size.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-ab}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 400 python -u tools/ab_image.py --variants "${VARIANTS:-hot_levels=0,hot_levels=0@split=1,hot_levels=3,hot_levels=3@split=1,hot_levels=4@split=1}" > $OUT/ab.json 2> $OUT/ab.log && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_emu -o run -- python3 tools/c4_emulate.py --config 3 --filters 10000000 --topics 2000000 --check 20000 > $OUT/c4emu_c3.json 2> $OUT/c4emu_c3.log
