#!/bin/bash
# C4 measurements on one MI355X: (1) rocprofv3 kernel trace of the sharded
# pipeline emulated at C3 size (walk with keys + merge kernels), (2) the full
# C4 emulation (100M filters, 8 shards, 8M-topic batch), (3) C4 replicated:
# all 100M filters in ONE engine (the image fits in 288 GB of HBM).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-c4}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_emu -o run -- python3 tools/c4_emulate.py --config 3 --filters 10000000 --topics 2000000 --check 20000 > $OUT/c4emu_c3.json 2> $OUT/c4emu_c3.log && \
timeout -k 10 600 python -u tools/c4_emulate.py > $OUT/c4emu.json 2> $OUT/c4emu.log && \
timeout -k 10 600 python -u bench.py --config 4 --mode replicated --check 0 --cpu-sample 0 > $OUT/bench_c4_repl.json 2> $OUT/bench_c4_repl.log
