#!/bin/bash
# HEAD numbers for DESIGN: C4 with the default walk order (range-local word
# hash, 24 bits) against arrival order and the global 16-bit sort, then the
# slice-size table (rocprofv3 kernel stats per size)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${TAG:-r04_u}
C4_AB="--ab-opt presort=0 --ab-opt presort=1" SKIP_PMC=1 T_BENCH=700 TAG=$TAG bash tools/c4_ab.sh || exit $?
STEPS="slices" SLICES="1000000 2000000 4000000" TAG=$TAG bash tools/gpu.sh || exit $?
