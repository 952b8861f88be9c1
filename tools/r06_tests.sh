#!/bin/bash
# Round 6 at the final sources:
#   PART=1  every -m gpu test but the full-size and config files, the smoke,
#           then the C2 and C5 bench lines
#   PART=2  the full-size (8M-topic C3) and config (C1-C5) tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${TAG:-r06_tests}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
case ${PART:-1} in
  1) STEPS="tests smoke" TAG=$TAG T_TESTS=900 \
       TESTS="tests --ignore=tests/test_gpu_fullsize.py --ignore=tests/test_gpu_configs.py" bash tools/gpu.sh || exit $?
     timeout -k 10 400 python -u bench.py --config 2 --steps 100 --warmup 10 --cpu-sample 200000 --no-extras \
       --weak-topics 0 > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.log" || exit $?
     timeout -k 10 500 python -u bench.py --config 5 --steps 10 --warmup 3 --cpu-sample 20000 --no-extras \
       --weak-topics 0 --check 2000 > "$OUT/bench_c5.json" 2> "$OUT/bench_c5.log" ;;
  2) STEPS="tests" TAG=${TAG}_big T_TESTS=1100 TESTS="tests/test_gpu_fullsize.py tests/test_gpu_configs.py" \
       bash tools/gpu.sh ;;
esac
