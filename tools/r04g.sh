STEPS="tests" TESTS="tests/test_gpu_parity.py tests/test_gpu_routed.py tests/test_gpu_shard.py" TAG=r04_g T_TESTS=400 bash tools/gpu.sh; rc=$?
[ $rc -le 1 ] || exit $rc
LIBS="base quad" ROUNDS=2 TAG=r04_g T_RUN=200 bash tools/ab_libs.sh || exit $?
PMC_DIR=r04_g/pmc_pair PASSES="wr" T_PMC=150 bash tools/pmc_passes.sh || exit $?
PMC_DIR=r04_g/pmc_quad PASSES="wr" T_PMC=150 BENCH_ARGS="--lib emqx_amd/variants/libtopicmatch_quad.so" bash tools/pmc_passes.sh || exit $?
