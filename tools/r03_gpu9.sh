# SC tree instances at F = 1, DL = n - 5: A/B against the round-3 start library, then the polar GPU tests
set -o pipefail
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out/r03"; cd "$R"
timeout -k 10 600 python3 tools/ab.py --cases polar_sc128,polar_sc256,polar_sc512,polar_sc,polar_sc_def,polar_sc2048,polar_sc4096 --reps 2 \
    build/lib_pre.so polarcode_and_ldpc_amd/_lib/libpolarldpc.so > gpurun_out/r03/ab_sc_tiers.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_polar.py tests/test_gpu_harness.py -x -v --timeout 300 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/r03/polar_tests_tiers.log 2>&1
