# SC rate-0 node skip and the MS register-cached adjacency: A/B against the
# libraries before each change, then the polar and LDPC tests
set -o pipefail
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out/r03"; cd "$R"
timeout -k 10 300 python3 tools/ab.py --cases polar_sc,polar_sc_def,polar_sc256,polar_l8 --reps 2 build/lib_pre.so \
    polarcode_and_ldpc_amd/_lib/libpolarldpc.so > gpurun_out/r03/ab_sc_skip.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/ab.py --cases ms_8192 --reps 3 build/lib_ri0.so \
    polarcode_and_ldpc_amd/_lib/libpolarldpc.so > gpurun_out/r03/ab_ms_regidx.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_polar.py tests/test_gpu_ldpc.py -x -v --timeout 300 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/r03/polar_ldpc_tests.log 2>&1
