# fused-top prefetch kept in flight (partial-sum words loaded before it, unconditional): A/B, then polar GPU tests
set -o pipefail
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out/r03"; cd "$R"
L=polarcode_and_ldpc_amd/_lib/libpolarldpc.so
timeout -k 10 500 python3 tools/ab.py --cases polar_l8,polar_l16,polar_l32,polar_4096,polar_sc256 --reps 3 build/lib_base.so "$L" build/lib_full.so \
    > gpurun_out/r03/ab_prefetch.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_polar.py -x -v --timeout 300 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/r03/polar_tests_prefetch.log 2>&1
