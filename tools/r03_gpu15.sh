# multi-word partial-sum walk with batched loads (WB = 4 product, 2 variant) and L=16 element-loop unroll 4 (v1): A/B vs HEAD, polar tests
set -o pipefail
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out/r03"; cd "$R"
L=polarcode_and_ldpc_amd/_lib/libpolarldpc.so
timeout -k 10 600 python3 tools/ab.py --cases polar_l8,polar_l16,polar_l32,polar_4096,polar_sc --reps 3 build/lib_v1.so "$L" \
    > gpurun_out/r03/ab_walk1.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_polar.py -x -v --timeout 300 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/r03/polar_tests_walk1.log 2>&1
