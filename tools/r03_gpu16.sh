# fused-top prefetch issued inside the element loop when it has an inner loop (IPC > unroll): A/B vs HEAD, polar tests
set -o pipefail
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out/r03"; cd "$R"
L=polarcode_and_ldpc_amd/_lib/libpolarldpc.so
timeout -k 10 600 python3 tools/ab.py --cases polar_l8,polar_l16,polar_l32,polar_4096 --reps 3 build/lib_base.so "$L" \
    > gpurun_out/r03/ab_pf_in.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_polar.py -x -v --timeout 300 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/r03/polar_tests_pf_in.log 2>&1
