# LDPC BP lane-per-check products: A/B against PL_LDPC_CPL=0 (same library), then the LDPC GPU tests;
# polar metric series path (build/lib_series.so) A/B
set -o pipefail
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out/r03"; cd "$R"
L=polarcode_and_ldpc_amd/_lib/libpolarldpc.so
timeout -k 10 400 python3 tools/ab.py --cases ldpc_bp,ldpc_bp_valid --reps 3 "$L@PL_LDPC_CPL=0" "$L" \
    > gpurun_out/r03/ab_ldpc_cpl.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_ldpc.py -x -v --timeout 300 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/r03/ldpc_tests_cpl.log 2>&1 || exit $?
timeout -k 10 400 python3 tools/ab.py --cases polar_l8,polar_l32,polar_4096 --reps 3 "$L" build/lib_series.so \
    > gpurun_out/r03/ab_polar_series.log 2>&1
