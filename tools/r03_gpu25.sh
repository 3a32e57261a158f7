# LDPC reg kernel with 192 threads per frame (EPT 8, VPT 3: 5 frames per CU) against 256: A/B + LDPC tests at 192
set -o pipefail
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out/r03"; cd "$R"
L=polarcode_and_ldpc_amd/_lib/libpolarldpc.so
timeout -k 10 600 python3 tools/ab.py --cases ldpc_bp,ldpc_bp_valid --reps 3 "$L" "$L@PL_LDPC_NT=192" \
    > gpurun_out/r03/ab_ldpc_nt192.log 2>&1 || exit $?
PL_LDPC_NT=192 timeout -k 10 600 python -u -m pytest tests/test_gpu_ldpc.py -x -v --timeout 300 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/r03/ldpc_tests_nt192.log 2>&1
