# SC rate-0 skip with the node table read a leaf ahead: A/B against the pre-change library
set -o pipefail
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out/r03"; cd "$R"
timeout -k 10 300 python3 tools/ab.py --cases polar_sc,polar_sc_def,polar_sc256 --reps 3 build/lib_pre.so \
    polarcode_and_ldpc_amd/_lib/libpolarldpc.so > gpurun_out/r03/ab_sc_skip3.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_polar.py -x -q -k "sc or SC" --timeout 200 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/r03/polar_tests_sc3.log 2>&1
