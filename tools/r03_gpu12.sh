# ordered pruning (full ordered list keeps its slots): A/B for list capacities 8/16/32 and N=4096, then the polar GPU tests
set -o pipefail
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out/r03"; cd "$R"
L=polarcode_and_ldpc_amd/_lib/libpolarldpc.so
timeout -k 10 500 python3 tools/ab.py --cases polar_l8,polar_l16,polar_l32,polar_4096 --reps 3 build/lib_op64.so "$L" build/lib_op8.so \
    > gpurun_out/r03/ab_ordered_prune.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_polar.py -x -v --timeout 300 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/r03/polar_tests_op.log 2>&1
