# bitonic L=32 ranks: A/B timing against the pre-change library, then the full validation
set -o pipefail
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out/r03"; cd "$R"
timeout -k 10 300 python3 tools/ab.py --cases polar_l32,polar_l8 --reps 2 build/lib_pre.so \
    polarcode_and_ldpc_amd/_lib/libpolarldpc.so > gpurun_out/r03/ab_bitonic.log 2>&1 || exit $?
bash tools/r03_full.sh r03b
