# frame epilogue (root partial-sum words 32 per round trip) and staging-loop unroll 2: A/B
set -o pipefail
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out/r03"; cd "$R"
L=polarcode_and_ldpc_amd/_lib/libpolarldpc.so
timeout -k 10 700 python3 tools/ab.py --cases polar_l8,polar_l32,polar_4096,polar_sc_def --reps 3 "$L" build/lib_epi.so build/lib_epist.so \
    > gpurun_out/r03/ab_epi.log 2>&1
