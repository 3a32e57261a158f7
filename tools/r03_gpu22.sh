# de-duplicated fused-top reads at N = 2048 / 4096 now that its prefetch overlaps (n <= 12 vs n <= 10)
set -o pipefail
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out/r03"; cd "$R"
L=polarcode_and_ldpc_amd/_lib/libpolarldpc.so
timeout -k 10 600 python3 tools/ab.py --cases polar_2048,polar_4096 --reps 3 "$L" build/lib_dd12.so \
    > gpurun_out/r03/ab_dedup12.log 2>&1
