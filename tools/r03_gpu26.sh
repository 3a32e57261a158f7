# LCAP = 8 fused top: D0 = 1 chunk loops fully unrolled (IPC 4), and the D0 = 2 prefetch inside its loop
set -o pipefail
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out/r03"; cd "$R"
L=polarcode_and_ldpc_amd/_lib/libpolarldpc.so
timeout -k 10 600 python3 tools/ab.py --cases polar_l8,polar_sc,polar_l32 --reps 6 "$L" build/lib_u4p.so \
    > gpurun_out/r03/ab_unr8b.log 2>&1
