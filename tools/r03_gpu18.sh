# SC instances: deeper in-flight loads (U 32 / unroll 16, U 16 / unroll 16) vs the new defaults (U 16 / unroll 8)
set -o pipefail
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out/r03"; cd "$R"
L=polarcode_and_ldpc_amd/_lib/libpolarldpc.so
timeout -k 10 600 python3 tools/ab.py --cases polar_sc,polar_sc_def,polar_sc256,polar_sc4096,polar_sc128,polar_sc512,polar_sc2048 --reps 3 "$L" build/lib_scd.so build/lib_sce.so \
    > gpurun_out/r03/ab_sc_knobs2.log 2>&1
