# LCAP = 8 fused top: two 16-byte pairs per lane per staged chunk (CH 2) with element-loop unroll 4 / 2 and in-loop prefetch
set -o pipefail
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out/r03"; cd "$R"
L=polarcode_and_ldpc_amd/_lib/libpolarldpc.so
timeout -k 10 600 python3 tools/ab.py --cases polar_l8,polar_sc --reps 3 "$L" build/lib_ch2a.so build/lib_ch2b.so build/lib_ch2c.so \
    > gpurun_out/r03/ab_ch2.log 2>&1
