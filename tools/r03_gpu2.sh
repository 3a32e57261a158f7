# round-3 GPU session 2: ablation timings of the polar tree kernel (diagnostic builds)
set -o pipefail
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out/r03"
cd "$R"
timeout -k 10 600 python3 tools/ab.py --cases polar_l8,polar_l32 --reps 2 build/lib_abl_base.so build/lib_abl_met.so \
    build/lib_abl_rank.so build/lib_abl_ws.so build/lib_abl_wsmet.so > gpurun_out/r03/ab_abl.log 2>&1
timeout -k 10 300 python3 tools/ab.py --cases ldpc_bp,ldpc_bp_valid --reps 3 polarcode_and_ldpc_amd/_lib/libpolarldpc.so build/lib_ilp.so > gpurun_out/r03/ab_ilp.log 2>&1
