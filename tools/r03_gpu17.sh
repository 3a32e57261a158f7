# SC instances: register budget (WPE 2), workspace pairs in flight (U 16), channel-loop unroll (8): A/B
set -o pipefail
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out/r03"; cd "$R"
L=polarcode_and_ldpc_amd/_lib/libpolarldpc.so
timeout -k 10 600 python3 tools/ab.py --cases polar_sc,polar_sc_def,polar_sc256,polar_sc4096 --reps 3 "$L" build/lib_sca.so build/lib_scb.so build/lib_scc.so \
    > gpurun_out/r03/ab_sc_knobs.log 2>&1
