# round-3 GPU session 1: LDPC vote A/B, then the stall / DRAM counter probe
set -o pipefail
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out/r03"
cd "$R"
timeout -k 10 300 python3 tools/ab.py --cases ldpc_bp,ldpc_bp_valid --reps 3 build/lib_base.so polarcode_and_ldpc_amd/_lib/libpolarldpc.so > gpurun_out/r03/ab_vote.log 2>&1 || exit $?
EXTRA_PASSES="TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" timeout -k 10 900 bash tools/probe_stalls.sh r03a
