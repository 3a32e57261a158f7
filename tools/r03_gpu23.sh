# AMDGPU machine-scheduler strategies (max-ilp, max-memory-clause) against the default, all bench kernels
set -o pipefail
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out/r03"; cd "$R"
L=polarcode_and_ldpc_amd/_lib/libpolarldpc.so
timeout -k 10 700 python3 tools/ab.py --cases polar_l8,polar_l32,polar_4096,polar_sc_def,ldpc_bp,ms_8192 --reps 3 "$L" build/lib_silp.so build/lib_smem.so \
    > gpurun_out/r03/ab_sched.log 2>&1
