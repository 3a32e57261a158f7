set -o pipefail
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out/r03"; cd "$R"
timeout -k 10 300 python3 tools/ab.py --cases ldpc_bp --reps 2 build/lib_lbase.so build/lib_latanh.so build/lib_ltanh.so \
    build/lib_lprod.so build/lib_lall.so > gpurun_out/r03/ab_ldpc_abl.log 2>&1 || exit $?
GROUPS_TO_RUN=g1 timeout -k 10 1000 bash tools/gpu_profile.sh r03c
