set -o pipefail
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out/r03"; cd "$R"
timeout -k 10 300 python3 tools/ab.py --cases ldpc_bp,ldpc_bp_valid --reps 3 build/lib_lbase.so build/lib_pipe.so > gpurun_out/r03/ab_ldpc_pipe.log 2>&1 || exit $?
GROUPS_TO_RUN=g2 timeout -k 10 900 bash tools/gpu_profile.sh r03c
