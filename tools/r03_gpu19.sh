# SC N=1024 LDS tiers after the deeper in-flight loads: DL = n-5 (default) vs n-4 / n-6 (diagnostic build)
set -o pipefail
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out/r03"; cd "$R"
D=build/lib_diag.so
timeout -k 10 600 python3 tools/ab.py --cases polar_sc,polar_sc_def --reps 3 "$D" "$D@PL_TREE_DLOFF=4" "$D@PL_TREE_DLOFF=6" \
    > gpurun_out/r03/ab_sc_dl2.log 2>&1
