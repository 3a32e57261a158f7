# fused-top depth after the prefetch fix: F = 3 (default) vs 4 / 2 (diagnostic build), L = 8 and 32
set -o pipefail
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out/r03"; cd "$R"
D=build/lib_diag.so
timeout -k 10 600 python3 tools/ab.py --cases polar_l8,polar_l32 --reps 3 "$D" "$D@PL_TREE_F=4" "$D@PL_TREE_F=2" \
    > gpurun_out/r03/ab_f4.log 2>&1
