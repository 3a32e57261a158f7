set -o pipefail
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out/r03"; cd "$R"
timeout -k 10 400 python3 tools/l32_diag.py > gpurun_out/r03/l32_diag.log 2>&1
