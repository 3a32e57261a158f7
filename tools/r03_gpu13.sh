# lists above 256 (lane kernel, 16-bit path slots): the large-list GPU test
set -o pipefail
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out/r03"; cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_gpu_polar.py -x -v --timeout 240 --timeout-method thread \
    -p no:cacheprovider -k "large_lists" > gpurun_out/r03/large_lists.log 2>&1
