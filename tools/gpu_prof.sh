# usage: bash tools/gpu_prof.sh <tag> [bench args...]
set -o pipefail
TAG=$1; shift
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/prof_$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
echo "start $(date)" > "$OUT/progress.txt"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 "$R/bench.py" --skip-cpu "$@" > "$OUT/bench_trace.json" 2> "$OUT/bench_trace.err" || exit $?
echo "trace done $(date)" >> "$OUT/progress.txt"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- \
    python3 "$R/bench.py" --skip-cpu "$@" > /dev/null 2> "$OUT/pmc_fetch.err" || exit $?
echo "fetch done $(date)" >> "$OUT/progress.txt"
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- \
    python3 "$R/bench.py" --skip-cpu "$@" > /dev/null 2> "$OUT/pmc_write.err" || exit $?
echo "write done $(date)" >> "$OUT/progress.txt"
