# One parameterised runner for GPU-box calls (replaces the round-3 one-off scripts):
#   gpurun -- 'bash tools/gpu_run.sh <command> ...'      outputs under gpurun_out/
#   full  <tag>                        -m gpu tests, smoke(), default bench.py      -> gpurun_out/full_<tag>/
#   tests <log> [pytest args]          pytest (default: tests -m gpu)                -> gpurun_out/<log>.log
#   bench <log> [bench.py args]        bench.py (stdout line + detail file)         -> gpurun_out/<log>.json
#   ab    <log> <cases> <reps> <lib[@VAR=VAL]>...   tools/ab.py A/B timing          -> gpurun_out/<log>.log
#   prof  <tag> [group]                tools/gpu_profile.sh (rocprofv3 trace + PMC)  -> gpurun_out/prof_<tag>/
# Every GPU step runs under its own timeout; the first failure ends the call.
set -o pipefail
R="$GRAFT_REPO_ROOT"; [ -n "$R" ] || R=$(cd "$(dirname "$0")/.." && pwd)
cd "$R" || exit 1
mkdir -p gpurun_out
cmd=$1; shift
case "$cmd" in
full)
    TAG=${1:-run}; OUT="gpurun_out/full_$TAG"; mkdir -p "$OUT"
    echo "start $(date)" > "$OUT/progress.txt"
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
        -p no:cacheprovider > "$OUT/pytest.log" 2>&1
    rc=$?; echo "pytest rc=$rc $(date)" >> "$OUT/progress.txt"; [ $rc -eq 0 ] || exit $rc
    timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit $?
    echo "smoke ok $(date)" >> "$OUT/progress.txt"
    timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --detail-out "$OUT/bench_detail.json" \
        > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
    echo "bench ok $(date)" >> "$OUT/progress.txt"
    ;;
tests)
    LOG=$1; shift; [ $# -gt 0 ] || set -- tests -m gpu
    timeout -k 10 900 python -u -m pytest "$@" -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
        > "gpurun_out/$LOG.log" 2>&1
    ;;
bench)
    LOG=$1; shift
    timeout -k 10 900 python -u bench.py --detail-out "gpurun_out/${LOG}_detail.json" "$@" \
        > "gpurun_out/$LOG.json" 2> "gpurun_out/$LOG.err"
    ;;
ab)
    LOG=$1; CASES=$2; REPS=$3; shift 3
    timeout -k 10 900 python3 tools/ab.py --cases "$CASES" --reps "$REPS" "$@" > "gpurun_out/$LOG.log" 2>&1
    ;;
prof)
    GROUPS_TO_RUN=${2:-g1 g2} timeout -k 10 1000 bash tools/gpu_profile.sh "$1"
    ;;
*)
    echo "unknown command: $cmd" >&2; exit 2 ;;
esac
