# round-3 full validation: GPU tests, smoke, default bench (one gpurun call)
set -o pipefail
TAG=${1:-r03}
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/full_$TAG"; mkdir -p "$OUT"
cd "$R"
echo "start $(date)" > "$OUT/progress.txt"
timeout -k 10 780 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > "$OUT/pytest.log" 2>&1
rc=$?
echo "pytest rc=$rc $(date)" >> "$OUT/progress.txt"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit $?
echo "smoke ok $(date)" >> "$OUT/progress.txt"
timeout -k 10 420 python -u bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
echo "bench ok $(date)" >> "$OUT/progress.txt"
