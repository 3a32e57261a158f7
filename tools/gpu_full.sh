# usage (on the GPU box): bash tools/gpu_full.sh <tag>
# One GPU call: parity tests, smoke, default bench, then tools/gpu_profile.sh.
set -o pipefail
TAG=${1:-run}
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/full_$TAG"; mkdir -p "$OUT"
cd "$R"
echo "start $(date)" > "$OUT/progress.txt"
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > "$OUT/pytest.log" 2>&1
rc=$?
echo "pytest rc=$rc $(date)" >> "$OUT/progress.txt"
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit $?
echo "smoke ok $(date)" >> "$OUT/progress.txt"
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
echo "bench ok $(date)" >> "$OUT/progress.txt"
bash "$R/tools/gpu_profile.sh" "$TAG"
