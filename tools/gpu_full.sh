# usage: bash tools/gpu_full.sh <tag>
# One GPU call: parity tests, smoke, default bench, rocprofv3 kernel trace + HBM PMC passes.
set -o pipefail
TAG=${1:-run}
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/full_$TAG"; mkdir -p "$OUT"
cd "$R"
echo "start $(date)" > "$OUT/progress.txt"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > "$OUT/pytest.log" 2>&1 || { echo "pytest failed $?" >> "$OUT/progress.txt"; exit 1; }
echo "pytest ok $(date)" >> "$OUT/progress.txt"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit $?
echo "smoke ok $(date)" >> "$OUT/progress.txt"
timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
echo "bench ok $(date)" >> "$OUT/progress.txt"
export TMPDIR=/tmp; cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 "$R/bench.py" --skip-cpu --skip-extra > "$OUT/bench_trace.json" 2> "$OUT/bench_trace.err" || exit $?
echo "trace ok $(date)" >> "$OUT/progress.txt"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- \
    python3 "$R/bench.py" --skip-cpu --skip-extra > /dev/null 2> "$OUT/pmc_fetch.err" || exit $?
echo "fetch ok $(date)" >> "$OUT/progress.txt"
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- \
    python3 "$R/bench.py" --skip-cpu --skip-extra > /dev/null 2> "$OUT/pmc_write.err" || exit $?
echo "write ok $(date)" >> "$OUT/progress.txt"
timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --output-format csv -d "$OUT/pmc_valu" -o run -- \
    python3 "$R/bench.py" --skip-cpu --skip-extra > /dev/null 2> "$OUT/pmc_valu.err" || exit $?
echo "valu ok $(date)" >> "$OUT/progress.txt"
