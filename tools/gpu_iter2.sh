# usage: bash tools/gpu_iter2.sh <tag> "<ENV=..;ENV=..>"  polar tree tests + bench sweep over env settings
set -o pipefail
TAG=${1:-it}; SETS=${2:-"X=0"}
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/iter_$TAG"; mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_polar.py -x -v --timeout 200 --timeout-method thread \
    -p no:cacheprovider -k "tree or scl_1024 or vs_oracle" > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
IFS=';' read -ra ARR <<< "$SETS"
for s in "${ARR[@]}"; do
  env $s timeout -k 10 300 python -u bench.py --skip-cpu --skip-ldpc > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
  python -c "import json;d=json.load(open('$OUT/bench.json'));print('$s', 'value',round(d['value'],1),'kernel_ms',round(d['roofline']['kernel_ms'],3))"
done
timeout -k 10 120 python -u tools/polar_stamps.py > "$OUT/stamps.json" 2> "$OUT/stamps.err" || exit $?
cat "$OUT/stamps.json"
