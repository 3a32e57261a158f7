# usage: bash tools/gpu_iter.sh <tag> [pytest -k expr]
# Kernel iteration: polar GPU parity tests, polar-only bench, phase stamps.
set -o pipefail
TAG=${1:-it}; KEXPR=${2:-}
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/iter_$TAG"; mkdir -p "$OUT"
cd "$R"
if [ -n "$KEXPR" ]; then KA=(-k "$KEXPR"); else KA=(); fi
timeout -k 10 600 python -u -m pytest tests/test_gpu_polar.py -x -v --timeout 200 --timeout-method thread \
    -p no:cacheprovider "${KA[@]}" > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -3 "$OUT/pytest.log"
timeout -k 10 300 python -u bench.py --skip-cpu --skip-ldpc > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
python -c "import json;d=json.load(open('$OUT/bench.json'));print('value',d['value'],'kernel_ms',d['roofline']['kernel_ms'])"
timeout -k 10 120 python -u tools/polar_stamps.py > "$OUT/stamps.json" 2> "$OUT/stamps.err" || exit $?
cat "$OUT/stamps.json"
