# usage: bash tools/gpu_tests.sh <tag> [pytest -k expr]   all GPU tests (or a subset)
set -o pipefail
TAG=${1:-t}; KEXPR=${2:-}
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/tests_$TAG"; mkdir -p "$OUT"
cd "$R"
if [ -n "$KEXPR" ]; then KA=(-k "$KEXPR"); else KA=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider "${KA[@]}" > "$OUT/pytest.log" 2>&1; rc=$?
tail -30 "$OUT/pytest.log"; exit $rc
