# usage: bash tools/gpu_polar_all.sh <tag>   all polar GPU tests + per-config kernel timing
set -o pipefail
TAG=${1:-pa}
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/pall_$TAG"; mkdir -p "$OUT"
cd "$R"
timeout -k 10 900 python -u -m pytest tests/test_gpu_polar.py -x -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 300 python -u tools/polar_configs.py > "$OUT/configs.jsonl" 2> "$OUT/configs.err" || { tail "$OUT/configs.err"; exit 1; }
cat "$OUT/configs.jsonl"
