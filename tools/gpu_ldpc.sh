# usage: bash tools/gpu_ldpc.sh <tag>   LDPC parity tests + kernel timing variants
set -o pipefail
TAG=${1:-l}
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/ldpc_$TAG"; mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_ldpc.py -x -v --timeout 200 --timeout-method thread \
    -p no:cacheprovider > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for S in "X=0" "PL_LDPC_KERNEL=generic" "PL_LDPC_KERNEL=check"; do
  echo "== $S"
  env $S timeout -k 10 300 python -u tools/ldpc_bench.py || exit $?
  env $S timeout -k 10 300 python -u tools/ldpc_bench.py --valid || exit $?
done
