# usage: bash tools/gpu_ab.sh <tag> [pytest -k expr]
# A/B of an experimental build (polarcode_and_ldpc_amd/_lib/libpolarldpc_exp.so, via
# PL_LIB_PATH) against the default one: polar + LDPC GPU tests on the
# experimental library, then alternating bench runs (no CPU baseline) of both.
set -o pipefail
TAG=${1:-ab}; KEXPR=${2:-not native_library_loaded}
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/ab_$TAG"; mkdir -p "$OUT"
cd "$R"
EXP="$R/polarcode_and_ldpc_amd/_lib/libpolarldpc_exp.so"
if [ -n "$KEXPR" ]; then KA=(-k "$KEXPR"); else KA=(); fi
PL_LIB_PATH="$EXP" timeout -k 10 600 python -u -m pytest tests/test_gpu_polar.py tests/test_gpu_ldpc.py -x -q --timeout 200 \
    --timeout-method thread -p no:cacheprovider "${KA[@]}" > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for rep in 1 2; do
  for v in base exp; do
    if [ $v = exp ]; then LP="$EXP"; else LP="$R/polarcode_and_ldpc_amd/_lib/libpolarldpc.so"; fi
    PL_LIB_PATH="$LP" timeout -k 10 300 python -u bench.py --skip-cpu > "$OUT/bench_$v$rep.json" 2> "$OUT/bench_$v$rep.err" || exit $?
    python -c "import json;d=json.load(open('$OUT/bench_$v$rep.json'));print('$v','polar',round(d['value'],1),round(d['roofline']['kernel_ms'],3),'ldpc',round(d['ldpc']['value'],1),round(d['ldpc']['kernel_ms'],3))"
  done
done
