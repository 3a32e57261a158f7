set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q --timeout 300 -p no:cacheprovider > gpurun_out/r3_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r3_pytest.log; [ $rc -le 1 ] || exit $rc
for F in 2 3 4; do timeout -k 10 120 python tools/polar_stamps.py --fused $F >> gpurun_out/r3_stamps.jsonl 2>>gpurun_out/r3_stamps.err || exit $?; done
bash tools/gpu_sweep.sh F3 "PL_POLAR_FUSED=2;PL_POLAR_FUSED=3;PL_POLAR_FUSED=4" --skip-ldpc --steps 3 --warmup 1
