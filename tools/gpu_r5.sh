set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x --timeout 300 -p no:cacheprovider > gpurun_out/r5_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r5_pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_sweep.sh v3b "PL_POLAR_LDS_BUDGET=16384;PL_POLAR_LDS_BUDGET=8192;PL_POLAR_LDS_BUDGET=0;PL_POLAR_LDS_BUDGET=16384 PL_POLAR_FUSED=4;PL_POLAR_LDS_BUDGET=8192 PL_POLAR_FUSED=4" --skip-ldpc --steps 3 --warmup 1 || exit $?
cd /tmp && timeout -k 10 120 rocprofv3 -L > "$GRAFT_REPO_ROOT/gpurun_out/r5_counters.txt" 2>&1 || true
