set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x --timeout 300 -p no:cacheprovider > gpurun_out/r4_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r4_pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_sweep.sh v3 "PL_POLAR_LDS_BUDGET=40960;PL_POLAR_LDS_BUDGET=16384;PL_POLAR_LDS_BUDGET=65536;PL_POLAR_FUSED=2;PL_POLAR_FUSED=4;PL_POLAR_FUSED=4 PL_POLAR_LDS_BUDGET=16384;PL_POLAR_KERNEL=group PL_POLAR_FUSED=4" --skip-ldpc --steps 3 --warmup 1
