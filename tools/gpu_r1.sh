set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
echo "start $(date)" > gpurun_out/r1_progress.txt
timeout -k 10 900 python -m pytest tests -m gpu -q --timeout 400 -p no:cacheprovider > gpurun_out/r1_pytest.log 2>&1
rc=$?
echo "pytest rc=$rc $(date)" >> gpurun_out/r1_progress.txt
exit $rc
