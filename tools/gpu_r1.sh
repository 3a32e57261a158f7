set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
echo "start $(date)" > gpurun_out/r1_progress.txt
timeout -k 10 900 python -m pytest tests -m gpu -x -q --timeout 400 -p no:cacheprovider > gpurun_out/r1_pytest.log 2>&1
rc=$?
echo "pytest rc=$rc $(date)" >> gpurun_out/r1_progress.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/r1_bench.json 2> gpurun_out/r1_bench.err
echo "bench rc=$? $(date)" >> gpurun_out/r1_progress.txt
