# long-block timing probe: the default bench with and without the CPU baseline legs
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/lp2
timeout -k 10 600 python -u bench.py --skip-cpu --steps 20 --warmup 5 > gpurun_out/lp2/full_skipcpu.json 2> gpurun_out/lp2/full_skipcpu.err || exit $?
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/lp2/full.json 2> gpurun_out/lp2/full.err || exit $?
