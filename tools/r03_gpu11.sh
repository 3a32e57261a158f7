# PC sampling of the headline polar decode (diagnostic): list the configurations, then one stochastic run
set -o pipefail
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out/r03/pcs"; cd "$R"
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/pcsample_polar.py 1 > gpurun_out/r03/pcs/plain.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 -L > gpurun_out/r03/pcs/list.log 2>&1
timeout -s KILL 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles \
    --pc-sampling-interval 1048576 -d gpurun_out/r03/pcs/stoch -o pcs --output-format csv \
    -- python3 tools/pcsample_polar.py 2 > gpurun_out/r03/pcs/stoch.log 2>&1
echo "stoch rc=$?"
ls -laR gpurun_out/r03/pcs | head -40
