# usage: bash tools/gpu_diag.sh <tag>
# Polar kernel diagnostics: phase stamps, SQ counter passes, resident-wave sweep.
set -o pipefail
TAG=${1:-diag}
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/diag_$TAG"; mkdir -p "$OUT"
cd "$R"
bash tools/gpu_sweep.sh "waves_$TAG" "PL_POLAR_WAVES=3072;PL_POLAR_WAVES=2048;PL_POLAR_WAVES=1536;PL_POLAR_WAVES=1024;PL_POLAR_WAVES=512" --skip-ldpc --steps 3 --warmup 1 || exit $?
export TMPDIR=/tmp; cd /tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $P --output-format csv -d "$OUT/p$i" -o run -- \
      python3 "$R/bench.py" --skip-cpu --skip-ldpc --steps 1 --warmup 0 > "$OUT/p$i.out" 2> "$OUT/p$i.err" || exit $?
done
