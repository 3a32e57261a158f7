# usage: bash tools/gpu_pmc2.sh <tag> [script args...]   SQ/TA/TD/TCP counter passes (default: polar bench)
set -o pipefail
TAG=${1:-pmc}; shift
if [ $# -gt 0 ]; then CMD=("$@"); else CMD=(bench.py --skip-cpu --skip-ldpc --steps 1 --warmup 0); fi
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/pmc2_$TAG"; mkdir -p "$OUT"
export TMPDIR=/tmp; cd /tmp
timeout -k 10 120 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VMEM"
P3="TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum TD_TD_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $P --output-format csv -d "$OUT/p$i" -o run -- \
      python3 "$R/${CMD[0]}" "${CMD[@]:1}" > "$OUT/p$i.out" 2> "$OUT/p$i.err" || echo "pass $i failed $?" >> "$OUT/fail.txt"
done
