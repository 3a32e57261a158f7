# usage (on the GPU box): bash tools/ldpc_pmc.sh <tag> [case=ldpc_bp] [lib[@VAR=VAL,...]]...
# PMC passes (stall breakdown, instruction mix, LDS) over tools/ab.py's worker
# for one case, once per library / environment; summaries into
# gpurun_out/ldpc_pmc_<tag>/ (csv per pass + summary.json via pmc_summary-style sums).
set -o pipefail
TAG=${1:-probe}; CASE=${2:-ldpc_bp}; shift 2
R="$GRAFT_REPO_ROOT"; [ -n "$R" ] || R=$(cd "$(dirname "$0")/.." && pwd)
OUT="$R/gpurun_out/ldpc_pmc_$TAG"; mkdir -p "$OUT"
export TMPDIR=/tmp; cd /tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64"
P3="SQ_BUSY_CYCLES SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_TRANS_F64 SQ_WAVES SQ_LDS_UNALIGNED_STALL"
li=0
for LIB in "$@"; do
  li=$((li+1))
  path=${LIB%%@*}; extra=""; [ "$path" != "$LIB" ] && extra=${LIB#*@}
  pi=0
  for C in "$P1" "$P2" "$P3"; do
    pi=$((pi+1))
    echo "lib $li ($LIB) pass $pi" >> "$OUT/progress.txt"
    (
      export PL_LIB_PATH="$R/$path"
      IFS=',' read -ra KV <<< "$extra"; for kv in "${KV[@]}"; do [ -n "$kv" ] && export "$kv"; done
      timeout -k 10 -s KILL 120 rocprofv3 --pmc $C --output-format csv -d "$OUT/l${li}_p$pi" -o run -- \
          python3 "$R/tools/ab.py" --worker "$CASE" > "$OUT/l${li}_p$pi.out" 2> "$OUT/l${li}_p$pi.err"
    ) || { echo "lib $li pass $pi rc=$?" >> "$OUT/progress.txt"; exit 1; }
  done
done
echo done >> "$OUT/progress.txt"
