# usage: bash tools/gpu_pmc.sh <tag> <script and args...>   (collects SQ counter passes)
set -o pipefail
TAG=$1; shift
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/pmc_$TAG"; mkdir -p "$OUT"
export TMPDIR=/tmp; cd /tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_ADD_F64 SQ_LDS_BANK_CONFLICT"
P3="SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INST_CYCLES_VMEM_RD"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P --output-format csv -d "$OUT/p$i" -o run -- python3 "$R/$@" > "$OUT/p$i.out" 2> "$OUT/p$i.err" || exit $?
done
