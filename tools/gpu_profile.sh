# usage (on the GPU box): bash tools/gpu_profile.sh <tag>
# rocprofv3 kernel trace + PMC passes at the bench's own batch sizes, in two
# section groups so that every decode kernel type is launched by ONE bench key
# per run (group g1: the headline, LDPC BP-20, CA-SCL L=32, configs[4] polar
# N=4096 and MS-20 without early stop at 131 072 frames; group g2: the default
# frozen set, the published SC configuration, configs[0] and MS-20 with early
# stop, and BP-20 on valid codewords), into gpurun_out/prof_<tag>/<group>/.  Summarise with
#   python tools/pmc_summary.py gpurun_out/prof_<tag> profiles/<round>_<tag>
# One counter group per run (rocprofv3 does not split passes), each run under
# its own time limit; the script stops at the first failing pass.
set -o pipefail
TAG=${1:-prof}
R="$GRAFT_REPO_ROOT"; BASE="$R/gpurun_out/prof_$TAG"; mkdir -p "$BASE"
export TMPDIR=/tmp; cd /tmp
# the profiled library build (bench.py compares it with the build it measures)
sha1sum "$R/polarcode_and_ldpc_amd/_lib/libpolarldpc.so" | cut -c1-16 > "$BASE/build_id.txt"
P_fetch="FETCH_SIZE"
P_write="WRITE_SIZE"
P_valu="SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_WAVES"
P_mix="SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_FLAT SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
P_l2="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"
P_wait="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS"
for G in ${GROUPS_TO_RUN:-g1 g2}; do
  case $G in
    g1) SECT="polar,ldpc,cascl,long_polar,long_ms_noes" ;;
    g2) SECT="polar_default,sc_default,config0,long_ms,ldpc_valid" ;;
  esac
  OUT="$BASE/$G"; mkdir -p "$OUT"
  ARGS="--skip-cpu --sections $SECT --long-batch 131072 --extra-steps 3"
  echo "$G start $(date)" >> "$BASE/progress.txt"
  timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
      python3 "$R/bench.py" $ARGS --steps 10 --warmup 2 > "$OUT/bench_trace.json" 2> "$OUT/trace.err" || exit $?
  echo "$G trace ok $(date)" >> "$BASE/progress.txt"
  for P in fetch write valu mix l2 wait; do
    eval C=\$P_$P
    timeout -k 10 -s KILL 300 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_$P" -o run -- \
        python3 "$R/bench.py" $ARGS --steps 2 --warmup 0 > "$OUT/pmc_$P.out" 2> "$OUT/pmc_$P.err" || exit $?
    echo "$G pmc $P ok $(date)" >> "$BASE/progress.txt"
  done
done
