# usage (on the GPU box): bash tools/gpu_profile.sh <tag>
# rocprofv3 kernel trace + PMC passes over the bench sections that each launch
# one decode kernel, into gpurun_out/prof_<tag>/.  Summarise with
#   python tools/pmc_summary.py gpurun_out/prof_<tag> profiles/<round>_<tag>
# One counter group per run (rocprofv3 does not split passes), each run under
# its own time limit; the script stops at the first failing pass.
set -o pipefail
TAG=${1:-prof}
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/prof_$TAG"; mkdir -p "$OUT"
export TMPDIR=/tmp; cd /tmp
SECT="polar,ldpc,cascl,long_polar,long_ms_noes"
ARGS="--skip-cpu --sections $SECT --long-batch 32768 --extra-steps 3"
echo "start $(date)" > "$OUT/progress.txt"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 "$R/bench.py" $ARGS --steps 10 --warmup 2 > "$OUT/bench_trace.json" 2> "$OUT/trace.err" || exit $?
echo "trace ok $(date)" >> "$OUT/progress.txt"
P_fetch="FETCH_SIZE"
P_write="WRITE_SIZE"
P_valu="SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_WAVES"
P_mix="SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_FLAT SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
P_l2="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"
for P in fetch write valu mix l2; do
  eval C=\$P_$P
  timeout -k 10 -s KILL 240 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_$P" -o run -- \
      python3 "$R/bench.py" $ARGS --steps 2 --warmup 0 > "$OUT/pmc_$P.out" 2> "$OUT/pmc_$P.err" || exit $?
  echo "pmc $P ok $(date)" >> "$OUT/progress.txt"
done
