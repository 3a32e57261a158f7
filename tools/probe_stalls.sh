# usage (on the GPU box): bash tools/probe_stalls.sh <tag>
# Counter list + one SQ stall-breakdown PMC pass (+ optional extra counter
# groups from $EXTRA_PASSES, ';'-separated) over the bench sections that each
# launch one decode kernel.  Output: gpurun_out/stall_<tag>/.
set -o pipefail
TAG=${1:-probe}
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/stall_$TAG"; mkdir -p "$OUT"
export TMPDIR=/tmp; cd /tmp
SECT=${SECT:-polar,ldpc,cascl}
ARGS="--skip-cpu --sections $SECT --extra-steps 2 --steps 2 --warmup 0"
timeout -k 10 -s KILL 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS"
i=0
IFS=';' read -ra PASSES <<< "$P1;${EXTRA_PASSES:-}"
for C in "${PASSES[@]}"; do
  [ -z "$C" ] && continue
  i=$((i+1))
  echo "pass $i: $C" >> "$OUT/progress.txt"
  timeout -k 10 -s KILL 240 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_$i" -o run -- \
      python3 "$R/bench.py" $ARGS > "$OUT/pmc_$i.out" 2> "$OUT/pmc_$i.err" || { echo "pass $i rc=$?" >> "$OUT/progress.txt"; exit 1; }
  echo "pass $i ok $(date)" >> "$OUT/progress.txt"
done
