# usage: bash tools/gpu_pmc3.sh <tag>   L2 hit rate / fabric stall passes over the polar bench
set -o pipefail
TAG=${1:-pmc3}
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/pmc3_$TAG"; mkdir -p "$OUT"
export TMPDIR=/tmp; cd /tmp
P1="TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT"
P2="TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum"
P3="TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $P --output-format csv -d "$OUT/p$i" -o run -- \
      python3 "$R/bench.py" --skip-cpu --skip-ldpc --steps 1 --warmup 0 > "$OUT/p$i.out" 2> "$OUT/p$i.err" || echo "pass $i failed $?" >> "$OUT/fail.txt"
done
