# HBM traffic of experimental builds (diagnostic), on the GPU box:
#   bash tools/pmc_ab.sh <tag> <sections> <lib>...
# for each library (PL_LIB_PATH) one FETCH_SIZE and one WRITE_SIZE pass of
# bench.py over <sections> at the bench's batches, into gpurun_out/pmcab_<tag>/
# <lib name>_<counter>/; summarise with python tools/pmc_kernel_sum.py.
set -o pipefail
TAG=$1; SECT=$2; shift 2
R="$GRAFT_REPO_ROOT"; [ -n "$R" ] || R=$(cd "$(dirname "$0")/.." && pwd)
BASE="$R/gpurun_out/pmcab_$TAG"; mkdir -p "$BASE"
export TMPDIR=/tmp; cd /tmp
for L in "$@"; do
  N=$(basename "$L" .so)
  export PL_LIB_PATH="$R/$L"
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 -s KILL 300 rocprofv3 --pmc $C --output-format csv -d "$BASE/${N}_$C" -o run -- \
        python3 "$R/bench.py" --skip-cpu --sections "$SECT" --long-batch 131072 --steps 2 --warmup 0 \
        > "$BASE/${N}_$C.out" 2> "$BASE/${N}_$C.err" || exit $?
    echo "$N $C ok $(date)" >> "$BASE/progress.txt"
  done
done
