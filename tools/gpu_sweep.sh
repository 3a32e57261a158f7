# usage: bash tools/gpu_sweep.sh <tag> "<ENV=.. settings>;<...>" [bench args]
set -o pipefail
TAG=$1; shift; SETS=$1; shift
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
OUT=gpurun_out/sweep_$TAG.jsonl; : > $OUT
IFS=';' read -ra ARR <<< "$SETS"
for s in "${ARR[@]}"; do
  echo "== $s $(date)" >> gpurun_out/sweep_$TAG.log
  env $s timeout -k 10 300 python bench.py --skip-cpu "$@" > gpurun_out/sweep_tmp.json 2>> gpurun_out/sweep_$TAG.log || exit $?
  python -c "import json,sys;d=json.load(open('gpurun_out/sweep_tmp.json'));print(json.dumps({'set':sys.argv[1],'value':d['value'],'kernel_ms':d['roofline']['kernel_ms'],'plan':d['plan'],'ldpc':d.get('ldpc',{}).get('value')}))" "$s" >> $OUT
done
