# A/B of environment settings on the default C3 bench (N = 1) on one box (run via gpurun):
#   tools/ab_env.sh TAG "VAR=v,VAR2=w" ["VAR=x" ...]   (the empty setting first: the default)
# Two alternations of a short bench (no CPU baselines, no C2 line, no rehearsal); one JSON line per run.
set -e
TAG="$1"; shift
O=gpurun_out/$TAG.jsonl
: > $O
run() {
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --no-c2 --rehearse= --no-stats \
   | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(json.dumps({'env': '$1', 'value': d['value'], 'cached': d['value_index_cached_transcript'], 'single_cached_ms': d['ms_per_proof_single_cached_transcript'], 'cores': d['host']['process_cores_busy']}))" >> $O
}
for i in 1 2; do
  run default
  for alt in "$@"; do
    ( IFS=','; for kv in $alt; do export "$kv"; done; run "$alt" )
  done
done
