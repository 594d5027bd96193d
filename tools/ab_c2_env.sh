# A/B of environment settings on BASELINE C2 alone (bench.py --config c2) on one box (run via gpurun):
#   tools/ab_c2_env.sh TAG "VAR=v,VAR2=w" ["VAR=x" ...]   (the unchanged environment first)
# AB_ARGS adds bench.py arguments to every run. Two alternations; one JSON line per run.
set -e
TAG="$1"; shift
O=gpurun_out/$TAG.jsonl
: > $O
read -r -a EXTRA <<< "${AB_ARGS:-}"
run() {
  timeout -k 10 300 python bench.py --config c2 --steps 10 --warmup 2 --no-cpu --rehearse= --no-stats "${EXTRA[@]}" \
   | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(json.dumps({'env': '$1', 'value': d['value'], 'cached': d['value_index_cached_transcript'], 'single_cached_ms': d['ms_per_proof_single_cached_transcript'], 'cores': d['host']['process_cores_busy'], 'hwq': d['config']['hw_queues'], 'inflight': d['config']['proofs_in_flight']}))" >> $O
}
for i in 1 2; do
  run default
  for alt in "$@"; do
    ( IFS=','; for kv in $alt; do export "$kv"; done; run "$alt" )
  done
done
