# A/B of library builds on BASELINE C2 (2^18, commitment stubbed) on one box (run via gpurun):
#   tools/ab_c2.sh TAG ALT.so [ARGS...]   (alternating default / ALT twice; ARGS go to bench.py)
set -e
TAG="$1"; ALT="$2"; shift; shift
O=gpurun_out/$TAG.jsonl
: > $O
run() {
  timeout -k 10 300 python bench.py --config c2 --steps 10 --warmup 2 --no-cpu --rehearse= --no-stats "$@" \
   | python -c "import json,sys,os; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(json.dumps({'build': os.environ.get('SPX_LIB_PATH', 'default'), 'value': d['value'], 'cached': d['value_index_cached_transcript'], 'single_cached_ms': d['ms_per_proof_single_cached_transcript'], 'cores': d['host']['process_cores_busy']}))" >> $O
}
for i in 1 2; do
  run "$@"
  SPX_LIB_PATH="$ALT" run "$@"
done
