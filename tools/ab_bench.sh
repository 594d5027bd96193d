# A/B of library builds / environment settings on one box (run via gpurun from the repo root):
#   tools/ab_bench.sh TAG ALT1 [ALT2 ...]
# Each ALT is an alternative .so (used through SPX_LIB_PATH) or VAR=value settings joined by ','
# (e.g. SPX_HASH_THREADS=8,SPX_LVL0=batch). AB_ARGS adds bench.py arguments to every run (e.g. --config c2). Rounds alternate the default and every alternative, twice, with a
# short bench (no CPU baseline, no C2 line); one JSON line per run into gpurun_out/<TAG>.jsonl.
set -e
TAG="$1"; shift
OUT="gpurun_out/$TAG.jsonl"
: > "$OUT"
read -r -a EXTRA <<< "${AB_ARGS:-}"  # split here, before any ALT changes IFS
run() {  # $1 = label; remaining environment already exported by the caller
  timeout -k 10 240 python bench.py --no-cpu --no-c2 --rehearse '' --steps 3 --warmup 1 "${EXTRA[@]}" \
    | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(json.dumps({'build': '$1', 'value': d['value'], 'ms_single_cached': d['ms_per_proof_single_cached_transcript'], 'kernels': d['kernels_ms_per_proof'], 'hbm_largest': d['roofline'].get('hbm_kernels', {}).get('largest_launches'), 'host': d.get('host'), 'value_cached': d.get('value_index_cached_transcript')}))" >> "$OUT"
}
for i in 1 2; do
  run default
  for alt in "$@"; do
    if [[ "$alt" == *=* ]]; then
      ( IFS=','; for kv in $alt; do export "$kv"; done; run "$alt" )
    else
      ( export SPX_LIB_PATH="$alt"; run "$alt" )
    fi
  done
done
