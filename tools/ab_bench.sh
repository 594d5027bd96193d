# A/B of library builds on one box (run via gpurun from the repo root):
#   tools/ab_bench.sh TAG ALT1.so [ALT2.so ...]
# Rounds alternate the default build and every alternative (SPX_LIB_PATH), twice, with a short
# bench (no CPU baseline, no C2 line); one JSON line per run into gpurun_out/<TAG>.jsonl.
set -e
TAG="$1"; shift
OUT="gpurun_out/$TAG.jsonl"
: > "$OUT"
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu --no-c2 --steps 3 --warmup 1 \
    | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(json.dumps({'build': 'default', 'round': $i, 'value': d['value'], 'ms_single_cached': d['ms_per_proof_single_cached_transcript'], 'kernels': d['kernels_ms_per_proof']}))" >> "$OUT"
  for alt in "$@"; do
    SPX_LIB_PATH="$alt" timeout -k 10 200 python bench.py --no-cpu --no-c2 --steps 3 --warmup 1 \
      | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(json.dumps({'build': '$alt', 'round': $i, 'value': d['value'], 'ms_single_cached': d['ms_per_proof_single_cached_transcript'], 'kernels': d['kernels_ms_per_proof']}))" >> "$OUT"
  done
done
