#!/bin/bash
# A/B of library builds / settings on ONE rank of a G-rank proof-sharded node (run via gpurun from the
# repo root):
#   tools/ab_vrank.sh TAG G ALT1 [ALT2 ...]
# Each ALT is an alternative .so (used through SPX_LIB_PATH), VAR=value settings joined by ',', or
# "args:<vrank_bench arguments>" (e.g. "args:--inflight 96"). Rounds alternate the default and every
# alternative, twice: tools/vrank_bench.py --G G --solo with the rank's own settings
# (bench.inflight_for(G) in flight, bench.hw_queues_for(G) queues), VRANK_PROOFS proofs per step
# (default 64) x VRANK_STEPS steps (default 5, as bench.py's rehearsal), one JSON line per run into
# gpurun_out/<TAG>.jsonl. VRANK_ARGS adds vrank_bench arguments to every run; AB_HWQ sets the hardware
# queues of every run, an ALT "AB_HWQ_ALT=n" those of one arm.
set -e
TAG="$1"; G="$2"; shift; shift
OUT="gpurun_out/$TAG.jsonl"
: > "$OUT"
read -r -a EXTRA <<< "${VRANK_ARGS:-}"
Q=$(python3 -c "import bench; print(bench.hw_queues_for($G))")
run() {  # $1 = label, $2 = extra arguments; remaining environment already exported by the caller
  read -r -a MORE <<< "${2:-}"
  GPU_MAX_HW_QUEUES=${AB_HWQ_ALT:-${AB_HWQ:-$Q}} SPX_BLOCKING_SYNC=1 timeout -k 10 300 python tools/vrank_bench.py --G "$G" --solo \
    --proofs "${VRANK_PROOFS:-64}" --steps "${VRANK_STEPS:-5}" --warmup 1 "${EXTRA[@]}" "${MORE[@]}" \
    | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); d['build']='$1'; print(json.dumps(d))" >> "$OUT"
}
for i in 1 2; do
  run default
  for alt in "$@"; do
    if [[ "$alt" == args:* ]]; then
      run "$alt" "${alt#args:}"
    elif [[ "$alt" == *=* ]]; then
      ( IFS=','; for kv in $alt; do export "$kv"; done; run "$alt" )
    else
      ( export SPX_LIB_PATH="$alt"; run "$alt" )
    fi
  done
done
