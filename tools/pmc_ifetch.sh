#!/bin/bash
# Instruction-fetch counters over the one-proof-in-flight bench (run via gpurun from the repo root):
#   tools/pmc_ifetch.sh <tag>
# Lists the available counters first; each pass only runs when every counter it names is listed.
set -eo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
TAG="${1:-r02}"
OUT="$ROOT/gpurun_out/ifetch_$TAG"
RAW="/tmp/ifetch_raw_$TAG"
mkdir -p "$OUT" "$RAW"
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=16
cd /tmp
timeout -s KILL 60 rocprofv3 -L > "$OUT/avail.txt" 2>&1 || true
B1="--steps 1 --warmup 1 --no-cpu --no-c2 --no-cached --inflight 1 --proofs-per-step 4 --no-stats"
pass() {  # $1 = name, rest = counters
  local name="$1"; shift
  for c in "$@"; do grep -qw "$c" "$OUT/avail.txt" || { echo "skip $name: $c not listed" >&2; return 0; }; done
  timeout -s KILL 240 rocprofv3 --pmc "$@" -d "$RAW/$name" -o run --output-format csv -- \
      python3 "$ROOT/bench.py" $B1 > "$OUT/bench_$name.json" 2> "$OUT/$name.err"
  find "$RAW/$name" -name "*counter_collection.csv" -exec cp {} "$OUT/$name.csv" \;
  echo "$name done" >&2
}
pass sqwait SQ_WAIT_INST_ANY SQ_IFETCH SQ_WAVE_CYCLES SQ_INSTS_VALU
pass sqc SQC_ICACHE_MISSES SQC_ICACHE_HITS
