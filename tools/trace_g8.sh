#!/bin/bash
# Kernel trace of ONE rank of a G-rank proof-sharded node (run via gpurun from the repo root):
#   tools/trace_g8.sh TAG [G] [extra vrank_bench args]
# tools/vrank_bench.py --solo with the rank's own settings (bench.inflight_for(G) proofs in flight,
# bench.hw_queues_for(G) hardware queues) under rocprofv3 --kernel-trace --stats, then
# tools/trace_busy.py over the trace. Writes gpurun_out/TAG_G<G>.json (the rehearsal's line),
# TAG_kernel_stats_G<G>.csv and TAG_busy_G<G>.txt.
set -eo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
TAG="$1"; G="${2:-8}"; shift; shift || true
OUT="$ROOT/gpurun_out"
RAW="/tmp/tg_$TAG"
mkdir -p "$OUT" "$RAW"
export TMPDIR=/tmp SPX_BLOCKING_SYNC=1
Q=$(python3 -c "import sys; sys.path.insert(0, '$ROOT'); import bench; print(bench.hw_queues_for($G))")
export GPU_MAX_HW_QUEUES=$Q
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$RAW/trace" -o run --output-format csv -- \
    python3 "$ROOT/tools/vrank_bench.py" --G "$G" --solo --proofs 128 --steps 1 --warmup 1 "$@" \
    > "$OUT/${TAG}_G${G}.json" 2> "$OUT/${TAG}_trace.err"
find "$RAW/trace" -name "*kernel_stats.csv" -exec cp {} "$OUT/${TAG}_kernel_stats_G${G}.csv" \;
KT=$(find "$RAW/trace" -name "*kernel_trace.csv" -print -quit)
TRACE_AFTER=k_sc1 TRACE_TOP=40 python3 "$ROOT/tools/trace_busy.py" "$KT" 0.3 0.9 > "$OUT/${TAG}_busy_G${G}.txt"
echo "trace_g8 done" >&2
