# Kernel trace of BASELINE C2's index-cached pipeline (tools/c2_cached.py; run via gpurun from the repo
# root):  [C2ARGS="--inflight 128 --group 8"] tools/c2_trace.sh TAG  -> gpurun_out/TAG.json (untraced line), TAG_traced.json,
# TAG_kernel_stats.csv, TAG_busy.txt (tools/trace_busy.py over the timed steps' part of the trace)
set -eo pipefail
C2ARGS="${C2ARGS:-}"
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
TAG="$1"
OUT="$ROOT/gpurun_out"
RAW="/tmp/c2t_$TAG"
mkdir -p "$OUT" "$RAW"
export TMPDIR=/tmp SPX_BLOCKING_SYNC=1 GPU_MAX_HW_QUEUES="${GPU_MAX_HW_QUEUES:-4}"
timeout -k 10 200 python3 "$ROOT/tools/c2_cached.py" --steps 8 $C2ARGS > "$OUT/$TAG.json"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$RAW/trace" -o run --output-format csv -- \
    python3 "$ROOT/tools/c2_cached.py" --steps ${TRACE_STEPS:-4} $C2ARGS > "$OUT/${TAG}_traced.json" 2> "$OUT/${TAG}_trace.err"
find "$RAW/trace" -name "*kernel_stats.csv" -exec cp {} "$OUT/${TAG}_kernel_stats.csv" \;
KT=$(find "$RAW/trace" -name "*kernel_trace.csv" -print -quit)
TRACE_TOP=40 python3 "$ROOT/tools/trace_busy.py" "$KT" 0.6 0.95 > "$OUT/${TAG}_busy.txt"
echo "c2_trace done" >&2
