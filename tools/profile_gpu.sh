#!/bin/bash
# GPU-box profiling recipe (run via gpurun from the repo root):
#   1. rocprofv3 --kernel-trace --stats over the default bench (per-kernel durations), and over a
#      one-proof-in-flight run (kernel durations without other proofs sharing the GPU)
#   2. two PMC passes (FETCH_SIZE, WRITE_SIZE: they do not fit one pass on gfx950) over a one-proof
#      bench run, plus the same two passes over tools/calib_stream (1 GiB read / write) to measure
#      the counters' byte scale, summarised by tools/pmc_summary.py into profiles/pmc_traffic.json
# Every GPU step has its own time limit; the first failure ends the script.
set -eo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
TAG="${1:-r01}"
OUT="$ROOT/gpurun_out/prof_$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu > "$OUT/bench_traced.json" 2> "$OUT/trace.err"
echo "trace done" >&2
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace1" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu --inflight 1 > "$OUT/bench_traced_inflight1.json" 2> "$OUT/trace1.err"
echo "trace (one proof in flight) done" >&2
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --steps 1 --warmup 1 --no-cpu --no-stats --inflight 1 > "$OUT/bench_fetch.json" 2> "$OUT/fetch.err"
echo "fetch done" >&2
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --steps 1 --warmup 1 --no-cpu --no-stats --inflight 1 > "$OUT/bench_write.json" 2> "$OUT/write.err"
echo "write done" >&2
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/cfetch" -o run --output-format csv -- "$ROOT/tools/calib_stream" > "$OUT/calib.txt" 2>&1
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -d "$OUT/cwrite" -o run --output-format csv -- "$ROOT/tools/calib_stream" >> "$OUT/calib.txt" 2>&1
python3 "$ROOT/tools/pmc_summary.py" --fetch "$OUT/fetch" --write "$OUT/write" --calib-fetch "$OUT/cfetch" \
    --calib-write "$OUT/cwrite" --out "$OUT/pmc_traffic.json"
# kernel_stats summaries are small: keep them next to the traffic summary
find "$OUT/trace" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
find "$OUT/trace1" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats_inflight1.csv" \;
echo "profile done: $OUT" >&2
