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
# raw traces are large (hundreds of MB of per-dispatch rows): they stay outside gpurun_out
RAW="/tmp/prof_raw_$TAG"
mkdir -p "$OUT" "$RAW"
export TMPDIR=/tmp
# rocprofv3's kernel tracing segfaults (inside its launch / sync interception, 10-20 s into the run)
# with bench.py's default of 16 hardware queues per process; the profiled runs use HIP's default 4
export GPU_MAX_HW_QUEUES="${PROF_HW_QUEUES:-4}"
[ -x "$ROOT/tools/calib_stream" ] || hipcc -O2 --offload-arch=gfx950 "$ROOT/tools/calib_stream.hip" -o "$ROOT/tools/calib_stream"
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$RAW/trace" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu > "$OUT/bench_traced.json" 2> "$OUT/trace.err"
echo "trace done" >&2
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$RAW/trace1" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu --inflight 1 > "$OUT/bench_traced_inflight1.json" 2> "$OUT/trace1.err"
echo "trace (one proof in flight) done" >&2
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d "$RAW/fetch" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --steps 1 --warmup 1 --no-cpu --no-stats --inflight 1 > "$OUT/bench_fetch.json" 2> "$OUT/fetch.err"
echo "fetch done" >&2
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d "$RAW/write" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --steps 1 --warmup 1 --no-cpu --no-stats --inflight 1 > "$OUT/bench_write.json" 2> "$OUT/write.err"
echo "write done" >&2
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d "$RAW/cfetch" -o run --output-format csv -- "$ROOT/tools/calib_stream" > "$OUT/calib.txt" 2>&1
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -d "$RAW/cwrite" -o run --output-format csv -- "$ROOT/tools/calib_stream" >> "$OUT/calib.txt" 2>&1
python3 "$ROOT/tools/pmc_summary.py" --fetch "$RAW/fetch" --write "$RAW/write" --calib-fetch "$RAW/cfetch" \
    --calib-write "$RAW/cwrite" --out "$OUT/pmc_traffic.json"
# kernel_stats summaries are small: keep them next to the traffic summary
find "$RAW/trace" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
find "$RAW/trace1" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats_inflight1.csv" \;
echo "profile done: $OUT" >&2
