#!/bin/bash
# GPU-box profiling recipe (run via gpurun from the repo root):  tools/profile_gpu.sh <tag>
#   1. rocprofv3 --kernel-trace --stats over the default bench configuration (16 proofs in flight,
#      16 hardware queues) and over a one-proof-in-flight run (kernel durations with nothing else
#      sharing the GPU)
#   2. PMC passes over a one-proof-in-flight run, one counter group per run (MI355X guide: separate
#      passes): FETCH_SIZE; WRITE_SIZE; SQ_INSTS_VALU / SQ_WAVES / SQ_INSTS_SALU / SQ_BUSY_CYCLES /
#      SQ_WAVE_CYCLES; plus FETCH_SIZE / WRITE_SIZE over tools/calib_stream (1 GiB read / write) to
#      measure the counters' byte scale. tools/pmc_summary.py -> pmc_kernels.json (per launch);
#      FETCH_SIZE / WRITE_SIZE over BASELINE C2 at 2^18 -> pmc_kernels_c2.json.
# Every GPU step has its own time limit; the first failure ends the script.
set -eo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
TAG="${1:-r02}"
OUT="$ROOT/gpurun_out/prof_$TAG"
# raw traces are large (hundreds of MB of per-dispatch rows): they stay outside gpurun_out
RAW="/tmp/prof_raw_$TAG"
mkdir -p "$OUT" "$RAW"
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES="${PROF_HW_QUEUES:-16}"
[ -x "$ROOT/tools/calib_stream" ] || hipcc -O2 --offload-arch=gfx950 "$ROOT/tools/calib_stream.hip" -o "$ROOT/tools/calib_stream"
cd /tmp
# one proof in flight, no index-cached runs: every G2 launch of the process is one of the three per
# proof that bench.py's "alone" statistics time (level 0, the two opening batches)
B1="--steps 1 --warmup 1 --no-cpu --no-c2 --no-cached --inflight 1 --proofs-per-step 4 --rehearse="
# BASELINE C2 (2^18, commitment stubbed): its own FETCH / WRITE passes for the c2 roofline's traffic
C2="--config c2 --steps 1 --warmup 1 --no-cpu --no-cached --inflight 1 --proofs-per-step 4 --rehearse="
if [ -z "$PROF_SKIP_TRACE" ]; then
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$RAW/trace" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu --no-c2 --rehearse= > "$OUT/bench_traced.json" 2> "$OUT/trace.err"
echo "trace done" >&2
find "$RAW/trace" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$RAW/trace1" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" $B1 > "$OUT/bench_traced_inflight1.json" 2> "$OUT/trace1.err"
echo "trace (one proof in flight) done" >&2
find "$RAW/trace1" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats_inflight1.csv" \;
fi
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d "$RAW/fetch" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" $B1 --no-stats > "$OUT/bench_fetch.json" 2> "$OUT/fetch.err"
echo "fetch done" >&2
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d "$RAW/write" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" $B1 --no-stats > "$OUT/bench_write.json" 2> "$OUT/write.err"
echo "write done" >&2
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d "$RAW/valu" \
    -o run --output-format csv -- python3 "$ROOT/bench.py" $B1 --no-stats > "$OUT/bench_valu.json" 2> "$OUT/valu.err"
echo "valu done" >&2
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d "$RAW/cfetch" -o run --output-format csv -- "$ROOT/tools/calib_stream" > "$OUT/calib.txt" 2>&1
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -d "$RAW/cwrite" -o run --output-format csv -- "$ROOT/tools/calib_stream" >> "$OUT/calib.txt" 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d "$RAW/c2fetch" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" $C2 --no-stats > "$OUT/bench_c2_fetch.json" 2> "$OUT/c2fetch.err"
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d "$RAW/c2write" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" $C2 --no-stats > "$OUT/bench_c2_write.json" 2> "$OUT/c2write.err"
echo "c2 fetch / write done" >&2
python3 "$ROOT/tools/pmc_summary.py" --fetch "$RAW/c2fetch" --write "$RAW/c2write" --calib-fetch "$RAW/cfetch" \
    --calib-write "$RAW/cwrite" --out "$OUT/pmc_kernels_c2.json"
python3 "$ROOT/tools/pmc_summary.py" --fetch "$RAW/fetch" --write "$RAW/write" --calib-fetch "$RAW/cfetch" \
    --calib-write "$RAW/cwrite" --valu "$RAW/valu" --bench "$OUT/bench_traced_inflight1.json" --out "$OUT/pmc_kernels.json"
echo "profile done: $OUT" >&2
