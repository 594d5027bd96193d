#!/bin/bash
# rocprofv3 kernel trace of one-proof-in-flight bench runs, reduced by tools/trace_gaps.py (run via
# gpurun from the repo root): gpurun_out/<TAG>_gaps.txt
set -eo pipefail
TAG="${1:-gaps}"
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=4
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/gaps_$TAG -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --steps 1 --warmup 1 --no-cpu --no-c2 --no-cached --inflight 1 --proofs-per-step 4 --rehearse= \
    > "$ROOT/gpurun_out/${TAG}_bench.json" 2> "$ROOT/gpurun_out/${TAG}_trace.err"
python3 "$ROOT/tools/trace_gaps.py" /tmp/gaps_$TAG > "$ROOT/gpurun_out/${TAG}_gaps.txt"
