#!/bin/bash
# Effective clock of the long kernels (run via gpurun from the repo root):  tools/pmc_clock.sh TAG
# One proof in flight at 2^20 (bench.py's "alone" launch mix), one PMC pass of GRBM_GUI_ACTIVE and
# SQ_INSTS_VALU with the kernel trace of the same pass, summarised by tools/pmc_clock.py.
set -eo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
TAG="$1"
OUT="$ROOT/gpurun_out"
RAW="/tmp/pc_$TAG"
mkdir -p "$OUT" "$RAW"
export TMPDIR=/tmp
cd /tmp
B1="--steps 1 --warmup 1 --no-cpu --no-c2 --no-cached --inflight 1 --proofs-per-step 4 --rehearse= --no-stats"
# shellcheck disable=SC2086
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_BUSY_CYCLES --kernel-trace -d "$RAW/pmc" -o run \
    --output-format csv -- python3 "$ROOT/bench.py" $B1 > /dev/null 2> "$OUT/${TAG}_clock.err"
python3 "$ROOT/tools/pmc_clock.py" "$RAW/pmc" --out "$OUT/${TAG}_clock.json" > "$OUT/${TAG}_clock.txt"
echo "pmc_clock done" >&2
