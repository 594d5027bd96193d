#!/bin/bash
# One PMC pass over ONE rank of a G-rank proof-sharded node (run via gpurun from the repo root):
#   tools/pmc_g8.sh TAG [G] [PROOFS]
# tools/vrank_bench.py --solo (PROOFS proofs, default 64, after one warm-up step) under rocprofv3 --pmc
# with SQ_WAVE_CYCLES, SQ_INSTS_VALU, SQ_WAVES, SQ_BUSY_CYCLES, SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_VALU,
# summarised by tools/slot_cost.py (register-file time per kernel family) -> gpurun_out/TAG_slot_cost.*
set -eo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
TAG="$1"; G="${2:-8}"; PROOFS="${3:-64}"
OUT="$ROOT/gpurun_out"
RAW="/tmp/pg_$TAG"
mkdir -p "$OUT" "$RAW"
export TMPDIR=/tmp SPX_BLOCKING_SYNC=1
Q=$(python3 -c "import sys; sys.path.insert(0, '$ROOT'); import bench; print(bench.hw_queues_for($G))")
export GPU_MAX_HW_QUEUES=$Q
cd /tmp
timeout -s KILL 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU \
    -d "$RAW/pmc" -o run --output-format csv -- python3 "$ROOT/tools/vrank_bench.py" --G "$G" --solo --proofs "$PROOFS" \
    --steps 1 --warmup 1 > "$OUT/${TAG}_pmc_run.json" 2> "$OUT/${TAG}_pmc.err"
# the memory probe proves one and the warm-up step PROOFS more: per-proof figures over all of them
python3 "$ROOT/tools/slot_cost.py" "$RAW/pmc" --proofs $((2 * PROOFS + 1)) --out "$OUT/${TAG}_slot_cost.json" \
    > "$OUT/${TAG}_slot_cost.txt"
echo "pmc_g8 done" >&2
