#!/bin/bash
# Quick per-kernel look (run via gpurun from the repo root):  tools/quickprof.sh TAG [PMC counters...]
# One proof in flight at 2^20 (bench.py's "alone" launch mix): rocprofv3 --kernel-trace --stats, then
# one PMC pass of the given SQ counters (default: VALU instructions, waves, busy / wave / wait cycles).
# Writes gpurun_out/TAG_kernel_stats.csv and gpurun_out/TAG_pmc.txt (per-kernel sums and launches).
set -eo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
TAG="$1"; shift
CNT="${*:-SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY}"
OUT="$ROOT/gpurun_out"
RAW="/tmp/qp_$TAG"
mkdir -p "$OUT" "$RAW"
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=16
cd /tmp
B1="--steps 1 --warmup 1 --no-cpu --no-c2 --no-cached --inflight 1 --proofs-per-step 4 --rehearse="
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$RAW/trace" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" $B1 > "$OUT/${TAG}_bench_traced.json" 2> "$OUT/${TAG}_trace.err"
find "$RAW/trace" -name "*kernel_stats.csv" -exec cp {} "$OUT/${TAG}_kernel_stats.csv" \;
# shellcheck disable=SC2086
timeout -s KILL 300 rocprofv3 --pmc $CNT -d "$RAW/pmc" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" $B1 --no-stats > /dev/null 2> "$OUT/${TAG}_pmc.err"
python3 - "$RAW/pmc" > "$OUT/${TAG}_pmc.txt" <<'EOF'
import csv, glob, os, sys
from collections import defaultdict
per = defaultdict(lambda: defaultdict(float))
disp = defaultdict(set)
for f in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"].split("(")[0][:60]
        per[k][row["Counter_Name"]] += float(row["Counter_Value"])
        disp[k].add((f, row.get("Dispatch_Id")))
for k in sorted(per, key=lambda k: -per[k].get("SQ_INSTS_VALU", 0)):
    n = len(disp[k])
    print("%-60s launches %5d  " % (k, n) + "  ".join("%s %.4g" % (c, v / n) for c, v in sorted(per[k].items())))
EOF
echo "quickprof done" >&2
