#!/bin/bash
# Gather granularity, run via gpurun from the repo root:
#   tools/gather_granularity.sh TAG   -> gpurun_out/TAG_gather.txt
# tools/ubench_gather (built here on the CPU: hipcc -O3 --offload-arch=gfx950 tools/ubench_gather.hip
# -o tools/ubench_gather) timed, then one rocprofv3 --pmc FETCH_SIZE pass over the same binary; the
# per-dispatch FETCH_SIZE (KB) is turned into bytes per gathered row, and the streaming read's bytes
# over its FETCH_SIZE give the counter's byte scale for 16-B-per-lane loads.
set -eo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
TAG="$1"
OUT="$ROOT/gpurun_out/${TAG}_gather.txt"
RAW="/tmp/gg_$TAG"
mkdir -p "$ROOT/gpurun_out" "$RAW"
export TMPDIR=/tmp
timeout -k 10 120 "$ROOT/tools/ubench_gather" > "$OUT"
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$RAW/pmc" -o run --output-format csv -- "$ROOT/tools/ubench_gather" > /dev/null
python3 - "$RAW/pmc" >> "$OUT" <<'PY'
import csv, glob, os, sys
from collections import defaultdict
rows = []
for f in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True):
    rows += list(csv.DictReader(open(f)))
per = defaultdict(list)
for r in rows:
    per[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]) * 1024.0)  # FETCH_SIZE is in KB
nrows = 1 << 22
stream = per.get("k_stream", [])
scale = (1 << 30) / (sum(stream[1:]) / max(1, len(stream) - 1)) if len(stream) > 1 else None
print("\nFETCH_SIZE per launch (warm-up launch excluded), bytes per gathered row:")
print("  stream calibration: 1 GiB read / FETCH_SIZE bytes = %.3f (the factor applied below)" % (scale or float("nan")))
for k, v in sorted(per.items()):
    if k == "k_stream" or len(v) < 2:
        continue
    fb = sum(v[1:]) / (len(v) - 1)
    print("  %-22s raw %8.1f B/row   x scale %8.1f B/row" % (k, fb / nrows, fb * (scale or 1) / nrows))
PY
echo "gather_granularity done" >&2
