"""Gaps between consecutive kernels on each HIP stream's queue around the G2 accumulation, from a
rocprofv3 --kernel-trace CSV (tools/trace_gaps.sh): for every k_accum_aff<Fq2> dispatch, the kernel
before it on the same queue, the idle gap between them and the accumulation's own duration. Used to
compare rocprofv3's kernel time with bench.py's HIP-event time (profiles)."""
import csv
import glob
import statistics
import sys

path = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(path)))
key = "Queue_Id" if "Queue_Id" in rows[0] else "Stream_Id"
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
last = {}
gaps, durs, prev_names = [], [], {}
for r in rows:
    q = r.get(key)
    name = r["Kernel_Name"]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if "k_accum_aff<spx::Fq2>" in name and q in last:
        pn, pe = last[q]
        gaps.append((s - pe) / 1e3)
        durs.append((e - s) / 1e3)
        short = pn.split("(")[0][-40:]
        prev_names[short] = prev_names.get(short, 0) + 1
    last[q] = (name, e)
print("accumulation launches with a predecessor on the same queue:", len(gaps))
print("duration us: mean %.1f median %.1f" % (statistics.mean(durs), statistics.median(durs)))
print("gap before it us: mean %.1f median %.1f max %.1f" % (statistics.mean(gaps), statistics.median(gaps), max(gaps)))
print("predecessors:", prev_names)
by = {}
for r in rows:
    if "k_accum_aff<spx::Fq2>" in r["Kernel_Name"]:
        g = r.get("Grid_Size") or r.get("Grid_Size_X") or "?"
        by.setdefault(g, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for g, v in sorted(by.items(), key=lambda x: -len(x[1])):
    print("grid %s: %d launches, mean %.1f us, min %.1f, max %.1f" % (g, len(v), statistics.mean(v), min(v), max(v)))

acc = [r for r in rows if "k_accum_aff<spx::Fq2>" in r["Kernel_Name"]]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in acc]
for lo in range(0, len(d), 30):
    seg = d[lo : lo + 30]
    print("launches %3d-%3d (time order): mean %.1f us" % (lo, lo + len(seg) - 1, statistics.mean(seg)))
print("last 9 launches (us):", " ".join("%.0f" % x for x in d[-9:]))
