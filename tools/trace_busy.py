"""GPU busy summary from a rocprofv3 --kernel-trace CSV: wall span, time with >= 1 kernel running,
and an estimate of SIMD occupancy (waves resident / 1024 SIMDs, one wave per SIMD for the
register-heavy curve kernels) per kernel family. Usage: trace_busy.py <kernel_trace.csv> [t0_frac t1_frac]
Environment: TRACE_AFTER=<name> starts the window at the first kernel whose name contains it (e.g.
k_sc1_round: skips setup); TRACE_TOP=<k> rows (default 20)."""
import os
import csv
import re
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
f0 = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
f1 = float(sys.argv[3]) if len(sys.argv) > 3 else 1.0
ev = []
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    grid = int(r.get("Grid_Size") or r.get("Grid_Size_X") or 0)
    wg = int(r.get("Workgroup_Size") or r.get("Workgroup_Size_X") or 64)
    ev.append((s, e, r["Kernel_Name"], grid, wg))
ev.sort()
after = os.environ.get("TRACE_AFTER")
if after:
    first = next(s for s, e, name, *_ in ev if after in name)
    ev = [x for x in ev if x[0] >= first]
T0, T1 = ev[0][0], max(e for _, e, *_ in ev)
lo, hi = T0 + f0 * (T1 - T0), T0 + f1 * (T1 - T0)
ev = [x for x in ev if x[0] >= lo and x[1] <= hi]
span = hi - lo
busy, cur_s, cur_e = 0, None, None
for s, e, *_ in ev:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
fam = defaultdict(lambda: [0.0, 0.0, 0])
for s, e, name, grid, wg in ev:
    short = re.sub(r"\(.*", "", name)
    short = re.sub(r"spx::Fe<spx::FqCfg>", "Fq", short)
    short = re.sub(r"spx::|void |rocprim::ROCPRIM_\w+::detail::", "", short)[:60]
    waves = max(1, grid // 64)
    d = e - s
    fam[short][0] += d
    fam[short][1] += min(waves, 1024) * d
    fam[short][2] += 1
print("span %.1f ms, >=1 kernel running %.1f%%, kernels %d" % (span / 1e6, 100 * busy / span, len(ev)))
# concurrency: time-weighted number of kernels running at once (hardware queues bound it)
pts = sorted([(s, 1) for s, e, *_ in ev] + [(e, -1) for s, e, *_ in ev])
hist = defaultdict(float)
cur, last = 0, pts[0][0] if pts else 0
for t, d in pts:
    hist[cur] += t - last
    cur += d
    last = t
tot_t = sum(hist.values()) or 1.0
avg = sum(k * v for k, v in hist.items()) / tot_t
print("concurrent kernels: time-weighted mean %.2f; share of time with >= k running: %s" % (
    avg, " ".join("%d:%.0f%%" % (k, 100 * sum(v for c, v in hist.items() if c >= k) / tot_t) for k in (1, 2, 4, 8, 12, 16, 24, 32))))
tot_occ = sum(v[1] for v in fam.values())
print("SIMD-occupancy estimate (sum min(waves,1024) x duration / 1024 x span): %.1f%%" % (100 * tot_occ / (1024 * span)))
for k, v in sorted(fam.items(), key=lambda kv: -kv[1][1])[: int(os.environ.get("TRACE_TOP", "20"))]:
    print("%-60s calls %6d  dur %9.1f ms  simd-share %5.1f%%" % (k, v[2], v[0] / 1e6, 100 * v[1] / (1024 * span)))
# timeline: occupancy estimate per 1/40 of the span (phases of the bench show up as plateaus)
nb = 40
occ = [0.0] * nb
w = span / nb
for s, e, name, grid, wg in ev:
    waves = min(max(1, grid // 64), 1024)
    b0, b1 = int((s - lo) // w), int((e - lo) // w)
    for b in range(max(0, b0), min(nb - 1, b1) + 1):
        a0, a1 = max(s, lo + b * w), min(e, lo + (b + 1) * w)
        if a1 > a0:
            occ[b] += waves * (a1 - a0)
print("timeline (%.0f ms bins): " % (w / 1e6) + " ".join("%d" % round(100 * o / (1024 * w)) for o in occ))
