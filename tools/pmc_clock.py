"""Effective shader clock per kernel from one rocprofv3 pass of `--pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU ...
--kernel-trace` (MI355X_MICROARCH.md "DVFS give-back": effective clock = GRBM_GUI_ACTIVE / 8 / kernel
wall time, rocprofv3 summing the counter over the 8 XCDs; reads high below ~0.3 ms per dispatch).

usage: python tools/pmc_clock.py DIR [--min-us 300] [--out FILE.json]
Per kernel: dispatches, mean duration, effective clock (GHz), VALU wave-instructions per dispatch and
cycles per VALU instruction per SIMD at that clock (1024 SIMDs)."""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--min-us", type=float, default=300.0)
    ap.add_argument("--out")
    a = ap.parse_args()
    cnt = defaultdict(dict)  # dispatch -> counter -> value
    name, span = {}, {}
    for f in glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            d = (f, row.get("Dispatch_Id") or row.get("Correlation_Id"))
            cnt[d][row["Counter_Name"]] = cnt[d].get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
            name[d] = row["Kernel_Name"].split("(")[0]
            if row.get("Start_Timestamp") and row.get("End_Timestamp"):
                span[d] = (int(row["Start_Timestamp"]), int(row["End_Timestamp"]))
    if not span:  # join with the kernel trace of the same pass by dispatch id
        tr = {}
        for f in glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                tr[row.get("Dispatch_Id") or row.get("Correlation_Id")] = (int(row["Start_Timestamp"]), int(row["End_Timestamp"]))
        for d in cnt:
            if d[1] in tr:
                span[d] = tr[d[1]]
    per = defaultdict(lambda: {"n": 0, "ns": 0.0, "grbm": 0.0, "valu": 0.0})
    for d, c in cnt.items():
        if d not in span or "GRBM_GUI_ACTIVE" not in c:
            continue
        ns = span[d][1] - span[d][0]
        if ns < a.min_us * 1e3:
            continue
        p = per[name[d]]
        p["n"] += 1
        p["ns"] += ns
        p["grbm"] += c["GRBM_GUI_ACTIVE"]
        p["valu"] += c.get("SQ_INSTS_VALU", 0.0)
    out = {}
    for k, p in sorted(per.items(), key=lambda kv: -kv[1]["ns"]):
        ghz = p["grbm"] / 8.0 / p["ns"]
        valu = p["valu"] / p["n"]
        us = p["ns"] / p["n"] / 1e3
        out[k] = {"dispatches": p["n"], "mean_us": round(us, 2), "effective_clock_GHz": round(ghz, 4),
                  "valu_per_dispatch": valu,
                  "cycles_per_valu_instr_per_simd": round(us * 1e-6 * ghz * 1e9 * 1024 / valu, 3) if valu else None}
        print("%-50s n %5d  %9.1f us  %.3f GHz  VALU %.4g  cyc/instr %s" % (
            k[:50], p["n"], us, ghz, valu, out[k]["cycles_per_valu_instr_per_simd"]))
    if a.out:
        json.dump({"source": "rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU --kernel-trace", "min_us": a.min_us,
                   "kernels": out}, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
