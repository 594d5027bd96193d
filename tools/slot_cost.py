"""Register-file time per kernel family from one rocprofv3 PMC pass (SQ_WAVE_CYCLES, SQ_INSTS_VALU,
SQ_WAVES, ...; rocprofv3 serialises the dispatches of a --pmc pass, so every dispatch is measured
alone). A wave holds its VGPRs for its whole life, and the curve kernels hold 198-256 of a lane's 512,
so on a full GPU the binding resource is register-file time, not wave count:
    rf_time = SQ_WAVE_CYCLES (quad-cycles, summed over waves) x 4 x VGPRs / 512
in SIMD-cycles. Its sum over a proof's kernels, / 1024 SIMDs / clock, bounds the proof's throughput
time from below; the kernels with the most rf_time per VALU instruction are the ones to fix.

usage: python tools/slot_cost.py PMC_DIR --proofs N [--clock-ghz 2.0] [--out FILE.json]"""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict


def short(name):
    s = re.sub(r"\(.*", "", name)
    s = re.sub(r"spx::Fe<spx::FqCfg>", "Fq", s)
    s = re.sub(r"spx::Fe<spx::FrCfg>", "Fr", s)
    s = re.sub(r"spx::|void |rocprim::ROCPRIM_\w+::detail::", "", s)
    return s[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--proofs", type=float, required=True, help="proofs the profiled process ran (per-proof figures)")
    ap.add_argument("--clock-ghz", type=float, default=2.0)
    ap.add_argument("--out")
    a = ap.parse_args()
    disp = defaultdict(dict)
    meta = {}
    for f in glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            d = (f, row.get("Dispatch_Id") or row.get("Correlation_Id"))
            disp[d][row["Counter_Name"]] = disp[d].get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
            vg = row.get("Arch_VGPR_Count") or row.get("VGPR_Count") or "0"
            meta[d] = (short(row["Kernel_Name"]), int(float(vg)))
    fam = defaultdict(lambda: defaultdict(float))
    for d, c in disp.items():
        k, vg = meta[d]
        f = fam[k]
        f["dispatches"] += 1
        f["vgprs"] = vg
        for cn, v in c.items():
            f[cn] += v
        f["rf_simd_cycles"] += c.get("SQ_WAVE_CYCLES", 0.0) * 4 * min(512, max(vg, 1)) / 512.0
    tot_rf = sum(f["rf_simd_cycles"] for f in fam.values())
    tot_valu = sum(f.get("SQ_INSTS_VALU", 0.0) for f in fam.values())
    out = {"proofs": a.proofs, "clock_GHz": a.clock_ghz,
           "rf_bound_ms_per_proof": tot_rf / a.proofs / 1024 / (a.clock_ghz * 1e9) * 1e3,
           "valu_per_proof": tot_valu / a.proofs, "kernels": {}}
    print("register-file time bound: %.3f ms per proof at %.2f GHz; VALU %.4g per proof" % (
        out["rf_bound_ms_per_proof"], a.clock_ghz, out["valu_per_proof"]))
    for k, f in sorted(fam.items(), key=lambda kv: -kv[1]["rf_simd_cycles"]):
        rf = f["rf_simd_cycles"]
        v = f.get("SQ_INSTS_VALU", 0.0)
        rec = {"dispatches_per_proof": f["dispatches"] / a.proofs, "vgprs": f["vgprs"],
               "rf_share": rf / tot_rf if tot_rf else 0.0, "valu_share": v / tot_valu if tot_valu else 0.0,
               "rf_cycles_per_valu": rf / v if v else None}
        out["kernels"][k] = rec
        print("%-60s disp/proof %6.1f vgpr %3d  rf %5.1f%%  valu %5.1f%%  rf-cyc/valu %s" % (
            k, rec["dispatches_per_proof"], f["vgprs"], 100 * rec["rf_share"], 100 * rec["valu_share"],
            "%.2f" % rec["rf_cycles_per_valu"] if v else "-"))
    if a.out:
        json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
