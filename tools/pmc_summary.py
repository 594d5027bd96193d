"""Summarise rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE collected in separate runs, as the
MI355X guide prescribes) into per-kernel HBM bytes per launch.

usage: python tools/pmc_summary.py --fetch DIR --write DIR [--calib-fetch DIR --calib-write DIR]
                                  [--valu DIR] --out profiles/X.json

--valu: a pass with SQ_INSTS_VALU (and SQ_WAVES, SQ_INSTS_SALU, SQ_BUSY_CYCLES ...): per-launch VALU
wave-instructions, the compute side of the MSM kernels' roofline (bench.py).

FETCH_SIZE / WRITE_SIZE are reported by rocprofv3 in KiB. On gfx950 FETCH_SIZE counts exactly half
of the bytes of a wide coalesced read (MI355X_MICROARCH.md, HBM section), so fetch bytes are
doubled. When --calib points at a run of tools/calib_stream (1 GiB read + 1 GiB write), the
correction factors are measured from it instead and recorded.
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def load_all(dirname):
    """every counter of a pass: {kernel: {counter: (sum, launches)}}"""
    per = defaultdict(lambda: defaultdict(lambda: [0.0, set()]))
    files = glob.glob(os.path.join(dirname, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit("no counter_collection.csv under %s" % dirname)
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                rec = per[row["Kernel_Name"]][row["Counter_Name"]]
                rec[0] += float(row["Counter_Value"])
                rec[1].add((f, row.get("Dispatch_Id") or row.get("Correlation_Id")))
    return {k: {c: (v[0], len(v[1])) for c, v in cs.items()} for k, cs in per.items()}


def load(dirname, counter, largest=False):
    """{kernel: (sum of the counter, dispatches)}; largest=True keeps only the dispatches whose value is at
    least half the kernel's maximum (e.g. the first rounds of a sumcheck, where the tables stream from HBM)"""
    per = defaultdict(lambda: defaultdict(float))
    files = glob.glob(os.path.join(dirname, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit("no counter_collection.csv under %s" % dirname)
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                per[row["Kernel_Name"]][(f, row.get("Dispatch_Id") or row.get("Correlation_Id"))] += float(row["Counter_Value"])
    out = {}
    for k, d in per.items():
        vals = list(d.values())
        if largest:
            top = max(vals)
            vals = [v for v in vals if v >= 0.5 * top]
        out[k] = (sum(vals), len(vals))
    return out


def short(name):
    return name.split("(")[0].replace("void ", "").replace("spx::", "").replace("Fe<FqCfg>", "Fq").replace("Fe<FrCfg>", "Fr")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--calib-fetch")
    ap.add_argument("--calib-write")
    ap.add_argument("--valu")
    ap.add_argument("--bench", help="bench.py JSON of a run with the same launch mix (its roofline kernel's "
                    "algorithmic bytes per launch are recorded, so a run with smaller launches can scale the counters)")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    unit = 1024.0  # KiB
    f_corr, w_corr, calib = 2.0, 1.0, None
    if a.calib_fetch and a.calib_write:
        cf = load(a.calib_fetch, "FETCH_SIZE")
        cw = load(a.calib_write, "WRITE_SIZE")
        rd = next(v for k, v in cf.items() if "k_calib_read" in k)
        wr = next(v for k, v in cw.items() if "k_calib_write" in k)
        f_corr = (1 << 30) / (rd[0] / rd[1] * unit)
        w_corr = (1 << 30) / (wr[0] / wr[1] * unit)
        calib = {"read_bytes": 1 << 30, "fetch_reported_bytes": rd[0] / rd[1] * unit, "fetch_correction": f_corr,
                 "write_bytes": 1 << 30, "write_reported_bytes": wr[0] / wr[1] * unit, "write_correction": w_corr}
    fe = load(a.fetch, "FETCH_SIZE")
    wr = load(a.write, "WRITE_SIZE")
    fel = load(a.fetch, "FETCH_SIZE", largest=True)
    wrl = load(a.write, "WRITE_SIZE", largest=True)
    out = {"unit": "bytes per launch", "fetch_correction": f_corr, "write_correction": w_corr, "calibration": calib,
           "kernels": {}}
    for k in sorted(set(fe) | set(wr)):
        fb, fn = fe.get(k, (0.0, 0))
        wb, wn = wr.get(k, (0.0, 0))
        rec = {
            "launches_fetch_pass": fn,
            "launches_write_pass": wn,
            "fetch_bytes": fb / fn * unit * f_corr if fn else None,
            "write_bytes": wb / wn * unit * w_corr if wn else None,
        }
        if rec["fetch_bytes"] is not None and rec["write_bytes"] is not None:
            rec["traffic_bytes"] = rec["fetch_bytes"] + rec["write_bytes"]
        lf, lw = fel.get(k), wrl.get(k)
        if lf and lw and lf[1] and lw[1]:
            rec["traffic_bytes_largest"] = lf[0] / lf[1] * unit * f_corr + lw[0] / lw[1] * unit * w_corr
        out["kernels"][short(k)] = rec
    if a.valu:
        out["valu_counters"] = "SQ_* per launch (SQ_INSTS_VALU = VALU wave-instructions)"
        for k, cs in load_all(a.valu).items():
            rec = out["kernels"].setdefault(short(k), {})
            for c, (tot, n) in cs.items():
                rec[c + "_per_launch"] = tot / n if n else None
                rec["launches_valu_pass"] = n
    if a.bench:
        try:
            rf = json.loads(open(a.bench).read().strip().splitlines()[-1]).get("roofline") or {}
            alg = (rf.get("hbm") or {}).get("algorithmic_bytes_per_launch")
            if alg and rf.get("kernel") in out["kernels"]:
                out["kernels"][rf["kernel"]]["alg_bytes_per_launch"] = alg
        except (OSError, ValueError, IndexError):
            pass
    json.dump(out, open(a.out, "w"), indent=1)
    print("wrote", a.out, len(out["kernels"]), "kernels")


if __name__ == "__main__":
    main()
