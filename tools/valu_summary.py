"""Per-kernel VALU instruction totals from a rocprofv3 --pmc SQ_INSTS_VALU pass (counter_collection.csv):
ideal time at full VALU issue = wave-instructions x 4 cycles / (1024 SIMDs x clock). Usage:
valu_summary.py <counter_collection.csv> <proofs in the run> [clock_GHz] [out.json]
Setup kernels (PP preprocessing / keygen) are reported but left out of the per-proof total."""
import json
import csv
import re
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
proofs = float(sys.argv[2])
ghz = float(sys.argv[3]) if len(sys.argv) > 3 else 2.4
SETUP = ("k_precompute", "k_fixed_base", "k_normalize", "k_aff_to_r29", "k_points_from_bytes", "k_points_to_canon",
         "__amd_rocclr")  # the last: PP window-copy blits (hipMemcpy2DAsync, prover.cpp pp_preprocess)
acc = defaultdict(lambda: defaultdict(float))
for r in rows:
    name = re.sub(r"\(.*", "", r["Kernel_Name"])
    name = re.sub(r"spx::Fe<spx::FqCfg>", "Fq", name)
    name = re.sub(r"spx::|void |rocprim::ROCPRIM_\w+::detail::", "", name)[:60]
    acc[name][r["Counter_Name"]] += float(r["Counter_Value"])
tot = 0.0
out = []
for k, v in acc.items():
    ins = v.get("SQ_INSTS_VALU", 0.0)
    ms = ins * 4 / (1024 * ghz * 1e9) * 1e3 / proofs
    if not k.startswith(SETUP):
        tot += ms
    out.append((ms, k, v))
out.sort(reverse=True)
print("ideal VALU-issue time per proof (proof kernels, setup excluded): %.2f ms" % tot)
for ms, k, v in out[:25]:
    print("%-60s %8.3f ms/proof  %s" % (k, ms, " ".join("%s=%.3g" % (c, x / proofs) for c, x in v.items())))
if len(sys.argv) > 4:
    json.dump({"clock_ghz": ghz, "proofs": proofs, "simds": 1024, "cycles_per_wave_instr": 4,
               "ideal_valu_ms_per_proof": tot,
               "kernels": {k: {"ideal_valu_ms_per_proof": ms, "setup": k.startswith(SETUP),
                               **{c: x / proofs for c, x in v.items()}} for ms, k, v in out}},
              open(sys.argv[4], "w"), indent=1)
