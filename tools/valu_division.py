"""Per-rank VALU division of a proof-sharded prove: SQ_INSTS_VALU per proof of the proof kernels (setup
excluded) at G ranks against G = 1, from two tools/valu_summary.py outputs of solo-rank rehearsals.
Prints the ratio  VALU(G) / (VALU(1) / G)  (1.0 = perfect division) and the kernels that divide worst.
usage: python tools/valu_division.py valu_G1.txt valu_G8.txt 8"""
import re
import sys

SETUP = ("k_precompute", "k_fixed_base", "k_normalize", "k_aff_to_r29", "k_points_from_bytes", "k_points_to_canon",
         "__amd_rocclr")


def load(path):
    d = {}
    for line in open(path):
        m = re.match(r"(\S.*?)\s{2,}([\d.]+) ms/proof.*SQ_INSTS_VALU=([\d.e+]+)", line)
        if m and not m.group(1).strip().startswith(SETUP):
            d[m.group(1).strip()] = float(m.group(3))
    return d


def main():
    a, b, G = load(sys.argv[1]), load(sys.argv[2]), int(sys.argv[3])
    ta, tb = sum(a.values()), sum(b.values())
    print("VALU per proof: G=1 %.4e, G=%d per rank %.4e, ratio to G=1/%d: %.3f" % (ta, G, tb, G, tb / (ta / G)))
    rows = sorted(((b.get(k, 0) - a.get(k, 0) / G, k) for k in set(a) | set(b)), reverse=True)
    for ex, k in rows[:8]:
        print("  excess %.2e  %-40s G=1 %.2e  G=%d %.2e" % (ex, k[:40], a.get(k, 0), G, b.get(k, 0)))


if __name__ == "__main__":
    main()
