"""Run by tests/test_gpu_sort_forms.py in a child process whose SPX_SORT_FORM (staged | direct) forces
one form of the MSM bucket sort (msm_common.hip) for every batch: MSMs with random, repeated and
degenerate scalars, a G = 1 proof, virtual-rank proofs at G = 2 and 8, crowded buckets and a forced
compacted-key overflow, each byte-equal to the oracle. Exit status 0 = all equal."""
import os
import random
import sys
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from conftest import ensure_oracle_lib, load_product  # noqa: E402

ensure_oracle_lib()
import oracle_c as oc  # noqa: E402

R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
spx = load_product()
ctx = spx.Context(0)
fails = []


def check(name, got, want):
    print("%-40s %s" % (name, "ok" if got == want else "DIFFERS"), flush=True)
    if got != want:
        fails.append(name)


def bases(nv, seed):
    b = oc.PP.keygen(nv, seed).serialize()
    n = 1 << nv
    g1 = b[24 : 24 + 96 * n]
    pos = 16
    for i in range(nv):
        pos += 8 + 96 * (n >> i)
    pos += 16
    return g1, b[pos : pos + 192 * n]


g1, g2 = bases(10, 5)
rs = random.Random(7)
for n in (1, 33, 1024):
    sc = b"".join(rs.randrange(R).to_bytes(32, "little") for _ in range(n))
    check("msm_g1 n=%d" % n, spx.msm_g1(ctx, g1[: 96 * n], sc), oc.msm_g1(g1[: 96 * n], sc, n))
    if n <= 700:
        check("msm_g2 n=%d" % n, spx.msm_g2(ctx, g2[: 192 * n], sc), oc.msm_g2(g2[: 192 * n], sc, n))
for s in (1, R - 1, 1 << 200):
    sc = s.to_bytes(32, "little") * 700
    check("msm_g2 equal scalars %x" % (s & 0xFFFF), spx.msm_g2(ctx, g2[: 192 * 700], sc), oc.msm_g2(g2[: 192 * 700], sc, 700))
sc = (0xDEADBEEF12345 * 977).to_bytes(32, "little") * 1024
check("msm_g1 repeated scalar", spx.msm_g1(ctx, g1[: 96 * 1024], sc), oc.msm_g1(g1[: 96 * 1024], sc, 1024))


def prove_ranks(G, inst, ppb, w=None):
    group = spx.CommGroup(G) if G > 1 else None
    out, errs = [None] * G, []

    def run(r):
        try:
            c = spx.Context(0)
            if group:
                c.set_comm_group(group, r)
            pp = spx.PublicParameter.load(c, ppb)
            pk = spx.MLArgumentForR1CS.index(c, *[spx.Csr(M.n, M.row_ptr, M.col, M.val) for M in inst.mats])
            out[r] = spx.MLArgumentForR1CS.prove(pk, inst.v_bytes, inst.w_bytes if w is None else w, pp)
        except Exception as e:
            errs.append(repr(e))

    ths = [threading.Thread(target=run, args=(r,)) for r in range(G)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=600)
    if errs:
        fails.append(repr(errs))
    return out


for G, log_n in ((1, 11), (2, 10), (8, 12)):
    inst = oc.Instance(0, log_n, 3, 300 + log_n, 0)
    ppb = oc.PP.keygen(log_n, 400 + log_n).serialize()
    want = oc.prove(inst.mats, inst.v_bytes, inst.w_bytes, oc.PP.load(ppb), 0, 0)
    for r, p in enumerate(prove_ranks(G, inst, ppb)):
        check("prove G=%d 2^%d rank %d" % (G, log_n, r), p, want)
# crowded buckets (equal witness values) at G = 4, then a forced overflow (halved capacity)
inst = oc.Instance(0, 9, 3, 959, 0)
ppb = oc.PP.keygen(9, 951).serialize()
w = (1).to_bytes(32, "little") * ((1 << 9) - (1 << 3))
want = oc.prove(inst.mats, inst.v_bytes, w, oc.PP.load(ppb), 0, 0)
for r, p in enumerate(prove_ranks(4, inst, ppb, w)):
    check("crowded G=4 rank %d" % r, p, want)
os.environ["SPX_MSM_CAP_SCALE"] = "0.5"
inst = oc.Instance(0, 10, 3, 910, 0)
ppb = oc.PP.keygen(10, 901).serialize()
want = oc.prove(inst.mats, inst.v_bytes, inst.w_bytes, oc.PP.load(ppb), 0, 0)
for r, p in enumerate(prove_ranks(4, inst, ppb)):
    check("overflow G=4 rank %d" % r, p, want)
print("FAILED: %s" % fails if fails else "all equal", flush=True)
sys.exit(1 if fails else 0)
