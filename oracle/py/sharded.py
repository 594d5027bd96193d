"""ORACLE — TEST INFRASTRUCTURE ONLY.

Python restatement of the product's SHARDED prove (r1cs-spartan_amd/csrc/prover.cpp):
G = 2^g ranks own contiguous blocks of the hypercube; variables bind LSB first, so each rank folds
locally for L - g rounds and exchanges only per-round partial sums (3 Fr) and per-MSM partial points;
the last g rounds / opening levels run on the gathered G-entry tables. `allgather(obj)` returns the
list of every rank's obj in rank order (in-process list, or torch.distributed gloo in the tests).

The result must equal the unsharded prover byte for byte (tests/test_sharded.py)."""
from bls12_381 import G1, G2, R, msm
from spartan import (
    INDEX_INFO_FIELDS,
    Proof,
    commitment_bytes,
    eval_on_x,
    is_pow2,
    log2_exact,
    matrix_bytes,
    open_proof_bytes,
    prover_msg_bytes,
    sum_over_y,
    vec_fr_bytes,
)
from bls12_381 import ser_fr, ser_u64
from transcript import Blake2s512Rng


def eq1(tau, t):
    return (1 - tau - t + 2 * tau * t) % R


def eq_block(r, base, count):
    out = []
    for x in range(base, base + count):
        v = 1
        for j, rj in enumerate(r):
            v = v * (rj if (x >> j) & 1 else (1 - rj)) % R
        out.append(v)
    return out


def fold(t, r):
    return [(t[2 * b] + r * (t[2 * b + 1] - t[2 * b])) % R for b in range(len(t) // 2)]


def sc1_message(Cc, tau_c, g, L):
    inv2 = pow(2, R - 2, R)
    out = []
    for t in range(L + 3):
        l0 = (t - 1) * (t - 2) * inv2 % R
        l1 = t * (t - 2) % R
        l2 = t * (t - 1) * inv2 % R
        Gt = (g[0] * l0 - g[1] * l1 + g[2] * l2) % R
        out.append(Cc * eq1(tau_c, t) % R * Gt % R)
    return out


def sum_points(curve, pts):
    acc = curve.inf
    for p in pts:
        acc = curve.add(acc, curve.from_affine(p))
    return curve.to_affine(acc)


def pair_sums(curve, bases):
    return [curve.to_affine(curve.add(curve.from_affine(bases[2 * b]), curve.from_affine(bases[2 * b + 1])))
            for b in range(len(bases) // 2)]


def open_sharded(pp, zl, L, point, G, rank, allgather):
    g = log2_exact(G)
    nl = (1 << L) // G
    proofs = [None] * L
    r = list(zl)
    parts = []
    for i in range(L - g):
        half = nl >> (i + 1)
        q = [(r[2 * b + 1] - r[2 * b]) % R for b in range(half)]
        r = fold(r, point[i])
        bases = pair_sums(G2, pp.powers_of_h[i])[rank * half : (rank + 1) * half]
        parts.append(G2.to_affine(msm(G2, bases, q)))
    allp = allgather(parts)
    for i in range(L - g):
        proofs[i] = sum_points(G2, [allp[k][i] for k in range(G)])
    rg = [x[0] for x in allgather(r)]
    for i in range(L - g, L):
        half = len(rg) // 2
        q = [(rg[2 * b + 1] - rg[2 * b]) % R for b in range(half)]
        rg = fold(rg, point[i])
        proofs[i] = G2.to_affine(msm(G2, pair_sums(G2, pp.powers_of_h[i]), q))
    return rg[0], (pp.h, proofs)


def prove_sharded(pk, v, w, pp, G, rank, allgather, fs=None):
    L, n = pk["log_n"], pk["n"]
    g = log2_exact(G)
    assert is_pow2(G) and L - g >= 1
    nl = n // G
    lo = rank * nl
    fs = fs or Blake2s512Rng()
    for M in ("A", "B", "C"):
        fs.feed(matrix_bytes(pk[M], n))
    fs.feed(vec_fr_bytes(v))
    log_v = log2_exact(len(v))
    z = [x % R for x in list(v) + list(w)]
    zl = z[lo : lo + nl]
    # commit
    part = G1.to_affine(msm(G1, pp.powers_of_g[0][lo : lo + nl], zl))
    com = (L, sum_points(G1, allgather(part)))
    fs.feed(commitment_bytes(com))
    r_v = [fs.rand_fr() for _ in range(log_v)]
    ev, prf = open_sharded(pp, zl, L, r_v + [0] * (L - log_v), G, rank, allgather)
    pm2 = (ev, prf)
    fs.feed(ser_fr(ev) + open_proof_bytes(prf))
    tau = [fs.rand_fr() for _ in range(L)]
    info = {"max_multiplicands": L + 2, "num_variables": L}
    pm3 = b"".join(ser_u64(info[f]) for f in INDEX_INFO_FIELDS)
    fs.feed(pm3)
    rows = lambda M: pk[M][lo : lo + nl]  # noqa: E731
    tabs = [sum_over_y(rows(M), z) for M in ("A", "B", "C")]
    E = eq_block(tau[1:], rank * (nl // 2), nl // 2)
    msgs1, r_x, Cc = [], [], 1
    for i in range(1, L - g + 1):
        if i >= 2:
            tabs = [fold(t, r_x[-1]) for t in tabs]
            E = [(E[2 * b] + E[2 * b + 1]) % R for b in range(len(E) // 2)]
        gs = [0, 0, 0]
        for b in range(len(tabs[0]) // 2):
            x0 = [t[2 * b] for t in tabs]
            x1 = [t[2 * b + 1] for t in tabs]
            y = [(2 * a1 - a0) % R for a0, a1 in zip(x0, x1)]
            for k, xs in enumerate((x0, x1, y)):
                gs[k] = (gs[k] + (xs[0] * xs[1] - xs[2]) * E[b]) % R
        gs = [sum(p[k] for p in allgather(gs)) % R for k in range(3)]
        m = sc1_message(Cc, tau[i - 1], gs, L)
        msgs1.append(m)
        fs.feed(prover_msg_bytes(m))
        ch = fs.rand_fr()
        r_x.append(ch)
        Cc = Cc * eq1(tau[i - 1], ch) % R
    mine = [fold(t, r_x[-1])[0] for t in tabs]
    allv = allgather(mine)
    tabs = [[allv[k][m] for k in range(G)] for m in range(3)]
    for i in range(L - g + 1, L + 1):
        c = i - 1
        gs = [0, 0, 0]
        for b in range(len(tabs[0]) // 2):
            e = 1
            for j in range(c + 1, L):
                e = e * (tau[j] if (b >> (j - c - 1)) & 1 else (1 - tau[j])) % R
            x0 = [t[2 * b] for t in tabs]
            x1 = [t[2 * b + 1] for t in tabs]
            y = [(2 * a1 - a0) % R for a0, a1 in zip(x0, x1)]
            for k, xs in enumerate((x0, x1, y)):
                gs[k] = (gs[k] + (xs[0] * xs[1] - xs[2]) * e) % R
        m = sc1_message(Cc, tau[c], gs, L)
        msgs1.append(m)
        fs.feed(prover_msg_bytes(m))
        ch = fs.rand_fr()
        r_x.append(ch)
        Cc = Cc * eq1(tau[c], ch) % R
        tabs = [fold(t, ch) for t in tabs]
    pm4 = tuple(t[0] for t in tabs)
    fs.feed(b"".join(ser_fr(x) for x in pm4))
    rabc = [fs.rand_fr() for _ in range(3)]
    mrx = [0] * nl
    for M, rm in zip(("A", "B", "C"), rabc):
        full = eval_on_x(pk[M], r_x)
        for y in range(nl):
            mrx[y] = (mrx[y] + rm * full[lo + y]) % R
    info2 = {"max_multiplicands": 2, "num_variables": L}
    pm5 = b"".join(ser_u64(info2[f]) for f in INDEX_INFO_FIELDS)
    fs.feed(pm5)
    Mt, Zt = mrx, zl
    msgs2, r_y = [], []

    def sc2_round(Mt, Zt):
        ps = [0, 0, 0]
        for b in range(len(Mt) // 2):
            m0, m1, z0, z1 = Mt[2 * b], Mt[2 * b + 1], Zt[2 * b], Zt[2 * b + 1]
            ps[0] += m0 * z0
            ps[1] += m1 * z1
            ps[2] += (2 * m1 - m0) * (2 * z1 - z0)
        return [p % R for p in ps]

    for i in range(1, L - g + 1):
        if i >= 2:
            Mt, Zt = fold(Mt, r_y[-1]), fold(Zt, r_y[-1])
        ps = [sum(p[k] for p in allgather(sc2_round(Mt, Zt))) % R for k in range(3)]
        msgs2.append(ps)
        fs.feed(prover_msg_bytes(ps))
        r_y.append(fs.rand_fr())
    allv = allgather([fold(Mt, r_y[-1])[0], fold(Zt, r_y[-1])[0]])
    Mt, Zt = [a[0] for a in allv], [a[1] for a in allv]
    for i in range(L - g + 1, L + 1):
        ps = sc2_round(Mt, Zt)
        msgs2.append(ps)
        fs.feed(prover_msg_bytes(ps))
        ch = fs.rand_fr()
        r_y.append(ch)
        Mt, Zt = fold(Mt, ch), fold(Zt, ch)
    ez, prf2 = open_sharded(pp, zl, L, r_y, G, rank, allgather)
    return Proof(com, pm2, pm3, msgs1, pm4, pm5, msgs2, (ez, prf2))


def prove_all_ranks_inprocess(pk, v, w, pp, G):
    """Run G ranks cooperatively in one process (generators yield at every allgather)."""
    import threading

    results = [None] * G
    slots = [None] * G
    barrier = threading.Barrier(G)

    def make(rank):
        def allgather(obj):
            slots[rank] = obj
            barrier.wait()
            out = list(slots)
            barrier.wait()
            return out

        return allgather

    def run(rank):
        results[rank] = prove_sharded(pk, v, w, pp, G, rank, make(rank)).to_bytes()

    ths = [threading.Thread(target=run, args=(r,)) for r in range(G)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    return results
