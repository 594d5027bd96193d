"""ORACLE — TEST INFRASTRUCTURE ONLY (checker for tests/, never the product path).

Reference-faithful pure-Python restatement of the reference prover / verifier, function by
function (small cases only):

  MLE / eq / R1CS-as-MLE   /root/reference/src/data_structures/eq.rs:5-20,
                           /root/reference/src/data_structures/r1cs_reader.rs:21-24,75-117
  sumcheck (linear-sumcheck AHPForMLSumcheck [upstream, unpinned]: convert_to_index,
           prover_init, prove_round, verify_round, check_and_generate_subclaim)
  mKZG                     /root/reference/src/commitment/setup.rs:27-105 (keygen),
                           commit.rs:17-29, open.rs:19-58, verify.rs:12-45
  AHP rounds               /root/reference/src/ahp/prover.rs:109-281, verifier.rs:143-512
  FS argument              /root/reference/src/lib.rs:58-212
  byte layout              /root/reference/src/data_structures/proof.rs:10-20 + ark-serialize

Conventions that live in unpinned upstream crates are reconstructed and flagged in
transcript.py / bls12_381.py; `INDEX_INFO_FIELDS` below is the reconstructed field list of
linear-sumcheck's `IndexInfo`.
"""
from bls12_381 import (
    R,
    G1,
    G2,
    fr_inv,
    msm,
    ser_u64,
    ser_fr,
    de_fr,
    g1_compress,
    g2_compress,
    g1_decompress,
    g2_decompress,
    g1_uncompressed,
    g2_uncompressed,
    g1_from_uncompressed,
    g2_from_uncompressed,
)
from transcript import Blake2s512Rng

# linear-sumcheck IndexInfo (CanonicalSerialize, field order) — reconstructed [upstream]
INDEX_INFO_FIELDS = ("max_multiplicands", "num_variables")


class InvalidArgument(Exception):
    """error.rs:7 Error::InvalidArgument"""


class WrongWitness(Exception):
    """error.rs:11 Error::WrongWitness"""


class SumCheckError(Exception):
    """error.rs:9 Error::SumCheckError"""


def log2_exact(n):
    return n.bit_length() - 1


def is_pow2(n):
    return n > 0 and n & (n - 1) == 0


# ----------------------------------------------------------------------------- MLE helpers
def fix_first(table, r):
    """Bind variable 0 (the LSB of the index) to r: T'[b] = T[2b](1-r) + T[2b+1] r."""
    one_minus = (1 - r) % R
    return [(table[2 * b] * one_minus + table[2 * b + 1] * r) % R for b in range(len(table) // 2)]


def mle_eval(table, point):
    """MLExtensionArray::eval_at [upstream]: point[0] binds variable 0 (LSB)."""
    assert len(table) == 1 << len(point)
    t = list(table)
    for r in point:
        t = fix_first(t, r)
    return t[0]


def eq_extension(t):
    """eq.rs:5-20 — log_n separate tables eq_i[x] = 2 t_i x_i - x_i - t_i + 1."""
    dim = len(t)
    out = []
    for i in range(dim):
        ti = t[i]
        poly = []
        for x in range(1 << dim):
            xi = (x >> i) & 1
            poly.append((2 * ti * xi - xi - ti + 1) % R)
        out.append(poly)
    return out


def eq_table(t):
    """Single table eq(t, x) = prod_i eq_i(x) (product form of eq_extension)."""
    tab = [1]
    for ti in reversed(t):
        tab = [v * e % R for v in tab for e in ((1 - ti) % R, ti)]
    # tab index: built with the last variable as MSB
    return tab


# ----------------------------------------------------------------------------- R1CS as MLE
def check_matrix(matrix, num_constraints):
    """MatrixExtension::new, r1cs_reader.rs:36-70."""
    if not is_pow2(num_constraints):
        raise InvalidArgument("num of constraints should be power of two")
    if len(matrix) != num_constraints:
        raise InvalidArgument("matrix size is inconsistent with number of constraints")
    for row in matrix:
        for _c, idx in row:
            if idx >= num_constraints:
                raise InvalidArgument("sparse index out of bound")


def sum_over_y(matrix, z):
    """r1cs_reader.rs:75-85 — Mz[x] = sum_{(a,y) in row x} a z[y]."""
    out = []
    for row in matrix:
        acc = 0
        for a, y in row:
            acc += a * z[y]
        out.append(acc % R)
    return out


def eval_on_x(matrix, r_x):
    """r1cs_reader.rs:91-117 — sparse MLE over 2s variables, index (y << s) + x, partially
    evaluated at r_x over the low s variables (SparseMLExtensionMap::eval_partial_at
    [upstream]: bind one variable at a time, new[k >> 1] += v * (r or 1 - r))."""
    n = len(matrix)
    s = log2_exact(n)
    if (1 << len(r_x)) != n:
        raise InvalidArgument("2^(r_x) should have size: num_constraints")
    cur = {}
    for x, row in enumerate(matrix):
        for val, y in row:
            cur[(y << s) + x] = val  # map insert (duplicate positions: last wins)
    for r in r_x:
        nxt = {}
        one_minus = (1 - r) % R
        for k, v in cur.items():
            w = v * (r if k & 1 else one_minus)
            nxt[k >> 1] = (nxt.get(k >> 1, 0) + w) % R
        cur = nxt
    ans = [0] * n
    for y, v in cur.items():
        ans[y] = v
    return ans


# ----------------------------------------------------------------------------- sumcheck
class MLSumcheckProver:
    """linear-sumcheck AHPForMLSumcheck prover [upstream]: products of MLE tables (coefficient
    one each), prove_round binds variable (round-1) with the last challenge, then evaluates
    P_round(t) = sum_b sum_products prod_j T_j(t, b) for t = 0..=max_multiplicands."""

    def __init__(self, products, num_vars):
        self.products = [[list(t) for t in p] for p in products]
        self.nv = num_vars
        self.max_multiplicands = max(len(p) for p in products)
        self.round = 0
        self.randomness = []

    def info_bytes(self):
        vals = {"max_multiplicands": self.max_multiplicands, "num_variables": self.nv}
        return b"".join(ser_u64(vals[f]) for f in INDEX_INFO_FIELDS)

    def prove_round(self, challenge):
        if challenge is not None:
            if self.round == 0:
                raise SumCheckError("first round should be prover first")
            self.randomness.append(challenge)
            self.products = [[fix_first(t, challenge) for t in p] for p in self.products]
        elif self.round > 0:
            raise SumCheckError("verifier message is empty")
        self.round += 1
        if self.round > self.nv:
            raise SumCheckError("prover is not active")
        deg = self.max_multiplicands
        sums = [0] * (deg + 1)
        half = len(self.products[0][0]) // 2
        for b in range(half):
            for t in range(deg + 1):
                for p in self.products:
                    prod = 1
                    for tab in p:
                        lo = tab[2 * b]
                        prod = prod * (lo + (tab[2 * b + 1] - lo) * t) % R
                    sums[t] += prod
        return [s % R for s in sums]


def interpolate_uni_poly(evals, x):
    """Value at x of the degree-(len-1) polynomial through (i, evals[i]), i = 0..len-1."""
    n = len(evals)
    x %= R
    total = 0
    for i in range(n):
        num = 1
        den = 1
        for j in range(n):
            if j != i:
                num = num * (x - j) % R
                den = den * (i - j) % R
        total += evals[i] * num * fr_inv(den)
    return total % R


def check_and_generate_subclaim(msgs, randomness, asserted_sum, nv, max_mult):
    """linear-sumcheck check_and_generate_subclaim [upstream]."""
    if len(msgs) != nv:
        raise InvalidArgument("insufficient rounds")
    expected = asserted_sum % R
    for evals, r in zip(msgs, randomness):
        if len(evals) != max_mult + 1:
            raise InvalidArgument("wrong number of evaluations")
        if (evals[0] + evals[1]) % R != expected:
            # linear_sumcheck::Error, surfaced by the reference verifier's `?` as Error::SumCheckError
            raise SumCheckError("Prover message is not consistent with the claim.")
        expected = interpolate_uni_poly(evals, r)
    return list(randomness), expected


# ----------------------------------------------------------------------------- mKZG
class PublicParameter:
    """commitment/data_structures.rs:9-17"""

    def __init__(self, nv, powers_of_g, powers_of_h, g, h):
        self.nv = nv
        self.powers_of_g = powers_of_g
        self.powers_of_h = powers_of_h
        self.g = g
        self.h = h

    def serialize_uncompressed(self):
        out = [ser_u64(self.nv), ser_u64(len(self.powers_of_g))]
        for lvl in self.powers_of_g:
            out.append(ser_u64(len(lvl)))
            out.extend(g1_uncompressed(p) for p in lvl)
        out.append(ser_u64(len(self.powers_of_h)))
        for lvl in self.powers_of_h:
            out.append(ser_u64(len(lvl)))
            out.extend(g2_uncompressed(p) for p in lvl)
        out.append(g1_uncompressed(self.g))
        out.append(g2_uncompressed(self.h))
        return b"".join(out)

    @staticmethod
    def deserialize_uncompressed(b):
        pos = 0

        def u64():
            nonlocal pos
            v = int.from_bytes(b[pos : pos + 8], "little")
            pos += 8
            return v

        nv = u64()
        pg = []
        for _ in range(u64()):
            k = u64()
            pg.append([g1_from_uncompressed(b[pos + 96 * i : pos + 96 * (i + 1)]) for i in range(k)])
            pos += 96 * k
        ph = []
        for _ in range(u64()):
            k = u64()
            ph.append([g2_from_uncompressed(b[pos + 192 * i : pos + 192 * (i + 1)]) for i in range(k)])
            pos += 192 * k
        g = g1_from_uncompressed(b[pos : pos + 96])
        pos += 96
        h = g2_from_uncompressed(b[pos : pos + 192])
        return PublicParameter(nv, pg, ph, g, h)


class VerifierParameter:
    """commitment/data_structures.rs:19-26"""

    def __init__(self, nv, g, h, g_mask_random):
        self.nv = nv
        self.g = g
        self.h = h
        self.g_mask_random = g_mask_random

    def serialize_uncompressed(self):
        """CanonicalSerialize::serialize_uncompressed field order: nv, g, h, g_mask_random."""
        return (ser_u64(self.nv) + g1_uncompressed(self.g) + g2_uncompressed(self.h) + ser_u64(len(self.g_mask_random))
                + b"".join(g1_uncompressed(x) for x in self.g_mask_random))


def _fixed_base_table(curve, base_aff, c, nwin):
    """ark-ec FixedBaseMSM::get_window_table [upstream]: table[w][d] = d * 2^(c w) * base."""
    table = []
    outer = curve.from_affine(base_aff)
    for _w in range(nwin):
        row = [curve.inf]
        cur = curve.inf
        for _d in range(1, 1 << c):
            cur = curve.add(cur, outer)
            row.append(cur)
        table.append(curve.batch_to_affine(row))
        for _ in range(c):
            outer = curve.dbl(outer)
    return table


def fixed_base_mul(curve, base_aff, scalars, c=6):
    """ark-ec FixedBaseMSM::multi_scalar_mul [upstream] semantics: s * base for every s,
    normalised to affine (batch_normalization_into_affine)."""
    nwin = (255 + c - 1) // c
    table = _fixed_base_table(curve, base_aff, c, nwin)
    res = []
    for s in scalars:
        acc = curve.inf
        for w in range(nwin):
            d = (s >> (c * w)) & ((1 << c) - 1)
            if d:
                acc = curve.madd(acc, table[w][d])
        res.append(acc)
    return curve.batch_to_affine(res)


def keygen_from_scalars(nv, g_scalar, h_scalar, t):
    """setup.rs:27-105 with the random draws supplied: g = g_scalar * G1gen,
    h = h_scalar * G2gen, trapdoor t. powers_of_g[i][x] = g^{eq(t[i..], x)} (2^(nv-i) points),
    same for h; vp.g_mask_random[i] = g^{t_i}."""
    g = G1.mul_affine(G1.gen, g_scalar)
    h = G2.mul_affine(G2.gen, h_scalar)
    pp_powers = []
    sizes = []
    for i in range(nv):
        tab = eq_table(t[i:])
        pp_powers.extend(tab)
        sizes.append(len(tab))
    pp_g = fixed_base_mul(G1, g, pp_powers)
    pp_h = fixed_base_mul(G2, h, pp_powers)
    powers_of_g, powers_of_h = [], []
    start = 0
    for size in sizes:
        powers_of_g.append(pp_g[start : start + size])
        powers_of_h.append(pp_h[start : start + size])
        start += size
    g_mask = fixed_base_mul(G1, g, t)
    return PublicParameter(nv, powers_of_g, powers_of_h, g, h), VerifierParameter(nv, g, h, g_mask), list(t)


def keygen(nv, draw_fr):
    """keygen with its random draws from `draw_fr()` in the reference's order
    (g, h, then t[0..nv]; setup.rs:28-34)."""
    gs = draw_fr()
    hs = draw_fr()
    t = [draw_fr() for _ in range(nv)]
    return keygen_from_scalars(nv, gs, hs, t)


def dummy_keygen_from_scalars(nv, g_scalar, h_scalar, t):
    """setup.rs:120-144 naive oracle (product of eq extensions, plain scalar mul)."""
    g = G1.mul_affine(G1.gen, g_scalar)
    h = G2.mul_affine(G2.gen, h_scalar)
    pg, ph = [], []
    for i in range(nv):
        ext = eq_extension(t[i:nv])
        vals = []
        for x in range(1 << (nv - i)):
            v = 1
            for e in ext:
                v = v * e[x] % R
            vals.append(v)
        pg.append([G1.mul_affine(g, v) for v in vals])
        ph.append([G2.mul_affine(h, v) for v in vals])
    return PublicParameter(nv, pg, ph, g, h)


def commit(pp, table):
    """commit.rs:17-29 — Commitment{nv, g_product = MSM(powers_of_g[0], into_repr(f))}."""
    nv = log2_exact(len(table))
    return nv, G1.to_affine(msm(G1, pp.powers_of_g[0], list(table)))


def commitment_bytes(com):
    nv, gp = com
    return ser_u64(nv) + g1_compress(gp)


def open_(pp, table, point):
    """open.rs:19-58 — returns (eval, Proof{h, proofs}, q)."""
    eval_result = mle_eval(table, point)
    nv = log2_exact(len(table))
    r = {nv: list(table)}
    q = {}
    proofs = []
    for i in range(nv):
        k = nv - i
        p = point[i]
        qk = [0] * (1 << (k - 1))
        rk1 = [0] * (1 << (k - 1))
        rk = r[k]
        for b in range(1 << (k - 1)):
            qk[b] = (rk[2 * b + 1] - rk[2 * b]) % R
            rk1[b] = (rk[2 * b] * (1 - p) + rk[2 * b + 1] * p) % R
        q[k] = qk
        r[k - 1] = rk1
        scalars = [qk[x >> 1] for x in range(1 << k)]
        proofs.append(G2.to_affine(msm(G2, pp.powers_of_h[i], scalars)))
    return eval_result, (pp.h, proofs), q


def open_proof_bytes(proof):
    h, proofs = proof
    return g2_compress(h) + ser_u64(len(proofs)) + b"".join(g2_compress(p) for p in proofs)


def mkzg_verify(vp, com, point, value, proof):
    """verify.rs:12-45: e(C - g^v, vp.h) == prod_{i < vp.nv} e(g^{t_i} - g^{p_i}, pi_i) (the proof's own
    h is not used, verify.rs:15)."""
    from pairing import product_of_pairings, is_one

    _nv, gp = com
    _h, proofs = proof
    left_pt = G1.to_affine(G1.add(G1.from_affine(gp), G1.neg(G1.mul(G1.from_affine(vp.g), value % R))))
    pairs = [(left_pt, vp.h)]
    for i in range(vp.nv):
        li = G1.add(G1.from_affine(vp.g_mask_random[i]), G1.neg(G1.mul(G1.from_affine(vp.g), point[i] % R)))
        pairs.append((G1.to_affine(G1.neg(li)), proofs[i]))
    return is_one(product_of_pairings(pairs))


# ----------------------------------------------------------------------------- serialization
def matrix_bytes(matrix, num_constraints):
    """CanonicalSerialize of MatrixExtension {constraint: Vec<Vec<(F, usize)>>, num_constraints}."""
    out = [ser_u64(len(matrix))]
    for row in matrix:
        out.append(ser_u64(len(row)))
        for coeff, col in row:
            out.append(ser_fr(coeff))
            out.append(ser_u64(col))
    out.append(ser_u64(num_constraints))
    return b"".join(out)


def vec_fr_bytes(v):
    return ser_u64(len(v)) + b"".join(ser_fr(x) for x in v)


def prover_msg_bytes(evals):
    return vec_fr_bytes(evals)


# ----------------------------------------------------------------------------- prover
class Proof:
    """proof.rs:10-20 (field order = byte order)."""

    def __init__(self, pm1, pm2, pm3, sc1, pm4, pm5, sc2, pm6):
        self.pm1, self.pm2, self.pm3, self.sc1 = pm1, pm2, pm3, sc1
        self.pm4, self.pm5, self.sc2, self.pm6 = pm4, pm5, sc2, pm6

    def pm1_bytes(self):
        return commitment_bytes(self.pm1)

    def pm2_bytes(self):
        z_rv_0, proof = self.pm2
        return ser_fr(z_rv_0) + open_proof_bytes(proof)

    def pm4_bytes(self):
        return b"".join(ser_fr(x) for x in self.pm4)

    def pm6_bytes(self):
        z_ry, proof = self.pm6
        return ser_fr(z_ry) + open_proof_bytes(proof)

    def to_bytes(self):
        return b"".join(
            [
                self.pm1_bytes(),
                self.pm2_bytes(),
                self.pm3,
                ser_u64(len(self.sc1)),
                b"".join(prover_msg_bytes(m) for m in self.sc1),
                self.pm4_bytes(),
                self.pm5,
                ser_u64(len(self.sc2)),
                b"".join(prover_msg_bytes(m) for m in self.sc2),
                self.pm6_bytes(),
            ]
        )

    @staticmethod
    def from_bytes(b):
        pos = 0

        def take(k):
            nonlocal pos
            out = b[pos : pos + k]
            if len(out) != k:
                raise InvalidArgument("truncated proof")
            pos += k
            return out

        def u64():
            return int.from_bytes(take(8), "little")

        def fr_():
            return de_fr(take(32))

        def open_proof():
            h = g2_decompress(take(96))
            k = u64()
            return (h, [g2_decompress(take(96)) for _ in range(k)])

        def msgs():
            out = []
            for _ in range(u64()):
                out.append([fr_() for _ in range(u64())])
            return out

        nv = u64()
        pm1 = (nv, g1_decompress(take(48)))
        pm2 = (fr_(), open_proof())
        pm3 = take(8 * len(INDEX_INFO_FIELDS))
        sc1 = msgs()
        pm4 = (fr_(), fr_(), fr_())
        pm5 = take(8 * len(INDEX_INFO_FIELDS))
        sc2 = msgs()
        pm6 = (fr_(), open_proof())
        if pos != len(b):
            raise InvalidArgument("trailing bytes")
        return Proof(pm1, pm2, pm3, sc1, pm4, pm5, sc2, pm6)


def index(A, B, C):
    """indexer.rs:41-64."""
    n = len(A)
    if not is_pow2(n):
        raise InvalidArgument("Matrix width should be a power of 2.")
    for M in (A, B, C):
        check_matrix(M, n)
    return {"A": A, "B": B, "C": C, "log_n": log2_exact(n), "n": n}


def prove(pk, v, w, pp, fs=None, trace=None):
    """lib.rs:58-146 with the AHP rounds of prover.rs:109-281 inlined. `fs` is the challenge
    source (default: Blake2s512Rng transcript); `trace`, if a dict, receives intermediates."""
    log_n = pk["log_n"]
    n = pk["n"]
    if fs is None:
        fs = Blake2s512Rng()
    fs.feed(matrix_bytes(pk["A"], n))
    fs.feed(matrix_bytes(pk["B"], n))
    fs.feed(matrix_bytes(pk["C"], n))
    fs.feed(vec_fr_bytes(v))
    # prover_init, prover.rs:109-121
    if not is_pow2(len(v)):
        raise InvalidArgument("public input should be power of two")
    if len(v) + len(w) != n:
        raise InvalidArgument("|v| + |w| != number of variables")
    log_v = log2_exact(len(v))
    # round 1, prover.rs:123-141
    z = [x % R for x in list(v) + list(w)]
    com = commit(pp, z)
    pm1_b = commitment_bytes(com)
    fs.feed(pm1_b)
    r_v = [fs.rand_fr() for _ in range(log_v)]
    # round 2, prover.rs:143-160
    point = r_v + [0] * (log_n - log_v)
    z_rv_0, proof_rv, _ = open_(pp, z, point)
    pm2 = (z_rv_0, proof_rv)
    fs.feed(ser_fr(z_rv_0) + open_proof_bytes(proof_rv))
    tau = [fs.rand_fr() for _ in range(log_n)]
    # round 3, prover.rs:163-196
    eq = eq_extension(tau)
    az = sum_over_y(pk["A"], z)
    bz = sum_over_y(pk["B"], z)
    cz = sum_over_y(pk["C"], z)
    neg_cz = [(-x) % R for x in cz]
    sc = MLSumcheckProver([[az, bz] + eq, [neg_cz] + eq], log_n)
    pm3 = sc.info_bytes()
    fs.feed(pm3)
    if trace is not None:
        trace.update(z=z, r_v=r_v, tau=tau, az=az, bz=bz, cz=cz, com=com)
    # sumcheck 1, lib.rs:86-103
    msgs1 = []
    ch = None
    chs1 = []
    for _ in range(log_n):
        m = sc.prove_round(ch)
        msgs1.append(m)
        fs.feed(prover_msg_bytes(m))
        ch = fs.rand_fr()
        chs1.append(ch)
    # round 4, prover.rs:210-228
    r_x = sc.randomness + [ch]
    va, vb, vc = mle_eval(az, r_x), mle_eval(bz, r_x), mle_eval(cz, r_x)
    pm4 = (va, vb, vc)
    fs.feed(b"".join(ser_fr(x) for x in pm4))
    r_a, r_b, r_c = fs.rand_fr(), fs.rand_fr(), fs.rand_fr()
    # round 5, prover.rs:230-255
    a_rx = [x * r_a % R for x in eval_on_x(pk["A"], r_x)]
    b_rx = [x * r_b % R for x in eval_on_x(pk["B"], r_x)]
    c_rx = [x * r_c % R for x in eval_on_x(pk["C"], r_x)]
    sc2 = MLSumcheckProver([[a_rx, z], [b_rx, z], [c_rx, z]], log_n)
    pm5 = sc2.info_bytes()
    fs.feed(pm5)
    if trace is not None:
        trace.update(r_x=r_x, r_abc=(r_a, r_b, r_c), m_rx=[(a + b + c) % R for a, b, c in zip(a_rx, b_rx, c_rx)])
    msgs2 = []
    ch = None
    for _ in range(log_n):
        m = sc2.prove_round(ch)
        msgs2.append(m)
        fs.feed(prover_msg_bytes(m))
        ch = fs.rand_fr()
    # round 6, prover.rs:268-281
    r_y = sc2.randomness + [ch]
    z_ry, proof_ry, _ = open_(pp, z, r_y)
    if trace is not None:
        trace.update(r_y=r_y, chs1=chs1)
    return Proof(com, pm2, pm3, msgs1, pm4, pm5, msgs2, (z_ry, proof_ry))


# ----------------------------------------------------------------------------- verifier
def verify(vk, v, proof, vp, fs=None, feed_matrices=None, eval_rr=None, check_pairings=True, out=None):
    """lib.rs:147-212 with verifier.rs:143-512. Raises on rejection, returns True on accept.

    Hooks for full-size tests (same checks, faster plumbing): `feed_matrices(fs)` absorbs A, B, C
    (default: matrix_bytes of vk's row lists); `eval_rr(r_x, r_y)` returns (A, B, C)(r_x, r_y)
    (default: eval_on_x + mle_eval); check_pairings=False skips the two mKZG pairing checks;
    `out`, if a dict, receives the opening points (r_v padded, r_y) and challenges."""
    log_n = vk["log_n"]
    n = vk["n"]
    if fs is None:
        fs = Blake2s512Rng()
    if feed_matrices is not None:
        feed_matrices(fs)
    else:
        fs.feed(matrix_bytes(vk["A"], n))
        fs.feed(matrix_bytes(vk["B"], n))
        fs.feed(matrix_bytes(vk["C"], n))
    fs.feed(vec_fr_bytes(v))
    if not is_pow2(len(v)) or len(v) > n:
        raise InvalidArgument("public input should be power of two and has size smaller than number of constraints")
    log_v = log2_exact(len(v))
    fs.feed(proof.pm1_bytes())
    r_v = [fs.rand_fr() for _ in range(log_v)]
    fs.feed(proof.pm2_bytes())
    tau = [fs.rand_fr() for _ in range(log_n)]
    info1 = dict(zip(INDEX_INFO_FIELDS, [int.from_bytes(proof.pm3[8 * i : 8 * i + 8], "little") for i in range(len(INDEX_INFO_FIELDS))]))
    if info1["num_variables"] != log_n:
        raise InvalidArgument("invalid sumcheck proposal")
    fs.feed(proof.pm3)
    if len(proof.sc1) != log_n or len(proof.sc2) != log_n:
        raise InvalidArgument("malformed sumcheck message")
    rand1 = []
    for m in proof.sc1:
        fs.feed(prover_msg_bytes(m))
        rand1.append(fs.rand_fr())
    fs.feed(proof.pm4_bytes())
    r_a, r_b, r_c = fs.rand_fr(), fs.rand_fr(), fs.rand_fr()
    info2 = dict(zip(INDEX_INFO_FIELDS, [int.from_bytes(proof.pm5[8 * i : 8 * i + 8], "little") for i in range(len(INDEX_INFO_FIELDS))]))
    if info2["num_variables"] != log_n:
        raise InvalidArgument("invalid sumcheck proposal")
    fs.feed(proof.pm5)
    rand2 = []
    for m in proof.sc2:
        fs.feed(prover_msg_bytes(m))
        rand2.append(fs.rand_fr())
    fs.feed(proof.pm6_bytes())
    # verify_sixth_round, verifier.rs:443-512
    com = proof.pm1
    z_rv_0, proof_rv = proof.pm2
    r_v0 = r_v + [0] * (log_n - log_v)
    if check_pairings and not mkzg_verify(vp, com, r_v0, z_rv_0, proof_rv):
        raise InvalidArgument("public witness failed in commitment check")
    if mle_eval([x % R for x in v], r_v) != z_rv_0:
        raise InvalidArgument("public witness is inconsistent with proof")
    r_x, expected1 = check_and_generate_subclaim(proof.sc1, rand1, 0, log_n, info1["max_multiplicands"])
    eq_rx = 1
    for i, ti in enumerate(tau):
        eq_rx = eq_rx * ((2 * ti * r_x[i] - r_x[i] - ti + 1) % R) % R
    va, vb, vc = proof.pm4
    if (va * vb - vc) * eq_rx % R != expected1:
        raise WrongWitness("first sumcheck has wrong subclaim")
    z_ry, proof_ry = proof.pm6
    claimed2 = (r_a * va + r_b * vb + r_c * vc) % R
    r_y, expected2 = check_and_generate_subclaim(proof.sc2, rand2, claimed2, log_n, info2["max_multiplicands"])
    if eval_rr is not None:
        a_rr, b_rr, c_rr = eval_rr(r_x, r_y)
    else:
        a_rr = mle_eval(eval_on_x(vk["A"], r_x), r_y)
        b_rr = mle_eval(eval_on_x(vk["B"], r_x), r_y)
        c_rr = mle_eval(eval_on_x(vk["C"], r_x), r_y)
    actual = (r_a * a_rr * z_ry + r_b * b_rr * z_ry + r_c * c_rr * z_ry) % R
    if expected2 != actual:
        raise WrongWitness("Cannot verify matrix A, B, C")
    if check_pairings and not mkzg_verify(vp, com, r_y, z_ry, proof_ry):
        raise WrongWitness("Cannot verify z_ry")
    if out is not None:
        out.update(r_v0=r_v0, r_y=r_y, r_x=r_x, tau=tau)
    return True
