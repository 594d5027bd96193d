"""ORACLE — TEST INFRASTRUCTURE ONLY (never shipped, never on the product path).

Pure-Python restatement of the BLS12-381 arithmetic the reference prover runs on.
The reference instantiates everything with `ark_bls12_381::Bls12_381`
(/root/reference/src/test_utils.rs:15-16, Cargo.toml:21-22); the arithmetic itself
lives in the upstream crates ark-ff / ark-ec / ark-bls12-381 / ark-serialize
[upstream, not in container; unpinned git deps, Cargo.toml:10-14,22].

What is restated here (published algorithms of those crates):
  * Fr (255-bit scalar field), Fq (381-bit base field), Fq2 = Fq[u]/(u^2+1).
  * Montgomery convention R = 2^256 for Fr, 2^384 for Fq (4x/6x u64 limbs) — used only
    where the reference's bytes depend on it (Fr::rand interprets raw limbs as Montgomery
    form, see transcript.py).
  * G1: y^2 = x^3 + 4 over Fq; G2: y^2 = x^3 + 4(u+1) over Fq2; Jacobian arithmetic.
  * ark-serialize byte layout: Fr = 32 B LE canonical; Fq = 48 B LE; Fq2 = c0 || c1;
    compressed SW points = x with flags in the top bits of the LAST byte
    (bit 6 = point at infinity, bit 7 = "positive y", i.e. y > -y, Fq2 ordered c1 then c0).
    These flag conventions are reconstructed ("unverified against upstream").

Pure-Python loops: small cases only.
"""

Q = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001

FR_BITS = 255
FQ_BITS = 381
FR_MONT_R = (1 << 256) % R
FR_MONT_RINV = pow(1 << 256, -1, R)
FQ_MONT_R = (1 << 384) % Q

G1_GEN = (
    0x17F1D3A73197D7942695638C4FA9AC0FC3688C4F9774B905A14E3A3F171BAC586C55E83FF97A1AEFFB3AF00ADB22C6BB,
    0x08B3F481E3AAA0F1A09E30ED741D8AE4FCF5E095D5D00AF600DB18CB2C04B3EDD03CC744A2888AE40CAA232946C5E7E1,
)
G2_GEN = (
    (
        0x024AA2B2F08F0A91260805272DC51051C6E47AD4FA403B02B4510B647AE3D1770BAC0326A805BBEFD48056C8C121BDB8,
        0x13E02B6052719F607DACD3A088274F65596BD0D09920B61AB5DA61BBDC7F5049334CF11213945D57E5AC7D055D042B7E,
    ),
    (
        0x0CE5D527727D6E118CC9CDC6DA2E351AADFD9BAA8CBDD3A76D429A695160D12C923AC9CC3BACA289E193548608B82801,
        0x0606C4A02EA734CC32ACD2B02BC28B99CB3E287E85A763AF267492AB572E99AB3F370D275CEC1DA1AAA9075FF05F79BE,
    ),
)


# ----------------------------------------------------------------------------- Fr
def fr(x):
    return x % R


def fr_inv(x):
    if x % R == 0:
        raise ZeroDivisionError("Fr inverse of zero")
    return pow(x, R - 2, R)


def fr_from_mont_limbs(v):
    """ark-ff Fp256(BigInteger256) holds the Montgomery form; value = v * R^-1."""
    return v * FR_MONT_RINV % R


def fr_to_mont(x):
    return x * FR_MONT_R % R


# ----------------------------------------------------------------------------- Fq2
def f2_add(a, b):
    return ((a[0] + b[0]) % Q, (a[1] + b[1]) % Q)


def f2_sub(a, b):
    return ((a[0] - b[0]) % Q, (a[1] - b[1]) % Q)


def f2_neg(a):
    return ((-a[0]) % Q, (-a[1]) % Q)


def f2_mul(a, b):
    a0, a1 = a
    b0, b1 = b
    t0 = a0 * b0
    t1 = a1 * b1
    return ((t0 - t1) % Q, ((a0 + a1) * (b0 + b1) - t0 - t1) % Q)


def f2_sqr(a):
    a0, a1 = a
    return ((a0 + a1) * (a0 - a1) % Q, 2 * a0 * a1 % Q)


def f2_muls(a, s):
    return (a[0] * s % Q, a[1] * s % Q)


def f2_inv(a):
    a0, a1 = a
    t = pow((a0 * a0 + a1 * a1) % Q, Q - 2, Q)
    return (a0 * t % Q, (-a1) * t % Q)


F2_ZERO = (0, 0)
F2_ONE = (1, 0)


class _Fq:
    """Field-op bundle for Fq (G1 coordinates)."""

    zero = 0
    one = 1

    @staticmethod
    def add(a, b):
        return (a + b) % Q

    @staticmethod
    def sub(a, b):
        return (a - b) % Q

    @staticmethod
    def mul(a, b):
        return a * b % Q

    @staticmethod
    def sqr(a):
        return a * a % Q

    @staticmethod
    def neg(a):
        return (-a) % Q

    @staticmethod
    def inv(a):
        return pow(a, Q - 2, Q)

    @staticmethod
    def small(k):
        return k % Q

    @staticmethod
    def is_zero(a):
        return a == 0

    @staticmethod
    def gt(a, b):  # ark-ff Ord on Fp compares canonical integers
        return a > b


class _Fq2:
    """Field-op bundle for Fq2 (G2 coordinates)."""

    zero = F2_ZERO
    one = F2_ONE
    add = staticmethod(f2_add)
    sub = staticmethod(f2_sub)
    mul = staticmethod(f2_mul)
    sqr = staticmethod(f2_sqr)
    neg = staticmethod(f2_neg)
    inv = staticmethod(f2_inv)

    @staticmethod
    def small(k):
        return (k % Q, 0)

    @staticmethod
    def is_zero(a):
        return a == F2_ZERO

    @staticmethod
    def gt(a, b):  # ark-ff Ord on QuadExtField: compare c1 first, then c0
        if a[1] != b[1]:
            return a[1] > b[1]
        return a[0] > b[0]


FQ = _Fq
FQ2 = _Fq2
G1_B = 4
G2_B = (4, 4)


# ----------------------------------------------------------------------------- curves
# Jacobian point: (X, Y, Z) with Z == zero meaning infinity. Affine: (x, y) or None.
class Curve:
    def __init__(self, F, b, gen, name):
        self.F = F
        self.b = b
        self.gen = gen
        self.name = name
        self.inf = (F.one, F.one, F.zero)

    def is_inf(self, P):
        return self.F.is_zero(P[2])

    def on_curve(self, A):
        if A is None:
            return True
        F = self.F
        x, y = A
        return F.sqr(y) == F.add(F.mul(F.sqr(x), x), self.b)

    def from_affine(self, A):
        if A is None:
            return self.inf
        return (A[0], A[1], self.F.one)

    def to_affine(self, P):
        F = self.F
        if F.is_zero(P[2]):
            return None
        zi = F.inv(P[2])
        zi2 = F.sqr(zi)
        return (F.mul(P[0], zi2), F.mul(P[1], F.mul(zi2, zi)))

    def dbl(self, P):
        F = self.F
        X, Y, Z = P
        if F.is_zero(Z) or F.is_zero(Y):
            return self.inf
        A = F.sqr(X)
        B = F.sqr(Y)
        C = F.sqr(B)
        D = F.sub(F.sqr(F.add(X, B)), F.add(A, C))
        D = F.add(D, D)
        E = F.add(F.add(A, A), A)
        Fv = F.sqr(E)
        X3 = F.sub(Fv, F.add(D, D))
        C8 = F.add(C, C)
        C8 = F.add(C8, C8)
        C8 = F.add(C8, C8)
        Y3 = F.sub(F.mul(E, F.sub(D, X3)), C8)
        Z3 = F.mul(F.add(Y, Y), Z)
        return (X3, Y3, Z3)

    def add(self, P, Qp):
        F = self.F
        if F.is_zero(P[2]):
            return Qp
        if F.is_zero(Qp[2]):
            return P
        X1, Y1, Z1 = P
        X2, Y2, Z2 = Qp
        Z1Z1 = F.sqr(Z1)
        Z2Z2 = F.sqr(Z2)
        U1 = F.mul(X1, Z2Z2)
        U2 = F.mul(X2, Z1Z1)
        S1 = F.mul(F.mul(Y1, Z2), Z2Z2)
        S2 = F.mul(F.mul(Y2, Z1), Z1Z1)
        if U1 == U2:
            if S1 == S2:
                return self.dbl(P)
            return self.inf
        H = F.sub(U2, U1)
        I = F.sqr(F.add(H, H))
        J = F.mul(H, I)
        r = F.sub(S2, S1)
        r = F.add(r, r)
        V = F.mul(U1, I)
        X3 = F.sub(F.sub(F.sqr(r), J), F.add(V, V))
        S1J = F.mul(S1, J)
        Y3 = F.sub(F.mul(r, F.sub(V, X3)), F.add(S1J, S1J))
        Z3 = F.mul(F.sub(F.sqr(F.add(Z1, Z2)), F.add(Z1Z1, Z2Z2)), H)
        return (X3, Y3, Z3)

    def madd(self, P, A):
        """P (Jacobian) + A (affine, not None)."""
        F = self.F
        if F.is_zero(P[2]):
            return (A[0], A[1], F.one)
        X1, Y1, Z1 = P
        Z1Z1 = F.sqr(Z1)
        U2 = F.mul(A[0], Z1Z1)
        S2 = F.mul(F.mul(A[1], Z1), Z1Z1)
        if U2 == X1:
            if S2 == Y1:
                return self.dbl(P)
            return self.inf
        H = F.sub(U2, X1)
        HH = F.sqr(H)
        I = F.add(HH, HH)
        I = F.add(I, I)
        J = F.mul(H, I)
        r = F.sub(S2, Y1)
        r = F.add(r, r)
        V = F.mul(X1, I)
        X3 = F.sub(F.sub(F.sqr(r), J), F.add(V, V))
        Y1J = F.mul(Y1, J)
        Y3 = F.sub(F.mul(r, F.sub(V, X3)), F.add(Y1J, Y1J))
        Z3 = F.sub(F.sub(F.sqr(F.add(Z1, H)), Z1Z1), HH)
        return (X3, Y3, Z3)

    def neg(self, P):
        return (P[0], self.F.neg(P[1]), P[2])

    def neg_affine(self, A):
        if A is None:
            return None
        return (A[0], self.F.neg(A[1]))

    def mul(self, P, k):
        """Jacobian P times integer k >= 0 (double-and-add, MSB first)."""
        acc = self.inf
        for bit in bin(k)[2:] if k > 0 else "":
            acc = self.dbl(acc)
            if bit == "1":
                acc = self.add(acc, P)
        return acc

    def mul_affine(self, A, k):
        return self.to_affine(self.mul(self.from_affine(A), k % R))

    def eq_proj(self, P, Qp):
        return self.to_affine(P) == self.to_affine(Qp)

    def batch_to_affine(self, pts):
        """Montgomery batch inversion (ark-ec batch_normalization semantics)."""
        F = self.F
        out = [None] * len(pts)
        prefix = []
        acc = F.one
        for P in pts:
            prefix.append(acc)
            if not F.is_zero(P[2]):
                acc = F.mul(acc, P[2])
        inv = F.inv(acc) if not F.is_zero(acc) else F.zero
        for i in range(len(pts) - 1, -1, -1):
            P = pts[i]
            if F.is_zero(P[2]):
                continue
            zi = F.mul(inv, prefix[i])
            inv = F.mul(inv, P[2])
            zi2 = F.sqr(zi)
            out[i] = (F.mul(P[0], zi2), F.mul(P[1], F.mul(zi2, zi)))
        return out


G1 = Curve(FQ, G1_B, G1_GEN, "G1")
G2 = Curve(FQ2, G2_B, G2_GEN, "G2")


# ----------------------------------------------------------------------------- MSM
def ceil_log2(x):
    """ark_std::log2: ceil(log2(x)), 0 for x == 0."""
    return 0 if x <= 1 else (x - 1).bit_length()


def msm_window_size(n):
    """ark-ec VariableBaseMSM window: c = 3 if N < 32 else ln_without_floats(N) + 2,
    ln_without_floats(N) = ceil_log2(N) * 69 / 100 [upstream]."""
    if n < 32:
        return 3
    return ceil_log2(n) * 69 // 100 + 2


def msm(curve, bases, scalars):
    """Restates ark-ec `VariableBaseMSM::multi_scalar_mul` [upstream] (single-thread,
    unsigned c-bit windows, 2^c-1 buckets, running-sum bucket reduction). Used at
    /root/reference/src/commitment/commit.rs:25 and open.rs:49. Scalars are canonical
    integers (`into_repr`). Returns a Jacobian point."""
    assert len(bases) == len(scalars)
    c = msm_window_size(len(scalars))
    num_bits = FR_BITS
    window_sums = []
    for w_start in range(0, num_bits, c):
        res = curve.inf
        buckets = [curve.inf] * ((1 << c) - 1)
        for s, base in zip(scalars, bases):
            if base is None:
                continue
            if s == 1:
                if w_start == 0:
                    res = curve.madd(res, base)
            else:
                d = (s >> w_start) & ((1 << c) - 1)
                if d:
                    buckets[d - 1] = curve.madd(buckets[d - 1], base)
        running = curve.inf
        for b in reversed(buckets):
            running = curve.add(running, b)
            res = curve.add(res, running)
        window_sums.append(res)
    total = curve.inf
    for ws in reversed(window_sums[1:]):
        total = curve.add(total, ws)
        for _ in range(c):
            total = curve.dbl(total)
    return curve.add(total, window_sums[0])


def msm_naive(curve, bases, scalars):
    acc = curve.inf
    for s, b in zip(scalars, bases):
        if b is not None and s % R:
            acc = curve.add(acc, curve.mul(curve.from_affine(b), s % R))
    return acc


# ----------------------------------------------------------------------------- serialization
def ser_u64(x):
    return int(x).to_bytes(8, "little")


def ser_fr(x):
    return (x % R).to_bytes(32, "little")


def de_fr(b):
    v = int.from_bytes(b[:32], "little")
    if v >= R:
        raise ValueError("non-canonical Fr")
    return v


def ser_fq(x, flags=0):
    b = bytearray((x % Q).to_bytes(48, "little"))
    b[47] |= flags
    return bytes(b)


def ser_fq2(x, flags=0):
    return ser_fq(x[0]) + ser_fq(x[1], flags)


FLAG_INF = 1 << 6
FLAG_POS_Y = 1 << 7


def _compress(curve, A, ser):
    F = curve.F
    if A is None:
        return ser(F.zero, FLAG_INF)
    x, y = A
    flags = FLAG_POS_Y if F.gt(y, F.neg(y)) else 0
    return ser(x, flags)


def g1_compress(A):
    return _compress(G1, A, ser_fq)


def g2_compress(A):
    return _compress(G2, A, ser_fq2)


def g1_uncompressed(A):
    if A is None:
        return ser_fq(0) + ser_fq(1, FLAG_INF)
    return ser_fq(A[0]) + ser_fq(A[1])


def g2_uncompressed(A):
    if A is None:
        return ser_fq2(F2_ZERO) + ser_fq2(F2_ONE, FLAG_INF)
    return ser_fq2(A[0]) + ser_fq2(A[1])


def _de_fq(b):
    v = int.from_bytes(b[:48], "little") & ((1 << 381) - 1)
    return v


def g1_from_uncompressed(b):
    if b[95] & FLAG_INF:
        return None
    return (_de_fq(b[0:48]), _de_fq(b[48:96]))


def g2_from_uncompressed(b):
    if b[191] & FLAG_INF:
        return None
    return ((_de_fq(b[0:48]), _de_fq(b[48:96])), (_de_fq(b[96:144]), _de_fq(b[144:192])))


def _sqrt_fq(a):
    # Q = 3 mod 4
    s = pow(a, (Q + 1) // 4, Q)
    return s if s * s % Q == a % Q else None


def _sqrt_fq2(a):
    # Algorithm 9 of "Square root computation over even extension fields" (q = 3 mod 4).
    a1 = _f2_pow(a, (Q - 3) // 4)
    alpha = f2_mul(a1, f2_mul(a1, a))
    x0 = f2_mul(a1, a)
    if alpha == (Q - 1, 0):
        x = f2_mul((0, 1), x0)
    else:
        b = _f2_pow(f2_add(F2_ONE, alpha), (Q - 1) // 2)
        x = f2_mul(b, x0)
    return x if f2_sqr(x) == a else None


def _f2_pow(a, e):
    acc = F2_ONE
    base = a
    while e:
        if e & 1:
            acc = f2_mul(acc, base)
        base = f2_sqr(base)
        e >>= 1
    return acc


def g1_decompress(b):
    flags = b[47] & 0xC0
    if flags & FLAG_INF:
        return None
    x = _de_fq(b[0:48])
    y = _sqrt_fq((x * x * x + 4) % Q)
    if y is None:
        raise ValueError("not on curve")
    pos = y > (-y) % Q
    if pos != bool(flags & FLAG_POS_Y):
        y = (-y) % Q
    return (x, y)


def g2_decompress(b):
    flags = b[95] & 0xC0
    if flags & FLAG_INF:
        return None
    x = (_de_fq(b[0:48]), _de_fq(b[48:96]))
    y = _sqrt_fq2(f2_add(f2_mul(f2_sqr(x), x), G2_B))
    if y is None:
        raise ValueError("not on curve")
    if FQ2.gt(y, f2_neg(y)) != bool(flags & FLAG_POS_Y):
        y = f2_neg(y)
    return (x, y)
