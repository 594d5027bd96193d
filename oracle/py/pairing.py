"""ORACLE — TEST INFRASTRUCTURE ONLY.

A (slow, pure-Python) bilinear pairing on BLS12-381 for the verifier side of the tests:
`E::pairing` / `E::product_of_pairings` used by /root/reference/src/commitment/verify.rs:12-45
[upstream ark-bls12-381, not in container]. Off the hot path (verify is a CPU
acceptance check).

Fq12 = Fq[w]/(w^12 - 2 w^6 + 2), Fq2 embedded by u -> w^6 - 1; G2 (on the twist
y^2 = x^3 + 4(u+1)) maps to E(Fq12) by (x, y) -> (x / w^2, y / w^3). Miller loop over
|x| = 0xd201000000010000 with affine doubling/addition in Fq2 and lines evaluated as sparse
Fq12 elements scaled by w^3 (a factor killed by the final exponentiation). The sign of x is
ignored, giving the inverse of the optimal-ate value: still bilinear and non-degenerate,
which is all an equality check of pairing products needs.
"""
from bls12_381 import Q, R, f2_add, f2_sub, f2_mul, f2_sqr, f2_inv, f2_muls, f2_neg

ATE = 0xD201000000010000
FINAL_EXP = (Q**12 - 1) // R
ONE12 = [1] + [0] * 11


def f12_mul(a, b):
    c = [0] * 23
    for i, ai in enumerate(a):
        if ai:
            for j, bj in enumerate(b):
                if bj:
                    c[i + j] += ai * bj
    for k in range(22, 11, -1):
        t = c[k]
        if t:
            c[k - 6] += 2 * t
            c[k - 12] -= 2 * t
    return [x % Q for x in c[:12]]


def f12_pow(a, e):
    acc = ONE12
    base = a
    while e:
        if e & 1:
            acc = f12_mul(acc, base)
        base = f12_mul(base, base)
        e >>= 1
    return acc


def _line(l, x1, y1, P):
    """w^3 * [slope*(xP - X1) - (yP - Y1)] for slope = l * w^-1, T1 = (x1 w^-2, y1 w^-3)."""
    xP, yP = P
    m = f2_mul(l, x1)
    c = [0] * 12
    c[0] = ((y1[0] - y1[1]) - (m[0] - m[1])) % Q
    c[6] = (y1[1] - m[1]) % Q
    c[2] = (l[0] - l[1]) * xP % Q
    c[8] = l[1] * xP % Q
    c[3] = (-yP) % Q
    return c


def _vertical(x1, P):
    """w^2 * (xP - X1)."""
    c = [0] * 12
    c[2] = P[0] % Q
    c[0] = (-(x1[0] - x1[1])) % Q
    c[6] = (-x1[1]) % Q
    return c


def miller_loop(Qa, P):
    """Qa: affine G2 point ((x0,x1),(y0,y1)); P: affine G1 point (x, y). None = infinity."""
    if Qa is None or P is None:
        return ONE12
    T = Qa
    f = ONE12
    for i in range(62, -1, -1):
        # doubling step
        x1, y1 = T
        lam = f2_mul(f2_muls(f2_sqr(x1), 3), f2_inv(f2_muls(y1, 2)))
        f = f12_mul(f12_mul(f, f), _line(lam, x1, y1, P))
        x3 = f2_sub(f2_sqr(lam), f2_muls(x1, 2))
        y3 = f2_sub(f2_mul(lam, f2_sub(x1, x3)), y1)
        T = (x3, y3)
        if (ATE >> i) & 1:
            x1, y1 = T
            x2, y2 = Qa
            if x1 == x2:
                if y1 == y2:
                    raise ValueError("unexpected doubling in addition step")
                f = f12_mul(f, _vertical(x1, P))
                T = None
                raise ValueError("unexpected T = -Q in Miller loop")
            lam = f2_mul(f2_sub(y2, y1), f2_inv(f2_sub(x2, x1)))
            f = f12_mul(f, _line(lam, x1, y1, P))
            x3 = f2_sub(f2_sub(f2_sqr(lam), x1), x2)
            y3 = f2_sub(f2_mul(lam, f2_sub(x1, x3)), y1)
            T = (x3, y3)
    return f


def final_exp(f):
    return f12_pow(f, FINAL_EXP)


def pairing(P, Qa):
    """e(P in G1, Q in G2) (affine inputs)."""
    return final_exp(miller_loop(Qa, P))


def product_of_pairings(pairs):
    """prod_i e(P_i, Q_i) with one final exponentiation."""
    f = ONE12
    for P, Qa in pairs:
        f = f12_mul(f, miller_loop(Qa, P))
    return final_exp(f)


def is_one(f):
    return f == ONE12
