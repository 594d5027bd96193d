"""The product's host pairing (spx_pairing_check: pairing.hpp, used by spx_verify for verify.rs:12-45)
on CPU: bilinearity and non-degeneracy on oracle-generated points, the mKZG verification equation of
a real opening (oracle keygen + open), and rejection of a wrong evaluation — no GPU needed."""
import pytest

from bls12_381 import G1, G2, R, g1_uncompressed, g2_uncompressed
from gen import SplitMix64
import spartan


def test_bilinearity(spx):
    a, b = 0x1234567890ABCDEF, 0xFEDCBA987654321
    P = G1.mul_affine(G1.gen, 7)
    Q = G2.mul_affine(G2.gen, 11)
    aP, bQ = G1.mul_affine(P, a), G2.mul_affine(Q, b)
    abP_neg = G1.neg_affine(G1.mul_affine(P, a * b % R)) if hasattr(G1, "neg_affine") else G1.to_affine(G1.neg(G1.mul(G1.from_affine(P), a * b % R)))
    g1 = [g1_uncompressed(aP), g1_uncompressed(abP_neg)]
    g2 = [g2_uncompressed(bQ), g2_uncompressed(Q)]
    assert spx.pairing_product_is_one(g1, g2)  # e(aP, bQ) e(-abP, Q) = 1
    g1_bad = [g1_uncompressed(aP), g1_uncompressed(G1.to_affine(G1.neg(G1.mul(G1.from_affine(P), (a * b + 1) % R))))]
    assert not spx.pairing_product_is_one(g1_bad, g2)
    assert not spx.pairing_product_is_one([g1_uncompressed(P)], [g2_uncompressed(Q)])  # non-degenerate
    assert spx.pairing_product_is_one([g1_uncompressed(None)], [g2_uncompressed(Q)])  # infinity -> 1


def test_mkzg_equation(spx):
    nv = 5
    rng = SplitMix64(33)
    pp, vp, t = spartan.keygen(nv, rng.next_fr)
    poly = [rng.next_fr() for _ in range(1 << nv)]
    point = [rng.next_fr() for _ in range(nv)]
    com = spartan.commit(pp, poly)
    ev, pf, _ = spartan.open_(pp, poly, point)

    def pairs(value):
        left = G1.to_affine(G1.add(G1.from_affine(com[1]), G1.neg(G1.mul(G1.from_affine(vp.g), value))))
        g1, g2 = [g1_uncompressed(left)], [g2_uncompressed(vp.h)]
        for i in range(nv):
            li = G1.add(G1.from_affine(vp.g_mask_random[i]), G1.neg(G1.mul(G1.from_affine(vp.g), point[i])))
            g1.append(g1_uncompressed(G1.to_affine(G1.neg(li))))
            g2.append(g2_uncompressed(pf[1][i]))
        return g1, g2

    assert spx.pairing_product_is_one(*pairs(ev))
    assert not spx.pairing_product_is_one(*pairs((ev + 1) % R))
