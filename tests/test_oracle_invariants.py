"""The reference's own tests, restated against the Python oracle (CPU). They pin the
MATHEMATICAL behaviour of the restatement (the reference ships no byte-level golden vectors):
  eq.rs:29-46, r1cs_reader.rs:127-145, commitment/commit.rs:53-66, commitment/setup.rs:146-156,
  commitment/verify.rs:60-95, ahp/tests.rs:8-75, benchmark.rs:11-50 (prove/serialize/verify)."""
import random

import pytest

from bls12_381 import G1, G2, R
from gen import SplitMix64, random_matrix, ref_shaped, uniform_3n
from pairing import pairing, f12_mul, ONE12
from spartan import (
    Proof,
    SumCheckError,
    WrongWitness,
    InvalidArgument,
    commit,
    dummy_keygen_from_scalars,
    eq_extension,
    eval_on_x,
    index,
    keygen,
    keygen_from_scalars,
    mkzg_verify,
    mle_eval,
    open_,
    prove,
    verify,
)
from transcript import InjectedChallenges


def bits_to_field_elements(bits, num_bits):  # test_utils.rs:39-49
    return [(bits >> i) & 1 for i in range(num_bits)]


def test_eq_functionality():  # eq.rs:29-46
    t = 0b101101001
    ext = eq_extension(bits_to_field_elements(t, 9))
    for x in range(1 << 9):
        v = 1
        for tab in ext:
            v = v * tab[x] % R
        assert v == (1 if x == t else 0)


def test_eval_on_x_sanity():  # r1cs_reader.rs:127-145
    matrix = random_matrix(6, 1 << 9, seed=3)
    expected = matrix[0b110010]
    point = [0, 1, 0, 0, 1, 1]
    got = eval_on_x(matrix, point)
    for val, idx in expected:
        assert got[idx] == val


def test_commit_equals_g_pow_f_of_t():  # commit.rs:53-66
    rng = SplitMix64(11)
    pp, vp, t = keygen(4, rng.next_fr)
    poly = [rng.next_fr() for _ in range(16)]
    _, gp = commit(pp, poly)
    assert gp == G1.mul_affine(pp.g, mle_eval(poly, t))


def test_keygen_matches_dummy_keygen():  # setup.rs:146-156
    rs = SplitMix64(5)
    gs, hs = rs.next_fr(), rs.next_fr()
    t = [rs.next_fr() for _ in range(4)]
    pp, _, _ = keygen_from_scalars(4, gs, hs, t)
    ref = dummy_keygen_from_scalars(4, gs, hs, t)
    assert pp.h == ref.h
    assert pp.powers_of_h == ref.powers_of_h
    assert pp.powers_of_g == ref.powers_of_g


def test_open_quotient_identity_and_verify():  # verify.rs:60-95 (nv reduced from 10 to 5 for CPU time)
    nv = 5
    rng = SplitMix64(17)
    pp, vp, s = keygen(nv, rng.next_fr)
    poly = [rng.next_fr() for _ in range(1 << nv)]
    point = [rng.next_fr() for _ in range(nv)]
    com = commit(pp, poly)
    ev, pf, q = open_(pp, poly, point)
    fx, ft = mle_eval(poly, s), mle_eval(poly, point)
    rhs = 0
    lhs_pair = pairing(G1.to_affine(G1.add(G1.from_affine(com[1]), G1.neg(G1.mul(G1.from_affine(vp.g), ft)))), pp.h)
    rhs_pair = ONE12
    for i in range(nv):
        k = nv - i
        q_i = [q[k][a >> 1] for a in range(1 << k)]
        qv = mle_eval(q_i, s[i:])
        rhs = (rhs + (s[i] - point[i]) * qv) % R
        assert G2.mul_affine(pp.h, qv) == pf[1][i], "open error"
        rhs_pair = f12_mul(rhs_pair, pairing(G1.mul_affine(vp.g, (s[i] - point[i]) % R), G2.mul_affine(pp.h, qv)))
    assert (fx - ft) % R == rhs
    assert lhs_pair == rhs_pair
    assert mkzg_verify(vp, com, point, ev, pf)
    assert not mkzg_verify(vp, com, point, (ev + 1) % R, pf)


@pytest.mark.parametrize("log_n,log_v", [(4, 2), (6, 2)])
def test_interactive_protocol_accepts(log_n, log_v):  # ahp/tests.rs:8-75 (verifier coins injected)
    A, B, C, v, w = ref_shaped(log_n, log_v, density=1, seed=log_n)
    pp, vp, _ = keygen(log_n, SplitMix64(9).next_fr)
    pk = index(A, B, C)
    pf = prove(pk, v, w, pp, fs=InjectedChallenges(123))
    assert verify(pk, v, pf, vp, fs=InjectedChallenges(123))


@pytest.mark.parametrize("gen,log_n,log_v", [("u3n", 5, 2), ("ref", 6, 5)])
def test_fs_prove_serialize_verify(gen, log_n, log_v):  # benchmark.rs:11-50
    A, B, C, v, w = (uniform_3n if gen == "u3n" else ref_shaped)(log_n, log_v)
    pp, vp, _ = keygen(log_n, SplitMix64(21).next_fr)
    pk = index(A, B, C)
    b = prove(pk, v, w, pp).to_bytes()
    pf = Proof.from_bytes(b)
    assert pf.to_bytes() == b
    assert verify(pk, v, pf, vp)


def test_wrong_witness_and_tampering_rejected():
    A, B, C, v, w = uniform_3n(4, 2, seed=5)
    pp, vp, _ = keygen(4, SplitMix64(1).next_fr)
    pk = index(A, B, C)
    w2 = list(w)
    w2[3] = (w2[3] + 1) % R
    with pytest.raises((WrongWitness, InvalidArgument, SumCheckError)):
        verify(pk, v, prove(pk, v, w2, pp), vp)
    b = bytearray(prove(pk, v, w, pp).to_bytes())
    b[200] ^= 1  # inside the z(r_v, 0) opening proof / sumcheck messages
    with pytest.raises(Exception):
        verify(pk, v, Proof.from_bytes(bytes(b)), vp)


def test_argument_errors():
    A, B, C, v, w = uniform_3n(3, 1, seed=1)
    pp, _, _ = keygen(3, SplitMix64(1).next_fr)
    with pytest.raises(InvalidArgument):
        index(A[:6], B[:6], C[:6])  # not a power of two (indexer.rs:49-51)
    bad = [list(r) for r in A]
    bad[0] = [(1, 99)]
    with pytest.raises(InvalidArgument):
        index(bad, B, C)  # sparse index out of bound (r1cs_reader.rs:55-63)
    pk = index(A, B, C)
    with pytest.raises(InvalidArgument):
        prove(pk, v + [1], w[:-1], pp)  # |v| not a power of two (prover.rs:114-116)
    with pytest.raises(InvalidArgument):
        prove(pk, v, w[:-1], pp)  # |v| + |w| != n (prover.rs:117-119)
