"""spx_verify (lib.rs:147-212, verifier.rs:143-512): the GPU-backed verifier accepts the prover's
proofs and rejects tampered ones with the reference's error kinds; its VerifierParameter bytes match
the oracle keygen's (setup.rs:91-101)."""
import pytest

import spartan
from gen import SplitMix64

pytestmark = pytest.mark.gpu

R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001


def _setup(spx, ctx, oc, kind, log_n, log_v, param=0, pp_seed=606):
    inst = oc.Instance(kind, log_n, log_v, 3000 + log_n, param)
    pp = spx.MLProofForR1CS.setup(ctx, log_n, pp_seed)
    mats = [spx.Csr(M.n, M.row_ptr, M.col, M.val) for M in inst.mats]
    pk = spx.MLArgumentForR1CS.index(ctx, *mats)
    return inst, pp, pk, spx.verifier_parameter(pp)


def test_vp_matches_oracle_keygen(spx, ctx):
    nv, seed = 6, 606
    pp = spx.MLProofForR1CS.setup(ctx, nv, seed)
    _pp, vp, _t = spartan.keygen(nv, SplitMix64(seed).next_fr)
    assert spx.verifier_parameter(pp) == vp.serialize_uncompressed()


@pytest.mark.parametrize("kind,log_n,log_v,param", [(0, 6, 2, 0), (0, 10, 5, 0), (1, 9, 3, 0), (2, 8, 3, 5 | (2 << 16))])
@pytest.mark.parametrize("mode", ["fs", "injected"])
def test_verify_accepts(spx, ctx, oc, kind, log_n, log_v, param, mode):
    inst, pp, pk, vp = _setup(spx, ctx, oc, kind, log_n, log_v, param)
    proof = spx.MLArgumentForR1CS.prove(pk, inst.v_bytes, inst.w_bytes, pp, mode=mode, seed=9)
    if kind == 2:  # ragged instances are unsatisfiable: the first sumcheck's subclaim must fail
        with pytest.raises((spx.WrongWitness, spx.SumCheckError)):
            spx.MLArgumentForR1CS.verify(pk, inst.v_bytes, proof, vp, mode=mode, seed=9)
        return
    assert spx.MLArgumentForR1CS.verify(pk, inst.v_bytes, proof, vp, mode=mode, seed=9)
    assert spx.MLArgumentForR1CS.verify(pk, inst.v_bytes, proof, vp, mode=mode, seed=9, cached=True)


def test_verify_rejects_tampering(spx, ctx, oc):
    log_n, log_v = 8, 3
    inst, pp, pk, vp = _setup(spx, ctx, oc, 0, log_n, log_v)
    proof = spx.MLArgumentForR1CS.prove(pk, inst.v_bytes, inst.w_bytes, pp)
    assert spx.MLArgumentForR1CS.verify(pk, inst.v_bytes, proof, vp)
    pf = spartan.Proof.from_bytes(proof)
    # a sumcheck-1 evaluation: transcript changes and round consistency fails
    bad = spartan.Proof.from_bytes(proof)
    bad.sc1[2][1] = (bad.sc1[2][1] + 1) % R
    with pytest.raises((spx.SumCheckError, spx.WrongWitness)):
        spx.MLArgumentForR1CS.verify(pk, inst.v_bytes, bad.to_bytes(), vp)
    # the claimed va: first subclaim check fails
    bad = spartan.Proof.from_bytes(proof)
    bad.pm4 = ((pf.pm4[0] + 1) % R, pf.pm4[1], pf.pm4[2])
    with pytest.raises((spx.SumCheckError, spx.WrongWitness)):
        spx.MLArgumentForR1CS.verify(pk, inst.v_bytes, bad.to_bytes(), vp)
    # z(r_y): the matrix claim fails
    bad = spartan.Proof.from_bytes(proof)
    bad.pm6 = ((pf.pm6[0] + 1) % R, pf.pm6[1])
    with pytest.raises((spx.WrongWitness, spx.SumCheckError)):
        spx.MLArgumentForR1CS.verify(pk, inst.v_bytes, bad.to_bytes(), vp)
    # one opening proof point replaced by another valid G2 point: pairing check fails
    bad = spartan.Proof.from_bytes(proof)
    z, (h, proofs) = pf.pm2
    bad.pm2 = (z, (h, [proofs[1]] + proofs[1:]))
    with pytest.raises(spx.InvalidArgument):
        spx.MLArgumentForR1CS.verify(pk, inst.v_bytes, bad.to_bytes(), vp)
    # a different public input
    v2 = bytearray(inst.v_bytes)
    v2[32] ^= 1
    with pytest.raises((spx.InvalidArgument, spx.WrongWitness, spx.SumCheckError)):
        spx.MLArgumentForR1CS.verify(pk, bytes(v2), proof, vp)
    # truncated bytes
    with pytest.raises(spx.SerializationError):
        spx.MLArgumentForR1CS.verify(pk, inst.v_bytes, proof[:-5], vp)


def test_verify_oracle_proof(spx, ctx, oc):
    """the oracle's proof (same PP) is accepted too: the verifier checks bytes, not their origin"""
    log_n, log_v = 7, 2
    inst, pp, pk, vp = _setup(spx, ctx, oc, 1, log_n, log_v)
    ppc = oc.PP.load(pp.serialize_uncompressed())
    proof = oc.prove(inst.mats, inst.v_bytes, inst.w_bytes, ppc, 0, 0)
    assert spx.MLArgumentForR1CS.verify(pk, inst.v_bytes, proof, vp)


def test_frontend_circuit_proves_and_verifies(spx, ctx):
    """a circuit stated through the R1CS front-end: x^3 + x + 5 = out (the classic example), padded
    square, proved on the GPU and accepted by the verifier; a wrong witness is rejected."""
    CS = spx.ConstraintSystem
    for x_val, ok in ((3, True), (4, False)):
        cs = CS()
        out = cs.new_input(35)  # 3^3 + 3 + 5
        x = cs.new_witness(x_val)
        x2 = cs.new_witness(x_val * x_val)
        x3 = cs.new_witness(x_val ** 3)
        cs.enforce([(1, x)], [(1, x)], [(1, x2)])
        cs.enforce([(1, x2)], [(1, x)], [(1, x3)])
        cs.enforce([(1, x3), (1, x), (5, CS.ONE)], [(1, CS.ONE)], [(1, out)])
        cs.new_input(0)  # |v| = 4 (a power of two: prover.rs:114-116)
        cs.new_input(0)
        cs.new_witness(0)  # 8 variables
        cs.make_square(8)  # 8 constraints (test_utils.rs:81-102)
        assert cs.is_satisfied() == ok
        a, b, c, v, w = cs.to_matrices()
        pk = spx.MLArgumentForR1CS.index(ctx, a, b, c)
        pp = spx.MLProofForR1CS.setup(ctx, 3, 11)
        proof = spx.MLArgumentForR1CS.prove(pk, v, w, pp)
        if ok:
            assert spx.MLArgumentForR1CS.verify(pk, v, proof, spx.verifier_parameter(pp))
        else:
            with pytest.raises((spx.WrongWitness, spx.SumCheckError)):
                spx.MLArgumentForR1CS.verify(pk, v, proof, spx.verifier_parameter(pp))
