"""The full-size verifier replay used by the 2^20 GPU test (tests/test_gpu_fullsize.py) against the
reference-faithful verifier: numpy matrix serialization == matrix_bytes, direct sparse
evaluation == eval_on_x + mle_eval, and the hooked verifier accepts/rejects exactly like the
default one (pairing checks included there)."""
import random

import pytest

import csr_fast
import spartan
from bls12_381 import R


def _rows(M):
    rp = list(M.row_ptr)
    return [[(int.from_bytes(M.val.raw[32 * k : 32 * k + 32], "little"), M.col[k]) for k in range(rp[x], rp[x + 1])]
            for x in range(M.n)]


@pytest.mark.parametrize("kind,log_n,param", [(0, 6, 0), (1, 7, 0), (2, 6, 4 | (1 << 16))])
def test_matrix_bytes_and_sparse_eval(oc, kind, log_n, param):
    inst = oc.Instance(kind, log_n, 3, 9000 + log_n, param)
    rs = random.Random(5)
    rx = [rs.randrange(R) for _ in range(log_n)]
    ry = [rs.randrange(R) for _ in range(log_n)]
    ex, ey = csr_fast.eq_table(rx), csr_fast.eq_table(ry)
    for M in inst.mats:
        rows = _rows(M)
        fast = csr_fast.matrix_bytes_csr(M.n, list(M.row_ptr), list(M.col)[: M.nnz], M.val.raw[: 32 * M.nnz])
        assert fast == spartan.matrix_bytes(rows, M.n)
        want = spartan.mle_eval(spartan.eval_on_x(rows, rx), ry)
        got = csr_fast.sparse_eval(M.n, list(M.row_ptr), list(M.col), M.val.raw, ex, ey)
        assert got == want


def test_hooked_verifier_matches_default(oc):
    log_n, log_v = 5, 2
    inst = oc.Instance(0, log_n, log_v, 4321)
    ppc = oc.PP.keygen(log_n, 99)
    proof_bytes = oc.prove(inst.mats, inst.v_bytes, inst.w_bytes, ppc, 0, 0)
    rows = [_rows(M) for M in inst.mats]
    vk = spartan.index(*rows)
    v = [int.from_bytes(inst.v_bytes[32 * i : 32 * i + 32], "little") for i in range(1 << log_v)]
    vp = None  # pairing checks are off in the hooked form (the default form is tested in test_oracle_invariants)

    def feed(fs):
        for M in inst.mats:
            fs.feed(csr_fast.matrix_bytes_csr(M.n, list(M.row_ptr), list(M.col)[: M.nnz], M.val.raw[: 32 * M.nnz]))

    def eval_rr(rx, ry):
        ex, ey = csr_fast.eq_table(rx), csr_fast.eq_table(ry)
        return tuple(csr_fast.sparse_eval(M.n, list(M.row_ptr), list(M.col), M.val.raw, ex, ey) for M in inst.mats)

    proof = spartan.Proof.from_bytes(proof_bytes)
    assert spartan.verify(vk, v, proof, vp, feed_matrices=feed, eval_rr=eval_rr, check_pairings=False)
    # a tampered sumcheck message is rejected by the hooked verifier too
    bad = spartan.Proof.from_bytes(proof_bytes)
    bad.sc2[1][0] = (bad.sc2[1][0] + 1) % R
    with pytest.raises((spartan.WrongWitness, spartan.InvalidArgument, spartan.SumCheckError)):
        spartan.verify(vk, v, bad, vp, feed_matrices=feed, eval_rr=eval_rr, check_pairings=False)
