"""BASELINE size (2^20 constraints, the bench workload) through size-independent properties — the
CPU oracle cannot prove at this size in test time, so the GPU proof is checked instead of compared:

* determinism across the product's execution modes: per-proof transcript, index-cached transcript,
  concurrent contexts (spx_prove_many) and 2 virtual ranks all give the same bytes;
* the verifier's complete transcript replay and every sumcheck relation (oracle/py/spartan.verify,
  verifier.rs:143-512) with the final matrix claim evaluated directly from the CSR;
* the commitment and all 2 x 20 opening proofs against the keygen trapdoor (commit.rs:53-66,
  verify.rs:60-95: C = g^{z(t)}, pi_i = h^{q_i(t_{i+1..})}, eval = z(point)) — the pairing equation
  without the pairings."""
import ctypes
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_fullsize_2_20(spx, ctx):
    sys.path.insert(0, ROOT)
    import bench
    import csr_fast
    import spartan
    from bls12_381 import G1, G2, R
    from gen import SplitMix64

    log_n, log_v, pp_seed = 20, 5, 0xC0FFEE
    n = 1 << log_n
    syn, mats, zb, nnz = bench.synth_instance(spx, 0, log_n, log_v, 0x5EED0000 + log_n)
    pp = spx.MLProofForR1CS.setup(ctx, log_n, pp_seed)
    pk = spx.IndexPK(ctx, bench.index_from_c(spx, ctx, mats), log_n)
    wit = spx.Witness(ctx, zb[: 32 << log_v], zb[32 << log_v :])
    proof = spx.MLArgumentForR1CS.prove_witness(pk, wit, pp)
    assert len(proof) == 21272
    assert spx.MLArgumentForR1CS.prove_witness(pk, wit, pp, cached=True) == proof
    ctx2 = spx.Context(0)
    assert all(p == proof for p in spx.MLArgumentForR1CS.prove_many([ctx, ctx2], pk, [wit] * 3, pp))

    # the same proof from 2 virtual ranks (sharded decomposition, in-process communicator)
    group = spx.CommGroup(2)
    rctx = [spx.Context(0) for _ in range(2)]
    for r, c in enumerate(rctx):
        c.set_comm_group(group, r)
    import threading

    res = [None, None]

    def rank(r):
        rpk = spx.IndexPK(rctx[r], bench.index_from_c(spx, rctx[r], mats), log_n)
        rw = spx.Witness(rctx[r], zb[: 32 << log_v], zb[32 << log_v :])
        res[r] = spx.MLArgumentForR1CS.prove_witness(rpk, rw, pp_r[r])

    pp_r = [spx.MLProofForR1CS.setup(c, log_n, pp_seed) for c in rctx]
    th = [threading.Thread(target=rank, args=(r,)) for r in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert res[0] == proof and res[1] == proof

    # verifier replay (all sumcheck relations, final claims)
    csr = []
    for m in mats:
        rp = np.ctypeslib.as_array(m.row_ptr, (n + 1,)).copy()
        k = int(rp[-1])
        col = np.ctypeslib.as_array(m.col, (max(k, 1),))[:k].copy()
        csr.append((rp, col, ctypes.string_at(m.val, 32 * k)))

    def feed(fs):
        for rp, col, val in csr:
            fs.feed(csr_fast.matrix_bytes_csr(n, rp, col, val))

    def eval_rr(rx, ry):
        ex, ey = csr_fast.eq_table(rx), csr_fast.eq_table(ry)
        return tuple(csr_fast.sparse_eval(n, rp.tolist(), col.tolist(), val, ex, ey) for rp, col, val in csr)

    z = [int.from_bytes(zb[32 * i : 32 * i + 32], "little") for i in range(n)]
    pf = spartan.Proof.from_bytes(proof)
    pts = {}
    assert spartan.verify({"log_n": log_n, "n": n}, z[: 1 << log_v], pf, None, feed_matrices=feed, eval_rr=eval_rr,
                          check_pairings=False, out=pts)
    # a corrupted sumcheck message must be rejected by the same replay
    bad = spartan.Proof.from_bytes(proof)
    bad.sc1[3][2] = (bad.sc1[3][2] + 1) % R
    with pytest.raises((spartan.WrongWitness, spartan.InvalidArgument, spartan.SumCheckError)):
        spartan.verify({"log_n": log_n, "n": n}, z[: 1 << log_v], bad, None, feed_matrices=feed, eval_rr=eval_rr,
                       check_pairings=False)

    # the product's verifier (GPU eval_on_x + host pairings) accepts it, and rejects the corrupted one
    vp = spx.verifier_parameter(pp)
    assert spx.MLArgumentForR1CS.verify(pk, zb[: 32 << log_v], proof, vp)
    with pytest.raises((spx.SumCheckError, spx.WrongWitness)):
        spx.MLArgumentForR1CS.verify(pk, zb[: 32 << log_v], bad.to_bytes(), vp)

    # commitment and openings against the trapdoor (draw order g, h, t: setup.rs:28-34)
    rng = SplitMix64(pp_seed)
    gs, hs = rng.next_fr(), rng.next_fr()
    t = [rng.next_fr() for _ in range(log_n)]
    assert pf.pm1[1] == G1.mul_affine(G1.gen, gs * spartan.mle_eval(z, t) % R)
    for (ev, (h, proofs)), point in ((pf.pm2, pts["r_v0"]), (pf.pm6, pts["r_y"])):
        assert h == G2.mul_affine(G2.gen, hs)
        r = z
        for i, p in enumerate(point):
            q = [(r[2 * b + 1] - r[2 * b]) % R for b in range(len(r) // 2)]
            r = spartan.fix_first(r, p)
            qv = spartan.mle_eval(q, t[i + 1 :])
            assert proofs[i] == G2.mul_affine(G2.gen, hs * qv % R), "opening proof %d" % i
        assert ev == r[0]
