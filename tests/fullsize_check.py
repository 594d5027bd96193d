"""Size-independent checks of a full-size GPU proof (test infrastructure; used at 2^20 and by the
sharded 2^22 / 2^24 tests, where the CPU oracle cannot prove in test time):

* the verifier's complete transcript replay and every sumcheck relation (oracle/py/spartan.verify,
  verifier.rs:143-512), with the final matrix claim (A, B, C)(r_x, r_y) evaluated by the C oracle
  directly from the CSR (orc_matrix_eval, eval_on_x's last-entry semantics);
* the commitment and every opening proof against the keygen trapdoor (commit.rs:53-66,
  verify.rs:60-95: C = g^{z(t)}, pi_i = h^{q_i(t_{i+1..})}, eval = z(point)): the pairing equation
  without the pairings, computed by the C oracle (orc_mle_eval, orc_open_trapdoor)."""
import ctypes

import numpy as np


def replay_and_trapdoor(oc, mats, zb, proof, log_n, log_v, pp_seed):
    import csr_fast
    import spartan
    from bls12_381 import G1, G2, R
    from gen import SplitMix64

    n = 1 << log_n
    # ctypes CSR views (the product's spx_csr or the oracle's CsrMatrix)
    mats = [m.csr() if hasattr(m, "csr") else m for m in mats]
    csr = []
    for m in mats:
        rp = np.ctypeslib.as_array(m.row_ptr, (n + 1,)).copy()
        k = int(rp[-1])
        col = np.ctypeslib.as_array(m.col, (max(k, 1),))[:k].copy()
        csr.append((rp, col, ctypes.string_at(m.val, 32 * k)))
    views = [oc.Csr(m.n, m.row_ptr, m.col, ctypes.cast(m.val, ctypes.POINTER(ctypes.c_uint8))) for m in mats]

    def feed(fs):
        for rp, col, val in csr:
            fs.feed(csr_fast.matrix_bytes_csr(n, rp, col, val))

    def eval_rr(rx, ry):
        return tuple(oc.matrix_eval(v, rx, ry) for v in views)

    v = [int.from_bytes(zb[32 * i : 32 * i + 32], "little") for i in range(1 << log_v)]
    pf = spartan.Proof.from_bytes(proof)
    pts = {}
    assert spartan.verify({"log_n": log_n, "n": n}, v, pf, None, feed_matrices=feed, eval_rr=eval_rr,
                          check_pairings=False, out=pts)
    # a corrupted sumcheck message must be rejected by the same replay
    bad = spartan.Proof.from_bytes(proof)
    bad.sc1[3][2] = (bad.sc1[3][2] + 1) % R
    rejected = False
    try:
        spartan.verify({"log_n": log_n, "n": n}, v, bad, None, feed_matrices=feed, eval_rr=eval_rr,
                       check_pairings=False)
    except (spartan.WrongWitness, spartan.InvalidArgument, spartan.SumCheckError):
        rejected = True
    assert rejected, "corrupted proof accepted by the replay"

    # commitment and openings against the trapdoor (draw order g, h, t: setup.rs:28-34)
    rng = SplitMix64(pp_seed)
    gs, hs = rng.next_fr(), rng.next_fr()
    t = [rng.next_fr() for _ in range(log_n)]
    assert pf.pm1[1] == G1.mul_affine(G1.gen, gs * oc.mle_eval(zb, log_n, t) % R), "commitment"
    for (ev, (h, proofs)), point in ((pf.pm2, pts["r_v0"]), (pf.pm6, pts["r_y"])):
        assert h == G2.mul_affine(G2.gen, hs)
        qv, want_ev = oc.open_trapdoor(zb, log_n, point, t)
        assert ev == want_ev, "opening evaluation"
        for i in range(log_n):
            assert proofs[i] == G2.mul_affine(G2.gen, hs * qv[i] % R), "opening proof %d" % i
    return bad.to_bytes()
