"""BASELINE size (2^20 constraints, the bench workload: circuit-3n):

* byte equality with the C oracle's proof of the same witness under the same PP (the oracle on the
  box's cores, ~30 s at 16: BASELINE C3 pinned byte for byte, /root/reference/src/lib.rs:58-146);

* determinism across the product's execution modes: per-proof transcript, index-cached transcript,
  concurrent contexts (spx_prove_many) and 2 virtual ranks all give the same bytes;
* the verifier's complete transcript replay and every sumcheck relation (oracle/py/spartan.verify,
  verifier.rs:143-512) with the final matrix claim evaluated directly from the CSR (C oracle);
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
def test_fullsize_2_20(spx, ctx, oc):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import bench

    log_n, log_v, pp_seed = 20, 5, 0xC0FFEE
    n = 1 << log_n
    # the bench workload (circuit-3n, fixed index) with one of its witnesses
    syn, mats, zb, nnz = bench.synth_one(spx, 3, log_n, log_v, 0x5EED0000 + log_n)
    pp = spx.MLProofForR1CS.setup(ctx, log_n, pp_seed)
    pk = spx.IndexPK(ctx, bench.index_from_c(spx, ctx, mats), log_n)
    wit = spx.Witness(ctx, zb[: 32 << log_v], zb[32 << log_v :])
    proof = spx.MLArgumentForR1CS.prove_witness(pk, wit, pp)
    assert len(proof) == 21272

    # the oracle's proof of the same witness (seed 0xB0B0) under the same PP, byte for byte
    inst = oc.Instance(3, log_n, log_v, 0x5EED0000 + log_n, 0xB0B0)
    assert inst.z_bytes == zb
    ppc = oc.PP.load(pp.serialize_uncompressed())
    oc.set_threads(bench.host_cores())
    try:
        want = oc.prove(inst.mats, inst.v_bytes, inst.w_bytes, ppc, 0, 0)
    finally:
        oc.set_threads(1)
    del ppc
    assert want == proof, "GPU proof differs from the oracle's at 2^20"
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

    # verifier replay (all sumcheck relations, final claims) and the trapdoor checks
    from fullsize_check import replay_and_trapdoor

    bad = replay_and_trapdoor(oc, mats, zb, proof, log_n, log_v, pp_seed)

    # the product's verifier (GPU eval_on_x + host pairings) accepts it, and rejects the corrupted one
    vp = spx.verifier_parameter(pp)
    assert spx.MLArgumentForR1CS.verify(pk, zb[: 32 << log_v], proof, vp)
    with pytest.raises((spx.SumCheckError, spx.WrongWitness)):
        spx.MLArgumentForR1CS.verify(pk, zb[: 32 << log_v], bad, vp)
