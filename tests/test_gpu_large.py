"""BASELINE configs C4 / C5 at their sizes on one GPU: 2^22 and 2^24 constraints (uniform-3n,
nnz = 3n), the proof sharded over 8 ranks (8 contexts with an in-process communicator on the one
GPU: the bench's N = 8 decomposition and exchanges, minus the transport) must equal the unsharded
proof byte for byte and the product's verifier must accept it.
* 2^22 (C4): the proof equals the C oracle's proof of the same instance under the same PP, byte
  for byte (the oracle on the box's cores, ~2 min at 16).
* 2^24 (C5): the oracle would take ~10 min, so the proof passes the oracle's complete transcript
  replay (every sumcheck relation, the final matrix claim from the CSR) and the commitment /
  opening checks against the keygen trapdoor instead (tests/fullsize_check.py)."""
import os
import sys
import threading

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
@pytest.mark.timeout(900)
@pytest.mark.parametrize("log_n", [22, 24])
def test_sharded_8_ranks_large(spx, ctx, oc, log_n):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import bench
    from fullsize_check import replay_and_trapdoor

    log_v, G = 5, 8
    syn, mats, zb, nnz = bench.synth_one(spx, 0, log_n, log_v, 0x5EED0000 + log_n)
    assert nnz == 3 << log_n
    v, w = zb[: 32 << log_v], zb[32 << log_v :]
    pp = spx.MLProofForR1CS.setup(ctx, log_n, 0xC0FFEE)
    pk = spx.IndexPK(ctx, bench.index_from_c(spx, ctx, mats), log_n)
    wit = spx.Witness(ctx, v, w)
    want = spx.MLArgumentForR1CS.prove_witness(pk, wit, pp)
    assert len(want) == spx.lib().spx_proof_size(log_n, log_v)
    assert spx.MLArgumentForR1CS.verify(pk, v, want, spx.verifier_parameter(pp))
    del wit

    group = spx.CommGroup(G)
    out, errs = [None] * G, []

    def rank(r):
        try:
            rctx = spx.Context(0)
            rctx.set_comm_group(group, r)
            rpk = spx.IndexPK(rctx, bench.index_from_c(spx, rctx, mats), log_n)
            rw = spx.Witness(rctx, v, w)
            out[r] = spx.MLArgumentForR1CS.prove_witness(rpk, rw, pp)
        except Exception as e:  # surfaced below
            errs.append(repr(e))

    ths = [threading.Thread(target=rank, args=(r,)) for r in range(G)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=900)
    assert not errs, errs
    for r in range(G):
        assert out[r] == want, "rank %d proof differs" % r
    if log_n == 22:
        inst = oc.Instance(0, log_n, log_v, 0x5EED0000 + log_n)
        assert inst.z_bytes == zb
        ppc = oc.PP.load(pp.serialize_uncompressed())
        oc.set_threads(bench.host_cores())
        try:
            ref = oc.prove(inst.mats, inst.v_bytes, inst.w_bytes, ppc, 0, 0)
        finally:
            oc.set_threads(1)
        assert ref == want, "GPU proof differs from the oracle's at 2^22"
    else:
        replay_and_trapdoor(oc, mats, zb, want, log_n, log_v, 0xC0FFEE)
