"""MSM batches of two proofs merged into one (spx_ctx_set_msm_pairing, prover.cpp msm_batch): with
several contexts in flight, a context that reaches a batch identical to one another context is
waiting with runs both as one; every proof must still equal the oracle's byte for byte, unsharded and
on the ranks of proof-sharded proofs (each rank's contexts pair among themselves), and a merged batch
whose compacted keys overflow makes both proofs rerun theirs dense."""
import os
import threading

import pytest

pytestmark = pytest.mark.gpu
WAIT_US = 200000  # long enough that the contexts in flight find each other in a test


def _setup(spx, oc, log_n, seed):
    inst = oc.Instance(0, log_n, 3, seed, 0)
    ppb = oc.PP.keygen(log_n, seed + 1).serialize()
    want = oc.prove(inst.mats, inst.v_bytes, inst.w_bytes, oc.PP.load(ppb), 0, 0)
    return inst, ppb, want


def test_pairing_unsharded_bit_exact(spx, oc):
    inst, ppb, want = _setup(spx, oc, 11, 7001)
    ctxs = [spx.Context(0) for _ in range(4)]
    for c in ctxs:
        c.set_msm_pairing(WAIT_US)
    pp = spx.PublicParameter.load(ctxs[0], ppb)
    pk = spx.MLArgumentForR1CS.index(ctxs[0], *[spx.Csr(M.n, M.row_ptr, M.col, M.val) for M in inst.mats])
    wit = spx.Witness(ctxs[0], inst.v_bytes, inst.w_bytes)
    got = spx.MLArgumentForR1CS.prove_many(ctxs, pk, [wit] * 8, pp)
    assert all(g == want for g in got)
    merged = sum(c.msm_pairing_stats()[0] for c in ctxs)
    assert merged > 0, "no MSM batch was merged"


def _prove_sharded(spx, inst, ppb, G, B, nproofs, cap_scale=None):
    groups = [spx.CommGroup(G) for _ in range(B)]
    out, errs, merged = [None] * G, [], [0] * G
    if cap_scale:
        os.environ["SPX_MSM_CAP_SCALE"] = cap_scale

    def rank(r):
        try:
            cs = [spx.Context(0) for _ in range(B)]
            for k, c in enumerate(cs):
                c.set_comm_group(groups[k], r)
                c.set_msm_pairing(WAIT_US)
            pp = spx.PublicParameter.load(cs[0], ppb)
            pk = spx.MLArgumentForR1CS.index(cs[0], *[spx.Csr(M.n, M.row_ptr, M.col, M.val) for M in inst.mats])
            w = spx.Witness(cs[0], inst.v_bytes, inst.w_bytes)
            out[r] = spx.MLArgumentForR1CS.prove_many(cs, pk, [w] * nproofs, pp)
            merged[r] = sum(c.msm_pairing_stats()[0] for c in cs)
        except Exception as e:  # surfaced below
            errs.append(repr(e))

    try:
        ts = [threading.Thread(target=rank, args=(r,)) for r in range(G)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=600)
    finally:
        if cap_scale:
            del os.environ["SPX_MSM_CAP_SCALE"]
    assert not errs, errs
    return out, merged


@pytest.mark.parametrize("G", [2, 8])
def test_pairing_sharded_bit_exact(spx, oc, G):
    inst, ppb, want = _setup(spx, oc, 12, 7100 + G)
    out, merged = _prove_sharded(spx, inst, ppb, G, 2, 4)
    for r in range(G):
        assert all(p == want for p in out[r]), "rank %d" % r
    assert sum(merged) > 0


def test_pairing_overflow_reruns_both(spx, oc):
    inst, ppb, want = _setup(spx, oc, 10, 7200)
    out, _ = _prove_sharded(spx, inst, ppb, 4, 2, 4, cap_scale="0.5")
    for r in range(4):
        assert all(p == want for p in out[r]), "rank %d" % r
