"""The product's sharded path (prover.cpp) on ONE GPU: G in-process ranks (one host
thread + context each, in-process communicator) must produce the single-rank proof byte for byte.
The MSMs split every instance by bucket range (MsmShard, kernels.hpp); the cases below also drive
their compacted-key overflow and the dense rerun. RCCL itself is exercised by bench.py --gpus N on
a multi-GPU node."""
import os
import threading

import pytest

pytestmark = pytest.mark.gpu


def _prove_ranks(spx, G, inst, ppb, w_bytes=None, lvl0=None):
    group = spx.CommGroup(G)
    out = [None] * G
    reruns = [0] * G
    errs = []
    w = inst.w_bytes if w_bytes is None else w_bytes

    def run(r):
        try:
            ctx = spx.Context(0)
            ctx.set_comm_group(group, r)
            if lvl0 is not None:
                ctx.set_lvl0_batch(lvl0[r])
            pp = spx.PublicParameter.load(ctx, ppb)
            mats = [spx.Csr(M.n, M.row_ptr, M.col, M.val) for M in inst.mats]
            pk = spx.MLArgumentForR1CS.index(ctx, *mats)
            out[r] = spx.MLArgumentForR1CS.prove(pk, inst.v_bytes, w, pp)
            reruns[r] = ctx.msm_reruns()
        except Exception as e:  # surfaced below
            errs.append(repr(e))

    ths = [threading.Thread(target=run, args=(r,)) for r in range(G)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=600)
    assert not errs, errs
    return out, sum(reruns)


@pytest.mark.parametrize("G,kind,log_n", [(2, 0, 6), (4, 0, 8), (8, 2, 9), (2, 1, 10), (8, 0, 12)])
def test_virtual_ranks_equal_single(spx, oc, G, kind, log_n):
    log_v = 3
    param = (3 | (2 << 16)) if kind == 2 else 0
    inst = oc.Instance(kind, log_n, log_v, 300 + log_n, param)
    ppb = oc.PP.keygen(log_n, 400 + log_n).serialize()
    want = oc.prove(inst.mats, inst.v_bytes, inst.w_bytes, oc.PP.load(ppb), 0, 0)
    out, reruns = _prove_ranks(spx, G, inst, ppb)
    for r in range(G):
        assert out[r] == want, "rank %d proof differs" % r
    assert reruns == 0, "uniform scalars overflowed the planned key capacity"


def test_virtual_ranks_forced_key_overflow(spx, oc):
    """SPX_MSM_CAP_SCALE=0.5 halves the compacted-key capacity: the first batches of every rank
    overflow, are rerun with one key slot per digit, and the proof stays byte-identical."""
    log_n, log_v, G = 10, 3, 4
    inst = oc.Instance(0, log_n, log_v, 900 + log_n, 0)
    ppb = oc.PP.keygen(log_n, 901).serialize()
    want = oc.prove(inst.mats, inst.v_bytes, inst.w_bytes, oc.PP.load(ppb), 0, 0)
    os.environ["SPX_MSM_CAP_SCALE"] = "0.5"
    try:
        out, reruns = _prove_ranks(spx, G, inst, ppb)
    finally:
        del os.environ["SPX_MSM_CAP_SCALE"]
    assert all(p == want for p in out)
    assert reruns > 0, "the halved capacity did not overflow"


# every 7-bit window digit of this scalar is 1: at 2^9 (commitment window c = 7) all of a
# commitment's digits land in bucket 0, i.e. on rank 0
_ONES7 = sum(1 << (7 * w) for w in range(37))


@pytest.mark.parametrize("fill", [_ONES7, 1, 0])
def test_virtual_ranks_crowded_buckets(spx, oc, fill):
    """a witness of equal values: every commitment digit of a window lands in one bucket (for
    _ONES7 all of them on rank 0: its compacted keys overflow and the batch is rerun dense), every
    opening quotient is 0. The proof is not a valid one (the witness does not satisfy the matrices);
    it must still equal the oracle's byte for byte."""
    log_n, log_v, G = 9, 3, 4
    inst = oc.Instance(0, log_n, log_v, 950 + log_n, 0)
    ppb = oc.PP.keygen(log_n, 951).serialize()
    w = fill.to_bytes(32, "little") * ((1 << log_n) - (1 << log_v))
    want = oc.prove(inst.mats, inst.v_bytes, w, oc.PP.load(ppb), 0, 0)
    out, reruns = _prove_ranks(spx, G, inst, ppb, w)
    assert all(p == want for p in out)
    if fill == _ONES7:
        assert reruns > 0, "crowded scalars did not overflow rank 0's keys"


def test_rehearsal_rank_runs(spx, oc):
    """spx_ctx_set_comm_rehearsal: one rank of a G-rank proof-sharded prove without peers (bench.py's node
    rehearsal). Its proofs are not valid; it must run the rank's whole path (compacted keys of its
    buckets included) and return a proof of the right size, and G = 1 must give the real proof."""
    log_n, log_v = 10, 3
    inst = oc.Instance(0, log_n, log_v, 970 + log_n, 0)
    ppb = oc.PP.keygen(log_n, 971).serialize()
    want = oc.prove(inst.mats, inst.v_bytes, inst.w_bytes, oc.PP.load(ppb), 0, 0)
    for G in (1, 4):
        ctx = spx.Context(0)
        ctx.set_comm_rehearsal(0, G)
        pp = spx.PublicParameter.load(ctx, ppb)
        mats = [spx.Csr(M.n, M.row_ptr, M.col, M.val) for M in inst.mats]
        pk = spx.MLArgumentForR1CS.index(ctx, *mats)
        got = spx.MLArgumentForR1CS.prove(pk, inst.v_bytes, inst.w_bytes, pp)
        assert len(got) == len(want)
        assert (got == want) == (G == 1)
        assert ctx.msm_reruns() == 0


def test_virtual_ranks_level0_in_first_batch(spx, oc):
    """spx_ctx_set_lvl0_batch(1) on every rank: the shared level-0 opening MSM inside the first
    opening's batch (bench.py's setting at G >= 4) gives the same bytes"""
    log_n, log_v, G = 10, 3, 4
    inst = oc.Instance(0, log_n, log_v, 980 + log_n, 0)
    ppb = oc.PP.keygen(log_n, 981).serialize()
    want = oc.prove(inst.mats, inst.v_bytes, inst.w_bytes, oc.PP.load(ppb), 0, 0)
    out, reruns = _prove_ranks(spx, G, inst, ppb, lvl0=[1] * G)
    assert all(p == want for p in out)


def test_virtual_ranks_level0_mode_mismatch(spx, oc):
    """ranks that disagree on the level-0 mode fail on their first sharded proof (no mismatched exchanges)"""
    log_n, log_v, G = 8, 3, 2
    inst = oc.Instance(0, log_n, log_v, 990 + log_n, 0)
    ppb = oc.PP.keygen(log_n, 991).serialize()
    with pytest.raises(AssertionError) as e:
        _prove_ranks(spx, G, inst, ppb, lvl0=[1, 0])
    assert "level-0 mode differs" in str(e.value)


@pytest.mark.parametrize("G", [1, 2, 4])
def test_derived_round_values_match_device(spx, oc, G):
    """From round 2 on a sumcheck round's value at 1 is derived on the host from the previous claim
    (prover.cpp). SPX_CHECK_DERIVED=1 makes the device compute it as well and fails the prove
    (SPX_SUMCHECK) on any difference: the identity is checked round by round, unsharded and over
    G virtual ranks, and the proof stays equal to the oracle's."""
    import threading

    log_n, log_v = 10, 3
    inst = oc.Instance(0, log_n, log_v, 808)
    ppc = oc.PP.keygen(log_n, 809)
    want = oc.prove(inst.mats, inst.v_bytes, inst.w_bytes, ppc, 0, 0)
    os.environ["SPX_CHECK_DERIVED"] = "1"
    try:
        group = spx.CommGroup(G) if G > 1 else None
        out, errs = [None] * G, []

        def rank(r):
            try:
                c = spx.Context(0)
                if group is not None:
                    c.set_comm_group(group, r)
                pp = spx.PublicParameter.load(c, ppc.serialize())
                pk = spx.MLArgumentForR1CS.index(c, *[spx.Csr(M.n, M.row_ptr, M.col, M.val) for M in inst.mats])
                out[r] = spx.MLArgumentForR1CS.prove(pk, inst.v_bytes, inst.w_bytes, pp)
            except Exception as e:
                errs.append(repr(e))

        ths = [threading.Thread(target=rank, args=(r,)) for r in range(G)]
        for t in ths:
            t.start()
        for t in ths:
            t.join(timeout=300)
    finally:
        del os.environ["SPX_CHECK_DERIVED"]
    assert not errs, errs
    assert all(o == want for o in out)
