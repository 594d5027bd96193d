"""The product's sharded path (prover.cpp) on ONE GPU: G in-process ranks (one host
thread + context each, in-process communicator) must produce the single-rank proof byte for byte.
RCCL itself is exercised by bench.py --gpus N on a multi-GPU node."""
import threading

import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("G,kind,log_n", [(2, 0, 6), (4, 0, 8), (8, 2, 9), (2, 1, 10)])
def test_virtual_ranks_equal_single(spx, oc, G, kind, log_n):
    log_v = 3
    param = (3 | (2 << 16)) if kind == 2 else 0
    inst = oc.Instance(kind, log_n, log_v, 300 + log_n, param)
    ppb = oc.PP.keygen(log_n, 400 + log_n).serialize()
    want = oc.prove(inst.mats, inst.v_bytes, inst.w_bytes, oc.PP.load(ppb), 0, 0)
    group = spx.CommGroup(G)
    out = [None] * G
    errs = []

    def run(r):
        try:
            ctx = spx.Context(0)
            ctx.set_comm_group(group, r)
            pp = spx.PublicParameter.load(ctx, ppb)
            mats = [spx.Csr(M.n, M.row_ptr, M.col, M.val) for M in inst.mats]
            pk = spx.MLArgumentForR1CS.index(ctx, *mats)
            out[r] = spx.MLArgumentForR1CS.prove(pk, inst.v_bytes, inst.w_bytes, pp)
        except Exception as e:  # surfaced below
            errs.append(repr(e))

    ths = [threading.Thread(target=run, args=(r,)) for r in range(G)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=600)
    assert not errs, errs
    for r in range(G):
        assert out[r] == want, "rank %d proof differs" % r
