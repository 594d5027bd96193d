"""The RCCL transport (comm_rccl.cpp; bench.py --comm rccl) on the one GPU of the test box: one
communicator per rank behind the ordered exchange hub (comm_hub.cpp), allgathers of the sizes a
sharded proof exchanges (3 Fr per sumcheck round, XYZZ bucket sums, a Blake2s state) and larger
ones, then proofs in flight on several contexts sharing it, byte-equal to the C oracle. RCCL refuses
two ranks on one device, so the multi-rank hub runs here over the in-process group (2 virtual ranks,
2 proofs in flight each: the sharded code path through the same hub interface) and across processes
over shared memory (tests/test_gpu_multiprocess.py); the driver's 8-GPU node runs the real thing."""
import threading

import pytest

pytestmark = pytest.mark.gpu


def _instance(spx, oc, c, log_n=10, log_v=3):
    inst = oc.Instance(3, log_n, log_v, 0x5EED0000 + log_n, 0xB0B0)
    ppc = oc.PP.keygen(log_n, 5150)
    pp = spx.PublicParameter.load(c, ppc.serialize())
    want = oc.prove(inst.mats, inst.v_bytes, inst.w_bytes, ppc, 0, 0)
    return inst, pp, want


def test_rccl_world1_allgather_and_prove(spx, oc):
    c = spx.Context(0)
    c.set_comm_rccl(spx.comm_unique_id(), 0, 1)
    for size in (1, 96, 192, 4096, 200000):
        data = bytes((i * 37 + size) & 0xFF for i in range(size))
        assert c.comm_allgather(data, 1) == [data]
    inst, pp, want = _instance(spx, oc, c)
    pk = spx.MLArgumentForR1CS.index(c, *[spx.Csr(M.n, M.row_ptr, M.col, M.val) for M in inst.mats])
    assert spx.MLArgumentForR1CS.prove(pk, inst.v_bytes, inst.w_bytes, pp) == want


def test_rccl_hub_proofs_in_flight(spx, oc):
    hub = spx.ExchangeHub.rccl(spx.comm_unique_id(), 0, 1, 0)
    ctxs = [spx.Context(0) for _ in range(4)]
    for j, c in enumerate(ctxs):
        c.set_comm_hub(hub, j)
    with pytest.raises(spx.InvalidArgument):
        spx.Context(0).set_comm_hub(hub, 0)  # channel taken
    inst, pp, want = _instance(spx, oc, ctxs[0])
    pk = spx.MLArgumentForR1CS.index(ctxs[0], *[spx.Csr(M.n, M.row_ptr, M.col, M.val) for M in inst.mats])
    wit = spx.Witness(ctxs[0], inst.v_bytes, inst.w_bytes)
    proofs = spx.MLArgumentForR1CS.prove_many(ctxs, pk, [wit] * 8, pp)
    assert proofs == [want] * 8
    # a one-rank prove skips its exchanges; each context's channel still reaches RCCL through the hub
    for j, c in enumerate(ctxs):
        assert c.comm_allgather(bytes([j]) * 96, 1) == [bytes([j]) * 96]
    st = hub.stats()
    assert st["served"] == 4 and st["rounds"] >= st["data_rounds"] >= 1
    hub.close()


def test_group_hub_two_virtual_ranks_in_flight(spx, oc):
    world, inflight = 2, 2
    g = spx.CommGroup(world)
    hubs = [spx.ExchangeHub.group(g, r) for r in range(world)]
    ctxs = [[spx.Context(0) for _ in range(inflight)] for _ in range(world)]
    for r in range(world):
        for j, c in enumerate(ctxs[r]):
            c.set_comm_hub(hubs[r], j)
    inst, pp, want = _instance(spx, oc, ctxs[0][0])
    mats = [spx.Csr(M.n, M.row_ptr, M.col, M.val) for M in inst.mats]
    pks = [spx.MLArgumentForR1CS.index(ctxs[r][0], *mats) for r in range(world)]
    wits = [spx.Witness(ctxs[r][0], inst.v_bytes, inst.w_bytes) for r in range(world)]
    out = [None] * world

    def rank_main(r):
        out[r] = spx.MLArgumentForR1CS.prove_many(ctxs[r], pks[r], [wits[r]] * 4, pp)

    ts = [threading.Thread(target=rank_main, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=240)
    assert not any(t.is_alive() for t in ts)
    assert out == [[want] * 4] * world
    for h in hubs:
        assert h.stats()["served"] > 0
        h.close()
