"""The RCCL transport (comm_rccl.cpp; bench.py --comm rccl) on the one GPU of the test box: a
one-rank communicator through ncclCommInitRank, allgathers of the sizes a sharded proof exchanges
(3 Fr per sumcheck round, one affine point per MSM, a Blake2s state) and larger ones, then a full
proof on a context that carries it, byte-equal to the C oracle. RCCL refuses two ranks on one
device, so the multi-rank exchange itself is covered by the shared-memory transport's
multi-process tests (tests/test_gpu_multiprocess.py) and by the driver's 8-GPU runs."""
import pytest

pytestmark = pytest.mark.gpu


def test_rccl_world1_allgather_and_prove(spx, oc):
    c = spx.Context(0)
    c.set_comm_rccl(spx.comm_unique_id(), 0, 1)
    for size in (1, 96, 192, 4096, 200000):
        data = bytes((i * 37 + size) & 0xFF for i in range(size))
        assert c.comm_allgather(data, 1) == [data]
    log_n, log_v = 10, 3
    inst = oc.Instance(3, log_n, log_v, 0x5EED0000 + log_n, 0xB0B0)
    ppc = oc.PP.keygen(log_n, 5150)
    pp = spx.PublicParameter.load(c, ppc.serialize())
    pk = spx.MLArgumentForR1CS.index(c, *[spx.Csr(M.n, M.row_ptr, M.col, M.val) for M in inst.mats])
    got = spx.MLArgumentForR1CS.prove(pk, inst.v_bytes, inst.w_bytes, pp)
    assert got == oc.prove(inst.mats, inst.v_bytes, inst.w_bytes, ppc, 0, 0)
