"""Sharded proof across real processes on the GPU box: 2 ranks (both on GPU 0), each with 2 proofs
in flight over shared-memory communicators, exactly the bench's N > 1 structure. Every proof of
both ranks must equal the oracle's unsharded proof byte for byte. The hub case shares one transport
per rank among 4 proofs in flight."""
import os

import pytest

from test_shm_comm import _run_workers


def _read(path):
    b = open(path, "rb").read()
    items, i = [], 0
    while i < len(b):
        n = int.from_bytes(b[i : i + 4], "little")
        items.append(b[i + 4 : i + 4 + n])
        i += 4 + n
    return items


@pytest.mark.gpu
@pytest.mark.parametrize("log_n,mode,inflight", [(8, "prove", 2), (11, "prove", 2), (10, "prove_hub", 4)])
def test_sharded_processes_bit_exact(spx, oc, log_n, mode, inflight):
    """mode prove_hub: all proofs in flight of a rank share ONE transport through the ordered exchange
    hub (comm_hub.cpp, the structure of bench.py --comm rccl), here over shared memory"""
    log_v = 3
    outs = _run_workers(spx, 2, mode, ["--log-n", str(log_n), "--log-v", str(log_v), "--inflight", str(inflight)],
                        timeout=300)
    per_rank = [_read(o) for o in outs]
    for o in outs:
        os.remove(o)
    proofs = [p for items in per_rank for p in items[:-1]]
    assert len(proofs) == 2 * 2 * inflight
    inst = oc.Instance(0, log_n, log_v, 0x5EED0000 + log_n)
    ppc = oc.PP.keygen(log_n, 77)
    assert per_rank[0][-1] == ppc.serialize()
    want = oc.prove(inst.mats, inst.v_bytes, inst.w_bytes, ppc, 0, 0)
    for p in proofs:
        assert p == want


@pytest.mark.gpu
def test_sharded_processes_refuse_mismatched_lvl0_mode(spx):
    """SPX_LVL0 shapes a proof's exchanges: ranks that read different values must both fail with
    InvalidArgument on their first sharded proof instead of exchanging mismatched messages"""
    outs = _run_workers(spx, 2, "lvl0_mismatch", ["--log-n", "8", "--log-v", "3"], timeout=300)
    res = [open(o).read() for o in outs]
    for o in outs:
        os.remove(o)
    for r in res:
        assert r.startswith("invalid") and "SPX_LVL0" in r, res
