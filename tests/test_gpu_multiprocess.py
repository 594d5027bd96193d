"""Sharded proof across real processes on the GPU box: 2 ranks (both on GPU 0), each with 2 proofs
in flight over shared-memory communicators, exactly the bench's N > 1 structure. Every proof of
both ranks must equal the oracle's unsharded proof byte for byte."""
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
@pytest.mark.parametrize("log_n", [8, 11])
def test_sharded_processes_bit_exact(spx, oc, log_n):
    log_v = 3
    outs = _run_workers(spx, 2, "prove", ["--log-n", str(log_n), "--log-v", str(log_v), "--inflight", "2"], timeout=300)
    per_rank = [_read(o) for o in outs]
    for o in outs:
        os.remove(o)
    proofs = [p for items in per_rank for p in items[:-1]]
    assert len(proofs) == 8
    inst = oc.Instance(0, log_n, log_v, 0x5EED0000 + log_n)
    ppc = oc.PP.keygen(log_n, 77)
    assert per_rank[0][-1] == ppc.serialize()
    want = oc.prove(inst.mats, inst.v_bytes, inst.w_bytes, ppc, 0, 0)
    for p in proofs:
        assert p == want
