"""Ordered exchange hub (comm_hub.cpp): many proofs in flight per rank share ONE collective
transport, each on a channel, and the hub matches their exchanges across ranks in rounds every
rank runs alike. Host-only here (no GPU): virtual ranks as threads over the in-process group, and
real processes over the shared-memory transport, with channels reached in random orders."""
import os
import sys
import threading

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from mp_worker import hub_check  # noqa: E402
from test_shm_comm import _run_workers  # noqa: E402


@pytest.mark.parametrize("world,channels", [(2, 4), (3, 8)])
def test_hub_virtual_ranks_random_orders(spx, world, channels):
    g = spx.CommGroup(world)
    hubs = [spx.ExchangeHub.group(g, r) for r in range(world)]
    errs = [None] * world

    def rank_main(r):
        errs[r] = hub_check(spx, hubs[r], r, world, channels, 40, 11)

    ts = [threading.Thread(target=rank_main, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in ts), "hub deadlock"
    assert errs == [[]] * world
    for h in hubs:
        st = h.stats()
        assert st["served"] == channels * 40
        assert st["data_rounds"] <= st["rounds"] and st["max_batch"] >= 1
        h.close()


def test_hub_size_disagreement_fails_on_every_rank(spx):
    g = spx.CommGroup(2)
    hubs = [spx.ExchangeHub.group(g, r) for r in range(2)]
    res = [None, None]

    def rank_main(r):
        try:
            hubs[r].allgather(3, b"x" * (10 + r))
            res[r] = "no error"
        except spx.InvalidArgument as e:
            res[r] = str(e)
        # the hub keeps serving other exchanges afterwards
        assert hubs[r].allgather(3, bytes([r])) == [b"\0", b"\1"]

    ts = [threading.Thread(target=rank_main, args=(r,)) for r in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=60)
    assert all("disagree" in x for x in res), res
    with pytest.raises(spx.InvalidArgument):
        hubs[0].allgather(64, b"")
    for h in hubs:
        h.close()


def test_hub_single_rank(spx):
    g = spx.CommGroup(1)
    h = spx.ExchangeHub.group(g, 0)
    assert h.allgather(0, b"abc") == [b"abc"]
    assert h.allgather(63, b"") == [b""]
    h.close()


@pytest.mark.parametrize("world", [2, 3])
def test_hub_processes_over_shm(spx, world):
    outs = _run_workers(spx, world, "hub")
    for o in outs:
        txt = open(o).read()
        assert txt.startswith("ok"), txt
        os.remove(o)
