"""The sharded (multi-GPU) decomposition of the prove (product: prover.cpp) equals
the unsharded prover byte for byte: in-process ranks, and world_size-2 torch.distributed gloo."""
import os

import pytest

from gen import SplitMix64, ragged, uniform_3n
from sharded import prove_all_ranks_inprocess, prove_sharded
from spartan import index, keygen, prove


@pytest.mark.parametrize("G", [2, 4])
def test_sharded_inprocess_equals_unsharded(G):
    A, B, C, v, w = uniform_3n(4, 2, seed=8)
    pp, _, _ = keygen(4, SplitMix64(2).next_fr)
    pk = index(A, B, C)
    want = prove(pk, v, w, pp).to_bytes()
    got = prove_all_ranks_inprocess(pk, v, w, pp, G)
    assert all(g == want for g in got)


def _gloo_worker(rank, world, port, q):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def allgather(obj):
        out = [None] * world
        dist.all_gather_object(out, obj)
        return out

    A, B, C, v, w = ragged(4, 2, 3, 11, dense_rows=1)
    pp, _, _ = keygen(4, SplitMix64(3).next_fr)
    pk = index(A, B, C)
    got = prove_sharded(pk, v, w, pp, world, rank, allgather).to_bytes()
    q.put((rank, got))
    dist.destroy_process_group()


def test_sharded_gloo_world2():
    import multiprocessing as mp
    import random

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + random.randrange(2000)
    ps = [ctx.Process(target=_gloo_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=300) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    A, B, C, v, w = ragged(4, 2, 3, 11, dense_rows=1)
    pp, _, _ = keygen(4, SplitMix64(3).next_fr)
    want = prove(index(A, B, C), v, w, pp).to_bytes()
    assert res[0] == want and res[1] == want
