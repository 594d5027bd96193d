"""Shared-memory communicator (the on-node transport of the sharded prover, DESIGN.md multi-GPU):
host-only allgathers across real processes, run here on CPU."""
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _run_workers(spx, world, mode, extra=(), timeout=120):
    name = spx.shm_name()
    outs, procs = [], []
    for r in range(world):
        out = os.path.join("/tmp", "%s_r%d.out" % (name, r))
        outs.append(out)
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "mp_worker.py"), "--mode", mode, "--name", name,
                                       "--rank", str(r), "--world", str(world), "--out", out, *extra]))
    try:
        for p in procs:
            assert p.wait(timeout=timeout) == 0
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    return outs


@pytest.mark.parametrize("world", [2, 3])
def test_shm_allgather_processes(spx, world):
    outs = _run_workers(spx, world, "allgather")
    for o in outs:
        assert open(o).read().startswith("ok")
        os.remove(o)


def test_shm_single_rank_and_errors(spx):
    c = spx.ShmComm(spx.shm_name(), 0, 1)
    assert c.allgather(b"abc") == [b"abc"]
    c.close()
    with pytest.raises(spx.InvalidArgument):
        spx.ShmComm(spx.shm_name(), 2, 2)
    with pytest.raises(spx.InvalidArgument):
        spx.ShmComm("bad/name", 0, 1)
    assert not [f for f in os.listdir("/dev/shm") if f.startswith("spx_")]
