"""The product's ordered exchange hub (comm_hub.cpp) over a torch.distributed process group
(spx_comm_hub_create_callback): world 2 over gloo on the CPU, real processes. Each rank drives 6
channels from threads that reach their exchanges in random orders (the structure of many proofs in
flight per rank sharing one collective), and every exchange returns every rank's payload in rank order.
The same hub runs over RCCL as torch.distributed backend "nccl" on a multi-GPU node."""
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))

WORKER = r"""
import os, sys
sys.path.insert(0, {here!r})
import torch.distributed as dist
from conftest import load_product
from mp_worker import hub_check
spx = load_product()
dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%s" % os.environ["PORT"],
                        rank=int(os.environ["RANK"]), world_size=2)
hub = spx.ExchangeHub.torch_group()
errs = hub_check(spx, hub, dist.get_rank(), 2, 6, 25, 17)
st = hub.stats()
hub.close()
dist.destroy_process_group()
print("served", st["served"], "errs", errs)
sys.exit(1 if errs or st["served"] != 6 * 25 else 0)
"""


def _free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_hub_over_torch_gloo_world2(spx):
    port = str(_free_port())
    code = WORKER.format(here=HERE)
    procs = [subprocess.Popen([sys.executable, "-c", code], env=dict(os.environ, RANK=str(r), PORT=port),
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(2)]
    outs = []
    try:
        for p in procs:
            o, e = p.communicate(timeout=240)
            outs.append((p.returncode, o, e[-2000:]))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for rc, o, e in outs:
        assert rc == 0, (o, e)
        assert "served 150" in o
