"""The N > 1 path end to end through the product, as the driver runs it: `bench.py --gpus 2` starts its
own two rank processes (no external launcher), both on GPU 0 here (SPX_BENCH_SAME_GPU=1), which prove
every proof sharded over the two ranks through the shared-memory transport, and also in batch mode.
bench.py itself asserts that the proofs of the two modes are equal witness by witness and that
distinct witnesses give distinct proofs; this test checks the line the launcher re-prints."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_gpus_2_same_gpu():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["SPX_BENCH_SAME_GPU"] = "1"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--log-n", "12", "--steps", "1",
           "--warmup", "1", "--no-cpu", "--no-c2", "--no-stats", "--rehearse=", "--groups=", "--inflight", "4",
           "--proofs-per-step", "8"]
    r = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["ranks_seen"] == [2, 2]
    assert d["value"] > 0 and d["value_batch_weak"] > 0
    assert d["config"]["parallelism"] == "proof-sharded over 2 ranks"
    assert d["value_comm_rccl"] is None and "RCCL refuses" in d["comm_rccl_skipped"]
