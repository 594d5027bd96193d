"""bench.py --gpus N starts its own N rank processes when no launcher set WORLD_SIZE (the driver's
`python bench.py --gpus N`); --launch-only ranks report what they were given and make no HIP call."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(n, extra_env=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(extra_env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--launch-only"],
                          env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=180)


@pytest.mark.parametrize("n", [2, 4])
def test_launcher_starts_n_ranks(n):
    r = _run(n)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # ONE JSON line, rank 0's
    d = json.loads(lines[0])
    assert d["n_gpus"] == n
    assert d["ranks_seen"] == [n] * n
    assert d["ranks"] == list(range(n)) and d["local_ranks"] == list(range(n))
    assert "launcher" in d


def test_launcher_fails_when_a_rank_fails():
    r = _run(2, {"SPX_LAUNCH_TEST_FAIL": "1"})
    assert r.returncode == 3
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert "rank 1 exited" in r.stderr
