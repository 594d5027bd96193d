"""The oracle's all-cores mode (OpenMP over MSM windows and sumcheck pairs; bench.py's
cpu_baseline_all_cores) gives the same proof bytes as the single-threaded reference restatement."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle", "py"))
import oracle_c as oc  # noqa: E402


def test_threads_same_proof():
    log_n, log_v = 10, 3
    inst = oc.Instance(0, log_n, log_v, 0x5EED0000 + log_n)
    pp = oc.PP.keygen(log_n, 7)
    try:
        oc.set_threads(1)
        one = oc.prove(inst.mats, inst.v_bytes, inst.w_bytes, pp, 0, 0)
        oc.set_threads(4)
        four = oc.prove(inst.mats, inst.v_bytes, inst.w_bytes, pp, 0, 0)
    finally:
        oc.set_threads(1)
    assert one == four
