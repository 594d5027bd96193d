"""BASELINE C2's index-cached pipeline alone (bench.py c2_line's last phase): 2^18 circuit-3n, commitment
stubbed, matrices absorbed once at index time, B proofs in flight. For traces and A/Bs of that phase:
  python tools/c2_cached.py [--inflight B] [--steps K]   -> one JSON line"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--inflight", type=int, default=bench.C2_INFLIGHT)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--group", type=int, default=1, help="lockstep group size (contexts = inflight / group)")
    ap.add_argument("--poll", type=int, default=bench.C2_SYNC_POLL_US, help="host wait: poll every POLL us (0: sync)")
    a = ap.parse_args()
    spx = bench.load_product()
    log_n, log_v, P = 18, 5, 64
    n = 1 << log_n
    ctxs = [spx.Context(0) for _ in range(max(1, a.inflight // a.group))]
    for c in ctxs:
        c.set_sync_poll(a.poll)
        c.set_group(a.group)
    syn, mats, zs, nnz = bench.synth_instance(spx, 3, log_n, log_v, 0x5EED0000 + log_n, P, 0xB0B0)
    pk = spx.IndexPK(ctxs[0], bench.index_from_c(spx, ctxs[0], mats), log_n)
    wits = [spx.Witness(ctxs[0], z[: 32 << log_v], z[32 << log_v:]) for z in zs]
    run = lambda k: spx.MLArgumentForR1CS.prove_many(ctxs, pk, wits * k, None, mode="fs", seed=7, cached=True,
                                                     commitment_stub=True)
    ref = run(1)
    t0 = time.perf_counter()
    pc = run(a.steps)
    el = time.perf_counter() - t0
    assert all(p == ref[i % P] for i, p in enumerate(pc))
    print(json.dumps({"inflight": a.inflight, "group": a.group, "poll_us": a.poll, "contexts": len(ctxs), "steps": a.steps, "proofs": len(pc),
                      "value_index_cached": round(a.steps * P * n / el, 1),
                      "ms_per_proof": round(el / (a.steps * P) * 1e3, 4),
                      "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES")}))


if __name__ == "__main__":
    main()
