"""Proof-sharded throughput with G VIRTUAL ranks in ONE process on one GPU (in-process communicator,
one thread per rank, B contexts per rank): the same prover code as bench.py --shard proof at N = G,
without multi-process GPU sharing, so rocprofv3 can trace it (one process) and its counters divide
the whole job's work by rank.

usage: python tools/vrank_bench.py --G 4 [--log-n 20] [--inflight 4] [--proofs 64] [--cached] [--steps 1]
Prints one JSON line: constraints/s, ms per proof, and the proofs' equality with rank 0's."""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--G", type=int, default=4)
    ap.add_argument("--log-n", type=int, default=20)
    ap.add_argument("--log-v", type=int, default=5)
    ap.add_argument("--inflight", type=int, default=0, help="contexts (proofs in flight) per rank (default: bench.inflight_for)")
    ap.add_argument("--lvl0", type=int, default=-2, help="level-0 opening MSM mode per context (default: bench.lvl0_for)")
    ap.add_argument("--proofs", type=int, default=64, help="proofs per step")
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--cached", action="store_true", help="index-cached matrix transcript")
    ap.add_argument("--sync-dir", default="", help="side-by-side runs: wait (after the warm-up) until --sync-n "
                    "processes have written a ready file into this directory, so their timed regions overlap")
    ap.add_argument("--sync-n", type=int, default=1)
    ap.add_argument("--solo", action="store_true",
                    help="rehearsal: one rank of the G, without peers (spx_ctx_set_comm_rehearsal), the GPU to "
                    "itself: its proof rate x n estimates an N = G node; its proofs are not valid")
    ap.add_argument("--ranks", default="0",
                    help="--solo: the ranks to rehearse one after the other ('all' = 0..G-1); the node runs at its "
                    "slowest rank, so node_estimate = the minimum over them")
    ap.add_argument("--exchange-ns", type=int, default=0,
                    help="--solo: charge every exchange this latency (SPX_REHEARSAL_EXCHANGE_NS; 0 = free)")
    ap.add_argument("--exchange-list", default="",
                    help="--solo: after the ranks, the slowest one again with every exchange charged each of these "
                    "latencies (ns, comma-separated)")
    a = ap.parse_args()
    if a.exchange_ns:
        os.environ["SPX_REHEARSAL_EXCHANGE_NS"] = str(a.exchange_ns)
    os.environ.setdefault("SPX_BLOCKING_SYNC", "1")
    os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")
    os.environ.setdefault("SPX_SYNC_POLL_US", str(bench.sync_poll_for(a.G)))
    spx = bench.load_product()
    G, B, P = a.G, a.inflight or bench.inflight_for(a.G), a.proofs
    world = G
    solo_ranks = [0]
    if a.solo:
        G = 1  # one rank object, acting as each rank of --ranks in turn
        solo_ranks = list(range(world)) if a.ranks == "all" else [int(x) for x in a.ranks.split(",")]
    groups = [spx.CommGroup(G) for _ in range(B)]
    ctxs = [[spx.Context(0) for _ in range(B)] for _ in range(G)]
    for r in range(G):
        for k in range(B):
            ctxs[r][k].set_lvl0_batch(bench.lvl0_for(world) if a.lvl0 == -2 else a.lvl0)
            if a.solo:
                ctxs[r][k].set_comm_rehearsal(solo_ranks[0], world)
            elif G > 1:
                ctxs[r][k].set_comm_group(groups[k], r)
    n = 1 << a.log_n
    syn, mats, zs, nnz = bench.synth_instance(spx, 3, a.log_n, a.log_v, 0x5EED0000 + a.log_n, P, 0xB0B0)
    pp = spx.MLProofForR1CS.setup(ctxs[0][0], a.log_n, 0xC0FFEE)
    pks = [None] * G

    def build(r):
        pks[r] = spx.IndexPK(ctxs[r][0], bench.index_from_c(spx, ctxs[r][0], mats), a.log_n)

    ths = [threading.Thread(target=build, args=(r,)) for r in range(G)]
    [t.start() for t in ths]
    [t.join() for t in ths]
    wits = [spx.Witness(ctxs[0][0], z[: 32 << a.log_v], z[32 << a.log_v :]) for z in zs]
    del zs
    mem = None
    if a.solo:  # proofs in flight capped by device memory, as bench.py does (one probe proof on context 0)
        nfit, mem = bench.fit_inflight(ctxs[0], lambda: spx.MLArgumentForR1CS.prove_witness(
            pks[0], wits[0], pp, cached=a.cached))
        del ctxs[0][nfit:]
        B = len(ctxs[0])

    def run(steps):
        out = [None] * G
        errs = []

        def rank(r):
            try:
                out[r] = spx.MLArgumentForR1CS.prove_many(ctxs[r], pks[r], wits * steps, pp, cached=a.cached)
            except Exception as e:
                errs.append(repr(e))

        t = [threading.Thread(target=rank, args=(r,)) for r in range(G)]
        t0, c0 = time.perf_counter(), time.process_time()
        [x.start() for x in t]
        [x.join() for x in t]
        el = time.perf_counter() - t0
        assert not errs, errs
        assert all(o == out[0] for o in out), "ranks disagree"
        return out[0], el, time.process_time() - c0

    def sync_barrier():
        if a.sync_dir:
            os.makedirs(a.sync_dir, exist_ok=True)
            open(os.path.join(a.sync_dir, "ready.%d" % os.getpid()), "w").close()
            t_wait = time.time()
            while len([f for f in os.listdir(a.sync_dir) if f.startswith("ready.")]) < a.sync_n:
                if time.time() - t_wait > 600:
                    raise SystemExit("side-by-side barrier timed out")
                time.sleep(0.01)

    per_rank, with_exchange = {}, {}
    cur = {"rank": solo_ranks[0]}

    def set_rank(rr, delay_ns):
        """solo contexts act as rank rr of `world`, each exchange charged delay_ns (read when the comm is set)"""
        os.environ["SPX_REHEARSAL_EXCHANGE_NS"] = str(delay_ns)
        for c in ctxs[0]:
            c.set_comm_rehearsal(rr, world)
        if rr != cur["rank"]:  # a rank's index holds its own rows and columns
            pks[0] = None
            pks[0] = spx.IndexPK(ctxs[0][0], bench.index_from_c(spx, ctxs[0][0], mats), a.log_n)
            cur["rank"] = rr

    if a.solo and (len(solo_ranks) > 1 or a.exchange_list):
        # every rank but the last: a warm-up step and the timed steps; the last is the main run below
        for rr in solo_ranks[:-1]:
            set_rank(rr, a.exchange_ns)
            if a.warmup:
                run(1)
            _, el_r, _ = run(a.steps)
            per_rank[rr] = round(a.steps * P * n / el_r, 1)
        set_rank(solo_ranks[-1], a.exchange_ns)
        if a.warmup:
            run(1)
    elif a.warmup:
        run(a.warmup)
    sync_barrier()
    hp0 = spx.host_phase_stats()
    proofs, el, cpu = run(a.steps)
    hp1 = spx.host_phase_stats()
    npf = max(1, len(proofs))
    host_phases = {k: {"cpu_ms": round((hp1[k][0] - hp0[k][0]) / npf * 1e3, 3),
                       "wall_ms": round((hp1[k][1] - hp0[k][1]) / npf * 1e3, 3)} for k in hp1}
    t_end = time.time()
    if a.solo:
        per_rank[solo_ranks[-1]] = round(a.steps * P * n / el, 1)
    node = min(per_rank.values()) if per_rank else None
    if a.solo and a.exchange_list:
        # the slowest rank again, every exchange charged each listed latency
        slow = min(per_rank, key=per_rank.get)
        for d in [int(x) for x in a.exchange_list.split(",")]:
            set_rank(slow, d)
            run(1)
            _, el_d, _ = run(a.steps)
            with_exchange[str(d)] = round(a.steps * P * n / el_d, 1)
        set_rank(slow, a.exchange_ns)
    print(json.dumps({"G": world, "solo_rank0": a.solo, "solo_ranks": solo_ranks if a.solo else None,
                      "per_rank": {str(k): v for k, v in sorted(per_rank.items())} if a.solo else None,
                      "exchange_ns": a.exchange_ns, "slowest_rank_with_exchange_ns": with_exchange or None, "t_start": round(t_end - el, 3), "t_end": round(t_end, 3), "inflight_per_rank": B, "proofs": len(proofs), "log_n": a.log_n, "cached": a.cached,
                      "value": round(a.steps * P * n / el, 1), "ms_per_proof": round(el / (a.steps * P) * 1e3, 3),
                      # strong scaling: every rank works on every proof, so the node finishes the batch when its
                      # slowest rank does (the minimum over the rehearsed ranks)
                      "node_estimate": node,
                      "node_spread": round(max(per_rank.values()) / node, 4) if per_rank else None,
                      "distinct": len(set(proofs)),
                      "msm_reruns": sum(c.msm_reruns() for cs in ctxs for c in cs), "device_memory": mem,
                      "process_cores_busy": round(cpu / el, 2),
                      "process_cpu_ms_per_proof": round(cpu / npf * 1e3, 3),
                      # per proof, on the proving threads (prove()'s phases), excluding the hashing pool
                      "host_phases_per_proof": host_phases}), flush=True)


if __name__ == "__main__":
    main()
