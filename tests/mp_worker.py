"""Worker for the multi-process tests: one rank of a sharded proof (GPU) or a host-only allgather
exercise of the shared-memory transport (CPU). Launched as a child process by the tests."""
import argparse
import importlib.util
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load_product():
    spec = importlib.util.spec_from_file_location("r1cs_spartan_amd", os.path.join(ROOT, "r1cs-spartan_amd", "__init__.py"))
    mod = importlib.util.module_from_spec(spec)
    sys.modules["r1cs_spartan_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


def allgather_check(spx, name, rank, world, out):
    c = spx.ShmComm(name, rank, world)
    res = []
    for size in (0, 1, 96, 4096, 200000):  # 200000 > one 64 KiB slot: chunked rounds
        mine = bytes(((rank * 131 + i * 7 + size) & 0xFF) for i in range(size))
        got = c.allgather(mine)
        for k in range(world):
            want = bytes(((k * 131 + i * 7 + size) & 0xFF) for i in range(size))
            if got[k] != want:
                raise SystemExit("allgather mismatch: size %d from rank %d" % (size, k))
        res.append(size)
    for i in range(200):  # many back-to-back small rounds (double-buffer reuse)
        got = c.allgather(bytes([rank, i & 0xFF]))
        if got != [bytes([k, i & 0xFF]) for k in range(world)]:
            raise SystemExit("allgather mismatch in round %d" % i)
    c.close()
    open(out, "w").write("ok %s" % res)


def hub_payload(rank, ch, i):
    size = (ch * 37 + i * 11) % 300  # sizes differ per (channel, exchange), agree across ranks
    return bytes(((rank * 89 + ch * 13 + i * 7 + j) & 0xFF) for j in range(size))


def hub_check(spx, hub, rank, world, channels, iters, seed):
    """`channels` threads on this rank, each a fixed sequence of `iters` exchanges on its channel,
    with random pauses so the ranks reach the channels in different orders."""
    import random
    import threading

    errs = []

    def worker(ch):
        rng = random.Random(seed * 1000 + rank * 100 + ch)
        try:
            for i in range(iters):
                if rng.random() < 0.3:
                    time.sleep(rng.random() * 0.002)
                got = hub.allgather(ch, hub_payload(rank, ch, i))
                if got != [hub_payload(k, ch, i) for k in range(world)]:
                    errs.append("mismatch ch %d exchange %d" % (ch, i))
                    return
        except Exception as e:  # reported below
            errs.append(repr(e))

    ts = [threading.Thread(target=worker, args=(ch,)) for ch in range(channels)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    return errs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=["allgather", "hub", "prove", "prove_hub", "lvl0_mismatch"], required=True)
    ap.add_argument("--name", required=True)
    ap.add_argument("--rank", type=int, required=True)
    ap.add_argument("--world", type=int, required=True)
    ap.add_argument("--log-n", type=int, default=10)
    ap.add_argument("--log-v", type=int, default=3)
    ap.add_argument("--inflight", type=int, default=1)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    spx = load_product()
    if a.mode == "allgather":
        allgather_check(spx, a.name, a.rank, a.world, a.out)
        return
    if a.mode == "hub":
        hub = spx.ExchangeHub.shm(a.name, a.rank, a.world)
        errs = hub_check(spx, hub, a.rank, a.world, 8, 60, 5)
        st = hub.stats()
        hub.close()
        open(a.out, "w").write(("ok %s" % st) if not errs else "fail %s" % errs[:3])
        return
    sys.path.insert(0, ROOT)
    import bench

    if a.mode == "lvl0_mismatch":
        # rank 1 alone reads SPX_LVL0=batch: the ranks' first sharded proof must refuse to run
        if a.rank == 1:
            os.environ["SPX_LVL0"] = "batch"
        ctx = spx.Context(0)
        ctx.set_comm_shm(a.name, a.rank, a.world)
        syn, mats, z, nnz = bench.synth_one(spx, 0, a.log_n, a.log_v, 0x5EED0000 + a.log_n)
        pp = spx.MLProofForR1CS.setup(ctx, a.log_n, 77)
        pk = spx.IndexPK(ctx, bench.index_from_c(spx, ctx, mats), a.log_n)
        try:
            spx.MLArgumentForR1CS.prove(pk, z[: 32 << a.log_v], z[32 << a.log_v :], pp)
            res = "proved"
        except spx.InvalidArgument as e:
            res = "invalid: %s" % e
        with open(a.out, "w") as f:
            f.write(res)
        return
    ctxs = [spx.Context(0) for _ in range(a.inflight)]
    hub = spx.ExchangeHub.shm(a.name, a.rank, a.world) if a.mode == "prove_hub" else None
    for k, c in enumerate(ctxs):
        if hub is not None:
            c.set_comm_hub(hub, k)  # every proof in flight through the one ordered transport
        else:
            c.set_comm_shm("%s_%d" % (a.name, k), a.rank, a.world)
    syn, mats, z, nnz = bench.synth_one(spx, 0, a.log_n, a.log_v, 0x5EED0000 + a.log_n)
    pp = spx.MLProofForR1CS.setup(ctxs[0], a.log_n, 77)
    pk = spx.IndexPK(ctxs[0], bench.index_from_c(spx, ctxs[0], mats), a.log_n)
    wit = spx.Witness(ctxs[0], z[: 32 << a.log_v], z[32 << a.log_v :])
    proofs = spx.MLArgumentForR1CS.prove_many(ctxs, pk, [wit] * (2 * a.inflight), pp)
    with open(a.out, "wb") as f:
        for p in proofs:
            f.write(len(p).to_bytes(4, "little") + p)
        ppb = pp.serialize_uncompressed()
        f.write(len(ppb).to_bytes(4, "little") + ppb)


if __name__ == "__main__":
    main()
