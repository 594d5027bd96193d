"""Latency of one allgather over the on-node shared-memory transport (comm_shm.cpp) among `world`
CPU processes: the exchange a rank of a proof-sharded prove makes per sumcheck round (96 B: three Fr)
and per MSM instance (384 B: one XYZZ G2 point). No GPU. Each rank process runs `iters` back-to-back
allgathers after a warm-up; the per-exchange time is rank 0's elapsed time / iters, minus the same
loop at world 1 (the ctypes call and the copy, which a rank inside the library does not pay).

usage: python tools/shm_latency.py [--world 8] [--iters 4000]  -> one JSON line
bench.py charges the 96-B figure to every exchange of a rehearsed rank (over_n1_with_exchange)."""
import argparse
import ctypes
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def worker(name, rank, world, iters, size, out):
    import bench

    spx = bench.load_product()
    L = spx.lib()
    h = ctypes.c_void_p()
    if L.spx_comm_shm_create(name.encode(), rank, world, ctypes.byref(h)) != 0:
        raise SystemExit("shm create failed")
    send = ctypes.create_string_buffer(size)
    recv = ctypes.create_string_buffer(size * world)
    f = L.spx_comm_shm_allgather
    for _ in range(200):
        f(h, send, recv, size)
    t0 = time.perf_counter()
    for _ in range(iters):
        f(h, send, recv, size)
    el = time.perf_counter() - t0
    f(h, send, recv, size)  # nobody leaves while a peer still needs the segment
    L.spx_comm_shm_destroy(h)
    if rank == 0:
        with open(out, "w") as fo:
            fo.write("%.9f" % (el / iters))


def measure(world, iters, size):
    import bench

    spx = bench.load_product()
    name = spx.shm_name()
    out = "/tmp/%s.lat" % name
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__), "--worker", name, str(r), str(world), str(iters),
                               str(size), out]) for r in range(world)]
    try:
        for p in procs:
            if p.wait(timeout=120) != 0:
                raise RuntimeError("shm latency worker failed")
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    v = float(open(out).read())
    os.remove(out)
    return v


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--worker":
        name, rank, world, iters, size, out = sys.argv[2:8]
        return worker(name, int(rank), int(world), int(iters), int(size), out)
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--iters", type=int, default=4000)
    a = ap.parse_args()
    res = {"world": a.world, "iters": a.iters, "cpus": os.cpu_count()}
    for size in (96, 384):
        t1 = measure(1, a.iters, size)
        tw = measure(a.world, a.iters, size)
        res["allgather_%dB_us" % size] = round((tw - t1) * 1e6, 3)
        res["call_overhead_%dB_us" % size] = round(t1 * 1e6, 3)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
