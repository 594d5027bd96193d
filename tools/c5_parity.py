"""BASELINE config C5 pinned byte for byte once: the 2^24 uniform-3n instance
(nnz = 3n), proved on the GPU sharded over 8 virtual ranks (8 contexts with an in-process
communicator: the N = 8 decomposition and exchanges, minus the transport), and proved by the C
oracle (oracle/c, the reference's algorithms; test infrastructure) on the box's cores under the
same PP. The two proofs must be equal byte for byte. Too long for the default GPU suite (~10 min of
oracle time), so it runs as this one-off and its log is committed (profiles/r05/).

usage: python tools/c5_parity.py [--log-n 24] --out gpurun_out/c5_parity.json
Prints a progress line every 30 s while the oracle runs."""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle", "py"))
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log-n", type=int, default=24)
    ap.add_argument("--log-v", type=int, default=5)
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--out", required=True)
    ap.add_argument("--commit", default="", help="the git revision of the tree being pinned (recorded; the GPU box has no .git)")
    a = ap.parse_args()
    log_n, log_v, G = a.log_n, a.log_v, a.ranks
    rec = {"log_n": log_n, "log_v": log_v, "generator": "uniform-3n (kind 0), seed 0x5EED0000 + log_n", "ranks": G,
           "pp": "GPU keygen, seed 0xC0FFEE", "t": {}, "commit": a.commit or None}
    t0 = time.perf_counter()

    def mark(k):
        rec["t"][k] = round(time.perf_counter() - t0, 1)
        print("%-24s %8.1f s" % (k, rec["t"][k]), flush=True)

    spx = bench.load_product()
    oc = bench.oracle()
    ctx = spx.Context(0)
    syn, mats, zb, nnz = bench.synth_one(spx, 0, log_n, log_v, 0x5EED0000 + log_n)
    rec["nnz"] = nnz
    v, w = zb[: 32 << log_v], zb[32 << log_v :]
    mark("generated")
    pp = spx.MLProofForR1CS.setup(ctx, log_n, 0xC0FFEE)
    mark("gpu keygen")
    group = spx.CommGroup(G)
    out, errs = [None] * G, []

    def rank(r):
        try:
            rctx = spx.Context(0)
            rctx.set_comm_group(group, r)
            rpk = spx.IndexPK(rctx, bench.index_from_c(spx, rctx, mats), log_n)
            rw = spx.Witness(rctx, v, w)
            out[r] = spx.MLArgumentForR1CS.prove_witness(rpk, rw, pp)
        except Exception as e:  # reported below
            errs.append(repr(e))

    ths = [threading.Thread(target=rank, args=(r,)) for r in range(G)]
    [t.start() for t in ths]
    [t.join() for t in ths]
    if errs:
        raise SystemExit("GPU prove failed: %s" % errs)
    if any(o != out[0] for o in out):
        raise SystemExit("the %d ranks' proofs differ" % G)
    gpu = out[0]
    rec["proof_bytes"] = len(gpu)
    mark("gpu proof (%d ranks)" % G)
    inst = oc.Instance(0, log_n, log_v, 0x5EED0000 + log_n)
    if inst.z_bytes != zb:
        raise SystemExit("oracle instance differs from the library generator's")
    ppc = oc.PP.load(pp.serialize_uncompressed())
    del pp
    mark("oracle pp loaded")
    threads = bench.host_cores()
    rec["oracle_threads"] = threads
    res, err = [], []

    def work():
        oc.set_threads(threads)
        try:
            res.append(oc.prove(inst.mats, inst.v_bytes, inst.w_bytes, ppc, 0, 0))
        except Exception as e:  # reported below
            err.append(repr(e))
        finally:
            oc.set_threads(1)

    th = threading.Thread(target=work)
    t1 = time.perf_counter()
    th.start()
    while th.is_alive():
        th.join(30)
        print("oracle proving on %d threads: %.0f s" % (threads, time.perf_counter() - t1), flush=True)
    if err:
        raise SystemExit("oracle failed: " + err[0])
    rec["oracle_s"] = round(time.perf_counter() - t1, 1)
    mark("oracle proof")
    rec["equal"] = res[0] == gpu
    rec["sha256_gpu"] = __import__("hashlib").sha256(gpu).hexdigest()
    rec["sha256_oracle"] = __import__("hashlib").sha256(res[0]).hexdigest()
    rec["cmd"] = "python tools/c5_parity.py --log-n %d --ranks %d" % (log_n, G)
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec), flush=True)
    if not rec["equal"]:
        raise SystemExit("PARITY FAILURE: the GPU proof differs from the oracle's at 2^%d" % log_n)


if __name__ == "__main__":
    main()
