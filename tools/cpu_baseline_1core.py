"""One-off CPU baseline at the metric's own size: the oracle's C restatement
(oracle/c: the reference's algorithms, single-threaded as the reference is configured,
/root/reference/Cargo.toml:10-27) proves BASELINE C3's 2^20 circuit-3n witness 0xB0B0 on ONE core,
under the GPU keygen's PP (seed 0xC0FFEE), and the product proves the same witness on the GPU: the
two proofs are compared byte for byte. Test infrastructure (the oracle is the thing timed here, as
in bench.py's cpu_baseline legs); run on the GPU box (it needs the GPU keygen and the GPU proof).

usage: python tools/cpu_baseline_1core.py --log-n 20 --out gpurun_out/cpu1_2_20.json
Prints a progress line every 30 s (the oracle runs in a worker thread) and writes one JSON record."""
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
    ap.add_argument("--log-n", type=int, default=20)
    ap.add_argument("--log-v", type=int, default=5)
    ap.add_argument("--threads", type=int, default=1)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    spx = bench.load_product()
    ctx = spx.Context(0)
    t0 = time.perf_counter()
    pp = spx.MLProofForR1CS.setup(ctx, a.log_n, 0xC0FFEE)
    pp_bytes = pp.serialize_uncompressed()
    syn, mats, zs, nnz = bench.synth_instance(spx, 3, a.log_n, a.log_v, 0x5EED0000 + a.log_n, 1, 0xB0B0)
    pk = spx.IndexPK(ctx, bench.index_from_c(spx, ctx, mats), a.log_n)
    gpu_proof = spx.MLArgumentForR1CS.prove(pk, zs[0][: 32 << a.log_v], zs[0][32 << a.log_v :], pp)
    print("setup + GPU proof %.1f s" % (time.perf_counter() - t0), flush=True)
    res, out_proof, err = {}, [], []

    def work():
        try:
            res.update(bench.cpu_baseline(3, a.log_n, a.log_v, 0.0, threads=a.threads, pp_bytes=pp_bytes, max_reps=1,
                                          out_proof=out_proof))
        except Exception as e:  # reported below
            err.append(repr(e))

    th = threading.Thread(target=work)
    t1 = time.perf_counter()
    th.start()
    while th.is_alive():
        th.join(30)
        print("oracle proving on %d core(s): %.0f s" % (a.threads, time.perf_counter() - t1), flush=True)
    if err:
        raise SystemExit("oracle failed: " + err[0])
    res["parity_vs_gpu"] = bool(out_proof) and out_proof[0] == gpu_proof
    res["proof_bytes"] = len(gpu_proof)
    res["host"] = {"cpu_count": os.cpu_count(), "affinity": len(os.sched_getaffinity(0))}
    res["cmd"] = "python tools/cpu_baseline_1core.py --log-n %d --threads %d" % (a.log_n, a.threads)
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res), flush=True)
    if not res["parity_vs_gpu"]:
        raise SystemExit("PARITY FAILURE: the oracle's proof differs from the GPU's")


if __name__ == "__main__":
    main()
