"""One-off CPU baselines at larger sizes than bench.py's bounded samples (run on the GPU box through
gpurun): the test oracle's reference-faithful C prover (oracle/c) on the bench workload
(circuit-3n, |v| = 32, FS transcript), all process cores at 2^20 (the metric's size) and 1 core at
2^16, with the PP from the GPU keygen loaded into the oracle. Prints one JSON line per measurement.
Test infrastructure: the oracle is the checker / baseline, never the product path."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main():
    spx = bench.load_product()
    ctx = spx.Context(0)
    cores = bench.host_cores()
    for log_n, threads in ((20, cores), (16, 1)):
        pp = spx.MLProofForR1CS.setup(ctx, log_n, 0xC0FFEE)
        ppb = pp.serialize_uncompressed()
        del pp
        t0 = time.perf_counter()
        r = bench.cpu_baseline(3, log_n, 5, 0.0, threads=threads, pp_bytes=ppb, max_reps=1)
        r["wall_s"] = round(time.perf_counter() - t0, 1)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
