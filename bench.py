#!/usr/bin/env python
"""bench.py — R1CS constraints proved per second (BASELINE.json metric) on N MI355X.

One proof = one complete `MLArgumentForR1CS::prove` (/root/reference/src/lib.rs:58-146) of a
synthetic uniform-3n R1CS instance (2^20 constraints, |v| = 32, nnz = 3n) with the
witness already resident in HBM: Fiat-Shamir transcript (including absorbing A, B, C on every
proof), G1 commit MSM, two mKZG openings (G2 MSMs), SpMVs, eq tables, both sumchecks, proof
serialization. Setup (keygen), index and witness upload are outside the timed region, as in
benchmark.rs:26-35.

One step = a batch of P = --proofs-per-step proofs (default 64); the K timed steps run as one
continuous pipeline of K x P proofs through spx_prove_many with B = --inflight (default 16) host
worker threads, each with its own HIP stream and MSM workspace, each proving its share back to
back, so the sequential host Blake2s absorption of the matrices (~150 MB per proof, one pool of
hashing threads per rank) overlaps other proofs' GPU work instead of idling the GPU.
value = constraints proved per second over the timed region (whole job). The single-proof latency
and the index-cached-transcript variant are reported beside it.

N > 1: one process per GPU (torch.distributed.run). Default (--shard batch): every rank proves its
own P proofs per step, with no data-path exchange ("scaling": "weak"; value = all ranks' proofs / the
max-over-ranks time). The same proofs split over all ranks are reported beside it as
value_proof_sharded: hypercube blocks, with per-round partials exchanged by an on-node shared-memory
allgather, one communicator per proof in flight; --comm rccl uses RCCL AllGather instead.
--shard proof makes that the headline ("strong").

Output: ONE JSON line on rank 0 (metric, value, roofline of the dominant kernel measured live with
HIP events on the library's stream, cpu_baseline from the test oracle on a bounded sample).
"""
import argparse
import ctypes
import importlib.util
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# measured VALU ceilings of the curve additions the MSM kernels run (tools/ubench29.hip with all 256 CUs
# busy, profiles/r01_ubench29_loose.txt, current loose-accumulator code): mixed additions per second
MADD_CEILING = {"msm_acc_g2": 2.216e9, "msm_acc_g1": 6.041e9}

# HIP kernel (short rocprofv3 name) behind each kernel-stats id
KSYM = {"sc1_round": "k_sc1_round", "sc2_round": "k_sc2_round", "spmv3": "k_sparse3<0>", "mtv3": "k_sparse3<1>",
        "open_level": "k_open_level", "eq_expand": "k_eq_expand", "msm_acc_g1": "k_accum_aff<Fq >",
        "msm_acc_g2": "k_accum_aff<Fq2>", "msm_accx_g1": "k_accum_xyzz<Fq >", "msm_accx_g2": "k_accum_xyzz<Fq2>"}
PMC_FILE = os.path.join(ROOT, "profiles", "pmc_traffic.json")


VALU_FILE = os.path.join(ROOT, "profiles", "pmc_valu.json")


def valu_issue(ms_per_proof, dom):
    """Compute-side roofline of the whole proof: the VALU wave-instructions every proof kernel issues
    (rocprofv3 SQ_INSTS_VALU pass, tools/valu_summary.py -> profiles/pmc_valu.json) at the full issue
    rate (4 cycles per wave-instruction on each of the 1024 SIMDs), against the measured time per proof."""
    try:
        d = json.load(open(VALU_FILE))
    except (OSError, ValueError):
        return None
    ideal = d["ideal_valu_ms_per_proof"]
    k = d["kernels"].get(KSYM.get(dom, ""), {})
    return {"ideal_ms_per_proof": round(ideal, 3), "ms_per_proof": round(ms_per_proof, 3),
            "frac": round(ideal / ms_per_proof, 4),
            "dominant_kernel_ideal_ms_per_proof": round(k.get("ideal_valu_ms_per_proof", 0.0), 3),
            "source": "profiles/pmc_valu.json (rocprofv3 --pmc SQ_INSTS_VALU, %g proofs, %g GHz)" % (d["proofs"], d["clock_ghz"])}


def pmc_traffic(kname):
    """HBM bytes per launch of `kname` from the committed rocprofv3 PMC passes (tools/pmc_summary.py)."""
    try:
        d = json.load(open(PMC_FILE))
    except (OSError, ValueError):
        return None
    sym = KSYM.get(kname)
    rec = d.get("kernels", {}).get(sym) if sym else None
    if not rec or rec.get("traffic_bytes") is None:
        return None
    return rec["traffic_bytes"]


KNAMES = ["sc1_round", "sc2_round", "spmv3", "mtv3", "open_level", "eq_expand", "msm_sort", "msm_acc_g1", "msm_acc_g2",
          "msm_accx_g1", "msm_accx_g2", "msm_reduce_g1", "msm_reduce_g2"]


def jobs_per_rank_step(P, world, sharded_head):
    """proofs one rank's GPU completes per step: P in batch mode; P / world of each proof's work sharded"""
    return P if not sharded_head else P / world * 1.0


def load_product():
    spec = importlib.util.spec_from_file_location("r1cs_spartan_amd", os.path.join(ROOT, "r1cs-spartan_amd", "__init__.py"))
    mod = importlib.util.module_from_spec(spec)
    sys.modules["r1cs_spartan_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


def synth_instance(spx, kind, log_n, log_v, seed):
    L = spx.lib()
    L.spx_synth_create.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, ctypes.POINTER(ctypes.c_void_p)]
    L.spx_synth_csr.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(spx._CCsr)]
    L.spx_synth_z.argtypes = [ctypes.c_void_p]
    L.spx_synth_z.restype = ctypes.c_void_p
    L.spx_synth_nnz.argtypes = [ctypes.c_void_p, ctypes.c_int]
    L.spx_synth_nnz.restype = ctypes.c_uint64
    L.spx_synth_free.argtypes = [ctypes.c_void_p]
    h = ctypes.c_void_p()
    spx._check(L.spx_synth_create(kind, log_n, log_v, seed, 0, ctypes.byref(h)))
    mats = []
    for m in range(3):
        c = spx._CCsr()
        spx._check(L.spx_synth_csr(h, m, ctypes.byref(c)))
        mats.append(c)
    n = 1 << log_n
    z = ctypes.string_at(L.spx_synth_z(h), 32 * n)
    nnz = sum(L.spx_synth_nnz(h, m) for m in range(3))
    return h, mats, z, nnz


def index_from_c(spx, ctx, mats):
    h = ctypes.c_void_p()
    a, b, c = mats
    spx._check(spx.lib().spx_index(ctx.h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c), ctypes.byref(h)))
    return h


def cpu_baseline(log_n, log_v, seconds_cap, threads=1):
    """Test-oracle C prover (reference-faithful algorithms) on a bounded sample: one thread (the
    reference is single-threaded as configured), or `threads` OpenMP threads over the MSM windows and
    sumcheck pairs (what ark-ec's `parallel` feature would split)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle", "py"))
    so = os.path.join(ROOT, "oracle", "liboracle.so")
    if not os.path.exists(so):
        import subprocess

        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
    import oracle_c as oc

    inst = oc.Instance(0, log_n, log_v, 0x5EED0000 + log_n)
    pp = oc.PP.keygen(log_n, 0xC0FFEE)
    oc.set_threads(threads)
    reps, t_total = 0, 0.0
    try:
        while True:
            t0 = time.perf_counter()
            oc.prove(inst.mats, inst.v_bytes, inst.w_bytes, pp, 0, 0)
            t_total += time.perf_counter() - t0
            reps += 1
            if t_total >= seconds_cap or reps >= 3:
                break
    finally:
        oc.set_threads(1)
    per = t_total / reps
    return {
        "value": (1 << log_n) / per,
        "unit": "constraints/s",
        "cores": threads,
        "kind": "port",
        "sample": "oracle/c reference-faithful prover (log_n eq tables, degree-(log_n+2) sumcheck, "
        "duplicated-scalar G2 MSMs, ark-ec Pippenger%s), uniform-3n 2^%d, |v|=%d, %d proof(s), %.2f s each, FS"
        % ("" if threads == 1 else ", %d OpenMP threads over MSM windows and sumcheck pairs" % threads,
           log_n, 1 << log_v, reps, per),
    }


def host_cores():
    """cores this process may use: OMP_NUM_THREADS (16 on the GPU box) or the affinity mask"""
    try:
        return max(1, int(os.environ.get("OMP_NUM_THREADS", "")))
    except ValueError:
        return max(1, min(16, len(os.sched_getaffinity(0))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--log-n", type=int, default=20)
    ap.add_argument("--log-v", type=int, default=5)
    ap.add_argument("--kind", type=int, default=0, help="0 uniform-3n, 1 ref-shaped")
    ap.add_argument("--mode", default="fs", choices=["fs", "injected"])
    ap.add_argument("--cpu-log-n", type=int, default=14)
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-stats", action="store_true")
    ap.add_argument("--shard", default="batch", choices=["batch", "proof"],
                    help="N > 1 headline: 'batch' = every rank proves its own proofs (weak scaling, no data-path "
                    "exchange); 'proof' = every proof split over all ranks (strong scaling, per-round exchange)")
    ap.add_argument("--no-sharded", action="store_true",
                    help="N > 1 with --shard batch: skip the secondary proof-sharded measurement")
    ap.add_argument("--comm", default="shm", choices=["shm", "rccl"],
                    help="N > 1 transport: on-node shared memory (default) or RCCL AllGather")
    ap.add_argument("--inflight", type=int, default=16, help="proofs in flight (worker contexts)")
    ap.add_argument("--proofs-per-step", type=int, default=64,
                    help="proofs per step (a multiple of --inflight); the K steps run as one pipeline of K x P proofs")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist

        # the gloo rendezvous prints connection notices on stdout: keep stdout for rank 0's JSON line
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group("gloo", init_method="env://", rank=rank, world_size=world)
            dist.barrier()
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)

    # host waits sleep rather than spin: with many proofs in flight the cores go to the transcript
    # hashing pool of spx_prove_many (measured: 31.2 vs 28.2 M constraints/s at 2^20 on one MI355X)
    os.environ.setdefault("SPX_BLOCKING_SYNC", "1")
    # 16 hardware queues per process (HIP default 4): a proof's small latency-bound kernels (sumcheck
    # rounds, bucket-weighting levels) then queue behind fewer of the other proofs' MSM launches
    # (measured 33.5 vs 31.1 M constraints/s at 2^20; 2 ranks on one GPU 23.9 vs 18.3)
    os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")
    spx = load_product()
    B = max(1, args.inflight)
    P = max(B, (args.proofs_per_step + B - 1) // B * B)  # proofs per step; each worker proves P / B of them
    # SPX_BENCH_SAME_GPU=1: every rank on GPU 0 (multi-rank rehearsal on a one-GPU box)
    device = 0 if os.environ.get("SPX_BENCH_SAME_GPU") == "1" else local
    sharded_head = world > 1 and args.shard == "proof"
    # batch mode (and N = 1): contexts with the local communicator, every rank proves whole proofs
    ctxs = [spx.Context(device) for _ in range(B)]
    ctx = ctxs[0]
    # proof-sharded contexts (N > 1): one communicator per proof in flight, every proof split over the ranks
    sctxs = []
    if world > 1 and (sharded_head or not args.no_sharded):
        sctxs = [spx.Context(device) for _ in range(B)]
        if args.comm == "rccl":
            uid = [[spx.comm_unique_id() for _ in range(B)] if rank == 0 else None]
            dist.broadcast_object_list(uid, src=0)
            for k, c in enumerate(sctxs):
                c.set_comm_rccl(uid[0][k], rank, world)
        else:
            name = [spx.shm_name() if rank == 0 else None]
            dist.broadcast_object_list(name, src=0)
            for k, c in enumerate(sctxs):
                c.set_comm_shm("%s_%d" % (name[0], k), rank, world)

    log_n, log_v = args.log_n, args.log_v
    n = 1 << log_n
    t0 = time.perf_counter()
    syn, mats, z, nnz = synth_instance(spx, args.kind, log_n, log_v, 0x5EED0000 + log_n)
    t_gen = time.perf_counter() - t0
    t0 = time.perf_counter()
    pp = spx.MLProofForR1CS.setup(ctx, log_n, 0xC0FFEE)
    t_setup = time.perf_counter() - t0
    t0 = time.perf_counter()
    pk = spx.IndexPK(ctx, index_from_c(spx, ctx, mats), log_n)
    spk = spx.IndexPK(sctxs[0], index_from_c(spx, sctxs[0], mats), log_n) if sctxs else None
    wit = spx.Witness(ctx, z[: 32 << log_v], z[32 << log_v :])
    t_index = time.perf_counter() - t0

    def barrier():
        if dist is not None:
            dist.barrier()

    def timed(fn):
        barrier()
        t0 = time.perf_counter()
        r = fn()
        barrier()
        return r, time.perf_counter() - t0

    def batch_fn(cs, k, steps, cached=False):
        return lambda: spx.MLArgumentForR1CS.prove_many(cs, k, [wit] * (P * steps), pp, mode=args.mode, seed=7,
                                                        cached=cached)

    def single_fn(k):
        def run():
            for _ in range(args.steps):
                r = spx.MLArgumentForR1CS.prove_witness(k, wit, pp, mode=args.mode, seed=7)
            return r
        return run

    # headline configuration
    hctxs, hpk = (sctxs, spk) if sharded_head else (ctxs, pk)
    hctx = hctxs[0]
    batch_fn(hctxs, hpk, max(1, args.warmup))()
    L = spx.lib()
    if not args.no_stats:
        spx._check(L.spx_kernel_stats_enable(hctx.h, 1))
    # ---- timed region (headline): K steps x P full proofs, pipelined over B workers
    proofs, elapsed = timed(batch_fn(hctxs, hpk, args.steps))
    stats = {}
    if not args.no_stats:
        for k, name in enumerate(KNAMES):
            cnt, kms, by, ops = ctypes.c_uint64(), ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
            spx._check(L.spx_kernel_stats(hctx.h, k, ctypes.byref(cnt), ctypes.byref(kms), ctypes.byref(by)))
            spx._check(L.spx_kernel_ops(hctx.h, k, ctypes.byref(ops)))
            if cnt.value:
                # per proof: ctx 0 proves P / B proofs per step
                per = args.steps * (P // B)
                stats[name] = {"launches": cnt.value / per, "ms": kms.value / per, "bytes": by.value / per,
                               "ops": ops.value / per}
        spx._check(L.spx_kernel_stats_enable(hctx.h, 0))
    assert all(p == proofs[0] for p in proofs), "concurrent proofs differ"
    proof = proofs[0]
    # ---- single-proof latency (one proof at a time) and its phase split
    p1, elapsed_single = timed(single_fn(hpk))
    assert p1 == proof, "single proof differs from the batched one"
    phases = hctx.last_timings()
    # ---- index-cached transcript variant (matrix absorption moved to index time; bit-identical)
    p2, elapsed_cached = timed(batch_fn(hctxs, hpk, args.steps, cached=True))
    assert all(p == proof for p in p2), "cached-transcript proof differs"
    # ---- N > 1, batch headline: the same proofs split over all ranks (throughput and latency)
    ms_s = ms_s1 = None
    if sctxs and not sharded_head:
        batch_fn(sctxs, spk, 1)()
        p3, el = timed(batch_fn(sctxs, spk, args.steps))
        assert all(p == proof for p in p3), "proof-sharded proof differs"
        p4, el1 = timed(single_fn(spk))
        assert p4 == proof, "proof-sharded single proof differs"
        ms_s, ms_s1 = el / args.steps * 1e3, el1 / args.steps * 1e3

    ms = elapsed / args.steps * 1e3  # per step (P proofs)
    ms_c = elapsed_cached / args.steps * 1e3
    ms_1 = elapsed_single / args.steps * 1e3
    if dist is not None:
        import torch

        t = torch.tensor([ms, ms_c, ms_1, ms_s or 0.0, ms_s1 or 0.0], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ms, ms_c, ms_1 = float(t[0]), float(t[1]), float(t[2])
        if ms_s is not None:
            ms_s, ms_s1 = float(t[3]), float(t[4])
    # whole-job throughput: in batch mode every rank proves P proofs per step, sharded all ranks share them
    jobs = P * (1 if sharded_head else world)
    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return

    roof = None
    if stats:
        # dominant kernel = largest share of a proof's GPU time when it runs alone (rocprofv3, one proof
        # in flight: profiles/*kernel_stats_inflight1*.csv). Live durations under P proofs in flight
        # overlap, so the latency-bound weighting-tree launches would otherwise look longest.
        dom = "msm_acc_g2" if "msm_acc_g2" in stats else max(stats, key=lambda k: stats[k]["ms"])
        d = stats[dom]
        avg_s = d["ms"] / d["launches"] / 1e3
        per_launch = d["bytes"] / d["launches"]
        ach = per_launch / avg_s / 1e9
        roof = {
            "kernel": dom,
            "bound": "hbm",
            "achieved": round(ach, 2),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4),
            "traffic": pmc_traffic(dom),
            "traffic_source": "profiles/pmc_traffic.json (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, separate passes)",
            "bytes_per_launch": per_launch,
            "avg_launch_us": round(avg_s * 1e6, 2),
            "note": "algorithmic bytes / live HIP-event duration; MSM bucket accumulation is integer-VALU bound (see DESIGN.md)",
        }
        if dom in MADD_CEILING and d["ops"]:
            per_proof_ops = d["ops"]  # mixed additions of one proof
            roof["valu"] = {
                "unit": "mixed additions/s",
                "ceiling": MADD_CEILING[dom],
                "ceiling_source": "tools/ubench29.hip, all CUs busy, L2-resident points (profiles/r01_ubench29_loose.txt)",
                # per launch, live duration (shares the GPU with the other proofs in flight)
                "achieved_per_launch": round(d["ops"] / d["launches"] / avg_s, 1),
                "frac_per_launch": round(d["ops"] / d["launches"] / avg_s / MADD_CEILING[dom], 4),
                # whole job: this kernel's additions of every proof in the timed region / wall time
                "achieved_job": round(per_proof_ops * (P if sharded_head else jobs) / (ms / 1e3), 1),
                "frac_job": round(per_proof_ops * (P if sharded_head else jobs) / (ms / 1e3) / MADD_CEILING[dom], 4),
            }
    if roof is not None:
        vi = valu_issue(ms / jobs_per_rank_step(P, world, sharded_head), roof["kernel"])
        if vi:
            roof["valu_issue"] = vi
    cpu = cpu_all = None
    if world == 1 and not args.no_cpu:
        cpu = cpu_baseline(args.cpu_log_n, args.log_v, args.cpu_seconds)
        cpu_all = cpu_baseline(args.cpu_log_n, args.log_v, args.cpu_seconds, threads=host_cores())
    out = {
        "metric": "R1CS constraints proved/sec at 2^%d" % log_n,
        "value": round(jobs * n / (ms / 1e3), 1),
        "unit": "constraints/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 3),
        "higher_is_better": True,
        "scaling": "strong" if sharded_head else "weak",
        "vs_baseline": None,
        "dtype": "bls12-381 Fr/Fq Montgomery (u32 limbs)",
        "data": "synthetic",
        "config": {
            "workload": "%s R1CS 2^%d constraints, |v|=%d, nnz=%d, full prove + commit + 2 openings, %s transcript, "
            "%d proofs per step, %d in flight" % ("uniform-3n" if args.kind == 0 else "ref-shaped", log_n, 1 << log_v,
                                                   nnz, args.mode.upper(), P, B),
            "log_n": log_n,
            "proofs_per_step": P,
            "proofs_in_flight": B,
            "parallelism": ("proof-sharded over %d ranks" % world) if sharded_head else ("%d independent ranks" % world),
            "comm": args.comm if sctxs else None,
        },
        "ms_per_proof_single": round(ms_1, 3),
        "value_single_proof": round(n / (ms_1 / 1e3), 1),
        "value_index_cached_transcript": round(jobs * n / (ms_c / 1e3), 1),
        "ms_per_step_index_cached_transcript": round(ms_c, 3),
        "phases_ms": {k: round(v / 1e3, 3) for k, v in phases.items()},
        "kernels_ms_per_proof": {k: round(v["ms"], 3) for k, v in stats.items()},
        "roofline": roof,
        "cpu_baseline": cpu,
        "cpu_baseline_all_cores": cpu_all,
        "setup_s": round(t_setup, 2),
        "index_s": round(t_index, 2),
        "gen_s": round(t_gen, 2),
        "proof_bytes": len(proof),
    }
    if ms_s is not None:
        # the same workload with every proof split over all ranks (hypercube blocks, per-round exchange)
        out["value_proof_sharded"] = round(P * n / (ms_s / 1e3), 1)
        out["ms_per_step_proof_sharded"] = round(ms_s, 3)
        out["ms_per_proof_single_proof_sharded"] = round(ms_s1, 3)
    print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
