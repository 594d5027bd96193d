#!/usr/bin/env python
"""bench.py — R1CS constraints proved per second (BASELINE.json metric) on N MI355X.

One proof = one complete `MLArgumentForR1CS::prove` (/root/reference/src/lib.rs:58-146) with the
witness already resident in HBM: Fiat-Shamir transcript (including absorbing A, B, C on every
proof), G1 commit MSM, two mKZG openings (G2 MSMs), SpMVs, eq tables, both sumchecks, proof
serialization. Setup (keygen), index and witness upload are outside the timed region, as in
benchmark.rs:26-35.

Workload (BASELINE config C3): the "circuit-3n" synthetic R1CS at 2^20 constraints, |v| = 32,
nnz = 3n: ONE index (A, B, C fixed) and W = --witnesses DISTINCT satisfying
witnesses (default: one per proof of a step), so every proof has its own transcript, challenges,
scalars and gather streams.

One step = P = --proofs-per-step proofs (default 64) over the W witnesses; the K timed steps run
as one continuous pipeline of K x P proofs through spx_prove_many with B = --inflight (default: inflight_for)
host worker threads, each with its own HIP stream and MSM workspace, so the sequential host Blake2s
absorption of the matrices (~150 MB per proof, one pool of hashing threads per rank) overlaps other
proofs' GPU work. value = constraints proved per second over the timed region (whole job).
Beside it: single-proof latency (with and without the index-cached transcript), the index-cached
throughput, BASELINE config C2 (2^18, sumcheck-only, commitment stubbed) with its own HBM roofline,
and CPU baselines (test oracle: 1 core at --cpu-log-n, all cores at --cpu-all-log-n).

N > 1: one process per GPU (torch.distributed.run). Default (--shard proof): every proof is split
over all ranks (hypercube blocks, per-round partials exchanged by an on-node
shared-memory allgather, one communicator per proof in flight; --comm rccl: one RCCL communicator per rank, shared by the
proofs in flight through the ordered exchange hub). Total work
per step is fixed ("scaling": "strong"). --shard batch makes every rank prove its own P proofs
("weak"); the other mode's value is reported beside the headline.

Output: ONE JSON line on rank 0 (metric, value, roofline of the dominant kernel measured live with
HIP events on the library's stream, cpu_baseline from the test oracle on a bounded sample).
"""
import argparse
import ctypes
import importlib.util
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# VALU issue peak: 1024 SIMDs x 32 lanes per cycle x 2.4 GHz (MI355X_MICROARCH.md: a wave64 VALU
# instruction issues over 2 cycles on a SIMD-32; = the 157.3 TFLOPS FP32 vector spec / 2 per FMA)
VALU_PEAK_WAVE_INSTR = 1024 * 2.4e9 / 2.0
PMC_FILE = os.path.join(ROOT, "profiles", "pmc_kernels.json")
# the same passes over the C2 workload (2^18, commitment stubbed): its launches' own counters
PMC_FILE_C2 = os.path.join(ROOT, "profiles", "pmc_kernels_c2.json")
ISSUE_FILE = os.path.join(ROOT, "profiles", "r02_ubench_issue.txt")
# effective shader clock of the long kernels (rocprofv3 --pmc GRBM_GUI_ACTIVE + the same pass's kernel
# trace, one proof in flight: tools/pmc_clock.sh; MI355X_MICROARCH.md "DVFS give-back")
CLOCK_FILE = os.path.join(ROOT, "profiles", "r05", "r05a_clock.json")
# the oracle's reference-faithful prover on ONE core at the metric's 2^20 on the GPU box (~220 s, too
# long for every bench run: tools/cpu_baseline_1core.py, run once, proof byte-equal to the GPU's)
CPU1_2_20_FILE = os.path.join(ROOT, "profiles", "r05", "r05a_cpu_baseline_1core_2_20.json")
# BASELINE C5 (2^24, 8 ranks) byte parity and the oracle's 16-core time there (tools/c5_parity.py)
# the newest committed 2^24 8-rank byte-parity record (tools/c5_parity.py --commit REV)
C5_FILE = next((f for f in (os.path.join(ROOT, "profiles", "r06", "r06_c5_parity_2_24.json"),
                            os.path.join(ROOT, "profiles", "r05", "r05d_c5_parity_2_24.json")) if os.path.exists(f)),
               os.path.join(ROOT, "profiles", "r05", "r05d_c5_parity_2_24.json"))
MADD_FILE = os.path.join(ROOT, "profiles", "r02_ubench_madd.txt")

# HIP kernel (short rocprofv3 name) behind each kernel-stats id
KSYM = {"sc1_round": "k_sc1_wave<true, false, false>", "sc2_round": "k_sc2_wave<true, false, false>", "spmv3": "k_spmv_sliced",
        "mtv3": "k_col_stream", "open_level": "k_open_fold_wave<3>", "eq_expand": "k_eq_expand", "msm_acc_g1": "k_accum_aff<Fq >",
        "msm_acc_g2": "k_accum_aff<Fq2>", "msm_accx_g1": "k_accum_xyzz<Fq >", "msm_accx_g2": "k_accum_xyzz<Fq2>"}
KNAMES = ["sc1_round", "sc2_round", "spmv3", "mtv3", "open_level", "eq_expand", "msm_sort", "msm_acc_g1", "msm_acc_g2",
          "msm_accx_g1", "msm_accx_g2", "msm_reduce_g1", "msm_reduce_g2"]
HBM_KERNELS = ["sc1_round", "sc2_round", "spmv3", "mtv3", "open_level", "eq_expand"]
KIND_NAMES = {0: "uniform-3n", 1: "ref-shaped", 3: "circuit-3n"}


def pmc_kernel(kname, path=PMC_FILE):
    """per-launch counters of `kname` from the committed rocprofv3 PMC passes (tools/pmc_summary.py)"""
    if not path:
        return None
    try:
        d = json.load(open(path))
    except (OSError, ValueError):
        return None
    sym = KSYM.get(kname)
    return d.get("kernels", {}).get(sym) if sym else None


def load_product():
    spec = importlib.util.spec_from_file_location("r1cs_spartan_amd", os.path.join(ROOT, "r1cs-spartan_amd", "__init__.py"))
    mod = importlib.util.module_from_spec(spec)
    sys.modules["r1cs_spartan_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


def synth_instance(spx, kind, log_n, log_v, seed, n_wit, wseed0):
    """the index's CSR views and n_wit witnesses (kind 3: distinct seeds wseed0..; else the generator's one)"""
    L = spx.lib()
    L.spx_synth_create.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64,
                                   ctypes.POINTER(ctypes.c_void_p)]
    L.spx_synth_csr.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(spx._CCsr)]
    L.spx_synth_z.argtypes = [ctypes.c_void_p]
    L.spx_synth_z.restype = ctypes.c_void_p
    L.spx_synth_nnz.argtypes = [ctypes.c_void_p, ctypes.c_int]
    L.spx_synth_nnz.restype = ctypes.c_uint64
    L.spx_synth_witnesses.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p]
    L.spx_synth_free.argtypes = [ctypes.c_void_p]
    h = ctypes.c_void_p()
    spx._check(L.spx_synth_create(kind, log_n, log_v, seed, wseed0, ctypes.byref(h)))
    mats = []
    for m in range(3):
        c = spx._CCsr()
        spx._check(L.spx_synth_csr(h, m, ctypes.byref(c)))
        mats.append(c)
    n = 1 << log_n
    if kind == 3:
        buf = ctypes.create_string_buffer(32 * n * n_wit)
        spx._check(L.spx_synth_witnesses(h, wseed0, n_wit, buf))
        base = ctypes.addressof(buf)
        zs = [ctypes.string_at(base + 32 * n * i, 32 * n) for i in range(n_wit)]
        del buf
    else:
        zs = [ctypes.string_at(L.spx_synth_z(h), 32 * n)]
    nnz = sum(L.spx_synth_nnz(h, m) for m in range(3))
    return h, mats, zs, nnz


def synth_one(spx, kind, log_n, log_v, seed):
    """(handle, CSR views, z bytes, nnz) of one generated instance (tests)"""
    h, mats, zs, nnz = synth_instance(spx, kind, log_n, log_v, seed, 1, 0xB0B0)
    return h, mats, zs[0], nnz


def index_from_c(spx, ctx, mats):
    h = ctypes.c_void_p()
    a, b, c = mats
    spx._check(spx.lib().spx_index(ctx.h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c), ctypes.byref(h)))
    return h


def oracle():
    sys.path.insert(0, os.path.join(ROOT, "oracle", "py"))
    so = os.path.join(ROOT, "oracle", "liboracle.so")
    if not os.path.exists(so):

        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
    import oracle_c as oc

    return oc


def cpu_baseline(kind, log_n, log_v, seconds_cap, threads=1, pp_bytes=None, stub=False, max_reps=3, out_proof=None):
    """Test-oracle C prover (reference-faithful algorithms: log_n eq tables, degree-(log_n+2) sumcheck,
    hash-map eval_on_x, duplicated-scalar G2 MSMs, ark-ec Pippenger) on a bounded sample of the same
    workload: one thread (the reference is single-threaded as configured), or `threads` OpenMP
    threads over the MSM windows and sumcheck pairs (what ark-ec's `parallel` feature would split).
    The proof of witness seed 0xB0B0 (FS transcript) is appended to `out_proof` when given: it is the
    oracle's proof of the GPU's first witness, so the caller can compare the two byte for byte."""
    oc = oracle()
    inst = oc.Instance(kind, log_n, log_v, 0x5EED0000 + log_n, 0xB0B0 if kind == 3 else 0)
    pp = None if stub else (oc.PP.load(pp_bytes) if pp_bytes else oc.PP.keygen(log_n, 0xC0FFEE))
    oc.set_threads(threads)
    reps, t_total = 0, 0.0
    try:
        while True:
            t0 = time.perf_counter()
            proof = oc.prove(inst.mats, inst.v_bytes, inst.w_bytes, pp, 0, 0, commitment_stub=stub)
            t_total += time.perf_counter() - t0
            reps += 1
            if out_proof is not None and reps == 1:
                out_proof.append(proof)
            if t_total >= seconds_cap or reps >= max_reps:
                break
    finally:
        oc.set_threads(1)
    per = t_total / reps
    return {
        "value": round((1 << log_n) / per, 1),
        "unit": "constraints/s",
        "cores": threads,
        "kind": "port",
        "sample": "oracle/c reference-faithful prover%s (log_n eq tables, degree-(log_n+2) sumcheck, hash-map "
        "eval_on_x%s%s), %s 2^%d, |v|=%d, %d proof(s), %.2f s each, FS"
        % (" with the commitment stubbed (C2)" if stub else "",
           "" if stub else ", duplicated-scalar G2 MSMs, ark-ec Pippenger",
           "" if threads == 1 else ", %d OpenMP threads over %ssumcheck pairs" % (threads, "" if stub else "MSM windows and "),
           KIND_NAMES.get(kind, str(kind)), log_n, 1 << log_v, reps, per),
        "log_n": log_n,
    }


def host_cores():
    """cores this process may use: OMP_NUM_THREADS (16 on the GPU box) or the affinity mask"""
    try:
        return max(1, int(os.environ.get("OMP_NUM_THREADS", "")))
    except ValueError:
        return max(1, min(16, len(os.sched_getaffinity(0))))


def issue_costs():
    """measured cycles per wave-instruction at 1 and 2 waves per SIMD (tools/ubench_issue.hip)"""
    try:
        txt = open(ISSUE_FILE).read()
    except OSError:
        return None
    out = {}
    for line in txt.splitlines():
        if "cycles per wave-instruction" in line and "x 8 chains" in line:  # 8 independent chains per lane
            name = line.split()[0]
            w = int(line.split("waves/SIMD")[1].split(":")[0])
            cyc = float(line.split("ms,")[1].split("cycles")[0])
            out["%s@%d" % (name, w)] = cyc
    return out


def kernel_stats(spx, L, hctx, per_proof_div):
    """HIP-event statistics of ctx's launches since enabling, per proof; 'largest' = the launches of each
    kernel with the most algorithmic bytes (round 1 of a sumcheck)"""
    L.spx_kernel_stats_largest.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_uint64),
                                           ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]
    stats = {}
    for k, name in enumerate(KNAMES):
        cnt, kms, by, ops = ctypes.c_uint64(), ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        spx._check(L.spx_kernel_stats(hctx.h, k, ctypes.byref(cnt), ctypes.byref(kms), ctypes.byref(by)))
        spx._check(L.spx_kernel_ops(hctx.h, k, ctypes.byref(ops)))
        bc, bms, bby = ctypes.c_uint64(), ctypes.c_double(), ctypes.c_double()
        spx._check(L.spx_kernel_stats_largest(hctx.h, k, ctypes.byref(bc), ctypes.byref(bms), ctypes.byref(bby)))
        if cnt.value:
            stats[name] = {"launches": cnt.value / per_proof_div, "ms": kms.value / per_proof_div,
                           "bytes": by.value / per_proof_div, "ops": ops.value / per_proof_div,
                           "largest": {"launches": bc.value, "ms": bms.value, "bytes": bby.value}}
    return stats


def roofline_valu(stats, dom):
    """dominant MSM kernel: VALU issue (SQ_INSTS_VALU per launch from the committed PMC pass) over the
    live HIP-event launch duration, against the chip's VALU issue peak; HBM side as secondary fields.
    The PMC pass is one whole proof on one rank; a proof sharded over G ranks gives each rank's launches
    part of its references, so the per-launch counters are scaled by this run's algorithmic bytes per
    launch over the profiled run's (pmc_kernels.json alg_bytes_per_launch)."""
    d = stats[dom]
    avg_s = d["ms"] / d["launches"] / 1e3
    per_launch = d["bytes"] / d["launches"]
    pm = dict(pmc_kernel(dom) or {})
    share = per_launch / pm["alg_bytes_per_launch"] if pm.get("alg_bytes_per_launch") else 1.0
    for key in ("SQ_INSTS_VALU_per_launch", "traffic_bytes"):
        if pm.get(key):
            pm[key] *= share
    insts = pm.get("SQ_INSTS_VALU_per_launch")
    roof = {
        "kernel": KSYM.get(dom, dom),
        "bound": "valu",
        "unit": "G VALU wave-instructions/s",
        "achieved": round(insts / avg_s / 1e9, 1) if insts else None,
        "peak": round(VALU_PEAK_WAVE_INSTR / 1e9, 1),
        "frac": round(insts / avg_s / VALU_PEAK_WAVE_INSTR, 4) if insts else None,
        "traffic": pm.get("traffic_bytes"),
        "avg_launch_us": round(avg_s * 1e6, 2),
        "valu_insts_per_launch": insts,
        "valu_source": "profiles/pmc_kernels.json (rocprofv3 --pmc SQ_INSTS_VALU, one proof in flight, same build)",
        "pmc_share": round(share, 4),
        "note": "integer big-number VALU work (v_mad_u64_u32 limb products), no MFMA; live HIP-event duration with "
        "one proof at a time",
    }
    ic = issue_costs()
    if ic and insts:
        # instruction-mix ceiling (two waves per SIMD): ~70% of a mixed addition's VALU instructions are
        # v_mad_u64_u32 (8 Fq2 products x 588 + 2 squares x 392 per lane), issue cost
        # ic[mad@2]; the rest are single-issue ALU ops (ic[v_add_u32@2])
        roof["issue_costs_cycles"] = ic
        cm, ca = ic.get("v_mad_u64_u32@2"), ic.get("v_add_u32@2")
        if cm and ca:
            mix = 0.7 * cm + 0.3 * ca
            roof["mix_ceiling_cycles_per_instr"] = round(mix, 2)
            roof["achieved_cycles_per_instr"] = round(avg_s * 1024 * 2.4e9 / insts, 2)
            roof["frac_vs_mix_ceiling"] = round(insts * mix / (1024 * 2.4e9) / avg_s, 4)
    clk = held_clock(KSYM.get(dom, dom))
    if clk and insts:
        # the clock the chip holds under this kernel (GRBM_GUI_ACTIVE / 8 / duration in the PMC pass),
        # carried to the live duration at the same cycle count: the issue peak and the cycles per
        # instruction at that clock instead of the 2.4 GHz maximum
        f = clk["effective_clock_GHz"] * 1e9 * clk["mean_us"] / (avg_s * 1e6)
        roof["held_clock"] = {
            "GHz": round(f / 1e9, 3), "pmc_GHz": clk["effective_clock_GHz"], "pmc_mean_us": clk["mean_us"],
            "peak_at_held_clock": round(1024 * f / 2.0 / 1e9, 1),
            "frac_at_held_clock": round(insts / avg_s / (1024 * f / 2.0), 4),
            "achieved_cycles_per_instr": round(avg_s * 1024 * f / insts, 3),
            "source": os.path.relpath(CLOCK_FILE, ROOT) + " (tools/pmc_clock.sh)"}
        if roof.get("mix_ceiling_cycles_per_instr"):
            roof["held_clock"]["frac_vs_mix_ceiling"] = round(
                roof["mix_ceiling_cycles_per_instr"] / roof["held_clock"]["achieved_cycles_per_instr"], 4)
    roof["hbm"] = {
        "algorithmic_bytes_per_launch": per_launch,
        "achieved_GBs": round(per_launch / avg_s / 1e9, 1),
        "peak_GBs": HBM_PEAK_GBS,
        "frac": round(per_launch / avg_s / 1e9 / HBM_PEAK_GBS, 4),
        "traffic_bytes_per_launch": pm.get("traffic_bytes"),
        "traffic_over_algorithmic": round(pm["traffic_bytes"] / per_launch, 3) if pm.get("traffic_bytes") else None,
        "traffic_source": "profiles/pmc_kernels.json (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, separate passes)",
    }
    if d.get("ops"):
        live = d["ops"] / d["launches"] / avg_s
        roof["mixed_additions_per_s_live"] = round(live, 1)
        rr = madd_register_resident()
        if rr and dom == "msm_acc_g2":
            # the same formula with every operand in registers (no loads, no bucket logic, full grid):
            # what the accumulation kernel would reach if its memory side and its grid tail were free
            roof["register_resident_madd_per_s"] = rr
            roof["frac_vs_register_resident_madd"] = round(live / rr, 4)
            roof["register_resident_source"] = os.path.relpath(MADD_FILE, ROOT) + " (tools/ubench_madd.hip, 2 waves/SIMD)"
    return roof


SETUP_KERNELS = ("k_fixed_base", "k_precompute", "k_normalize", "k_aff_to_r29", "k_to_mont", "k_points_",
                 "__amd_rocclr_copyBufferRect")


def whole_proof_valu(ms_per_proof):
    """every per-proof kernel's VALU wave-instructions (committed PMC pass, one proof in flight; setup and
    PP-preprocessing kernels excluded), issued in the measured throughput time per proof, against the chip's
    VALU issue peak: how busy the batch keeps the vector ALUs"""
    try:
        ks = json.load(open(PMC_FILE))["kernels"]
    except (OSError, ValueError, KeyError):
        return None
    proofs = (ks.get("k_accum_aff<Fq >") or {}).get("launches_valu_pass")  # one commitment MSM per proof
    if not proofs or not ms_per_proof:
        return None
    tot = 0.0
    for k, v in ks.items():
        if k.startswith(SETUP_KERNELS):
            continue
        vi, n = v.get("SQ_INSTS_VALU_per_launch"), v.get("launches_valu_pass")
        if vi and n:
            tot += vi * n
    per = tot / proofs
    ach = per / (ms_per_proof / 1e3)
    return {"valu_insts_per_proof": round(per), "ms_per_proof": round(ms_per_proof, 3),
            "achieved": round(ach / 1e9, 1), "peak": round(VALU_PEAK_WAVE_INSTR / 1e9, 1), "unit": "G VALU wave-instructions/s",
            "frac": round(ach / VALU_PEAK_WAVE_INSTR, 4),
            "source": "profiles/pmc_kernels.json (per-proof kernels of the PMC pass, %d proofs)" % proofs}


def held_clock(sym):
    """{effective_clock_GHz, mean_us} of kernel `sym` from the committed GRBM_GUI_ACTIVE pass"""
    try:
        ks = json.load(open(CLOCK_FILE))["kernels"]
    except (OSError, ValueError, KeyError):
        return None
    for k, v in ks.items():  # "void spx::k_accum_aff<spx::Fe<spx::FqCfg> >" -> "k_accum_aff<Fq >"
        if k.replace("void ", "").replace("spx::", "").replace("Fe<FqCfg>", "Fq") == sym:
            return v
    return None


def committed_record(path):
    try:
        d = json.load(open(path))
    except (OSError, ValueError):
        return None
    d["source"] = os.path.relpath(path, ROOT)
    return d


def madd_register_resident():
    """lane-pair G2 mixed additions per second of x29_madd on register-resident operands"""
    try:
        for line in open(MADD_FILE):
            if line.startswith("chains 1 madd") and "waves/SIMD 2" in line:
                return float(line.split(",")[-1].split("G iterations/s")[0]) * 1e9
    except OSError:
        pass
    return None


def roofline_hbm(stats, pmc_path=PMC_FILE):
    """dominant HBM-streaming kernel (largest device time per proof among the sumcheck / SpMV / eq / fold
    kernels), priced on its largest launches (round 1: the tables stream from HBM; later rounds shrink
    into the caches and are launch-latency bound). `traffic` comes from the PMC passes over the SAME
    workload (pmc_path), or is null when there is none."""
    cands = [k for k in HBM_KERNELS if k in stats]
    if not cands:
        return None
    dom = max(cands, key=lambda k: stats[k]["ms"])
    d = stats[dom]
    big = d["largest"]
    avg_s = big["ms"] / big["launches"] / 1e3
    per_launch = big["bytes"] / big["launches"]
    ach = per_launch / avg_s / 1e9
    pm = pmc_kernel(dom, pmc_path) or {}
    return {"kernel": KSYM.get(dom, dom), "bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": pm.get("traffic_bytes_largest"),
            "bytes_per_launch": per_launch, "avg_launch_us": round(avg_s * 1e6, 2),
            "all_launches": {"launches_per_proof": d["launches"], "ms_per_proof": round(d["ms"], 4),
                             "GBs": round(d["bytes"] / (d["ms"] / 1e3) / 1e9, 1)},
            "largest_launches": {k: largest_rate(stats[k]) for k in cands},
            "note": "algorithmic bytes of the kernel's largest launch / its HIP-event duration, one proof at a time"}


def largest_rate(d):
    """the largest launches of one HBM kernel: algorithmic MB per launch, HIP-event us, GB/s, fraction of HBM peak"""
    big = d["largest"]
    us = big["ms"] / big["launches"] * 1e3
    mb = big["bytes"] / big["launches"] / 1e6
    gbs = mb / us * 1e3
    return {"MB": round(mb, 2), "us": round(us, 2), "GBs": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4)}


# BASELINE C2 (commitment stubbed): its proofs are ~100x shorter than a full proof's absorption, so
# the host's cores, not the GPU, set the per-proof-absorbed rate, and the runtime's spinning waits took
# 13-15 of the 16 (profiles/r05/r05u_c2ab.jsonl). Its contexts poll their waits every 20 us
# (C2_SYNC_POLL_US): 445 -> 525 M constraints/s at 16 in flight, 534-557 M at 32 (index-cached 746 ->
# 783-794 M). 8 / 16 / 32 hardware queues instead of 4: 542-666 M index-cached (r05w_c2_hwq.jsonl).
# (Round 4, spinning: 32 in flight on 4 queues had halved the index-cached rate against 16.)
# Lockstep groups (spx_ctx_set_group, round 5): each context proves C2_GROUP proofs at a time, every
# step of the group (sumcheck round, SpMV, eq table, eval_on_x, opening fold) one launch and every
# round one wait. One-at-a-time C2 proofs left the GPU idle 65% of the time behind the 4 hardware
# queues (r05zg_c2_busy.txt); index-cached 790 M -> 1,454 - 1,461 M with 16 contexts x 8 and the
# sumcheck rounds grouped (more queues: lower; profiles/r05/r05zh_c2group.jsonl, r05zi_c2group.jsonl),
# 2,114 - 2,190 M with every step grouped (r05zl_c2group.jsonl; 64 / 128 / 192 / 256 in flight: 1,987 /
# 2,142 - 2,165 / 2,114 - 2,122 / 2,137 - 2,190 M). C2_INFLIGHT counts proofs in flight.
C2_INFLIGHT = int(os.environ.get("SPX_BENCH_C2_INFLIGHT", "128"))
C2_GROUP = int(os.environ.get("SPX_BENCH_C2_GROUP", "8"))  # (A/B: up to 16, spx_ctx_set_group's limit)
C2_SYNC_POLL_US = 20


def c2_contexts(spx, device, inflight):
    """the C2 contexts: inflight / C2_GROUP lockstep groups, polling waits"""
    cs = [spx.Context(device) for _ in range(max(1, inflight // C2_GROUP))]
    for c in cs:
        c.set_sync_poll(C2_SYNC_POLL_US)
        c.set_group(C2_GROUP)
    return cs


def inflight_for(g):
    """proofs in flight per rank for proofs sharded over g ranks (1: unsharded). N = 1 with the round-4
    hashing pool (16 hardware queues, profiles/r04/r04a[k-n]_ab_inflight.jsonl): 16 -> 61.0, 24 -> 62.2,
    32 -> 62.8, 48 -> 62.9, 64 -> 62.7 M constraints/s (round 3 found 16 best while host hashing still
    limited, r03ak); a rank of a 4- or 8-rank proof has 1/g of every kernel's work, so 8 g there"""
    return 32 if g <= 2 else min(64, 8 * g)


def hw_queues_for(g):
    """hardware queues per process (GPU_MAX_HW_QUEUES): 4, HIP's default and the GPU box's preset, for
    N <= 2 (round 4, 32 in flight: 4 -> 62.8 vs 32 -> 60.4 M, 24 in flight: 62.2 vs 60.9 M with 24 queues,
    profiles/r04/r04a{i,j}_ab_inflight.jsonl; 8 queues no better, r04ah_ab_hwq8.jsonl); 32 when 4- or
    8-rank proofs keep 32-64 in flight (profiles/r03/r03aj_g8_knobs.jsonl: 64 in flight on 32 queues
    +18% over 16 on 16)"""
    return 4 if g <= 2 else 32


def sync_poll_for(g):
    """SPX_SYNC_POLL_US for proofs sharded over g ranks: host waits poll an event every 50 us instead of
    spinning in the HSA runtime (~0.2 ms of a core per wait). A rank of a g-rank proof replays every
    proof's host work at g times the single-GPU proof rate: at g = 8 the spinning took ~9 of its 16
    cores; polling halves the proving threads' CPU at equal throughput (profiles/r05/r05g_poll.jsonl,
    r05h_poll_inflight.jsonl). At g <= 2 the spinning has cores to spare and polling adds ~40 us per
    wait to a proof's latency: kept off."""
    return 50 if g >= 4 else 0


# device memory kept free beyond the contexts' own footprint (HIP runtime, fragmentation, the
# index-cached runs' second-stream MSM workspace, per-launch temporaries)
FIT_RESERVE = 8 << 30


def fit_inflight(ctxs, probe, reserve=FIT_RESERVE):
    """how many of `ctxs` fit the device: probe() runs one proof on ctxs[0] (its grow-only scratch,
    slots and MSM workspace reach their steady size, as every context's first proof makes them);
    per-context bytes = the drop in free device memory. Returns (count, record). At 2^20 nothing
    binds (~1.4 GiB per context); at 2^24 a context takes ~3 GiB beside ~90 GiB of PP, so a rank's
    64 in flight would not fit."""
    f0, total = ctxs[0].mem_info()
    probe()
    f1, _ = ctxs[0].mem_info()
    per = max(f0 - f1, 1)
    fit = int(min(len(ctxs), 1 + max(0, (f1 - reserve) // per)))
    return fit, {"free_before_GiB": round(f0 / 2**30, 2), "free_after_one_GiB": round(f1 / 2**30, 2),
                 "per_context_GiB": round(per / 2**30, 3), "total_GiB": round(total / 2**30, 2),
                 "reserve_GiB": round(reserve / 2**30, 2), "contexts": fit, "wanted": len(ctxs)}


def lvl0_for(g):
    """level-0 opening MSM inside the first opening's batch (one MSM pipeline less per proof) for proofs
    sharded over g >= 4 ranks, where a rank's small MSMs are latency-bound; beside the commitment otherwise"""
    return 1 if g >= 4 else 0


def free_port():
    import socket

    s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n, argv):
    """`bench.py --gpus N` without an external launcher (WORLD_SIZE unset): start N rank processes
    (this script again, one per GPU, RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in their environment)
    BEFORE this process makes any GPU call, wait for them, and re-print rank 0's JSON line. A rank that
    fails ends the others (by their exact PIDs) and the launcher exits with its status. Nothing here
    touches HIP, and no process is replaced (exec) by another."""
    import tempfile

    port = os.environ.get("MASTER_PORT") or str(free_port())
    base = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=port, WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n))
    out0 = tempfile.TemporaryFile(mode="w+")
    procs = []
    for r in range(n):
        env = dict(base, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env,
                                      stdout=out0 if r == 0 else subprocess.DEVNULL))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            st = p.poll()
            if st is None:
                continue
            live.remove(p)
            if st != 0 and rc == 0:
                rc = st if st > 0 else 128 - st
                sys.stderr.write("bench.py launcher: rank %d exited with %d; stopping the others\n" % (procs.index(p), st))
                for q in live:
                    q.terminate()
        time.sleep(0.2)
    for p in procs:
        p.wait()
    if rc:
        return rc
    out0.seek(0)
    lines = [ln for ln in out0.read().splitlines() if ln.strip().startswith("{")]
    if not lines:
        sys.stderr.write("bench.py launcher: rank 0 printed no JSON line\n")
        return 1
    d = json.loads(lines[-1])
    d["launcher"] = "bench.py --gpus %d: %d rank processes started by bench.py itself (no external launcher)" % (n, n)
    print(json.dumps(d), flush=True)
    return 0


def init_dist(rank, world):
    """gloo process group (rank 0's stdout is kept for its JSON line: rendezvous notices go to stderr)"""
    import torch.distributed as dist

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
    return dist


def launch_only(rank, world, local):
    """--launch-only: the rank reports what the launch gave it, with no HIP call (CPU test of the launcher)"""
    seen = {"rank": rank, "local_rank": local, "world": world}
    if os.environ.get("SPX_LAUNCH_TEST_FAIL") == str(rank):  # launcher test: this rank fails
        sys.exit(3)
    dist = init_dist(rank, world) if world > 1 else None
    allseen = [seen]
    if dist is not None:
        allseen = [None] * world
        dist.all_gather_object(allseen, seen)
    if rank == 0:
        print(json.dumps({"launch_only": True, "n_gpus": world, "ranks_seen": [s["world"] for s in allseen],
                          "ranks": [s["rank"] for s in allseen], "local_ranks": [s["local_rank"] for s in allseen]}),
              flush=True)
    if dist is not None:
        dist.destroy_process_group()


def comm_seen(ctx, rank, world):
    """world size the context's product communicator actually spans: one allgather of every rank's id
    on it (entries must come back in rank order)"""
    got = ctx.comm_allgather(rank.to_bytes(4, "little"), world)
    ids = [int.from_bytes(g, "little") for g in got]
    if ids != list(range(world)):
        raise RuntimeError("communicator returned rank ids %s, expected 0..%d" % (ids, world - 1))
    return len(ids)


def shm_exchange_latency(world):
    """one shared-memory allgather among `world` CPU processes (tools/shm_latency.py; no GPU): the latency
    charged to every exchange of a rehearsed rank in the with-exchange variant"""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "shm_latency.py"), "--world", str(world), "--iters", "4000"],
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=300)
    if r.returncode != 0:
        raise RuntimeError("shm latency measurement failed: %s" % r.stderr[-2000:])
    return json.loads(r.stdout.strip().splitlines()[-1])


# the with-exchange variants of the largest rehearsal: the measured shm allgather latency, and a
# pessimistic 50 us per exchange (a futex wake-up on every exchange instead of a spinning peer)
REHEARSAL_PESSIMISTIC_NS = 50000


def run_rehearsal(args, log_n, log_v, P):
    """N = 1: rehearsal of a G-GPU node, proof-sharded. This GPU runs ONE rank of every proof at a time,
    with no peers: every exchange returns its own contribution (spx_ctx_set_comm_rehearsal), so the rank
    does a real rank's device and host work for its 1/G of the buckets, blocks and hashing. EVERY rank
    r = 0..G-1 is rehearsed in turn (ranks own different blocks, bucket residues and whole instances),
    and the node runs at its slowest rank: the node estimate is the MINIMUM over the ranks' proof rates x
    n (per-rank values and their spread are reported). Exchanges are free in that estimate; for the
    largest G the slowest rank is run again with every exchange charged the shared-memory allgather
    latency measured among G CPU processes (tools/shm_latency.py), and with a pessimistic 50 us
    (over_n1_with_exchange). The proofs of a rehearsal are not valid and are not checked.
    Each G runs in a child process of its own (tools/vrank_bench.py --solo --ranks all), with the
    settings an N = G rank runs with: inflight_for(G) proofs in flight, lvl0_for(G), hw_queues_for(G)
    hardware queues and sync_poll_for(G). The children run BEFORE this process creates its own contexts:
    their streams hold hardware queues too, and 4 of this process's beside a child's 32 oversubscribed
    the GPU's queues (a G = 8 child measured 377 M constraints/s beside them against 400-403 M alone,
    profiles/r05/r05y_bench.json, r05z_steps.jsonl)."""
    rehearsal = {"method": "every rank r = 0..G-1 of a G-rank proof-sharded prove on this GPU in turn, no peers, matrices "
                 "absorbed per proof (1/G of them by the rank), in a child process (tools/vrank_bench.py --solo --ranks "
                 "all) run before the headline; node value = the slowest rank's proof rate x n",
                 "proofs_in_flight": {}, "hw_queues": {}, "values": {}, "per_rank": {}, "spread_max_over_min": {},
                 "msm_reruns": {}, "device_memory": {}}
    gs = [int(x) for x in args.rehearse.split(",") if x.strip()]
    gmax = max(gs) if gs else 0
    lat = None
    if gmax > 1:
        try:
            lat = shm_exchange_latency(gmax)
        except Exception as e:  # reported, the estimate without exchanges stands
            rehearsal["exchange_latency_error"] = repr(e)
        rehearsal["exchange_latency"] = lat
    for G in gs:
        env = dict(os.environ, GPU_MAX_HW_QUEUES=str(hw_queues_for(G)))
        env.setdefault("SPX_SYNC_POLL_US", str(sync_poll_for(G)))
        cmd = [sys.executable, os.path.join(ROOT, "tools", "vrank_bench.py"), "--G", str(G), "--solo", "--ranks", "all",
               "--log-n", str(log_n), "--log-v", str(log_v), "--proofs", str(P),
               "--steps", str(min(args.steps, args.rehearse_steps)),
               "--warmup", "1"] + (["--inflight", str(args.inflight)] if args.inflight else [])
        if G == gmax and lat:
            meas = max(lat["allgather_96B_us"], lat["allgather_384B_us"])
            cmd += ["--exchange-list", "%d,%d" % (max(1, int(meas * 1e3)), REHEARSAL_PESSIMISTIC_NS)]
        r = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=1200)
        if r.returncode != 0:
            raise RuntimeError("rehearsal G=%d failed: %s" % (G, r.stderr[-2000:]))
        d = json.loads(r.stdout.strip().splitlines()[-1])
        rehearsal["values"][str(G)] = d["node_estimate"]
        rehearsal["per_rank"][str(G)] = d["per_rank"]
        rehearsal["spread_max_over_min"][str(G)] = d["node_spread"]
        rehearsal["proofs_in_flight"][str(G)] = d["inflight_per_rank"]
        rehearsal["hw_queues"][str(G)] = hw_queues_for(G)
        rehearsal["msm_reruns"][str(G)] = d["msm_reruns"]
        rehearsal["device_memory"][str(G)] = d.get("device_memory")
        if d.get("slowest_rank_with_exchange_ns"):
            rehearsal["slowest_rank_with_exchange_ns"] = {str(G): d["slowest_rank_with_exchange_ns"]}
    return rehearsal


T_START = time.perf_counter()
PHASE = ["start"]


def heartbeat(period=30.0):
    """a progress line on stderr every `period` s (long silent phases: the rehearsal children, the 1-core
    CPU leg of ~220 s), so a supervisor watching the output sees the run alive"""
    import threading

    def beat():
        while True:
            time.sleep(period)
            sys.stderr.write("bench.py: %.0f s, %s\n" % (time.perf_counter() - T_START, PHASE[0]))
            sys.stderr.flush()

    threading.Thread(target=beat, daemon=True).start()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c3", choices=["c3", "c2"],
                    help="c3: full prove + commit (BASELINE configs C3-C5); c2: sumcheck-only, commitment stubbed")
    ap.add_argument("--log-n", type=int, default=None, help="default 20 (c3) / 18 (c2)")
    ap.add_argument("--log-v", type=int, default=5)
    ap.add_argument("--kind", type=int, default=3, help="3 circuit-3n (distinct witnesses), 0 uniform-3n, 1 ref-shaped")
    ap.add_argument("--witnesses", type=int, default=0, help="distinct witnesses (kind 3; default: one per proof of a step)")
    ap.add_argument("--mode", default="fs", choices=["fs", "injected"])
    ap.add_argument("--cpu-log-n", type=int, default=20,
                    help="1-core CPU baseline (cpu_baseline) size: the metric's 2^20 by default (one proof, ~220 s, run "
                    "last; skipped if the run has already taken --cpu-budget-s, the committed record then stands in)")
    ap.add_argument("--cpu-small-log-n", type=int, default=16, help="extra 1-core sample size (one proof ~17 s)")
    ap.add_argument("--cpu-budget-s", type=float, default=330.0,
                    help="wall seconds of the run after which the long 1-core leg is skipped")
    ap.add_argument("--cpu-all-log-n", type=int, default=20,
                    help="all-cores CPU baseline sample size (default: the metric's 2^20, one proof ~30 s on 16 cores)")
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-stats", action="store_true")
    ap.add_argument("--no-cached", action="store_true",
                    help="skip the index-cached transcript runs (profiling: one launch mix in the whole process)")
    ap.add_argument("--no-c2", action="store_true", help="skip the C2 (sumcheck-only) line of the default run")
    ap.add_argument("--shard", default="proof", choices=["batch", "proof"],
                    help="N > 1 headline: 'proof' = every proof split over all ranks (strong, per-round exchange); "
                    "'batch' = every rank proves its own proofs (weak, no data-path exchange)")
    ap.add_argument("--no-other", action="store_true", help="N > 1: skip the other shard mode's measurement")
    ap.add_argument("--groups", default="2",
                    help="N >= 4: also measure proof groups of these sizes K (N / K groups of K ranks, every proof sharded "
                    "over its group's K GPUs); '' to skip")
    ap.add_argument("--rehearse", default="2,4,8",
                    help="N = 1: world sizes G for the one-rank rehearsal of a G-GPU proof-sharded node ('' to skip)")
    ap.add_argument("--rehearse-steps", type=int, default=10,
                    help="steps of P proofs timed per rehearsed rank (at most --steps)")
    ap.add_argument("--comm", default="shm", choices=["shm", "rccl"],
                    help="N > 1 headline transport: on-node shared memory (default) or RCCL AllGather (one communicator "
                    "per rank shared by the proofs in flight through the ordered exchange hub; proof groups stay on shm). "
                    "The other transport is measured beside it (value_comm_<other>) unless --one-comm")
    ap.add_argument("--one-comm", action="store_true", help="N > 1: measure the headline transport only")
    ap.add_argument("--comm-deadline", type=float, default=300.0,
                    help="N > 1: seconds the second transport's measurement may take before the line is printed without it")
    ap.add_argument("--launch-only", action="store_true",
                    help="start the ranks and report RANK / WORLD_SIZE without any HIP call (launcher test)")
    ap.add_argument("--inflight", type=int, default=0,
                    help="proofs in flight per rank (worker contexts); default: 16 for unsharded and 2-rank proofs, "
                    "8 x G (at most 64) for proofs sharded over G >= 4 ranks (inflight_for)")
    ap.add_argument("--proofs-per-step", type=int, default=64,
                    help="proofs per step (a multiple of --inflight); the K steps run as one pipeline of K x P proofs")
    args = ap.parse_args()
    heartbeat()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # the driver's `python bench.py --gpus N`: this process becomes the launcher of N ranks
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    stub = args.config == "c2"
    log_n = args.log_n or (18 if stub else 20)
    log_v = args.log_v
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and args.gpus != 1:
        raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    if args.launch_only:
        return launch_only(rank, world, local)
    dist = init_dist(rank, world) if world > 1 else None

    # host waits sleep rather than spin: with many proofs in flight the cores go to the transcript
    # hashing pool of spx_prove_many (measured: 31.2 vs 28.2 M constraints/s at 2^20 on one MI355X)
    os.environ.setdefault("SPX_BLOCKING_SYNC", "1")
    # hardware queues per process (HIP default 4): a proof's small latency-bound kernels (sumcheck
    # rounds, bucket-weighting levels) then queue behind fewer of the other proofs' MSM launches
    # (set for G >= 4 even where the environment presets HIP's default 4; kept from the environment
    # otherwise, so an A/B can vary it)
    if world >= 4:
        os.environ["GPU_MAX_HW_QUEUES"] = str(hw_queues_for(world))
        os.environ.setdefault("SPX_SYNC_POLL_US", str(sync_poll_for(world)))
    else:
        os.environ.setdefault("GPU_MAX_HW_QUEUES", str(hw_queues_for(world)))
    # contexts of the unsharded (batch) proofs (C2: one per lockstep group of C2_GROUP proofs)
    Bb = max(1, (args.inflight or C2_INFLIGHT) // C2_GROUP) if stub else (args.inflight or inflight_for(1))
    Bs = args.inflight or inflight_for(world)  # contexts of the proofs sharded over all ranks
    Bm = max(Bb, Bs, inflight_for(2))
    P = max(Bm, (args.proofs_per_step + Bm - 1) // Bm * Bm)  # proofs per step; each worker proves P / B of them
    # the G-GPU rehearsals first, in child processes, while this process holds no GPU queue (run_rehearsal)
    PHASE[0] = "rehearsals"
    rehearsal = run_rehearsal(args, log_n, log_v, P) if world == 1 and args.rehearse and not stub else None
    PHASE[0] = "setup and headline"
    spx = load_product()
    L = spx.lib()
    # SPX_BENCH_SAME_GPU=1: every rank on GPU 0 (multi-rank rehearsal on a one-GPU box)
    device = 0 if os.environ.get("SPX_BENCH_SAME_GPU") == "1" else local
    sharded_head = world > 1 and args.shard == "proof"
    need_batch = world == 1 or not sharded_head or not args.no_other
    need_sharded = world > 1 and (sharded_head or not args.no_other)

    def attach(cs, comm):
        """put the sharded contexts on one transport; returns the RCCL hub (stats) or None"""
        if comm == "rccl":
            # ONE communicator per rank; every proof in flight exchanges through its own channel of
            # the ordered hub (comm_hub.cpp), context j on channel j on every rank
            uid = [spx.comm_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(uid, src=0)
            hub = spx.ExchangeHub.rccl(uid[0], rank, world, device)
            for j, c in enumerate(cs):
                c.set_comm_hub(hub, j)
            return hub
        name = [spx.shm_name() if rank == 0 else None]
        dist.broadcast_object_list(name, src=0)
        for j, c in enumerate(cs):
            c.set_comm_shm("%s_%d" % (name[0], j), rank, world)
        return None

    def make_sharded(k):
        cs = [spx.Context(device) for _ in range(k)]
        for c in cs:
            c.set_lvl0_batch(lvl0_for(world))
        return cs, attach(cs, args.comm)

    if not need_batch:
        ctxs = []
    elif stub:
        ctxs = c2_contexts(spx, device, Bb * C2_GROUP)
    else:
        ctxs = [spx.Context(device) for _ in range(Bb)]
    sctxs, hub = make_sharded(Bs) if need_sharded else ([], None)
    ctx = (ctxs or sctxs)[0]
    # the world size each rank's product communicator spans (one allgather of the rank ids on it)
    seen = comm_seen(sctxs[0], rank, world) if sctxs else world
    ranks_seen = [seen]
    if dist is not None:
        ranks_seen = [None] * world
        dist.all_gather_object(ranks_seen, seen)

    n = 1 << log_n
    W = (args.witnesses or P) if args.kind == 3 else 1
    t0 = time.perf_counter()
    syn, mats, zs, nnz = synth_instance(spx, args.kind, log_n, log_v, 0x5EED0000 + log_n, W, 0xB0B0)
    t_gen = time.perf_counter() - t0
    t0 = time.perf_counter()
    pp = None if stub else spx.MLProofForR1CS.setup(ctx, log_n, 0xC0FFEE)
    t_setup = time.perf_counter() - t0
    t0 = time.perf_counter()
    pk = spx.IndexPK(ctxs[0], index_from_c(spx, ctxs[0], mats), log_n) if ctxs else None
    spk = spx.IndexPK(sctxs[0], index_from_c(spx, sctxs[0], mats), log_n) if sctxs else None
    wits = [spx.Witness(ctx, z[: 32 << log_v], z[32 << log_v :]) for z in zs]
    v0 = zs[0][: 32 << log_v]
    del zs
    t_index = time.perf_counter() - t0

    def barrier():
        if dist is not None:
            dist.barrier()

    cpu_busy = {}  # this process's CPU seconds (all threads) per second of a timed run, by label

    def timed(fn, label=None):
        barrier()
        t0, c0 = time.perf_counter(), time.process_time()
        r = fn()
        c1 = time.process_time()
        barrier()
        el = time.perf_counter() - t0
        if label:
            cpu_busy[label] = round((c1 - c0) / el, 2)
        return r, el

    def batch_fn(cs, k, steps, cached=False):
        wl = [wits[i % W] for i in range(P * steps)]
        return lambda: spx.MLArgumentForR1CS.prove_many(cs, k, wl, pp, mode=args.mode, seed=7, cached=cached,
                                                        commitment_stub=stub)

    def single_fn(c, k, cached=False):
        def run():
            for _ in range(args.steps):
                r = spx.MLArgumentForR1CS.prove_witness(k, wits[0], pp, mode=args.mode, seed=7, cached=cached,
                                                        commitment_stub=stub)
            return r
        return run

    def check_batch(proofs, ref=None):
        ref = ref or proofs[:W]
        assert all(p == ref[i % W] for i, p in enumerate(proofs)), "proofs of the same witness differ"
        assert len(set(ref)) == len(ref), "distinct witnesses gave equal proofs"
        return ref

    # headline configuration
    hctxs, hpk = (sctxs, spk) if sharded_head else (ctxs, pk)
    hctx = hctxs[0]
    # proofs in flight capped by device memory: one probe proof (uncached and index-cached) on the
    # first context measures a context's footprint; every rank keeps the same count (min over ranks)
    grouped = stub and not sharded_head  # C2: each context proves C2_GROUP proofs in lockstep

    def probe():
        for cached in (False, True):
            if grouped:  # a group's scratch is ~C2_GROUP times one proof's: probe with one whole group
                spx.MLArgumentForR1CS.prove_many([hctxs[0]], hpk, [wits[i % W] for i in range(C2_GROUP)], pp,
                                                 mode=args.mode, seed=7, cached=cached, commitment_stub=stub)
            else:
                spx.MLArgumentForR1CS.prove_witness(hpk, wits[0], pp, mode=args.mode, seed=7, cached=cached,
                                                    commitment_stub=stub)
    nfit, mem_fit = fit_inflight(hctxs, probe)
    if dist is not None:
        import torch

        tf = torch.tensor([nfit], dtype=torch.int64)
        dist.all_reduce(tf, op=dist.ReduceOp.MIN)
        nfit = int(tf[0])
    if nfit < len(hctxs):
        sys.stderr.write("bench.py: %d of %d contexts fit the device memory (%s)\n" % (nfit, len(hctxs), mem_fit))
        del hctxs[nfit:]
    mem_fit["contexts"] = len(hctxs)
    batch_fn(hctxs, hpk, max(1, args.warmup))()
    if not args.no_stats:
        spx._check(L.spx_kernel_stats_enable(hctx.h, 1))
    # ---- timed region (headline): K steps x P full proofs, pipelined over B workers
    hs0, hp0 = spx.hash_stats(), spx.host_phase_stats()
    proofs, elapsed = timed(batch_fn(hctxs, hpk, args.steps), "headline")
    hs1, hp1 = spx.hash_stats(), spx.host_phase_stats()
    stats = {}
    if not args.no_stats:
        stats = kernel_stats(spx, L, hctx, args.steps * (P // len(hctxs)))  # ctx 0 proves P / B proofs per step
        spx._check(L.spx_kernel_stats_enable(hctx.h, 0))
    ref = check_batch(proofs)
    # ---- single-proof latency (one proof at a time), with and without the index-cached transcript.
    # Kernel durations with one proof at a time (no other proof sharing the GPU) come from the
    # per-proof-absorbed loop: the same launch mix as the batched proofs (level 0 as its own MSM)
    if not args.no_stats:
        spx._check(L.spx_kernel_stats_enable(hctx.h, 1))
    p1, elapsed_single = timed(single_fn(hctx, hpk))
    assert p1 == ref[0], "single proof differs from the batched one"
    phases = hctx.last_timings()
    alone = {}
    if not args.no_stats:
        alone = kernel_stats(spx, L, hctx, args.steps)
        spx._check(L.spx_kernel_stats_enable(hctx.h, 0))
    elapsed_single_c = elapsed_cached = None
    phases_c = {}
    if not args.no_cached:
        p1c, elapsed_single_c = timed(single_fn(hctx, hpk, cached=True))
        assert p1c == ref[0], "cached-transcript single proof differs"
        phases_c = hctx.last_timings()
    # ---- index-cached transcript throughput (matrix absorption moved to index time; bit-identical)
    if not args.no_cached:
        # one untimed step first: every context's workspaces grow to the cached form's batches (an
        # unsharded cached proof runs level 0 inside its first opening batch) outside the timed region
        batch_fn(hctxs, hpk, 1, cached=True)()
        p2, elapsed_cached = timed(batch_fn(hctxs, hpk, args.steps, cached=True), "index_cached")
        check_batch(p2, ref)
    # ---- N > 1: the other shard mode (throughput, and the proof-sharded single-proof latency)
    other = None
    if world > 1 and not args.no_other:
        octxs, opk = (ctxs, pk) if sharded_head else (sctxs, spk)
        batch_fn(octxs, opk, 1)()
        p3, el = timed(batch_fn(octxs, opk, args.steps))
        check_batch(p3, ref)
        el1 = None
        if not sharded_head:
            p4, el1 = timed(single_fn(octxs[0], opk))
            assert p4 == ref[0], "proof-sharded single proof differs"
        other = [el, el1]
    if hub is not None:
        hub_stats = hub.stats()
        hub.close()
    else:
        hub_stats = None
    # ---- N >= 4: proof groups (every proof sharded over K ranks, N / K groups side by side)
    grouped = {}
    if world >= 4 and not args.no_other and args.groups and not stub:
        for K in [int(x) for x in args.groups.split(",") if x.strip()]:
            if K < 2 or K >= world or world % K:
                continue
            gname = [spx.shm_name() if rank == 0 else None]
            dist.broadcast_object_list(gname, src=0)
            gctxs = [spx.Context(device) for _ in range(args.inflight or inflight_for(K))]
            for j, c in enumerate(gctxs):
                c.set_lvl0_batch(lvl0_for(K))
                c.set_comm_shm("%s_g%d_%d" % (gname[0], rank // K, j), rank % K, K)
            gpk = spx.IndexPK(gctxs[0], index_from_c(spx, gctxs[0], mats), log_n)
            batch_fn(gctxs, gpk, 1)()
            pg, elg = timed(batch_fn(gctxs, gpk, args.steps), "groups_%d" % K)
            check_batch(pg, ref)
            # the same groups with the index-cached transcript: a group's K ranks absorb the matrices
            # of all its proofs (proof i by its rank i mod K), i.e. N / K times the hashing of the
            # proof-sharded headline on the same host; this separates that host cost from the GPU's
            pgc, elgc = timed(batch_fn(gctxs, gpk, args.steps, cached=True), "groups_%d_index_cached" % K)
            check_batch(pgc, ref)
            grouped[K] = (elg, elgc)
            del gctxs, gpk

    ms = elapsed / args.steps * 1e3  # per step (P proofs)
    ms_c = elapsed_cached / args.steps * 1e3 if elapsed_cached else 0.0
    ms_1 = elapsed_single / args.steps * 1e3
    ms_1c = elapsed_single_c / args.steps * 1e3 if elapsed_single_c else 0.0
    ms_o = ms_o1 = None
    ms_g = {}
    if dist is not None:
        import torch

        for K in sorted(grouped):  # max over ranks, in the same order on every rank
            tg = torch.tensor([grouped[K][0] / args.steps * 1e3, grouped[K][1] / args.steps * 1e3], dtype=torch.float64)
            dist.all_reduce(tg, op=dist.ReduceOp.MAX)
            ms_g[K] = (float(tg[0]), float(tg[1]))
        t = torch.tensor([ms, ms_c, ms_1, ms_1c, (other[0] / args.steps * 1e3) if other else 0.0,
                          (other[1] / args.steps * 1e3) if other and other[1] else 0.0], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ms, ms_c, ms_1, ms_1c = float(t[0]), float(t[1]), float(t[2]), float(t[3])
        if other:
            ms_o, ms_o1 = float(t[4]), (float(t[5]) or None)
    # whole-job throughput: in batch mode every rank proves P proofs per step, sharded all ranks share them
    jobs = P * (1 if sharded_head else world)
    def make_out():  # rank 0: the JSON line
        roof = None
        if alone:
            if stub:
                roof = roofline_hbm(alone, PMC_FILE_C2 if log_n == 18 else None)
            else:
                dom = "msm_acc_g2" if "msm_acc_g2" in alone else max(alone, key=lambda k: alone[k]["ms"])
                roof = roofline_valu(alone, dom)
                if dom in stats:  # the same kernel while 16 proofs share the GPU
                    d = stats[dom]
                    roof["avg_launch_us_shared"] = round(d["ms"] / d["launches"] * 1e3, 2)
                hb = roofline_hbm(alone, PMC_FILE if log_n == 20 else None)
                if hb:
                    roof["hbm_kernels"] = hb
                if world == 1:
                    wp = whole_proof_valu(ms / P)
                    if wp:
                        roof["whole_proof"] = wp
        cpu = cpu_all = parity = None
        if world == 1 and not args.no_cpu:
            def gpu_pp_bytes(k):
                # the GPU keygen's PP (seed 0xC0FFEE, as the oracle's keygen would make it), loaded into the
                # oracle: a CPU keygen at 2^16+ would dominate the run
                if k == log_n and pp is not None:
                    return pp.serialize_uncompressed()
                pp_s = spx.MLProofForR1CS.setup(ctx, k, 0xC0FFEE)
                b = pp_s.serialize_uncompressed()
                del pp_s
                return b

            # the 1-core sample at the small size now; the one at the metric's size runs last (run_cpu1)
            PHASE[0] = "CPU baselines (small sample, all cores)"
            one_log_n = args.cpu_small_log_n if not stub else 16
            cpu = cpu_baseline(args.kind, one_log_n, log_v, args.cpu_seconds, stub=stub, max_reps=1,
                               pp_bytes=None if stub else gpu_pp_bytes(one_log_n))
            all_log_n = args.cpu_all_log_n if not stub else log_n
            pp_bytes = None if stub else gpu_pp_bytes(all_log_n)
            oracle_proof = []
            cpu_all = cpu_baseline(args.kind, all_log_n, log_v, args.cpu_seconds, threads=host_cores(), pp_bytes=pp_bytes,
                                   stub=stub, max_reps=1, out_proof=oracle_proof)
            del pp_bytes
            if all_log_n == log_n and args.kind == 3 and args.mode == "fs" and oracle_proof:
                # the oracle just proved witness 0xB0B0 under the same index and PP: the GPU's ref[0]
                parity = oracle_proof[0] == ref[0]
                if not parity:
                    sys.stderr.write("bench.py: PARITY FAILURE: the GPU proof differs from the oracle's at 2^%d\n" % log_n)
        wl = "%s R1CS 2^%d constraints, |v|=%d, nnz=%d, %s, %s transcript, %s, %d proofs per step, %d in flight" % (
            KIND_NAMES.get(args.kind, str(args.kind)), log_n, 1 << log_v, nnz,
            "sumcheck-only, commitment stubbed (BASELINE C2)" if stub else "full prove + commit + 2 openings",
            args.mode.upper(), ("one index, %d distinct witnesses" % W) if args.kind == 3 else "one witness", P,
            len(hctxs) * (C2_GROUP if stub and not sharded_head else 1))
        if stub and not sharded_head:
            wl += " (%d lockstep groups of %d)" % (len(hctxs), C2_GROUP)
        out = {
            "metric": "R1CS constraints proved/sec at 2^%d%s" % (log_n, " (sumcheck-only, commitment stubbed)" if stub else ""),
            "value": round(jobs * n / (ms / 1e3), 1),
            "unit": "constraints/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            # --shard proof (default): the same proofs split over however many ranks (N = 1 included)
            "scaling": "strong" if (sharded_head or (world == 1 and args.shard == "proof")) else "weak",
            "vs_baseline": None,
            "dtype": "bls12-381 Fr/Fq Montgomery (u32 limbs)",
            "data": "synthetic",
            "config": {
                "workload": wl,
                "log_n": log_n,
                "baseline_config": "C2" if stub else "C3",
                "distinct_witnesses": W,
                "proofs_per_step": P,
                "proofs_in_flight": len(hctxs) * (C2_GROUP if stub and not sharded_head else 1),
                "lockstep_group": C2_GROUP if stub and not sharded_head else 1,
                "parallelism": ("proof-sharded over %d ranks" % world) if sharded_head else ("%d independent ranks" % world),
                "comm": args.comm if sctxs else None,
                "hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES", "0")) or None,  # hardware queues per process
            },
            "ms_per_proof_single": round(ms_1, 3),
            "value_single_proof": round(n / (ms_1 / 1e3), 1),
            "ms_per_proof_single_cached_transcript": round(ms_1c, 3) if ms_1c else None,
            "value_single_proof_cached_transcript": round(n / (ms_1c / 1e3), 1) if ms_1c else None,
            "value_index_cached_transcript": round(jobs * n / (ms_c / 1e3), 1) if ms_c else None,
            "ms_per_step_index_cached_transcript": round(ms_c, 3) if ms_c else None,
            "phases_ms": {k: round(v / 1e3, 3) for k, v in phases.items()},
            "phases_ms_cached_transcript": {k: round(v / 1e3, 3) for k, v in phases_c.items()},
            "kernels_ms_per_proof": {k: round(v["ms"], 3) for k, v in alone.items()},
            "kernels_ms_per_proof_shared": {k: round(v["ms"], 3) for k, v in stats.items()},
            "roofline": roof,
            "cpu_baseline": cpu,
            "cpu_baseline_all_cores": cpu_all,
            "setup_s": round(t_setup, 2),
            "index_s": round(t_index, 2),
            "gen_s": round(t_gen, 2),
            "proof_bytes": len(ref[0]),
            # the first witness's proof byte-equal to the test oracle's, proved in this run (cpu_baseline_all_cores)
            "parity_2_%d" % log_n: parity,
            "ranks_seen": ranks_seen,
            "device_memory": mem_fit,
        }
        if hub_stats is not None:
            out["comm_%s_hub_stats_rank0" % args.comm] = hub_stats
        # host side: the machine's cores, the ones this process uses, and how many of them the per-proof
        # sequential Blake2s absorption of A, B, C keeps busy at the measured rate (proofs/s x seconds each)
        # (the pool's own clock over the timed region: multi-buffer lanes hash several proofs per job)
        hash_s = phases.get("transcript_matrices", 0.0) / 1e6
        pool_s, pool_n = hs1[0] - hs0[0], hs1[1] - hs0[1]
        if world == 1 and log_n == 20 and not stub and args.kind == 3:
            # the headline's baseline at the metric's own size: one core, 2^20 (committed record)
            c1 = committed_record(CPU1_2_20_FILE)
            if c1:  # the cross-check of the in-run 1-core 2^20 leg (run last, make_out)
                c1["gpu_value_over_it"] = round(out["value"] / c1["value"], 1)
                out["cpu_baseline_1core_2_20_record"] = c1
        c5 = committed_record(C5_FILE)
        if c5 and not stub:
            out["c5_parity_2_24"] = {"equal": c5.get("equal"), "ranks": c5.get("ranks"), "proof_bytes": c5.get("proof_bytes"),
                                     "oracle_cores": c5.get("oracle_threads"), "oracle_s": c5.get("oracle_s"),
                                     "oracle_constraints_per_s": round((1 << 24) / c5["oracle_s"], 1) if c5.get("oracle_s") else None,
                                     # the revision the record pins (round 5's record predates the field:
                                     # it was made at 239b49d)
                                     "commit": c5.get("commit") or "239b49d",
                                     "source": c5["source"]}
        out["host"] = {"cpu_count": os.cpu_count(), "cores_used": host_cores(),
                       "hashing_lanes": hs1[2],
                       "hashing_core_s_per_proof": round(pool_s / pool_n, 4) if pool_n else None,
                       "hashing_s_single_proof_scalar": round(hash_s, 4),
                       "hashing_cores_busy": round(pool_s / elapsed, 2) if pool_n else 0.0,
                       # summed over the proof workers: time a proof waited for its absorption
                       "hashing_wait_ms_per_proof": round((hs1[3] - hs0[3]) / pool_n * 1e3, 2) if pool_n else None,
                       # the whole process's CPU use (proof workers, HIP runtime, hashing pool) in cores
                       "process_cores_busy": cpu_busy,
                       # the proving threads' CPU per proof by prove() phase over the headline run (ms); a
                       # rank of a sharded proof does all of it for every proof (it does not divide by N)
                       "proving_thread_cpu_ms_per_proof": {
                           k: round((hp1[k][0] - hp0[k][0]) / max(1, len(proofs)) * 1e3, 3) for k in hp1}}
        for K, (mg, mgc) in ms_g.items():
            out.setdefault("value_proof_groups", {})[str(K)] = {
                "value": round(P * (world // K) * n / (mg / 1e3), 1), "ms_per_step": round(mg, 3),
                "value_index_cached_transcript": round(P * (world // K) * n / (mgc / 1e3), 1),
                "layout": "%d groups of %d ranks, every proof sharded over its group (%d proofs per group per step)" % (
                    world // K, K, P)}
        if ms_o is not None:
            if sharded_head:  # the other mode: every rank proves whole proofs
                out["value_batch_weak"] = round(P * world * n / (ms_o / 1e3), 1)
                out["ms_per_step_batch_weak"] = round(ms_o, 3)
            else:
                out["value_proof_sharded"] = round(P * n / (ms_o / 1e3), 1)
                out["ms_per_step_proof_sharded"] = round(ms_o, 3)
                out["ms_per_proof_single_proof_sharded"] = round(ms_o1, 3) if ms_o1 else None
        if rehearsal:
            rehearsal["over_n1"] = {g: round(v / out["value"], 3) for g, v in rehearsal["values"].items()}
            rehearsal["over_n1_rank0"] = {g: round(pr["0"] / out["value"], 3) for g, pr in rehearsal["per_rank"].items()
                                          if pr and "0" in pr}
            if rehearsal.get("slowest_rank_with_exchange_ns"):
                rehearsal["over_n1_with_exchange"] = {g: {ns: round(v / out["value"], 3) for ns, v in d.items()}
                                                      for g, d in rehearsal["slowest_rank_with_exchange_ns"].items()}
            out["proof_sharded_rehearsal"] = rehearsal
        if not stub and world == 1 and not args.no_c2:
            PHASE[0] = "C2 line"
            out["c2"] = c2_line(spx, L, args, args.inflight or C2_INFLIGHT)
        if cpu is not None:
            PHASE[0] = "1-core CPU baseline at 2^%d" % args.cpu_log_n
            # cpu_baseline: one core at the metric's size, timed in this run (last: ~220 s of CPU)
            out["cpu_baseline_1core_2_%d" % one_log_n] = cpu
            out["cpu_baseline"] = cpu
            big = args.cpu_log_n
            if big != one_log_n and not stub:
                if time.perf_counter() - T_START > args.cpu_budget_s:
                    out["cpu_baseline_note"] = ("the 1-core 2^%d leg was skipped: the run had taken %.0f s (> %.0f s); "
                                                "cpu_baseline is the 2^%d sample, cpu_baseline_1core_2_20 the committed record"
                                                % (big, time.perf_counter() - T_START, args.cpu_budget_s, one_log_n))
                else:
                    p1 = []
                    c1 = cpu_baseline(args.kind, big, log_v, args.cpu_seconds, max_reps=1, out_proof=p1,
                                      pp_bytes=pp.serialize_uncompressed() if big == log_n and pp is not None else None)
                    if big == log_n and args.kind == 3 and args.mode == "fs" and p1:
                        c1["proof_equals_gpu"] = p1[0] == ref[0]  # the GPU's proof of the same witness
                    c1["gpu_value_over_it"] = round(out["value"] / c1["value"], 1)
                    out["cpu_baseline"] = c1
                    out["cpu_baseline_1core_2_%d" % big] = c1
                    rec = out.get("cpu_baseline_1core_2_20_record")
                    if rec and big == 20:
                        c1["committed_record_value"] = rec["value"]
        return out

    out = make_out() if rank == 0 else None
    # ---- N > 1, last: the same proof-sharded pipeline on the other transport (shm <-> RCCL over xGMI), so
    # one run reports both. The contexts, index and witnesses stay; only their communicator changes. It
    # runs after the headline is complete, under a watchdog: if the transport hangs (a collective that
    # never completes), rank 0 prints the line without it after --comm-deadline seconds and every rank
    # exits, so a failing second transport never costs the headline.
    if sctxs and not args.one_comm:
        alt = "rccl" if args.comm == "shm" else "shm"
        if alt == "rccl" and os.environ.get("SPX_BENCH_SAME_GPU") == "1":
            if out is not None:
                out["value_comm_%s" % alt] = None
                out["comm_%s_skipped" % alt] = "every rank on GPU 0: RCCL refuses two ranks on one device"
        else:
            import threading

            def expire():
                if out is not None:
                    out["value_comm_%s" % alt] = None
                    out["comm_%s_error" % alt] = "did not finish within %d s" % args.comm_deadline
                    print(json.dumps(out), flush=True)
                sys.stderr.flush()
                os._exit(0)

            dog = threading.Timer(args.comm_deadline, expire)
            dog.daemon = True
            dog.start()
            try:
                hub_x = attach(sctxs, alt)
                batch_fn(sctxs, spk, 1)()
                px, elx = timed(batch_fn(sctxs, spk, args.steps))
                check_batch(px, ref)
                err = None
            except Exception as e:  # recorded; the other ranks' collectives end by the watchdog
                hub_x, elx, err = None, 0.0, repr(e)
            import torch

            tx = torch.tensor([elx / args.steps * 1e3], dtype=torch.float64)
            dist.all_reduce(tx, op=dist.ReduceOp.MAX)
            dog.cancel()
            if out is not None:
                if err is None:
                    ms_x = float(tx[0])
                    out["value_comm_%s" % alt] = round(jobs * n / (ms_x / 1e3), 1)
                    out["ms_per_step_comm_%s" % alt] = round(ms_x, 3)
                    if hub_x is not None:
                        out["comm_%s_hub_stats_rank0" % alt] = hub_x.stats()
                else:
                    out["value_comm_%s" % alt] = None
                    out["comm_%s_error" % alt] = err
            if hub_x is not None:
                hub_x.close()  # the contexts keep it alive
    if out is None:
        if dist is not None:
            dist.destroy_process_group()
        return
    print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def c2_line(spx, L, args, B):
    """BASELINE config C2 beside the headline: 2^18 circuit-3n, sumcheck-only (commitment stubbed), the
    same pipeline, its HBM-bound dominant kernel and the oracle's stubbed prover on all host cores."""
    log_n, log_v, P = 18, args.log_v, 64
    n = 1 << log_n
    ctxs = c2_contexts(spx, 0, B)
    syn, mats, zs, nnz = synth_instance(spx, 3, log_n, log_v, 0x5EED0000 + log_n, P, 0xB0B0)
    pk = spx.IndexPK(ctxs[0], index_from_c(spx, ctxs[0], mats), log_n)
    wits = [spx.Witness(ctxs[0], z[: 32 << log_v], z[32 << log_v :]) for z in zs]
    steps = max(1, args.steps)
    run = lambda k: spx.MLArgumentForR1CS.prove_many(ctxs, pk, wits * k, None, mode=args.mode, seed=7,
                                                     commitment_stub=True)
    run(1)
    hs0 = spx.hash_stats()
    t0 = time.perf_counter()
    proofs = run(steps)
    el = time.perf_counter() - t0
    hs1 = spx.hash_stats()
    assert all(p == proofs[i % P] for i, p in enumerate(proofs))
    spx._check(L.spx_kernel_stats_enable(ctxs[0].h, 1))
    t0 = time.perf_counter()
    for _ in range(steps):
        p1 = spx.MLArgumentForR1CS.prove_witness(pk, wits[0], None, mode=args.mode, seed=7, cached=True,
                                                 commitment_stub=True)
    el1 = (time.perf_counter() - t0) / steps
    stats = kernel_stats(spx, L, ctxs[0], steps)
    spx._check(L.spx_kernel_stats_enable(ctxs[0].h, 0))
    assert p1 == proofs[0]
    # one lockstep group alone (the launches the pipeline runs: each step of C2_GROUP proofs in one launch)
    spx._check(L.spx_kernel_stats_enable(ctxs[0].h, 1))
    for _ in range(steps):
        pg = spx.MLArgumentForR1CS.prove_many([ctxs[0]], pk, wits[:C2_GROUP], None, mode=args.mode, seed=7, cached=True,
                                              commitment_stub=True)
    gstats = kernel_stats(spx, L, ctxs[0], steps * C2_GROUP)
    spx._check(L.spx_kernel_stats_enable(ctxs[0].h, 0))
    assert pg == proofs[:C2_GROUP]
    rgroup = roofline_hbm(gstats, None)
    if rgroup:
        # traffic: the group kernel's own PMC pass (profiles/pmc_kernels_c2.json: the C2 profile run proves
        # its proofs in a group), e.g. k_sc1_wave<...> -> k_sc1_wave_group<...>
        sym = rgroup["kernel"]
        gsym = sym.split("<")[0] + "_group" + (sym[sym.index("<"):] if "<" in sym else "")
        try:
            gk = json.load(open(PMC_FILE_C2)).get("kernels", {}).get(gsym) or {}
        except (OSError, ValueError):
            gk = {}
        rgroup["traffic"] = gk.get("traffic_bytes_largest")
        rgroup["traffic_kernel"] = gsym if gk else None
        rgroup["note"] = ("one lockstep group of %d proofs alone: algorithmic bytes of the kernel's largest group "
                          "launch (all %d proofs) / its HIP-event duration; traffic from the group kernel's PMC "
                          "passes" % (C2_GROUP, C2_GROUP))
    # the same pipeline with the matrices absorbed once at index time (bit-identical proofs): the GPU
    # side's capacity, which the per-proof host hashing hides in `value`
    t0 = time.perf_counter()
    pc = spx.MLArgumentForR1CS.prove_many(ctxs, pk, wits * steps, None, mode=args.mode, seed=7, cached=True,
                                          commitment_stub=True)
    elc = time.perf_counter() - t0
    assert all(p == proofs[i % P] for i, p in enumerate(pc))
    res = {
        "metric": "R1CS constraints proved/sec at 2^18 (sumcheck-only, commitment stubbed)",
        "value": round(steps * P * n / el, 1),
        "unit": "constraints/s",
        "workload": "circuit-3n 2^18, |v|=%d, nnz=%d, %d distinct witnesses, FS transcript, %d in flight "
                    "(%d lockstep groups of %d)" % (1 << log_v, nnz, P, len(ctxs) * C2_GROUP, len(ctxs), C2_GROUP),
        "ms_per_proof_single_cached_transcript": round(el1 * 1e3, 3),
        "value_index_cached_transcript": round(steps * P * n / elc, 1),
        "kernels_ms_per_proof": {k: round(v["ms"], 4) for k, v in stats.items()},
        "roofline": roofline_hbm(stats, PMC_FILE_C2),
        "roofline_group": rgroup,
        "hashing_cores_busy": round((hs1[0] - hs0[0]) / el, 2),
    }
    # the whole pipeline against HBM: the algorithmic bytes of every instrumented launch per proof in the
    # pipeline's own launch mix (one lockstep group alone: each step of C2_GROUP proofs in one launch, the
    # SpMV's index streamed once per group), times the proof rate, over 8 TB/s
    alg = sum(v["bytes"] for v in gstats.values())
    if alg:
        rate_c, rate = steps * P / elc, steps * P / el
        res["hbm_pipeline"] = {
            "alg_bytes_per_proof": round(alg, 1), "alg_bytes_per_constraint": round(alg / n, 2),
            "peak_GBs": HBM_PEAK_GBS,
            "frac_index_cached": round(alg * rate_c / (HBM_PEAK_GBS * 1e9), 4),
            "frac_per_proof_absorbed": round(alg * rate / (HBM_PEAK_GBS * 1e9), 4),
            "by_kernel_bytes_per_proof": {k: round(v["bytes"], 1) for k, v in gstats.items()},
            "note": "algorithmic bytes (kp_end of every launch of one lockstep group alone, per proof) x proofs/s of "
                    "the pipeline / 8 TB/s; per-proof-absorbed runs at the hashing pool's rate"}
    if not args.no_cpu:
        op = []
        res["cpu_baseline_all_cores"] = cpu_baseline(3, log_n, log_v, args.cpu_seconds, threads=host_cores(), stub=True,
                                                     max_reps=1, out_proof=op)
        if args.mode == "fs" and op:
            # the oracle's stubbed proof of witness 0xB0B0 against the GPU's proof of the same witness
            res["parity_2_18"] = op[0] == proofs[0]
            if not res["parity_2_18"]:
                sys.stderr.write("bench.py: PARITY FAILURE: the GPU C2 proof differs from the oracle's at 2^18\n")
    return res


if __name__ == "__main__":
    main()
