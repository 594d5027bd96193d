"""bench.py's roofline bookkeeping (host logic, no GPU): the per-launch PMC counters are scaled to the
run's launch size, and the whole-proof VALU rate counts only per-proof kernels."""
import importlib.util
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _pmc():
    return json.load(open(os.path.join(ROOT, "profiles", "pmc_kernels.json")))["kernels"]


def test_valu_roofline_scales_counters_to_the_launch(bench):
    pm = _pmc()["k_accum_aff<Fq2>"]
    alg = pm["alg_bytes_per_launch"]
    full = {"msm_acc_g2": {"launches": 3.0, "ms": 3 * 4.0, "bytes": 3 * alg, "ops": 0.0}}
    half = {"msm_acc_g2": {"launches": 3.0, "ms": 3 * 2.0, "bytes": 3 * alg / 2, "ops": 0.0}}
    a = bench.roofline_valu(full, "msm_acc_g2")
    b = bench.roofline_valu(half, "msm_acc_g2")
    assert a["pmc_share"] == pytest.approx(1.0)
    assert b["pmc_share"] == pytest.approx(0.5)
    assert b["valu_insts_per_launch"] == pytest.approx(a["valu_insts_per_launch"] / 2)
    # half the work in half the time: the same issue rate, the same traffic ratio
    assert b["frac"] == pytest.approx(a["frac"], rel=1e-3)
    assert b["hbm"]["traffic_over_algorithmic"] == pytest.approx(a["hbm"]["traffic_over_algorithmic"], rel=1e-3)
    assert 0 < a["frac"] < 1


def test_whole_proof_valu_excludes_setup_kernels(bench):
    ks = _pmc()
    wp = bench.whole_proof_valu(17.5)
    proofs = ks["k_accum_aff<Fq >"]["launches_valu_pass"]
    setup = sum(v["SQ_INSTS_VALU_per_launch"] * v["launches_valu_pass"] for k, v in ks.items()
                if k.startswith(bench.SETUP_KERNELS) and v.get("SQ_INSTS_VALU_per_launch"))
    every = sum(v["SQ_INSTS_VALU_per_launch"] * v["launches_valu_pass"] for v in ks.values()
                if v.get("SQ_INSTS_VALU_per_launch") and v.get("launches_valu_pass"))
    assert setup > 0
    assert wp["valu_insts_per_proof"] == pytest.approx((every - setup) / proofs, rel=1e-6)
    # the accumulation kernels alone are most of a proof's instructions
    acc = sum(ks[k]["SQ_INSTS_VALU_per_launch"] * ks[k]["launches_valu_pass"] for k in ("k_accum_aff<Fq2>", "k_accum_aff<Fq >"))
    assert acc / proofs < wp["valu_insts_per_proof"] < 1.3 * acc / proofs
    assert 0 < wp["frac"] < 1


def test_settings_by_sharding_degree(bench):
    """proofs in flight / hardware queues / level-0 mode per sharding degree: the
    measured optima, every in-flight count divides the default 64 proofs per step, and the RCCL hub's
    64 channels cover the largest"""
    assert [bench.inflight_for(g) for g in (1, 2, 4, 8, 16)] == [32, 32, 32, 64, 64]
    assert [bench.hw_queues_for(g) for g in (1, 2, 4, 8)] == [4, 4, 32, 32]
    assert [bench.lvl0_for(g) for g in (1, 2, 4, 8)] == [0, 0, 1, 1]
    assert [bench.sync_poll_for(g) for g in (1, 2, 4, 8)] == [0, 0, 50, 50]
    for g in (1, 2, 4, 8):
        assert 64 % bench.inflight_for(g) == 0
        assert bench.hw_queues_for(g) <= 32  # gpurun / the pool refuse more


def test_hbm_largest_launch_rates(bench):
    """every HBM kernel's largest launch: algorithmic MB over its HIP-event duration"""
    r = bench.largest_rate({"largest": {"launches": 2, "ms": 0.1, "bytes": 2 * 176e6}})
    assert r["MB"] == pytest.approx(176.0)
    assert r["us"] == pytest.approx(50.0)
    assert r["GBs"] == pytest.approx(3520.0)
    assert r["frac"] == pytest.approx(0.44)


def test_held_clock_restates_the_roofline(bench):
    """the GRBM_GUI_ACTIVE pass's clock carried to the live launch duration: at the measured duration of
    the PMC pass itself the held clock is the pass's clock, and the cycles per instruction follow"""
    clk = bench.held_clock("k_accum_aff<Fq2>")
    assert clk and 1.5 < clk["effective_clock_GHz"] < 2.5
    pm = _pmc()["k_accum_aff<Fq2>"]
    alg = pm["alg_bytes_per_launch"]
    ms = clk["mean_us"] / 1e3
    r = bench.roofline_valu({"msm_acc_g2": {"launches": 1.0, "ms": ms, "bytes": alg, "ops": 0.0}}, "msm_acc_g2")
    h = r["held_clock"]
    assert h["GHz"] == pytest.approx(clk["effective_clock_GHz"], rel=1e-3)
    want = ms * 1e-3 * 1024 * clk["effective_clock_GHz"] * 1e9 / r["valu_insts_per_launch"]
    assert h["achieved_cycles_per_instr"] == pytest.approx(want, rel=1e-3)
    assert h["frac_at_held_clock"] > r["frac"]  # the held clock's peak is below the 2.4 GHz one


def test_committed_cpu_baselines(bench):
    c1 = bench.committed_record(bench.CPU1_2_20_FILE)
    assert c1["cores"] == 1 and c1["log_n"] == 20 and c1["parity_vs_gpu"] is True
    c5 = bench.committed_record(bench.C5_FILE)
    assert c5["equal"] is True and c5["log_n"] == 24 and c5["ranks"] == 8
