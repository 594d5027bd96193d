"""Lockstep groups (spx_ctx_set_group, csrc/prover.cpp prove_group): spx_prove_many proving k stubbed-
commitment proofs of one index at a time, each sumcheck round of the k proofs in one launch. Every
proof's bytes must equal its own one-at-a-time proof (which tests/test_c2.py pins to the C oracle, up to
BASELINE C2's 2^18), for every group size, a ragged last group, both transcript forms and modes, and at
sizes that take every round kernel: the wave-transposed large rounds with and without the second-launch
reduction, and the small fold rounds."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _instance(spx, ctx, log_n, log_v, nwit):
    sys.path.insert(0, ROOT)
    import bench

    syn, mats, zs, nnz = bench.synth_instance(spx, 3, log_n, log_v, 0x5EED0000 + log_n, nwit, 0xB0B0)
    pk = spx.IndexPK(ctx, bench.index_from_c(spx, ctx, mats), log_n)
    wits = [spx.Witness(ctx, z[: 32 << log_v], z[32 << log_v :]) for z in zs]
    return syn, pk, wits


@pytest.mark.gpu
@pytest.mark.parametrize("log_n", [6, 16])
@pytest.mark.parametrize("mode", ["fs", "injected"])
def test_group_equals_single(spx, ctx, oc, log_n, mode):
    log_v = 3
    syn, pk, wits = _instance(spx, ctx, log_n, log_v, 7)
    want = [spx.MLArgumentForR1CS.prove_witness(pk, w, None, mode=mode, seed=5, commitment_stub=True) for w in wits]
    for k in (2, 3, 8, 16):
        ctxs = [spx.Context(0) for _ in range(2)]
        for c in ctxs:
            c.set_group(k)
        for cached in (False, True):
            got = spx.MLArgumentForR1CS.prove_many(ctxs, pk, wits, None, mode=mode, seed=5, cached=cached,
                                                   commitment_stub=True)
            assert got == want, (k, cached)
    if log_n == 6:  # the oracle's proof of witness 0 (the generator's 0xB0B0 witness) at a small size
        inst = oc.Instance(3, log_n, log_v, 0x5EED0000 + log_n, 0xB0B0)
        assert oc.prove(inst.mats, inst.v_bytes, inst.w_bytes, None, 1 if mode == "injected" else 0, 5,
                        commitment_stub=True) == want[0]


@pytest.mark.gpu
def test_group_c2_size(spx, ctx):
    """BASELINE C2's size, 2^18: a group of 8 and a ragged group of 3, then one group of 11 (group size
    16), against one-at-a-time proofs"""
    log_n, log_v = 18, 5
    syn, pk, wits = _instance(spx, ctx, log_n, log_v, 11)
    want = [spx.MLArgumentForR1CS.prove_witness(pk, w, None, cached=True, commitment_stub=True) for w in wits]
    c = spx.Context(0)
    c.set_group(8)
    assert spx.MLArgumentForR1CS.prove_many([c], pk, wits, None, cached=True, commitment_stub=True) == want
    c.set_group(16)  # one group of 11: more than one tail launch's 8 proofs
    assert spx.MLArgumentForR1CS.prove_many([c], pk, wits, None, cached=True, commitment_stub=True) == want


@pytest.mark.gpu
def test_group_leaves_full_proofs_alone(spx, ctx, oc):
    """a context with a group size still proves full (MSM) proofs one at a time, with their own bytes"""
    log_n, log_v = 8, 3
    syn, pk, wits = _instance(spx, ctx, log_n, log_v, 3)
    pp = spx.MLProofForR1CS.setup(ctx, log_n, 77)
    want = [spx.MLArgumentForR1CS.prove_witness(pk, w, pp) for w in wits]
    c = spx.Context(0)
    c.set_group(4)
    assert spx.MLArgumentForR1CS.prove_many([c], pk, wits, pp) == want


@pytest.mark.gpu
def test_group_size_checked(spx, ctx):
    c = spx.Context(0)
    for bad in (0, 17, -1):
        with pytest.raises(spx.InvalidArgument):
            c.set_group(bad)
    c.set_group(1)


@pytest.mark.gpu
def test_group_with_device_checked_identities(spx, ctx, monkeypatch):
    """SPX_CHECK_DERIVED=1: every round also computes the derived value on the device and checks it, so
    every round of a group takes its G(1) / P(1) form: the large rounds' NEED1 group kernels and the small
    rounds' per-proof launches inside a group (launch_sc1_round_group's fallback). Same bytes."""
    log_n, log_v = 16, 3
    syn, pk, wits = _instance(spx, ctx, log_n, log_v, 5)
    want = [spx.MLArgumentForR1CS.prove_witness(pk, w, None, seed=5, commitment_stub=True) for w in wits]
    monkeypatch.setenv("SPX_CHECK_DERIVED", "1")
    c = spx.Context(0)
    c.set_group(4)
    assert spx.MLArgumentForR1CS.prove_many([c], pk, wits, None, seed=5, commitment_stub=True) == want
