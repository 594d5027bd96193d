"""BASELINE config C2: "2^18 constraints, sumcheck-only, commitment stubbed" (SURVEY §8(d)).

The stub is defined as the proof prove() (/root/reference/src/lib.rs:58-146) outputs under the
public parameter whose every group element is the identity: the commitment, h and every opening
proof are the point at infinity, while the evaluations of z at (r_v, 0..0) and r_y, both sumchecks
and the transcript are computed in full. That definition is pinned on the CPU (the oracle's stub
equals the oracle's full prove under an all-identity PP), then the GPU stub is checked against the
oracle byte for byte, up to the BASELINE size 2^18 (no MSM work, so the C oracle finishes in
seconds on the box's cores)."""
import os
import struct
import threading

import pytest


def identity_pp_bytes(nv):
    """PublicParameter (ark-serialize uncompressed) with every point = infinity."""
    g1 = bytearray(96)
    g1[48] = 1
    g1[95] |= 0x40
    g2 = bytearray(192)
    g2[96] = 1
    g2[191] |= 0x40
    b = bytearray(struct.pack("<QQ", nv, nv))
    for i in range(nv):
        b += struct.pack("<Q", 1 << (nv - i)) + bytes(g1) * (1 << (nv - i))
    b += struct.pack("<Q", nv)
    for i in range(nv):
        b += struct.pack("<Q", 1 << (nv - i)) + bytes(g2) * (1 << (nv - i))
    return bytes(b + g1 + g2)


@pytest.mark.parametrize("kind,log_n,log_v", [(0, 6, 2), (1, 8, 3), (2, 7, 2)])
@pytest.mark.parametrize("mode", [0, 1])
def test_oracle_stub_is_identity_pp(oc, kind, log_n, log_v, mode):
    param = (3 | (1 << 16)) if kind == 2 else 0
    inst = oc.Instance(kind, log_n, log_v, 500 + log_n, param)
    pp = oc.PP.load(identity_pp_bytes(log_n))
    full = oc.prove(inst.mats, inst.v_bytes, inst.w_bytes, pp, mode, 3)
    stub = oc.prove(inst.mats, inst.v_bytes, inst.w_bytes, None, mode, 3, commitment_stub=True)
    assert full == stub


def test_abi_stub_needs_no_pp_but_full_prove_does(spx):
    """argument checks of the C ABI that run without a GPU: a null pp is refused unless stubbed."""
    with pytest.raises(spx.InvalidArgument):
        spx._pp_handle(None, False)
    assert spx._pp_handle(None, True) is None


@pytest.mark.gpu
@pytest.mark.parametrize("kind,log_n,log_v", [(0, 2, 1), (0, 8, 3), (1, 10, 4), (2, 9, 3), (0, 12, 5)])
@pytest.mark.parametrize("mode", ["fs", "injected"])
def test_gpu_stub_bit_exact(spx, ctx, oc, kind, log_n, log_v, mode):
    param = (3 | (1 << 16)) if kind == 2 else 0
    inst = oc.Instance(kind, log_n, log_v, 600 + log_n, param)
    pk = spx.MLArgumentForR1CS.index(ctx, *[spx.Csr(M.n, M.row_ptr, M.col, M.val) for M in inst.mats])
    got = spx.MLArgumentForR1CS.prove(pk, inst.v_bytes, inst.w_bytes, None, mode=mode, seed=8, commitment_stub=True)
    want = oc.prove(inst.mats, inst.v_bytes, inst.w_bytes, None, 1 if mode == "injected" else 0, 8,
                    commitment_stub=True)
    assert got == want


@pytest.mark.gpu
def test_gpu_full_prove_under_identity_pp_equals_stub(spx, ctx, oc):
    """The product's full path (MSMs included) under the all-identity PP gives the stub's bytes."""
    log_n = 7
    inst = oc.Instance(0, log_n, 3, 777)
    pp = spx.PublicParameter.load(ctx, identity_pp_bytes(log_n))
    pk = spx.MLArgumentForR1CS.index(ctx, *[spx.Csr(M.n, M.row_ptr, M.col, M.val) for M in inst.mats])
    full = spx.MLArgumentForR1CS.prove(pk, inst.v_bytes, inst.w_bytes, pp)
    stub = spx.MLArgumentForR1CS.prove(pk, inst.v_bytes, inst.w_bytes, None, commitment_stub=True)
    assert full == stub


@pytest.mark.gpu
@pytest.mark.parametrize("G", [2, 4])
def test_gpu_stub_sharded(spx, oc, G):
    log_n = 9
    inst = oc.Instance(0, log_n, 3, 900 + G)
    want = oc.prove(inst.mats, inst.v_bytes, inst.w_bytes, None, 0, 0, commitment_stub=True)
    group = spx.CommGroup(G)
    out, errs = [None] * G, []

    def run(r):
        try:
            c = spx.Context(0)
            c.set_comm_group(group, r)
            pk = spx.MLArgumentForR1CS.index(c, *[spx.Csr(M.n, M.row_ptr, M.col, M.val) for M in inst.mats])
            out[r] = spx.MLArgumentForR1CS.prove(pk, inst.v_bytes, inst.w_bytes, None, commitment_stub=True)
        except Exception as e:  # surfaced below
            errs.append(repr(e))

    ths = [threading.Thread(target=run, args=(r,)) for r in range(G)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=300)
    assert not errs, errs
    assert all(o == want for o in out)


@pytest.mark.gpu
def test_gpu_stub_bit_exact_2_18(spx, ctx, oc):
    """BASELINE config C2 at its own size: 2^18 uniform-3n, |v| = 32, FS transcript, byte-equal to the
    reference-faithful C oracle (log_n eq tables, degree-(log_n+2) sumcheck-1, hash-map eval_on_x),
    run on the box's cores."""
    log_n = 18
    inst = oc.Instance(0, log_n, 5, 0x5EED0000 + log_n)
    pk = spx.MLArgumentForR1CS.index(ctx, *[spx.Csr(M.n, M.row_ptr, M.col, M.val) for M in inst.mats])
    got = spx.MLArgumentForR1CS.prove(pk, inst.v_bytes, inst.w_bytes, None, commitment_stub=True)
    oc.set_threads(min(16, os.cpu_count() or 1))
    try:
        want = oc.prove(inst.mats, inst.v_bytes, inst.w_bytes, None, 0, 0, commitment_stub=True)
    finally:
        oc.set_threads(1)
    assert len(got) == len(want) == 18040
    assert got == want
