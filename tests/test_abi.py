"""Boundary checks that need no GPU: libspartan_hip.so loads, exports every function declared in
include/spartan_hip.h, its host-only entry points (synthetic generators, proof sizing) agree with
the oracle, and a compute call without a GPU fails loudly (no CPU fallback)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(os.path.join(ROOT, "include", "spartan_hip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"\b(spx_[a-z0-9_]+)\s*\(", src)
    return sorted(set(names))


def test_header_symbols_exported(spx):
    L = spx.lib()
    names = declared_functions()
    assert len(names) >= 30
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    assert set(spx.EXPORTED) <= set(names)
    assert b"gfx950" in L.spx_version()


def test_proof_size_matches_oracle_layout(spx, oc):
    for log_n in (4, 10, 20):
        # spartan.py byte layout: pm1 56, open 32+96+8+96L (x2), infos 16 (x2), sc1, pm4 96, sc2
        L = log_n
        want = 56 + 2 * (32 + 96 + 8 + 96 * L) + 32 + 8 + L * (8 + 32 * (L + 3)) + 96 + 8 + L * (8 + 96)
        assert spx.lib().spx_proof_size(log_n, 5) == want
    assert spx.lib().spx_proof_size(20, 5) == 21272  # matches the 2^20 bench proof length


@pytest.mark.parametrize("kind,log_n,log_v", [(0, 6, 2), (1, 7, 3), (0, 9, 5), (3, 6, 2), (3, 10, 5)])
def test_library_generators_match_oracle(spx, oc, kind, log_n, log_v):
    L = spx.lib()
    L.spx_synth_create.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, ctypes.POINTER(ctypes.c_void_p)]
    L.spx_synth_csr.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(spx._CCsr)]
    L.spx_synth_z.argtypes = [ctypes.c_void_p]
    L.spx_synth_z.restype = ctypes.c_void_p
    L.spx_synth_free.argtypes = [ctypes.c_void_p]
    seed = 0x5EED0000 + log_n
    h = ctypes.c_void_p()
    assert L.spx_synth_create(kind, log_n, log_v, seed, 0, ctypes.byref(h)) == 0
    I = oc.Instance(kind, log_n, log_v, seed, 0)
    n = 1 << log_n
    assert ctypes.string_at(L.spx_synth_z(h), 32 * n) == I.z_bytes
    for m in range(3):
        c = spx._CCsr()
        assert L.spx_synth_csr(h, m, ctypes.byref(c)) == 0
        nnz = c.row_ptr[n]
        M = I.mats[m]
        assert [c.row_ptr[i] for i in range(n + 1)] == [M.row_ptr[i] for i in range(n + 1)]
        assert [c.col[i] for i in range(nnz)] == [M.col[i] for i in range(nnz)]
        assert ctypes.string_at(c.val, 32 * nnz) == M.val.raw[: 32 * nnz]
    L.spx_synth_free(h)


def test_library_circuit_witnesses_match_oracle(spx, oc):
    """spx_synth_witnesses (kind 3): the witness of every seed equals the oracle generator's."""
    L = spx.lib()
    L.spx_synth_create.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, ctypes.POINTER(ctypes.c_void_p)]
    L.spx_synth_witnesses.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p]
    L.spx_synth_free.argtypes = [ctypes.c_void_p]
    log_n, log_v, seed = 8, 3, 4321
    h = ctypes.c_void_p()
    assert L.spx_synth_create(3, log_n, log_v, seed, 0, ctypes.byref(h)) == 0
    n, k = 1 << log_n, 5
    buf = ctypes.create_string_buffer(32 * n * k)
    assert L.spx_synth_witnesses(h, 100, k, buf) == 0
    for i in range(k):
        assert buf.raw[32 * n * i : 32 * n * (i + 1)] == oc.Instance(3, log_n, log_v, seed, 100 + i).z_bytes
    L.spx_synth_free(h)


def test_no_cpu_fallback_without_gpu(spx):
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(spx.SpartanError):
        spx.Context(0)


def test_sumcheck_round_argument_checks(spx):
    """spx.sumcheck_round checks its buffers before the native call, which reads 32 n bytes of both
    tables and 32 bytes of r_prev (no context is touched: these fail on any machine)"""
    with pytest.raises(spx.InvalidArgument):  # g shorter than f
        spx.sumcheck_round(None, [1, 2, 3, 4], [1, 2, 3])
    with pytest.raises(spx.InvalidArgument):  # not a whole number of 32-byte elements
        spx.sumcheck_round(None, b"\x01" * 100, b"\x01" * 100)
    with pytest.raises(spx.InvalidArgument):  # r_prev of the wrong size
        spx.sumcheck_round(None, [1, 2, 3, 4], [1, 2, 3, 4], b"\x01" * 16)
