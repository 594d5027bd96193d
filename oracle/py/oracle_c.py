"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes binding of the C restatement (oracle/liboracle.so, built by oracle/Makefile).
Loaded only by tests/, bench.py's cpu_baseline leg and __graft_entry__.smoke().
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(_HERE), "liboracle.so")

u8p = ctypes.POINTER(ctypes.c_uint8)


class Csr(ctypes.Structure):
    _fields_ = [
        ("n", ctypes.c_uint64),
        ("row_ptr", ctypes.POINTER(ctypes.c_uint64)),
        ("col", ctypes.POINTER(ctypes.c_uint32)),
        ("val", u8p),
    ]


_lib = None


def lib():
    global _lib
    if _lib is None:
        L = ctypes.CDLL(LIB_PATH)
        L.orc_gen.restype = ctypes.c_void_p
        L.orc_gen.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64]
        L.orc_inst_nnz.restype = ctypes.c_uint64
        L.orc_inst_nnz.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.orc_inst_log_v.argtypes = [ctypes.c_void_p]
        L.orc_inst_export.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.orc_inst_z.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.orc_inst_free.argtypes = [ctypes.c_void_p]
        L.orc_keygen.restype = ctypes.c_void_p
        L.orc_keygen.argtypes = [ctypes.c_int, ctypes.c_uint64]
        L.orc_pp_load.restype = ctypes.c_void_p
        L.orc_pp_load.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
        L.orc_pp_serialize.restype = ctypes.c_size_t
        L.orc_pp_serialize.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
        L.orc_pp_trapdoor.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.orc_pp_free.argtypes = [ctypes.c_void_p]
        L.orc_sum_over_y.argtypes = [ctypes.POINTER(Csr), ctypes.c_char_p, ctypes.c_void_p]
        L.orc_eval_on_x.argtypes = [ctypes.POINTER(Csr), ctypes.c_char_p, ctypes.c_void_p]
        L.orc_msm_g1.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_void_p]
        L.orc_msm_g2.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_void_p]
        L.orc_commit.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_void_p]
        L.orc_open.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_void_p, ctypes.c_void_p]
        L.orc_set_threads.argtypes = [ctypes.c_int]
        L.orc_get_threads.restype = ctypes.c_int
        L.orc_prove.restype = ctypes.c_int
        L.orc_prove.argtypes = [
            ctypes.POINTER(Csr),
            ctypes.POINTER(Csr),
            ctypes.POINTER(Csr),
            ctypes.c_char_p,
            ctypes.c_size_t,
            ctypes.c_char_p,
            ctypes.c_size_t,
            ctypes.c_void_p,
            ctypes.c_int,
            ctypes.c_uint64,
            ctypes.c_void_p,
            ctypes.c_size_t,
            ctypes.POINTER(ctypes.c_size_t),
        ]
        L.orc_matrix_eval.argtypes = [ctypes.POINTER(Csr), ctypes.c_char_p, ctypes.c_char_p, ctypes.c_void_p]
        L.orc_open_trapdoor.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_char_p,
                                        ctypes.c_void_p, ctypes.c_void_p]
        L.orc_mle_eval.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_void_p]
        L.orc_last_error.restype = ctypes.c_char_p
        _lib = L
    return _lib


GEN_UNIFORM_3N, GEN_REF_SHAPED, GEN_RAGGED, GEN_CIRCUIT_3N = 0, 1, 2, 3


class CsrMatrix:
    """Host CSR in the ABI byte layout (numpy-free: plain ctypes arrays)."""

    def __init__(self, n, row_ptr, col, val_bytes):
        self.n = n
        self.row_ptr = (ctypes.c_uint64 * (n + 1))(*row_ptr) if not isinstance(row_ptr, ctypes.Array) else row_ptr
        nnz = self.row_ptr[n]
        self.col = (ctypes.c_uint32 * max(nnz, 1))(*col) if not isinstance(col, ctypes.Array) else col
        self.val = ctypes.create_string_buffer(bytes(val_bytes), max(len(val_bytes), 1))
        self.nnz = nnz

    def csr(self):
        return Csr(self.n, self.row_ptr, self.col, ctypes.cast(self.val, u8p))

    @staticmethod
    def from_rows(rows):
        n = len(rows)
        rp = [0]
        col = []
        val = bytearray()
        for row in rows:
            for coeff, c in row:
                col.append(c)
                val += int(coeff).to_bytes(32, "little")
            rp.append(len(col))
        return CsrMatrix(n, rp, col, bytes(val))

    def to_rows(self):
        out = []
        vb = self.val.raw
        for x in range(self.n):
            row = []
            for k in range(self.row_ptr[x], self.row_ptr[x + 1]):
                row.append((int.from_bytes(vb[32 * k : 32 * k + 32], "little"), self.col[k]))
            out.append(row)
        return out


class Instance:
    def __init__(self, kind, log_n, log_v, seed, param=0):
        L = lib()
        h = L.orc_gen(kind, log_n, log_v, seed, param)
        self.log_n, self.log_v, self.n = log_n, log_v, 1 << log_n
        self.mats = []
        for m in range(3):
            nnz = L.orc_inst_nnz(h, m)
            rp = (ctypes.c_uint64 * (self.n + 1))()
            col = (ctypes.c_uint32 * max(nnz, 1))()
            val = ctypes.create_string_buffer(max(32 * nnz, 1))
            L.orc_inst_export(h, m, rp, col, val)
            M = CsrMatrix.__new__(CsrMatrix)
            M.n, M.row_ptr, M.col, M.val, M.nnz = self.n, rp, col, val, nnz
            self.mats.append(M)
        zb = ctypes.create_string_buffer(32 * self.n)
        L.orc_inst_z(h, zb)
        self.z_bytes = zb.raw
        L.orc_inst_free(h)

    @property
    def v_bytes(self):
        return self.z_bytes[: 32 << self.log_v]

    @property
    def w_bytes(self):
        return self.z_bytes[32 << self.log_v :]


class PP:
    def __init__(self, handle):
        self.h = handle

    @staticmethod
    def keygen(nv, seed):
        return PP(lib().orc_keygen(nv, seed))

    @staticmethod
    def load(b):
        h = lib().orc_pp_load(b, len(b))
        if not h:
            raise ValueError(lib().orc_last_error().decode())
        return PP(h)

    def serialize(self):
        L = lib()
        need = L.orc_pp_serialize(self.h, None, 0)
        buf = ctypes.create_string_buffer(need)
        L.orc_pp_serialize(self.h, buf, need)
        return buf.raw

    def trapdoor(self, nv):
        buf = ctypes.create_string_buffer(32 * max(nv, 1))
        lib().orc_pp_trapdoor(self.h, buf)
        return [int.from_bytes(buf.raw[32 * i : 32 * i + 32], "little") for i in range(nv)]

    def __del__(self):
        try:
            if self.h:
                lib().orc_pp_free(self.h)
        except Exception:
            pass


def sum_over_y(M, z_bytes):
    out = ctypes.create_string_buffer(32 * M.n)
    c = M.csr()
    lib().orc_sum_over_y(ctypes.byref(c), z_bytes, out)
    return out.raw


def eval_on_x(M, r_x_bytes):
    out = ctypes.create_string_buffer(32 * M.n)
    c = M.csr()
    lib().orc_eval_on_x(ctypes.byref(c), r_x_bytes, out)
    return out.raw


def msm_g1(bases, scalars, n):
    out = ctypes.create_string_buffer(96)
    lib().orc_msm_g1(bases, scalars, n, out)
    return out.raw


def msm_g2(bases, scalars, n):
    out = ctypes.create_string_buffer(192)
    lib().orc_msm_g2(bases, scalars, n, out)
    return out.raw


def commit(pp, table_bytes, nv):
    out = ctypes.create_string_buffer(56)
    lib().orc_commit(pp.h, table_bytes, nv, out)
    return out.raw


def open_(pp, table_bytes, nv, point_bytes):
    ev = ctypes.create_string_buffer(32)
    pf = ctypes.create_string_buffer(96 + 8 + 96 * nv)
    lib().orc_open(pp.h, table_bytes, nv, point_bytes, ev, pf)
    return ev.raw, pf.raw


def set_threads(k):
    """OpenMP threads for the oracle's MSM windows and sumcheck rounds (1 = the reference's single thread)."""
    lib().orc_set_threads(int(k))


def prove(mats, v_bytes, w_bytes, pp, mode=0, inj_seed=0, commitment_stub=False):
    """mode 0 = FS, 1 = injected; commitment_stub: BASELINE config C2 (pp may be None)."""
    L = lib()
    if commitment_stub:
        mode |= 2
    A, B, C = (m.csr() for m in mats)
    n = mats[0].n
    cap = 64 * 1024 + 64 * n.bit_length() * 64
    out = ctypes.create_string_buffer(cap)
    ln = ctypes.c_size_t(0)
    rc = L.orc_prove(
        ctypes.byref(A),
        ctypes.byref(B),
        ctypes.byref(C),
        v_bytes,
        len(v_bytes) // 32,
        w_bytes,
        len(w_bytes) // 32,
        pp.h if pp is not None else None,
        mode,
        inj_seed,
        out,
        cap,
        ctypes.byref(ln),
    )
    if rc:
        raise RuntimeError("orc_prove failed (%d): %s" % (rc, L.orc_last_error().decode()))
    return out.raw[: ln.value]


def _frb(xs):
    return b"".join(int(x).to_bytes(32, "little") for x in xs)


def matrix_eval(M, r_x, r_y):
    """M(r_x, r_y) with eval_on_x's last-entry semantics; M a CsrMatrix or a ctypes Csr view"""
    out = ctypes.create_string_buffer(32)
    c = M.csr() if hasattr(M, "csr") else M
    lib().orc_matrix_eval(ctypes.byref(c), _frb(r_x), _frb(r_y), out)
    return int.from_bytes(out.raw, "little")


def open_trapdoor(table_bytes, nv, point, t):
    """([q_i(t[i+1..])] for every level, z(point)) of an mKZG opening"""
    qv = ctypes.create_string_buffer(32 * max(nv, 1))
    ev = ctypes.create_string_buffer(32)
    lib().orc_open_trapdoor(table_bytes, nv, _frb(point), _frb(t), qv, ev)
    return [int.from_bytes(qv.raw[32 * i : 32 * i + 32], "little") for i in range(nv)], int.from_bytes(ev.raw, "little")


def mle_eval(table_bytes, nv, point):
    out = ctypes.create_string_buffer(32)
    lib().orc_mle_eval(table_bytes, nv, _frb(point), out)
    return int.from_bytes(out.raw, "little")
