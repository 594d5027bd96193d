"""r1cs-spartan_amd — MI355X-native drop-in for the proving hot path of tsunrise/r1cs-spartan.

Host-side mirror of the reference interface over the C ABI of libspartan_hip.so
(include/spartan_hip.h). Names, argument meaning and errors follow the reference:

  MLArgumentForR1CS.index(A, B, C) -> IndexPK          /root/reference/src/lib.rs:45-51
  MLArgumentForR1CS.prove(pk, v, w, pp) -> bytes       /root/reference/src/lib.rs:58-146
  MLProofForR1CS.setup(nv, seed) -> PublicParameter    /root/reference/src/ahp/setup.rs:13-16
  MLPolyCommit.commit / open                           /root/reference/src/commitment/{commit,open}.rs
  MatrixExtension.sum_over_y / eval_on_x               /root/reference/src/data_structures/r1cs_reader.rs
  InvalidArgument / SumCheckError / WrongWitness / SerializationError   src/error.rs:5-14

The product path is the HIP library only: importing this module loads libspartan_hip.so and
raises if it is missing; there is no CPU fallback. Field elements are Python ints (canonical) or
32-byte little-endian canonical byte strings; matrices are `Matrix<F>` = list of rows of
(coeff, col) or a `Csr` (row_ptr / col / val bytes).

The directory name contains a hyphen, so load it with importlib (see __graft_entry__.py):
    spec = importlib.util.spec_from_file_location("r1cs_spartan_amd", ".../__init__.py")
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SPX_LIB_PATH") or os.path.join(_HERE, "libspartan_hip.so")  # override: A/B builds

R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001


class SpartanError(Exception):
    code = -1


class InvalidArgument(SpartanError):
    code = 1


class SumCheckError(SpartanError):
    code = 2


class WrongWitness(SpartanError):
    code = 3


class SerializationError(SpartanError):
    code = 4


class DeviceError(SpartanError):
    code = 5


_ERRORS = {1: InvalidArgument, 2: SumCheckError, 3: WrongWitness, 4: SerializationError, 5: DeviceError}


class _CCsr(ctypes.Structure):
    _fields_ = [
        ("n", ctypes.c_uint64),
        ("row_ptr", ctypes.POINTER(ctypes.c_uint64)),
        ("col", ctypes.POINTER(ctypes.c_uint32)),
        ("val", ctypes.POINTER(ctypes.c_uint8)),
    ]


class _Opts(ctypes.Structure):
    _fields_ = [("mode", ctypes.c_int), ("inj_seed", ctypes.c_uint64), ("cached_matrix_transcript", ctypes.c_int),
                ("commitment_stub", ctypes.c_int)]


EXPORTED = [
    "spx_last_error",
    "spx_version",
    "spx_ctx_create",
    "spx_ctx_destroy",
    "spx_comm_unique_id",
    "spx_ctx_set_comm_rccl",
    "spx_ctx_set_comm_shm",
    "spx_comm_shm_create",
    "spx_comm_shm_allgather",
    "spx_comm_shm_destroy",
    "spx_comm_group_create",
    "spx_comm_group_destroy",
    "spx_ctx_set_comm_group",
    "spx_ctx_set_comm_rehearsal",
    "spx_ctx_set_lvl0_batch",
    "spx_comm_hub_create_rccl",
    "spx_comm_hub_create_shm",
    "spx_comm_hub_create_group",
    "spx_comm_hub_create_callback",
    "spx_ctx_set_comm_hub",
    "spx_comm_hub_allgather",
    "spx_comm_hub_stats",
    "spx_comm_hub_destroy",
    "spx_ctx_comm_allgather",
    "spx_msm_reruns",
    "spx_ctx_mem_info",
    "spx_ctx_set_sync_poll",
    "spx_ctx_set_group",
    "spx_host_phase_stats",
    "spx_pp_load",
    "spx_pp_generate",
    "spx_pp_serialize",
    "spx_pp_free",
    "spx_index",
    "spx_index_free",
    "spx_witness_upload",
    "spx_witness_free",
    "spx_proof_size",
    "spx_prove",
    "spx_prove_witness",
    "spx_prove_many",
    "spx_hash_stats",
    "spx_last_timings",
    "spx_cs_create",
    "spx_cs_free",
    "spx_cs_new_input",
    "spx_cs_new_witness",
    "spx_cs_enforce",
    "spx_cs_make_square",
    "spx_cs_counts",
    "spx_cs_is_satisfied",
    "spx_cs_matrices",
    "spx_verify",
    "spx_vp_from_pp",
    "spx_pairing_check",
    "spx_prover_init",
    "spx_prover_first_round",
    "spx_prover_second_round",
    "spx_prover_third_round",
    "spx_prove_first_sumcheck_round",
    "spx_prove_fourth_round",
    "spx_prove_fifth_round",
    "spx_prove_second_sumcheck_round",
    "spx_prove_sixth_round",
    "spx_prover_free",
    "spx_sumcheck_round",
    "spx_sum_over_y",
    "spx_eval_on_x",
    "spx_msm_g1",
    "spx_msm_g2",
    "spx_commit",
    "spx_open",
]

_lib = None


def lib():
    """Load libspartan_hip.so (fails loudly: the HIP path is the only product path)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError("libspartan_hip.so not built (run __graft_entry__.build()): %s" % LIB_PATH)
    L = ctypes.CDLL(LIB_PATH)
    vp = ctypes.c_void_p
    sz = ctypes.c_size_t
    u8p = ctypes.c_char_p
    L.spx_last_error.restype = ctypes.c_char_p
    L.spx_version.restype = ctypes.c_char_p
    L.spx_ctx_create.argtypes = [ctypes.c_int, ctypes.POINTER(vp)]
    L.spx_ctx_destroy.argtypes = [vp]
    L.spx_comm_unique_id.argtypes = [ctypes.c_void_p]
    L.spx_ctx_set_comm_rccl.argtypes = [vp, u8p, ctypes.c_int, ctypes.c_int]
    L.spx_ctx_set_comm_shm.argtypes = [vp, ctypes.c_char_p, ctypes.c_int, ctypes.c_int]
    L.spx_comm_shm_create.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.POINTER(vp)]
    L.spx_comm_shm_allgather.argtypes = [vp, ctypes.c_void_p, ctypes.c_void_p, sz]
    L.spx_comm_shm_destroy.argtypes = [vp]
    L.spx_comm_group_create.argtypes = [ctypes.c_int, ctypes.POINTER(vp)]
    L.spx_comm_group_destroy.argtypes = [vp]
    L.spx_ctx_set_comm_group.argtypes = [vp, vp, ctypes.c_int]
    if hasattr(L, "spx_ctx_set_comm_rehearsal") or not os.environ.get("SPX_LIB_PATH"):  # A/B builds may predate it
        L.spx_ctx_set_comm_rehearsal.argtypes = [vp, ctypes.c_int, ctypes.c_int]
    if hasattr(L, "spx_msm_reruns") or not os.environ.get("SPX_LIB_PATH"):
        L.spx_msm_reruns.argtypes = [vp, ctypes.POINTER(ctypes.c_uint64)]
    if hasattr(L, "spx_ctx_set_sync_poll") or not os.environ.get("SPX_LIB_PATH"):
        L.spx_ctx_set_sync_poll.argtypes = [vp, ctypes.c_int]
    if hasattr(L, "spx_ctx_set_group") or not os.environ.get("SPX_LIB_PATH"):
        L.spx_ctx_set_group.argtypes = [vp, ctypes.c_int]
    if hasattr(L, "spx_ctx_mem_info") or not os.environ.get("SPX_LIB_PATH"):
        L.spx_ctx_mem_info.argtypes = [vp, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
    if hasattr(L, "spx_ctx_set_lvl0_batch"):  # A/B builds may predate it
        L.spx_ctx_set_lvl0_batch.argtypes = [vp, ctypes.c_int]
    if hasattr(L, "spx_comm_hub_create_rccl") or not os.environ.get("SPX_LIB_PATH"):  # A/B builds may predate the hub
        L.spx_comm_hub_create_rccl.argtypes = [u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(vp)]
        L.spx_comm_hub_create_shm.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.POINTER(vp)]
        L.spx_comm_hub_create_group.argtypes = [vp, ctypes.c_int, ctypes.POINTER(vp)]
        if hasattr(L, "spx_comm_hub_create_callback") or not os.environ.get("SPX_LIB_PATH"):
            L.spx_comm_hub_create_callback.argtypes = [ALLGATHER_FN, vp, ctypes.c_int, ctypes.c_int, ctypes.POINTER(vp)]
        L.spx_ctx_set_comm_hub.argtypes = [vp, vp, ctypes.c_int]
        L.spx_comm_hub_allgather.argtypes = [vp, ctypes.c_int, ctypes.c_char_p, ctypes.c_void_p, sz]
        L.spx_comm_hub_stats.argtypes = [vp, ctypes.c_void_p]
        L.spx_comm_hub_destroy.argtypes = [vp]
    L.spx_ctx_comm_allgather.argtypes = [vp, ctypes.c_char_p, ctypes.c_void_p, sz]
    L.spx_pp_load.argtypes = [vp, u8p, sz, ctypes.POINTER(vp)]
    L.spx_pp_generate.argtypes = [vp, ctypes.c_int, ctypes.c_uint64, ctypes.POINTER(vp)]
    L.spx_pp_serialize.argtypes = [vp, ctypes.c_void_p, sz, ctypes.POINTER(sz)]
    L.spx_pp_free.argtypes = [vp]
    L.spx_index.argtypes = [vp, ctypes.POINTER(_CCsr), ctypes.POINTER(_CCsr), ctypes.POINTER(_CCsr), ctypes.POINTER(vp)]
    L.spx_index_free.argtypes = [vp]
    L.spx_witness_upload.argtypes = [vp, u8p, sz, u8p, sz, ctypes.POINTER(vp)]
    L.spx_witness_free.argtypes = [vp]
    L.spx_proof_size.restype = sz
    L.spx_proof_size.argtypes = [ctypes.c_int, ctypes.c_int]
    L.spx_prove.argtypes = [vp, vp, u8p, sz, u8p, sz, vp, ctypes.POINTER(_Opts), ctypes.c_void_p, sz, ctypes.POINTER(sz)]
    L.spx_prove_witness.argtypes = [vp, vp, vp, vp, ctypes.POINTER(_Opts), ctypes.c_void_p, sz, ctypes.POINTER(sz)]
    L.spx_prove_many.argtypes = [ctypes.POINTER(vp), ctypes.c_int, vp, ctypes.POINTER(vp), ctypes.c_int, vp,
                                 ctypes.POINTER(_Opts), ctypes.c_void_p, sz, ctypes.POINTER(sz)]
    L.spx_verify.argtypes = [vp, vp, u8p, sz, u8p, sz, u8p, sz, ctypes.POINTER(_Opts)]
    if hasattr(L, "spx_hash_stats") or not os.environ.get("SPX_LIB_PATH"):
        L.spx_hash_stats.argtypes = [ctypes.POINTER(ctypes.c_uint64)]
    L.spx_vp_from_pp.argtypes = [vp, ctypes.c_void_p, sz, ctypes.POINTER(sz)]
    L.spx_pairing_check.argtypes = [u8p, u8p, sz, ctypes.POINTER(ctypes.c_int)]
    L.spx_cs_create.argtypes = [ctypes.POINTER(vp)]
    L.spx_cs_free.argtypes = [vp]
    L.spx_cs_new_input.argtypes = [vp, u8p, ctypes.POINTER(ctypes.c_uint64)]
    L.spx_cs_new_witness.argtypes = [vp, u8p, ctypes.POINTER(ctypes.c_uint64)]
    L.spx_cs_enforce.argtypes = [vp, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    L.spx_cs_make_square.argtypes = [vp, ctypes.c_uint64]
    L.spx_cs_counts.argtypes = [vp, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    L.spx_cs_is_satisfied.argtypes = [vp, ctypes.POINTER(ctypes.c_int)]
    L.spx_cs_matrices.argtypes = [vp, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    L.spx_last_timings.argtypes = [vp, ctypes.POINTER(ctypes.c_double), ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
    psz = ctypes.POINTER(sz)
    if hasattr(L, "spx_prover_init") or not os.environ.get("SPX_LIB_PATH"):  # A/B builds may predate it
        L.spx_prover_init.argtypes = [vp, vp, u8p, sz, u8p, sz, ctypes.POINTER(vp)]
        L.spx_prover_first_round.argtypes = [vp, vp, ctypes.c_void_p, sz, psz]
        L.spx_prover_second_round.argtypes = [vp, u8p, sz, vp, ctypes.c_void_p, sz, psz]
        L.spx_prover_third_round.argtypes = [vp, u8p, sz, ctypes.c_void_p, sz, psz]
        L.spx_prove_first_sumcheck_round.argtypes = [vp, u8p, ctypes.c_void_p, sz, psz]
        L.spx_prove_fourth_round.argtypes = [vp, u8p, ctypes.c_void_p, sz, psz]
        L.spx_prove_fifth_round.argtypes = [vp, u8p, ctypes.c_void_p, sz, psz]
        L.spx_prove_second_sumcheck_round.argtypes = [vp, u8p, ctypes.c_void_p, sz, psz]
        L.spx_prove_sixth_round.argtypes = [vp, u8p, vp, ctypes.c_void_p, sz, psz]
        L.spx_prover_free.argtypes = [vp]
        L.spx_sumcheck_round.argtypes = [vp, u8p, u8p, sz, u8p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    L.spx_sum_over_y.argtypes = [vp, ctypes.POINTER(_CCsr), u8p, ctypes.c_void_p]
    L.spx_eval_on_x.argtypes = [vp, ctypes.POINTER(_CCsr), u8p, ctypes.c_void_p]
    L.spx_msm_g1.argtypes = [vp, u8p, u8p, sz, ctypes.c_void_p]
    L.spx_msm_g2.argtypes = [vp, u8p, u8p, sz, ctypes.c_void_p]
    L.spx_commit.argtypes = [vp, vp, u8p, ctypes.c_int, ctypes.c_void_p]
    L.spx_open.argtypes = [vp, vp, u8p, ctypes.c_int, u8p, ctypes.c_void_p, ctypes.c_void_p]
    for name in EXPORTED:
        if name not in ("spx_last_error", "spx_version", "spx_proof_size"):
            if os.environ.get("SPX_LIB_PATH") and not hasattr(L, name):
                continue  # an older A/B build (tools/ab_bench.sh); the in-tree library must export all
            getattr(L, name).restype = ctypes.c_int
    _lib = L
    return L


def _check(rc):
    if rc != 0:
        msg = lib().spx_last_error().decode(errors="replace")
        raise _ERRORS.get(rc, SpartanError)(msg)


# ------------------------------------------------------------------ data helpers
def fr_bytes(values):
    """Canonical ints -> concatenated 32-byte LE images."""
    return b"".join((int(x) % R).to_bytes(32, "little") for x in values)


def fr_ints(b):
    return [int.from_bytes(b[32 * i : 32 * i + 32], "little") for i in range(len(b) // 32)]


class Csr:
    """CSR image of an ark-relations `Matrix<F>` (row order and in-row order preserved)."""

    def __init__(self, n, row_ptr, col, val_bytes):
        self.n = int(n)
        self.row_ptr = row_ptr if isinstance(row_ptr, ctypes.Array) else (ctypes.c_uint64 * (self.n + 1))(*row_ptr)
        nnz = int(self.row_ptr[self.n])
        self.col = col if isinstance(col, ctypes.Array) else (ctypes.c_uint32 * max(nnz, 1))(*col)
        self.val = val_bytes if isinstance(val_bytes, ctypes.Array) else ctypes.create_string_buffer(bytes(val_bytes), max(len(val_bytes), 1))
        self.nnz = nnz

    @staticmethod
    def from_rows(rows):
        rp, col, val = [0], [], bytearray()
        for row in rows:
            for coeff, c in row:
                col.append(int(c))
                val += (int(coeff) % R).to_bytes(32, "little")
            rp.append(len(col))
        return Csr(len(rows), rp, col, bytes(val))

    def c(self):
        return _CCsr(self.n, self.row_ptr, self.col, ctypes.cast(self.val, ctypes.POINTER(ctypes.c_uint8)))


def _as_csr(m):
    return m if isinstance(m, Csr) else Csr.from_rows(m)


def _as_bytes(v):
    if isinstance(v, (bytes, bytearray)):
        return bytes(v)
    return fr_bytes(v)


# ------------------------------------------------------------------ handles
class Context:
    """One GPU (one rank). Everything else is created against a context."""

    def __init__(self, device=0):
        h = ctypes.c_void_p()
        _check(lib().spx_ctx_create(int(device), ctypes.byref(h)))
        self.h = h

    def close(self):
        if self.h:
            lib().spx_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_comm_rccl(self, unique_id, rank, world):
        _check(lib().spx_ctx_set_comm_rccl(self.h, bytes(unique_id), int(rank), int(world)))

    def set_comm_shm(self, name, rank, world):
        """On-node shared-memory communicator; every rank passes the same name (one per context)."""
        _check(lib().spx_ctx_set_comm_shm(self.h, name.encode(), int(rank), int(world)))

    def set_comm_group(self, group, rank):
        _check(lib().spx_ctx_set_comm_group(self.h, group.h, int(rank)))

    def set_comm_hub(self, hub, channel):
        """exchanges through channel `channel` of an ExchangeHub (context j of every rank on channel j)"""
        _check(lib().spx_ctx_set_comm_hub(self.h, hub.h, int(channel)))

    def set_comm_rehearsal(self, rank, world):
        """one rank of a world-rank proof-sharded prove without its peers (throughput rehearsal; the
        proofs are not valid)"""
        _check(lib().spx_ctx_set_comm_rehearsal(self.h, int(rank), int(world)))

    def set_lvl0_batch(self, mode):
        """where the shared level-0 opening MSM runs: 1 inside the first opening's batch, 0 beside the
        commitment, -1 the process default (SPX_LVL0); the same on every rank of a sharded prove"""
        _check(lib().spx_ctx_set_lvl0_batch(self.h, int(mode)))

    def comm_allgather(self, data, world):
        """one allgather of `data` on this context's communicator -> list of world byte strings"""
        data = bytes(data)
        out = ctypes.create_string_buffer(max(1, len(data) * world))
        _check(lib().spx_ctx_comm_allgather(self.h, data, out, len(data)))
        return [out.raw[k * len(data) : (k + 1) * len(data)] for k in range(world)]

    def set_sync_poll(self, us):
        """host waits of this context: poll an event every `us` microseconds (0: hipStreamSynchronize,
        -1: the process default; spx_ctx_set_sync_poll)"""
        _check(lib().spx_ctx_set_sync_poll(self.h, int(us)))

    def set_group(self, k):
        """spx_prove_many runs this context's stubbed-commitment proofs k at a time in lockstep (one launch
        per sumcheck round for the k proofs; 1 = one at a time; spx_ctx_set_group)"""
        _check(lib().spx_ctx_set_group(self.h, int(k)))

    def mem_info(self):
        """(free, total) bytes of this context's device (spx_ctx_mem_info)"""
        f, t = ctypes.c_uint64(), ctypes.c_uint64()
        _check(lib().spx_ctx_mem_info(self.h, ctypes.byref(f), ctypes.byref(t)))
        return f.value, t.value

    def msm_reruns(self):
        """MSM batches rerun with dense keys after a compacted-key overflow (spx_msm_reruns)"""
        v = ctypes.c_uint64(0)
        _check(lib().spx_msm_reruns(self.h, ctypes.byref(v)))
        return v.value

    def last_timings(self):
        buf = (ctypes.c_double * 32)()
        n = ctypes.c_int(0)
        _check(lib().spx_last_timings(self.h, buf, 32, ctypes.byref(n)))
        names = ["transcript_matrices", "commit", "open_rv", "sumcheck1", "eval_on_x", "sumcheck2", "open_ry", "total"]
        return {names[i] if i < len(names) else str(i): buf[i] for i in range(min(n.value, 32))}


class CommGroup:
    """In-process communicator for `world` contexts (tests of the sharded path on one node)."""

    def __init__(self, world):
        h = ctypes.c_void_p()
        _check(lib().spx_comm_group_create(int(world), ctypes.byref(h)))
        self.h, self.world = h, int(world)

    def __del__(self):
        try:
            if self.h:
                lib().spx_comm_group_destroy(self.h)
        except Exception:
            pass


class ShmComm:
    """Standalone host allgather over the shared-memory transport (no GPU needed)."""

    def __init__(self, name, rank, world):
        h = ctypes.c_void_p()
        _check(lib().spx_comm_shm_create(name.encode(), int(rank), int(world), ctypes.byref(h)))
        self.h, self.world = h, int(world)

    def allgather(self, data):
        data = bytes(data)
        out = ctypes.create_string_buffer(len(data) * self.world)
        _check(lib().spx_comm_shm_allgather(self.h, data, out, len(data)))
        return [out.raw[k * len(data) : (k + 1) * len(data)] for k in range(self.world)]

    def close(self):
        if self.h:
            lib().spx_comm_shm_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# spx_allgather_fn: (user, send, recv, bytes) -> 0 on success
ALLGATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t)


class ExchangeHub:
    """One collective transport per rank shared by every proof in flight, ordered by channel
    (comm_hub.cpp): ExchangeHub.rccl(uid, rank, world, device), .shm(name, rank, world),
    .group(CommGroup, rank) or .torch_group(process_group) (a torch.distributed group: gloo on the CPU,
    RCCL as backend "nccl")."""

    def __init__(self, h, world):
        self.h, self.world = h, int(world)

    @classmethod
    def rccl(cls, unique_id, rank, world, device=0):
        h = ctypes.c_void_p()
        _check(lib().spx_comm_hub_create_rccl(bytes(unique_id), int(rank), int(world), int(device), ctypes.byref(h)))
        return cls(h, world)

    @classmethod
    def shm(cls, name, rank, world):
        h = ctypes.c_void_p()
        _check(lib().spx_comm_hub_create_shm(name.encode(), int(rank), int(world), ctypes.byref(h)))
        return cls(h, world)

    @classmethod
    def group(cls, group, rank):
        h = ctypes.c_void_p()
        _check(lib().spx_comm_hub_create_group(group.h, int(rank), ctypes.byref(h)))
        return cls(h, group.world)

    @classmethod
    def torch_group(cls, group=None):
        """the hub over a torch.distributed process group (spx_comm_hub_create_callback): the hub's thread
        calls dist.all_gather on uint8 tensors (CPU tensors for gloo, the current device's otherwise)"""
        import torch
        import torch.distributed as dist

        rank, world = dist.get_rank(group), dist.get_world_size(group)
        dev = "cpu" if dist.get_backend(group) == "gloo" else "cuda:%d" % torch.cuda.current_device()

        def fn(_user, send, recv, nbytes):
            try:
                if nbytes == 0:
                    return 0
                t = torch.frombuffer(bytearray(ctypes.string_at(send, nbytes)), dtype=torch.uint8).to(dev)
                outs = [torch.empty(nbytes, dtype=torch.uint8, device=dev) for _ in range(world)]
                dist.all_gather(outs, t, group=group)
                buf = torch.cat(outs).cpu().numpy().tobytes()
                ctypes.memmove(recv, buf, len(buf))
                return 0
            except Exception:  # reported to the waiting exchange as SPX_DEVICE
                return 1

        cb = ALLGATHER_FN(fn)
        h = ctypes.c_void_p()
        _check(lib().spx_comm_hub_create_callback(cb, None, rank, world, ctypes.byref(h)))
        hub = cls(h, world)
        hub._cb = cb  # the C side holds the function pointer: keep the thunk alive with the hub
        return hub

    def allgather(self, channel, data):
        data = bytes(data)
        out = ctypes.create_string_buffer(max(1, len(data) * self.world))
        _check(lib().spx_comm_hub_allgather(self.h, int(channel), data, out, len(data)))
        return [out.raw[k * len(data) : (k + 1) * len(data)] for k in range(self.world)]

    def stats(self):
        """control rounds, data rounds, exchanges served, largest batch in one round, idle rounds (matched
        nothing: a peer had not reached the exchange yet)"""
        out = (ctypes.c_uint64 * 5)()
        _check(lib().spx_comm_hub_stats(self.h, out))
        return dict(zip(("rounds", "data_rounds", "served", "max_batch", "idle_rounds"), list(out)))

    def close(self):
        if self.h:
            lib().spx_comm_hub_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def hash_stats():
    """(seconds, proofs, lane width, seconds the proof workers waited for an absorption) of
    spx_prove_many's matrix absorption so far (process-wide)"""
    out = (ctypes.c_uint64 * 4)()
    _check(lib().spx_hash_stats(out))
    return out[0] / 1e9, out[1], out[2], out[3] / 1e9


HOST_PHASES = ["transcript_matrices", "commit", "open_rv", "sumcheck1", "eval_on_x", "sumcheck2", "open_ry"]


def host_phase_stats():
    """{phase: (thread CPU s, wall s, count)} of prove() on this process's proving threads
    (spx_host_phase_stats; cumulative since load)"""
    a = (ctypes.c_uint64 * 21)()
    _check(lib().spx_host_phase_stats(a))
    return {p: (a[3 * i] / 1e9, a[3 * i + 1] / 1e9, a[3 * i + 2]) for i, p in enumerate(HOST_PHASES)}


def shm_name():
    """A fresh segment name (rank 0 draws it and distributes it)."""
    return "spx_%016x" % int.from_bytes(os.urandom(8), "little")


def comm_unique_id():
    buf = ctypes.create_string_buffer(128)
    _check(lib().spx_comm_unique_id(buf))
    return buf.raw


class PublicParameter:
    """commitment/data_structures.rs:9-17, resident in HBM with its window tables."""

    def __init__(self, ctx, h, nv):
        self.ctx, self.h, self.nv = ctx, h, nv

    @staticmethod
    def load(ctx, data):
        h = ctypes.c_void_p()
        _check(lib().spx_pp_load(ctx.h, bytes(data), len(data), ctypes.byref(h)))
        return PublicParameter(ctx, h, int.from_bytes(data[:8], "little"))

    def serialize_uncompressed(self):
        n = ctypes.c_size_t(0)
        _check(lib().spx_pp_serialize(self.h, None, 0, ctypes.byref(n)))
        buf = ctypes.create_string_buffer(n.value)
        _check(lib().spx_pp_serialize(self.h, buf, n.value, ctypes.byref(n)))
        return buf.raw

    def __del__(self):
        try:
            if self.h:
                lib().spx_pp_free(self.h)
        except Exception:
            pass


class IndexPK:
    """ahp/indexer.rs:9-17 (prover key)."""

    def __init__(self, ctx, h, log_n):
        self.ctx, self.h, self.log_n = ctx, h, log_n

    def __del__(self):
        try:
            if self.h:
                lib().spx_index_free(self.h)
        except Exception:
            pass


class Witness:
    """z = v || w resident in HBM (the benchmarked form of prove's input)."""

    def __init__(self, ctx, v, w):
        vb, wb = _as_bytes(v), _as_bytes(w)
        h = ctypes.c_void_p()
        _check(lib().spx_witness_upload(ctx.h, vb, len(vb) // 32, wb, len(wb) // 32, ctypes.byref(h)))
        self.ctx, self.h = ctx, h

    def __del__(self):
        try:
            if self.h:
                lib().spx_witness_free(self.h)
        except Exception:
            pass


def _opts(mode, seed, cached, stub=False):
    return _Opts(1 if mode == "injected" else 0, int(seed), 1 if cached else 0, 1 if stub else 0)


def _pp_handle(pp, stub):
    if pp is None:
        if not stub:
            raise InvalidArgument("a public parameter is required unless commitment_stub=True")
        return None
    return pp.h


class MLProofForR1CS:
    @staticmethod
    def setup(ctx, nv, seed):
        """GPU keygen with setup.rs semantics; draws (g, h, t) from SplitMix64(seed)."""
        h = ctypes.c_void_p()
        _check(lib().spx_pp_generate(ctx.h, int(nv), int(seed), ctypes.byref(h)))
        return PublicParameter(ctx, h, nv)


class MLArgumentForR1CS:
    @staticmethod
    def index(ctx, matrix_a, matrix_b, matrix_c):
        A, B, C = (_as_csr(m) for m in (matrix_a, matrix_b, matrix_c))
        h = ctypes.c_void_p()
        ca, cb, cc = A.c(), B.c(), C.c()
        _check(lib().spx_index(ctx.h, ctypes.byref(ca), ctypes.byref(cb), ctypes.byref(cc), ctypes.byref(h)))
        return IndexPK(ctx, h, A.n.bit_length() - 1)

    @staticmethod
    def prove(pk, v, w, pp, mode="fs", seed=0, cached=False, commitment_stub=False):
        """Proof bytes (ark-serialize compressed, proof.rs:10-20 field order).
        commitment_stub=True is BASELINE config C2 (sumcheck-only): the proof prove() gives under a
        public parameter whose every group element is the identity; no MSM runs and pp may be None."""
        vb, wb = _as_bytes(v), _as_bytes(w)
        cap = lib().spx_proof_size(pk.log_n, 0)
        out = ctypes.create_string_buffer(cap)
        n = ctypes.c_size_t(0)
        o = _opts(mode, seed, cached, commitment_stub)
        _check(lib().spx_prove(pk.ctx.h, pk.h, vb, len(vb) // 32, wb, len(wb) // 32, _pp_handle(pp, commitment_stub),
                               ctypes.byref(o), out, cap, ctypes.byref(n)))
        return out.raw[: n.value]

    @staticmethod
    def prove_witness(pk, wit, pp, mode="fs", seed=0, cached=False, commitment_stub=False):
        cap = lib().spx_proof_size(pk.log_n, 0)
        out = ctypes.create_string_buffer(cap)
        n = ctypes.c_size_t(0)
        o = _opts(mode, seed, cached, commitment_stub)
        _check(lib().spx_prove_witness(pk.ctx.h, pk.h, wit.h, _pp_handle(pp, commitment_stub), ctypes.byref(o), out, cap,
                                       ctypes.byref(n)))
        return out.raw[: n.value]


    @staticmethod
    def prove_many(ctxs, pk, wits, pp, mode="fs", seed=0, cached=False, commitment_stub=False):
        """Proves every witness in `wits` concurrently, one worker per context (spx_prove_many)."""
        cap = lib().spx_proof_size(pk.log_n, 0)
        n = len(wits)
        out = ctypes.create_string_buffer(cap * max(n, 1))
        lens = (ctypes.c_size_t * max(n, 1))()
        ch = (ctypes.c_void_p * len(ctxs))(*[c.h for c in ctxs])
        wh = (ctypes.c_void_p * max(n, 1))(*[w.h for w in wits])
        o = _opts(mode, seed, cached, commitment_stub)
        _check(lib().spx_prove_many(ch, len(ctxs), pk.h, wh, n, _pp_handle(pp, commitment_stub), ctypes.byref(o), out,
                                    cap, lens))
        raw = out.raw
        return [raw[i * cap : i * cap + lens[i]] for i in range(n)]


    @staticmethod
    def verify(pk, v, proof, vp, mode="fs", seed=0, cached=False):
        """lib.rs:147-212: True on acceptance; the reference's Err(...) raises the mapped exception."""
        vb = _as_bytes(v)
        o = _opts(mode, seed, cached)
        _check(lib().spx_verify(pk.ctx.h, pk.h, vb, len(vb) // 32, bytes(proof), len(proof), bytes(vp), len(vp),
                                ctypes.byref(o)))
        return True


class InteractiveProver:
    """The reference's round-level prover (src/ahp/prover.rs:109-281) over spx_prover_*: construct
    with MLArgumentForR1CS-style inputs (prover_init), then call the rounds in the reference's order
    with the verifier messages (canonical ints or 32-byte strings); each returns the prover message
    as ark-serialize compressed bytes. Challenges of the sumcheck rounds: None first, then the
    previous round's challenge (AHPForMLSumcheck::prove_round)."""

    _CAP = 1 << 16

    def __init__(self, pk, v, w):
        vb, wb = _as_bytes(v), _as_bytes(w)
        h = ctypes.c_void_p()
        _check(lib().spx_prover_init(pk.ctx.h, pk.h, vb, len(vb) // 32, wb, len(wb) // 32, ctypes.byref(h)))
        self.pk, self.h = pk, h

    def _call(self, fn, *args):
        out = ctypes.create_string_buffer(self._CAP)
        n = ctypes.c_size_t(0)
        _check(fn(self.h, *args, out, self._CAP, ctypes.byref(n)))
        return out.raw[: n.value]

    @staticmethod
    def _one(x):
        return None if x is None else _as_bytes([x] if isinstance(x, int) else x)

    def prover_first_round(self, pp):
        return self._call(lib().spx_prover_first_round, pp.h)

    def prover_second_round(self, r_v, pp):
        b = _as_bytes(r_v)
        return self._call(lib().spx_prover_second_round, b, len(b) // 32, pp.h)

    def prover_third_round(self, tau):
        b = _as_bytes(tau)
        return self._call(lib().spx_prover_third_round, b, len(b) // 32)

    def prove_first_sumcheck_round(self, challenge=None):
        return self._call(lib().spx_prove_first_sumcheck_round, self._one(challenge))

    def prove_fourth_round(self, last_random_point):
        return self._call(lib().spx_prove_fourth_round, self._one(last_random_point))

    def prove_fifth_round(self, r_a, r_b, r_c):
        return self._call(lib().spx_prove_fifth_round, _as_bytes([r_a, r_b, r_c]))

    def prove_second_sumcheck_round(self, challenge=None):
        return self._call(lib().spx_prove_second_sumcheck_round, self._one(challenge))

    def prove_sixth_round(self, last_random_point, pp):
        return self._call(lib().spx_prove_sixth_round, self._one(last_random_point), pp.h)

    def close(self):
        if self.h:
            lib().spx_prover_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def sumcheck_round(ctx, f, g, r_prev=None):
    """One AHPForMLSumcheck::prove_round of sum_b f(b) g(b) (spx_sumcheck_round): returns
    ([P(0), P(1), P(2)] as 32-byte strings, f', g') with f', g' the tables bound to r_prev (None in
    the first round)."""
    fb, gb = _as_bytes(f), _as_bytes(g)
    # the native side reads 32 n bytes from both tables and 32 from r_prev: check before the call
    if len(fb) != len(gb) or len(fb) % 32:
        raise InvalidArgument("f and g must be equal-length tables of 32-byte field elements")
    n = len(fb) // 32
    ev = ctypes.create_string_buffer(96)
    fo = ctypes.create_string_buffer(max(16 * n, 1))
    go = ctypes.create_string_buffer(max(16 * n, 1))
    rb = None if r_prev is None else _as_bytes([r_prev] if isinstance(r_prev, int) else r_prev)
    if rb is not None and len(rb) != 32:
        raise InvalidArgument("r_prev must be one 32-byte field element")
    _check(lib().spx_sumcheck_round(ctx.h, fb, gb, n, rb, ev, fo, go))
    evals = [ev.raw[32 * k : 32 * k + 32] for k in range(3)]
    if r_prev is None:
        return evals, None, None
    return evals, fo.raw[: 16 * n], go.raw[: 16 * n]


class _Lc(ctypes.Structure):
    _fields_ = [("vars", ctypes.POINTER(ctypes.c_uint64)), ("coeffs", ctypes.c_char_p), ("len", ctypes.c_size_t)]


class ConstraintSystem:
    """R1CS front-end with ark-relations semantics (spx_cs_*): variable ONE = instance 0, inputs
    numbered before witnesses, compactified rows, make_square as test_utils.rs:81-102."""

    ONE = 0

    def __init__(self):
        L = lib()
        L.spx_cs_last_error.restype = ctypes.c_char_p
        h = ctypes.c_void_p()
        self._chk(L.spx_cs_create(ctypes.byref(h)))
        self.h = h

    @staticmethod
    def _chk(rc):
        if rc != 0:
            raise _ERRORS.get(rc, SpartanError)(lib().spx_cs_last_error().decode(errors="replace"))

    def _new(self, fn, value):
        v = ctypes.c_uint64()
        self._chk(fn(self.h, (int(value) % R).to_bytes(32, "little"), ctypes.byref(v)))
        return v.value

    def new_input(self, value):
        return self._new(lib().spx_cs_new_input, value)

    def new_witness(self, value):
        return self._new(lib().spx_cs_new_witness, value)

    @staticmethod
    def _lc(terms):
        terms = list(terms)
        vars_ = (ctypes.c_uint64 * max(len(terms), 1))(*[int(v) for _, v in terms])
        co = b"".join((int(c) % R).to_bytes(32, "little") for c, _ in terms)
        return _Lc(vars_, co, len(terms)), vars_

    def enforce(self, a, b, c):
        """a * b == c over lists of (coefficient, variable)."""
        la, ka = self._lc(a)
        lb, kb = self._lc(b)
        lc, kc = self._lc(c)
        self._chk(lib().spx_cs_enforce(self.h, ctypes.byref(la), ctypes.byref(lb), ctypes.byref(lc)))

    def make_square(self, num_formatted_variables):
        self._chk(lib().spx_cs_make_square(self.h, int(num_formatted_variables)))

    def counts(self):
        a, b, c = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        self._chk(lib().spx_cs_counts(self.h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)))
        return a.value, b.value, c.value

    def is_satisfied(self):
        ok = ctypes.c_int()
        self._chk(lib().spx_cs_is_satisfied(self.h, ctypes.byref(ok)))
        return ok.value == 1

    def to_matrices(self):
        """(A, B, C as Csr, v bytes, w bytes) — the inputs of MLArgumentForR1CS.index / prove."""
        cs = [_CCsr(), _CCsr(), _CCsr()]
        v, w = ctypes.c_void_p(), ctypes.c_void_p()
        self._chk(lib().spx_cs_matrices(self.h, *[ctypes.byref(x) for x in cs], ctypes.byref(v), ctypes.byref(w)))
        ncons, ninst, nwit = self.counts()
        out = []
        for x in cs:
            n = x.n
            rp = [x.row_ptr[i] for i in range(n + 1)]
            nnz = rp[-1]
            col = [x.col[i] for i in range(nnz)]
            val = ctypes.string_at(x.val, 32 * nnz) if nnz else b""
            out.append(Csr(n, rp, col, val))
        vb = ctypes.string_at(v, 32 * ninst)
        wb = ctypes.string_at(w, 32 * nwit) if nwit else b""
        return out[0], out[1], out[2], vb, wb

    def __del__(self):
        try:
            if self.h:
                lib().spx_cs_free(self.h)
        except Exception:
            pass


def verifier_parameter(pp):
    """VerifierParameter bytes (uncompressed) of a keygen-generated PP (setup.rs:91-101)."""
    cap = 8 + 96 + 192 + 8 + 96 * 64
    out = ctypes.create_string_buffer(cap)
    n = ctypes.c_size_t(0)
    _check(lib().spx_vp_from_pp(pp.h, out, cap, ctypes.byref(n)))
    return out.raw[: n.value]


def pairing_product_is_one(g1_uncompressed, g2_uncompressed):
    """prod_i e(P_i, Q_i) == 1 (host pairing; lists of uncompressed point bytes)."""
    n = len(g1_uncompressed)
    assert n == len(g2_uncompressed)
    r = ctypes.c_int(0)
    _check(lib().spx_pairing_check(b"".join(g1_uncompressed), b"".join(g2_uncompressed), n, ctypes.byref(r)))
    return r.value == 1


class MatrixExtension:
    @staticmethod
    def sum_over_y(ctx, matrix, z):
        M = _as_csr(matrix)
        zb = _as_bytes(z)
        out = ctypes.create_string_buffer(32 * M.n)
        c = M.c()
        _check(lib().spx_sum_over_y(ctx.h, ctypes.byref(c), zb, out))
        return out.raw

    @staticmethod
    def eval_on_x(ctx, matrix, r_x):
        M = _as_csr(matrix)
        rb = _as_bytes(r_x)
        out = ctypes.create_string_buffer(32 * M.n)
        c = M.c()
        _check(lib().spx_eval_on_x(ctx.h, ctypes.byref(c), rb, out))
        return out.raw


class MLPolyCommit:
    @staticmethod
    def commit(pp, table):
        tb = _as_bytes(table)
        out = ctypes.create_string_buffer(56)
        _check(lib().spx_commit(pp.ctx.h, pp.h, tb, (len(tb) // 32).bit_length() - 1, out))
        return out.raw

    @staticmethod
    def open(pp, table, point):
        tb, pb = _as_bytes(table), _as_bytes(point)
        nv = len(pb) // 32
        ev = ctypes.create_string_buffer(32)
        pf = ctypes.create_string_buffer(96 + 8 + 96 * nv)
        _check(lib().spx_open(pp.ctx.h, pp.h, tb, nv, pb, ev, pf))
        return ev.raw, pf.raw


def msm_g1(ctx, bases_uncompressed, scalars):
    sb = _as_bytes(scalars)
    out = ctypes.create_string_buffer(96)
    _check(lib().spx_msm_g1(ctx.h, bytes(bases_uncompressed), sb, len(sb) // 32, out))
    return out.raw


def msm_g2(ctx, bases_uncompressed, scalars):
    sb = _as_bytes(scalars)
    out = ctypes.create_string_buffer(192)
    _check(lib().spx_msm_g2(ctx.h, bytes(bases_uncompressed), sb, len(sb) // 32, out))
    return out.raw
