"""Full-size helpers for the tests' verifier replay (test infrastructure, like the rest of oracle/).

Same byte stream / values as spartan.matrix_bytes and spartan.eval_on_x + mle_eval
(r1cs_reader.rs:8-13 serialization; r1cs_reader.rs:91-117 semantics), computed from CSR arrays with
numpy so a 2^20 instance (3M entries) takes seconds instead of minutes."""
import numpy as np

from bls12_381 import R


def matrix_bytes_csr(n, row_ptr, col, val_bytes):
    """CanonicalSerialize of MatrixExtension{constraint: Vec<Vec<(F, usize)>>, num_constraints} from CSR.
    val_bytes: 32-byte canonical LE Fr per entry."""
    rp = np.asarray(row_ptr, dtype=np.uint64)
    cols = np.asarray(col, dtype=np.uint64)
    nnz = int(rp[-1])
    vals = np.frombuffer(val_bytes, dtype=np.uint8, count=32 * nnz).reshape(nnz, 32)
    total = 8 + 8 * n + 40 * nnz + 8
    out = np.zeros(total, dtype=np.uint8)
    out[0:8] = np.frombuffer(np.uint64(n).tobytes(), dtype=np.uint8)
    rows = np.arange(n, dtype=np.uint64)
    row_pos = 8 + 8 * rows + 40 * rp[:-1]
    lens = (rp[1:] - rp[:-1]).astype(np.uint64)
    out[(row_pos[:, None] + np.arange(8, dtype=np.uint64)).ravel()] = lens.view(np.uint8)
    if nnz:
        row_of = np.repeat(rows, lens.astype(np.int64))
        k = np.arange(nnz, dtype=np.uint64)
        pos = 16 + 8 * row_of + 40 * k
        out[(pos[:, None] + np.arange(32, dtype=np.uint64)).ravel()] = vals.ravel()
        out[(pos[:, None] + 32 + np.arange(8, dtype=np.uint64)).ravel()] = cols.view(np.uint8)
    out[total - 8 :] = np.frombuffer(np.uint64(n).tobytes(), dtype=np.uint8)
    return out.tobytes()


def eq_table(point):
    """eq(point, x) for all x, variable 0 = LSB of x."""
    t = [1]
    for r in point:
        one_m = (1 - r) % R
        t = [v * one_m % R for v in t] + [v * r % R for v in t]
    return t


def sparse_eval(n, row_ptr, col, val_bytes, eqx, eqy):
    """M(r_x, r_y) = sum_{(x, y, a) in M} a eq(r_x, x) eq(r_y, y); rows are x (constraints), columns y.
    A row that repeats a column contributes only its last entry for it (eval_on_x's map insert,
    r1cs_reader.rs:98-108)."""
    rp = list(row_ptr)
    acc = 0
    for x in range(n):
        ex = eqx[x]
        row = {}
        for k in range(rp[x], rp[x + 1]):
            row[col[k]] = int.from_bytes(val_bytes[32 * k : 32 * k + 32], "little")
        for y, a in row.items():
            acc += a * eqy[y] % R * ex
    return acc % R
