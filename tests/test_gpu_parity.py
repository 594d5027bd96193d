"""GPU parity: the HIP library (through its C ABI) against the C oracle (reference-faithful
restatement, itself pinned to the Python oracle + pairing verifier by the CPU tests) on the same
seeded inputs. Integer/field/point work: bit-exact byte equality everywhere."""
import random

import pytest

pytestmark = pytest.mark.gpu

R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001


def _scalars(n, seed):
    rs = random.Random(seed)
    out = [rs.randrange(R) for _ in range(n)]
    specials = [0, 1, R - 1, 2, (1 << 255) % R, (1 << 128)]
    for i, s in enumerate(specials[: max(0, n - 1)]):
        out[(i * 7919) % n] = s
    return b"".join(x.to_bytes(32, "little") for x in out)


def _pp_bases(oc, nv, seed):
    """uncompressed G1 / G2 bases from an oracle keygen (level 0: 2^nv points each)."""
    b = oc.PP.keygen(nv, seed).serialize()
    n = 1 << nv
    g1 = b[24 : 24 + 96 * n]
    pos = 16
    for i in range(nv):
        pos += 8 + 96 * (n >> i)
    pos += 8 + 8
    g2 = b[pos : pos + 192 * n]
    return g1, g2


@pytest.mark.parametrize("n", [1, 3, 32, 257, 1024])
def test_msm_g1(spx, ctx, oc, n):
    g1, _ = _pp_bases(oc, 10, 5)
    sc = _scalars(n, n)
    assert spx.msm_g1(ctx, g1[: 96 * n], sc) == oc.msm_g1(g1[: 96 * n], sc, n)


@pytest.mark.parametrize("n", [1, 2, 33, 700])
def test_msm_g2(spx, ctx, oc, n):
    _, g2 = _pp_bases(oc, 10, 6)
    sc = _scalars(n, 100 + n)
    assert spx.msm_g2(ctx, g2[: 192 * n], sc) == oc.msm_g2(g2[: 192 * n], sc, n)


def test_msm_repeated_scalar(spx, ctx, oc):
    """all scalars equal: one bucket per window gets every point (multi-level accumulation)."""
    n = 4096
    g1, _ = _pp_bases(oc, 12, 7)
    s = (0xDEADBEEF12345 * 977).to_bytes(32, "little")
    assert spx.msm_g1(ctx, g1[: 96 * n], s * n) == oc.msm_g1(g1[: 96 * n], s * n, n)


@pytest.mark.parametrize("scalar", [1, R - 1, 1 << 200])
def test_msm_g2_degenerate_scalars(spx, ctx, oc, scalar):
    """every scalar equal: each window's references pile into one bucket, past the capacity
    layout's per-bucket slots, so the exact counting-sort fallback runs."""
    n = 700
    _, g2 = _pp_bases(oc, 10, 8)
    s = scalar.to_bytes(32, "little")
    assert spx.msm_g2(ctx, g2[: 192 * n], s * n) == oc.msm_g2(g2[: 192 * n], s * n, n)


@pytest.mark.parametrize("group", ["g1", "g2"])
def test_msm_repeated_bases_doubling_and_cancellation(spx, ctx, oc, group):
    """bases repeated inside one bucket: the accumulation meets P + P (its doubling branch) and
    P + (-P) (scalars s and r - s give opposite digits: the infinity branch), on every window."""
    g1, g2 = _pp_bases(oc, 4, 11)
    w = 96 if group == "g1" else 192
    src = g1 if group == "g1" else g2
    pts = [src[w * i : w * (i + 1)] for i in range(3)]
    s = (0x1234567890ABCDEF1234567 * 131).to_bytes(32, "little")
    t = (R - int.from_bytes(s, "little")).to_bytes(32, "little")
    u = (0xFEDCBA9876543210 << 64 | 77).to_bytes(32, "little")
    bases, sc = [], []
    for k, (pi, reps) in enumerate([(0, 8), (1, 5), (2, 3)]):
        bases += [pts[pi]] * reps
        sc += [s] * reps
    bases += [pts[0], pts[1], pts[1], pts[2]]  # cancellations against the runs above, and a new scalar
    sc += [t, t, u, u]
    b, c, n = b"".join(bases), b"".join(sc), len(bases)
    if group == "g1":
        assert spx.msm_g1(ctx, b, c) == oc.msm_g1(b, c, n)
    else:
        assert spx.msm_g2(ctx, b, c) == oc.msm_g2(b, c, n)


@pytest.mark.parametrize("nv", [3, 6])
def test_keygen_matches_oracle(spx, ctx, oc, nv):
    pp = spx.MLProofForR1CS.setup(ctx, nv, 4242)
    assert pp.serialize_uncompressed() == oc.PP.keygen(nv, 4242).serialize()


@pytest.mark.parametrize("which", ["g1", "g2"])
def test_pp_load_rejects_off_curve_point(spx, ctx, oc, which):
    """a PP whose point is not on the curve is refused (SerializationError), as ark's deserialization does"""
    nv = 4
    b = bytearray(oc.PP.keygen(nv, 9).serialize())
    off = 24 + 96 * 3 + 5 if which == "g1" else 16 + sum(8 + 96 * (16 >> i) for i in range(nv)) + 16 + 192 * 2 + 7
    b[off] ^= 0x01  # a canonical coordinate that no longer satisfies y^2 = x^3 + b
    with pytest.raises(spx.SerializationError):
        spx.PublicParameter.load(ctx, bytes(b))


def test_pp_load_roundtrip(spx, ctx, oc):
    b = oc.PP.keygen(5, 9).serialize()
    assert spx.PublicParameter.load(ctx, b).serialize_uncompressed() == b


@pytest.mark.parametrize("kind,log_n,param", [(0, 8, 0), (2, 9, 5 | (2 << 16)), (1, 10, 0)])
def test_sum_over_y_and_eval_on_x(spx, ctx, oc, kind, log_n, param):
    inst = oc.Instance(kind, log_n, 3, 77 + log_n, param)
    rs = random.Random(log_n)
    r_x = b"".join(rs.randrange(R).to_bytes(32, "little") for _ in range(log_n))
    for M in inst.mats:
        P = spx.Csr(M.n, M.row_ptr, M.col, M.val)
        assert spx.MatrixExtension.sum_over_y(ctx, P, inst.z_bytes) == oc.sum_over_y(M, inst.z_bytes)
        assert spx.MatrixExtension.eval_on_x(ctx, P, r_x) == oc.eval_on_x(M, r_x)


def _with_duplicates(oc, M, seed):
    """M with repeated columns inside rows: about a third of the rows get one or two extra entries
    whose column repeats an earlier entry of the same row, with a fresh value, sometimes between
    other entries. MatrixExtension::new accepts such rows (r1cs_reader.rs:52-60); sum_over_y adds
    every entry, eval_on_x keeps the last one per (x, y) (r1cs_reader.rs:98-108)."""
    rs = random.Random(seed)
    rows = []
    for row in M.to_rows():
        row = list(row)
        if row and rs.random() < 0.35:
            for _ in range(rs.choice((1, 1, 2))):
                col = rs.choice(row)[1]
                row.insert(rs.randrange(len(row) + 1), (rs.randrange(R), col))
        rows.append(row)
    return oc.CsrMatrix.from_rows(rows)


@pytest.mark.parametrize("kind,log_n,param", [(0, 8, 0), (2, 9, 5 | (2 << 16))])
def test_sum_over_y_and_eval_on_x_duplicates(spx, ctx, oc, kind, log_n, param):
    inst = oc.Instance(kind, log_n, 3, 91 + log_n, param)
    rs = random.Random(7 * log_n)
    r_x = b"".join(rs.randrange(R).to_bytes(32, "little") for _ in range(log_n))
    for m, M0 in enumerate(inst.mats):
        M = _with_duplicates(oc, M0, 1000 * log_n + m)
        assert M.nnz > M0.nnz
        P = spx.Csr(M.n, M.row_ptr, M.col, M.val)
        assert spx.MatrixExtension.sum_over_y(ctx, P, inst.z_bytes) == oc.sum_over_y(M, inst.z_bytes)
        assert spx.MatrixExtension.eval_on_x(ctx, P, r_x) == oc.eval_on_x(M, r_x)


@pytest.mark.parametrize("kind,log_n,log_v", [(0, 6, 2), (2, 9, 3), (0, 11, 5)])
@pytest.mark.parametrize("mode", ["fs", "injected"])
def test_prove_bit_exact_duplicates(spx, ctx, oc, kind, log_n, log_v, mode):
    """Full proofs over matrices with repeated (x, y) entries: the transcript hashes every entry,
    Az/Bz/Cz sum them, the eval_on_x pass keeps the last one."""
    param = (3 | (1 << 16)) if kind == 2 else 0
    inst = oc.Instance(kind, log_n, log_v, 3000 + log_n, param)
    mats_o = [_with_duplicates(oc, M, 77 * log_n + m) for m, M in enumerate(inst.mats)]
    ppc = oc.PP.keygen(log_n, 4000 + log_n)
    pp = spx.PublicParameter.load(ctx, ppc.serialize())
    pk = spx.MLArgumentForR1CS.index(ctx, *[spx.Csr(M.n, M.row_ptr, M.col, M.val) for M in mats_o])
    got = spx.MLArgumentForR1CS.prove(pk, inst.v_bytes, inst.w_bytes, pp, mode=mode, seed=66)
    want = oc.prove(mats_o, inst.v_bytes, inst.w_bytes, ppc, 1 if mode == "injected" else 0, 66)
    assert got == want


@pytest.mark.parametrize("nv", [1, 4, 9])
def test_commit_open(spx, ctx, oc, nv):
    ppc = oc.PP.keygen(nv, 31 + nv)
    pp = spx.PublicParameter.load(ctx, ppc.serialize())
    table = _scalars(1 << nv, nv)
    rs = random.Random(nv)
    point = b"".join(rs.randrange(R).to_bytes(32, "little") for _ in range(nv))
    assert spx.MLPolyCommit.commit(pp, table) == oc.commit(ppc, table, nv)
    assert spx.MLPolyCommit.open(pp, table, point) == oc.open_(ppc, table, nv, point)


CASES = [(0, 2, 1), (0, 4, 2), (0, 6, 3), (1, 7, 2), (2, 6, 2), (0, 10, 5), (1, 11, 5), (0, 12, 5), (3, 9, 3), (3, 12, 5)]


@pytest.mark.parametrize("kind,log_n,log_v", CASES)
@pytest.mark.parametrize("mode", ["fs", "injected"])
def test_prove_bit_exact(spx, ctx, oc, kind, log_n, log_v, mode):
    param = (3 | (1 << 16)) if kind == 2 else 0
    if kind == 1 and log_v < 2:
        pytest.skip("ref-shaped needs > 3 public inputs")
    inst = oc.Instance(kind, log_n, log_v, 1000 + log_n, param)
    ppc = oc.PP.keygen(log_n, 2000 + log_n)
    pp = spx.PublicParameter.load(ctx, ppc.serialize())
    mats = [spx.Csr(M.n, M.row_ptr, M.col, M.val) for M in inst.mats]
    pk = spx.MLArgumentForR1CS.index(ctx, *mats)
    got = spx.MLArgumentForR1CS.prove(pk, inst.v_bytes, inst.w_bytes, pp, mode=mode, seed=55)
    want = oc.prove(inst.mats, inst.v_bytes, inst.w_bytes, ppc, 1 if mode == "injected" else 0, 55)
    assert len(got) == len(want)
    if got != want:
        i = next(k for k in range(len(got)) if got[k] != want[k])
        pytest.fail("proof differs from oracle at byte %d of %d" % (i, len(got)))


@pytest.mark.parametrize("cached", [False, True])
def test_prove_many_concurrent(spx, ctx, oc, cached):
    """spx_prove_many: several contexts (streams, MSM workspaces) proving concurrently from one index;
    every proof bit-exact vs the oracle, with and without the index-cached matrix transcript."""
    log_n, log_v = 10, 4
    inst = oc.Instance(0, log_n, log_v, 4242)
    ppc = oc.PP.keygen(log_n, 4343)
    pp = spx.PublicParameter.load(ctx, ppc.serialize())
    mats = [spx.Csr(M.n, M.row_ptr, M.col, M.val) for M in inst.mats]
    pk = spx.MLArgumentForR1CS.index(ctx, *mats)
    wit = spx.Witness(ctx, inst.v_bytes, inst.w_bytes)
    ctxs = [ctx] + [spx.Context(0) for _ in range(2)]
    want = oc.prove(inst.mats, inst.v_bytes, inst.w_bytes, ppc, 0, 0)
    got = spx.MLArgumentForR1CS.prove_many(ctxs, pk, [wit] * 7, pp, cached=cached)
    assert len(got) == 7
    for g in got:
        assert g == want


def test_prove_bit_exact_2_16(spx, ctx, oc):
    """The largest bit-exact case vs the C oracle (2^16 constraints, ~30 s of oracle time); the PP
    comes from the GPU keygen and is loaded into the oracle."""
    log_n, log_v = 16, 5
    inst = oc.Instance(0, log_n, log_v, 0x5EED0000 + log_n)
    pp = spx.MLProofForR1CS.setup(ctx, log_n, 0xC0FFEE)
    ppc = oc.PP.load(pp.serialize_uncompressed())
    mats = [spx.Csr(M.n, M.row_ptr, M.col, M.val) for M in inst.mats]
    pk = spx.MLArgumentForR1CS.index(ctx, *mats)
    got = spx.MLArgumentForR1CS.prove(pk, inst.v_bytes, inst.w_bytes, pp)
    assert got == oc.prove(inst.mats, inst.v_bytes, inst.w_bytes, ppc, 0, 0)


def _with_long_columns(oc, M, seed, extra):
    """M plus entries that make some columns long: column 0 (z[0] = 1, as real circuits use ONE) in
    every row, and columns c in `extra` (c -> count) in `count` random rows each, so columns of the
    eval_on_x stream cross the long-column threshold (kernels.hpp: kLongCol = 62 entries: 62 stays
    short, 63 goes to the chunked path) and rows gain repeated columns too."""
    rs = random.Random(seed)
    rows = [list(r) for r in M.to_rows()]
    n = len(rows)
    for row in rows:
        row.append((rs.randrange(R), 0))
    for c, cnt in extra.items():
        for x in rs.sample(range(n), cnt):
            rows[x].insert(rs.randrange(len(rows[x]) + 1), (rs.randrange(R), c))
    return oc.CsrMatrix.from_rows(rows)


def _sparse_columns(oc, n, seed):
    """a matrix whose entries fall in a few columns: most columns are empty"""
    rs = random.Random(seed)
    rows = [[(rs.randrange(R), rs.choice((1, 2, 3, n - 1)))] if rs.random() < 0.7 else [] for _ in range(n)]
    return oc.CsrMatrix.from_rows(rows)


@pytest.mark.parametrize("log_n", [7, 10, 13])
def test_eval_on_x_long_and_empty_columns(spx, ctx, oc, log_n):
    inst = oc.Instance(0, log_n, 3, 505 + log_n)
    rs = random.Random(log_n)
    r_x = b"".join(rs.randrange(R).to_bytes(32, "little") for _ in range(log_n))
    n = 1 << log_n
    mats = [_with_long_columns(oc, inst.mats[0], log_n, {5: 62, 7: 63, 9: min(n, 4500)}), _sparse_columns(oc, n, log_n)]
    for M in mats:
        P = spx.Csr(M.n, M.row_ptr, M.col, M.val)
        assert spx.MatrixExtension.eval_on_x(ctx, P, r_x) == oc.eval_on_x(M, r_x)
        assert spx.MatrixExtension.sum_over_y(ctx, P, inst.z_bytes) == oc.sum_over_y(M, inst.z_bytes)


@pytest.mark.parametrize("mode", ["fs", "injected"])
def test_prove_bit_exact_long_columns(spx, ctx, oc, mode):
    """Full proofs whose matrices have long columns (chunked path) next to short and empty ones."""
    log_n, log_v = 11, 3
    inst = oc.Instance(0, log_n, log_v, 6000 + log_n)
    mats_o = [_with_long_columns(oc, inst.mats[0], 1, {5: 62, 7: 63, 11: 300}),
              _with_long_columns(oc, inst.mats[1], 2, {6: 100}), _sparse_columns(oc, 1 << log_n, 3)]
    ppc = oc.PP.keygen(log_n, 6100)
    pp = spx.PublicParameter.load(ctx, ppc.serialize())
    pk = spx.MLArgumentForR1CS.index(ctx, *[spx.Csr(M.n, M.row_ptr, M.col, M.val) for M in mats_o])
    got = spx.MLArgumentForR1CS.prove(pk, inst.v_bytes, inst.w_bytes, pp, mode=mode, seed=67)
    want = oc.prove(mats_o, inst.v_bytes, inst.w_bytes, ppc, 1 if mode == "injected" else 0, 67)
    assert got == want
