"""R1CS front-end (spx_cs_*, ark-relations ConstraintSystem semantics), host only:
TestSynthesizer's constraints (constraints.rs:39-110, restated by the oracle's ref_shaped) entered
through the builder and padded with make_square (test_utils.rs:81-102) must export exactly the
oracle's matrices and assignment; satisfiability checks and both padding branches."""
import pytest

import gen
from bls12_381 import R


def _build(spx, raw_cons, inst_vals, wit_vals):
    cs = spx.ConstraintSystem()
    var = {("i", 0): spx.ConstraintSystem.ONE}
    for k, v in enumerate(inst_vals[1:], start=1):
        var[("i", k)] = cs.new_input(v)
    for k, v in enumerate(wit_vals):
        var[("w", k)] = cs.new_witness(v)
    for a, b, c in raw_cons:
        cs.enforce([(x, var[u]) for x, u in a], [(x, var[u]) for x, u in b], [(x, var[u]) for x, u in c])
    return cs


def _rows(M):
    rp = [M.row_ptr[i] for i in range(M.n + 1)]
    return [[(int.from_bytes(M.val.raw[32 * k : 32 * k + 32], "little"), M.col[k]) for k in range(rp[x], rp[x + 1])]
            for x in range(M.n)]


@pytest.mark.parametrize("log_n,log_v,density", [(5, 3, 0), (7, 4, 3), (8, 3, 200)])
def test_test_synthesizer_through_builder(spx, log_n, log_v, density):
    A, B, C, inst, wit, raw, nfmt = gen.ref_shaped(log_n, log_v, density, seed=77 + log_n, raw=True)
    cs = _build(spx, raw, inst, wit)
    assert cs.is_satisfied()
    cs.make_square(nfmt)
    assert cs.counts() == (1 << log_n, len(inst), len(wit))
    a, b, c, v, w = cs.to_matrices()
    assert (_rows(a), _rows(b), _rows(c)) == (A, B, C)
    assert v == b"".join(x.to_bytes(32, "little") for x in inst)
    assert w == b"".join(x.to_bytes(32, "little") for x in wit)


def test_compactify_and_satisfaction(spx):
    cs = spx.ConstraintSystem()
    x = cs.new_input(3)
    y = cs.new_witness(5)
    z = cs.new_witness(15)
    # (x + x - x) * (y + 0 x) == z, duplicate and zero terms compactified away
    cs.enforce([(1, x), (1, x), (R - 1, x)], [(1, y), (0, x)], [(1, z)])
    assert cs.is_satisfied()
    a, b, c, v, w = cs.to_matrices()
    assert _rows(a) == [[(1, 1)]] and _rows(b) == [[(1, 2)]] and _rows(c) == [[(1, 3)]]
    cs.enforce([(1, y)], [(1, y)], [(1, z)])  # 25 != 15
    assert not cs.is_satisfied()


def test_make_square_branches(spx):
    cs = spx.ConstraintSystem()
    a = cs.new_input(2)
    cs.enforce([(1, a)], [(1, a)], [(4, spx.ConstraintSystem.ONE)])
    cs.make_square(4)  # more variables than constraints: 0 * 0 = 0 rows
    assert cs.counts() == (4, 2, 0)
    cs2 = spx.ConstraintSystem()
    b = cs2.new_input(1)
    for _ in range(4):
        cs2.enforce([(1, b)], [(1, b)], [(1, b)])
    cs2.make_square(2)  # more constraints than variables: witnesses of value one
    assert cs2.counts() == (4, 2, 2)
    assert cs2.is_satisfied()


def test_bad_variables_rejected(spx):
    cs = spx.ConstraintSystem()
    with pytest.raises(spx.InvalidArgument):
        cs.enforce([(1, 5)], [], [])  # unknown instance variable
    with pytest.raises(spx.InvalidArgument):
        cs.enforce([(1, (1 << 63) | 0)], [], [])  # unknown witness variable
