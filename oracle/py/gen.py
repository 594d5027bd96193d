"""ORACLE — TEST INFRASTRUCTURE ONLY.

Deterministic synthetic-input generators shared (draw for draw) with the C oracle
(oracle/c/gen.c) and the product's instance generator, so that large instances are
regenerated on the GPU box instead of shipped.

PRNG: SplitMix64. `next_fr` = 4 x next_u64 as little-endian limbs, top limb masked to 63
bits, rejected while >= r; the value is CANONICAL (this is our generator, not Fr::rand).

Generators:
  * `uniform_3n(log_n, log_v, seed)` — SURVEY §8(d) primary: satisfiable, one entry per row in
    each of A, B, C (uniform random columns), C's coefficient chosen so Az∘Bz = Cz.
  * `ref_shaped(log_n, log_v, density, seed)` — restates the reference's TestSynthesizer
    (/root/reference/src/data_structures/constraints.rs:39-110) + make_matrices_square
    (/root/reference/src/test_utils.rs:81-102) + generate_circuit_with_random_input
    (test_utils.rs:51-79) with ark-relations matrix conventions [upstream]: column 0 = One,
    instance variables next, witnesses after; each row's entries sorted by column with
    duplicate variables merged. Draws come from SplitMix64 instead of test_rng().
  * `circuit_3n(log_n, log_v, seed, wseed)` — the benchmark's fixed index with many witnesses:
    rows x < n - |v| define a fresh private variable o_x (Fisher-Yates permutation of the private
    columns) by (alpha, a) x (beta, b) = (1, o_x) over variables defined earlier; the last |v| rows
    are (alpha, a) x (1, One) = (alpha, a). `wseed` draws the public inputs; the rest follows.
  * `random_matrix(log_size, nnz, seed)` — restates test_utils.rs:18-37 (row lists in
    insertion order, unique (x, y) positions).
A matrix is a list of n rows, each a list of (coeff, col) — ark-relations `Matrix<F>`.
"""
from bls12_381 import R, fr_inv

MASK64 = (1 << 64) - 1


class SplitMix64:
    def __init__(self, seed):
        self.state = seed & MASK64

    def next_u64(self):
        self.state = (self.state + 0x9E3779B97F4A7C15) & MASK64
        z = self.state
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK64
        return z ^ (z >> 31)

    def next_fr(self):
        while True:
            l0 = self.next_u64()
            l1 = self.next_u64()
            l2 = self.next_u64()
            l3 = self.next_u64() & ((1 << 63) - 1)
            v = l0 | (l1 << 64) | (l2 << 128) | (l3 << 192)
            if v < R:
                return v

    def next_fr_nonzero(self):
        while True:
            v = self.next_fr()
            if v:
                return v

    def below(self, k):
        """Uniform-ish integer in [0, k) (our own rule; stands in for rand's gen_range)."""
        return self.next_u64() % k


def default_seed(log_n):
    return 0x5EED0000 + log_n


def uniform_3n(log_n, log_v=5, seed=None):
    n = 1 << log_n
    if seed is None:
        seed = default_seed(log_n)
    rng = SplitMix64(seed)
    z = [1] + [rng.next_fr_nonzero() for _ in range(n - 1)]
    A, B, C = [], [], []
    m = n - 1
    for _x in range(n):
        a = rng.next_u64() & m
        alpha = rng.next_fr()
        b = rng.next_u64() & m
        beta = rng.next_fr()
        c = rng.next_u64() & m
        gamma = alpha * z[a] % R * beta % R * z[b] % R * fr_inv(z[c]) % R
        A.append([(alpha, a)])
        B.append([(beta, b)])
        C.append([(gamma, c)])
    nv = 1 << log_v
    return A, B, C, z[:nv], z[nv:]


def circuit_3n(log_n, log_v=5, seed=None, wseed=0):
    n, nv = 1 << log_n, 1 << log_v
    if seed is None:
        seed = default_seed(log_n)
    rng = SplitMix64(seed)
    perm = list(range(nv, n))
    for i in range(len(perm) - 1, 0, -1):
        j = rng.next_u64() % (i + 1)
        perm[i], perm[j] = perm[j], perm[i]
    avail = list(range(nv))
    A, B, C = [], [], []
    for x in range(n):
        a = avail[rng.next_u64() % len(avail)]
        alpha = rng.next_fr()
        A.append([(alpha, a)])
        if x + nv < n:
            b = avail[rng.next_u64() % len(avail)]
            B.append([(rng.next_fr(), b)])
            C.append([(1, perm[x])])
            avail.append(perm[x])
        else:
            B.append([(1, 0)])
            C.append([(alpha, a)])
    w = SplitMix64(wseed)
    z = [0] * n
    z[0] = 1
    for i in range(1, nv):
        z[i] = w.next_fr_nonzero()
    for x in range(n - nv):
        (al, a), (be, b), (_one, o) = A[x][0], B[x][0], C[x][0]
        z[o] = al * z[a] % R * be % R * z[b] % R
    return A, B, C, z[:nv], z[nv:]


def _row_from_terms(terms):
    """Compactify a list of (coeff, col): sort by column, merge duplicates, drop zeros."""
    acc = {}
    for coeff, col in terms:
        acc[col] = (acc.get(col, 0) + coeff) % R
    return [(acc[c], c) for c in sorted(acc) if acc[c] != 0]


def ref_shaped(log_n, log_v=5, density=0, seed=None, raw=False):
    n = 1 << log_n
    num_public = 1 << log_v
    num_private = n - num_public
    assert num_public > 3
    if seed is None:
        seed = default_seed(log_n) ^ 0xA5A5
    rng = SplitMix64(seed)
    # variables: ("i", k) instance k (k=0 is One), ("w", k) witness k
    inst_vals = [1]
    wit_vals = []
    cons = []  # (a_terms, b_terms, c_terms) with terms over variables

    def new_input(val):
        inst_vals.append(val)
        return ("i", len(inst_vals) - 1)

    def new_witness(val):
        wit_vals.append(val)
        return ("w", len(wit_vals) - 1)

    one = ("i", 0)
    assignments = []
    a_val = rng.next_fr()
    a_var = new_input(a_val)
    assignments.append((a_val, a_var))
    b_val = rng.next_fr()
    b_var = new_input(b_val)
    assignments.append((a_val, a_var))  # sic: constraints.rs:47 pushes (a_val, a_var) again
    for _ in range(num_public - 3):
        val = rng.next_fr()
        var = new_input(val)
        assignments.append((val, var))
    num_sparse = (num_private - 1) * (510 - density) // 510
    for i in range(num_sparse):
        off_idx = 2 + rng.below(num_public - 3)  # gen_range(2, num_public - 1)
        off_val, off_var = assignments[off_idx]
        if i % 2 != 0:
            c_val = a_val * ((b_val + off_val) % R) % R
            c_var = new_witness(c_val)
            cons.append(([(1, a_var)], [(1, b_var), (1, off_var)], [(1, c_var)]))
        else:
            c_val = (a_val + b_val + off_val) % R
            c_var = new_witness(c_val)
            cons.append(([(1, a_var), (1, b_var), (1, off_var)], [(1, one)], [(1, c_var)]))
        assignments.append((c_val, c_var))
        a_val, a_var = b_val, b_var
        b_val, b_var = c_val, c_var
    for _ in range(num_sparse, num_private):
        lc = [(1, var) for (_v, var) in assignments]
        c_val = 0
        for val, _var in assignments:
            c_val = (c_val + val) % R
        c_val = c_val * c_val % R
        c_var = new_witness(c_val)
        cons.append((lc, list(lc), [(1, c_var)]))
    raw_cons = [tuple(list(x) for x in k) for k in cons]
    # make_matrices_square: add 0*0 = 0 constraints
    while len(cons) < num_public + num_private:
        cons.append(([], [], []))
    ninst = len(inst_vals)

    def col(var):
        kind, k = var
        return k if kind == "i" else ninst + k

    A = [_row_from_terms([(c, col(v)) for c, v in a]) for a, _b, _c in cons]
    B = [_row_from_terms([(c, col(v)) for c, v in b]) for _a, b, _c in cons]
    C = [_row_from_terms([(c, col(v)) for c, v in cc]) for _a, _b, cc in cons]
    assert ninst == num_public and ninst + len(wit_vals) == n
    if raw:  # the constraints before padding, over ("i", k) / ("w", k) variables (front-end tests)
        return A, B, C, inst_vals, wit_vals, raw_cons, num_public + num_private
    return A, B, C, inst_vals, wit_vals


def random_matrix(log_size, num_non_zero, seed):
    bound = 1 << log_size
    rng = SplitMix64(seed)
    mat = [[] for _ in range(bound)]
    added = set()
    for _ in range(num_non_zero):
        x = rng.next_u64() & (bound - 1)
        y = rng.next_u64() & (bound - 1)
        while (x, y) in added:
            x = rng.next_u64() & (bound - 1)
            y = rng.next_u64() & (bound - 1)
        added.add((x, y))
        mat[x].append((rng.next_fr(), y))
    return mat


def ragged(log_n, log_v, max_row, seed, dense_rows=0):
    """Unsatisfiable stress instance: rows with 0..max_row entries (empty rows included),
    plus `dense_rows` rows of ~7n/8 entries in A and B (nnz skew). Columns are unsorted but
    distinct within a row: ark-relations matrices never repeat a (row, col) position, and the
    reference's eval_on_x (hash-map keyed) and sum_over_y (summing) would disagree if they did."""
    n = 1 << log_n
    rng = SplitMix64(seed)
    z = [1] + [rng.next_fr() for _ in range(n - 1)]
    mats = []
    for _m in range(3):
        rows = []
        for _x in range(n):
            k = min(rng.below(max_row + 1), n)
            cols = []
            while len(cols) < k:
                y = rng.next_u64() & (n - 1)
                if y not in cols:
                    cols.append(y)
            rows.append([(rng.next_fr(), y) for y in cols])
        mats.append(rows)
    for d in range(dense_rows):
        x = rng.next_u64() & (n - 1)
        for m in (0, 1):
            mats[m][x] = [(rng.next_fr(), y) for y in range(n) if rng.below(8) != 0]
    nv = 1 << log_v
    return mats[0], mats[1], mats[2], z[:nv], z[nv:]
