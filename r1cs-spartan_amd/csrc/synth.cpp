// Synthetic R1CS instances for the benchmark and large-size tests, generated on
// the host from SplitMix64 so multi-million-constraint instances are regenerated on the GPU box
// instead of shipped. Same draw order as the test oracle's generators (tests check equality).
//   kind 0 "uniform-3n": z[0] = 1, z[i] uniform non-zero; each row has one entry in A, B, C at
//          uniform columns; C's coefficient makes Az o Bz = Cz (satisfiable, nnz = 3n).
//   kind 1 "ref-shaped": the reference's TestSynthesizer chain circuit
//          (/root/reference/src/data_structures/constraints.rs:39-110, density 0 by default) padded
//          square (test_utils.rs:81-102): one dense row of ~n entries in A and B.
//   kind 3 "circuit-3n": a FIXED index with many satisfying witnesses (the benchmark proves distinct
//          witnesses of one index). Rows x < n - |v| each define a fresh output variable o_x (a random
//          permutation of the private columns): A = (alpha, a), B = (beta, b), C = (1, o_x) with a, b
//          drawn uniformly from the variables defined so far, so z[o_x] = alpha z[a] beta z[b]. The
//          last |v| rows are (alpha, a) x (1, One) = (alpha, a). The witness seed draws the public
//          inputs z[1..|v|); every private value follows from them. nnz = 3n; scalars uniform.
#include "../../include/spartan_hip.h"

#include <algorithm>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "host_ff.hpp"

using spx::host::Fr;

namespace {
struct Sm {
    uint64_t s;
    uint64_t next() {
        s += 0x9E3779B97F4A7C15ULL;
        uint64_t z = s;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
        return z ^ (z >> 31);
    }
    // canonical draw kept as canonical limbs (no Montgomery round trip for values we only store)
    void fr_canon(uint64_t c[4]) {
        for (;;) {
            c[0] = next(), c[1] = next(), c[2] = next(), c[3] = next() & 0x7FFFFFFFFFFFFFFFULL;
            if (!Fr::geq_p(c)) return;
        }
    }
};
struct Mat {
    std::vector<uint64_t> rp;
    std::vector<uint32_t> col;
    std::vector<uint8_t> val;
    void push(uint32_t c, const uint64_t v[4]) {
        col.push_back(c);
        val.insert(val.end(), (const uint8_t*)v, (const uint8_t*)v + 32);
    }
};
}  // namespace

struct spx_synth {
    int kind = 0, log_n = 0, log_v = 0;
    uint64_t n = 0;
    Mat m[3];
    std::vector<uint8_t> z;  // canonical bytes
};

static Fr fr_at(const Mat& M, uint64_t k) {
    uint64_t c[4];
    memcpy(c, &M.val[32 * k], 32);
    return Fr::from_canon(c);
}

// kind 3: the witness of `wseed` for the circuit in S.m (canonical bytes into out, 32 n)
static void circuit_witness(const spx_synth& S, uint64_t wseed, uint8_t* out) {
    const uint64_t n = S.n, nv = 1ull << S.log_v;
    Sm w{wseed};
    std::vector<Fr> z(n);
    z[0] = Fr::one();
    uint64_t c[4];
    for (uint64_t i = 1; i < nv; ++i) {
        do w.fr_canon(c);
        while (!(c[0] | c[1] | c[2] | c[3]));
        z[i] = Fr::from_canon(c);
    }
    for (uint64_t x = 0; x + nv < n; ++x)
        z[S.m[2].col[x]] = fr_at(S.m[0], x) * z[S.m[0].col[x]] * fr_at(S.m[1], x) * z[S.m[1].col[x]];
    for (uint64_t i = 0; i < n; ++i) spx::host::fr_to_bytes(out + 32 * i, z[i]);
}

static void gen_circuit(spx_synth& S, uint64_t seed, uint64_t wseed) {
    const uint64_t n = S.n, nv = 1ull << S.log_v;
    if (nv < 2 || nv >= n) throw std::invalid_argument("circuit-3n needs 2 <= |v| < n");
    Sm r{seed};
    std::vector<uint32_t> perm(n - nv);
    for (uint64_t i = 0; i < n - nv; ++i) perm[i] = (uint32_t)(nv + i);
    for (uint64_t i = n - nv - 1; i >= 1; --i) std::swap(perm[i], perm[r.next() % (i + 1)]);
    std::vector<uint32_t> avail;
    avail.reserve(n);
    for (uint64_t i = 0; i < nv; ++i) avail.push_back((uint32_t)i);
    for (int k = 0; k < 3; ++k) {
        S.m[k].rp.resize(n + 1);
        S.m[k].col.reserve(n);
        S.m[k].val.reserve(32 * n);
        for (uint64_t x = 0; x <= n; ++x) S.m[k].rp[x] = x;
    }
    uint64_t c[4];
    const uint64_t one[4] = {1, 0, 0, 0};
    for (uint64_t x = 0; x < n; ++x) {
        const uint32_t a = avail[r.next() % avail.size()];
        r.fr_canon(c);
        S.m[0].push(a, c);
        if (x + nv < n) {
            const uint32_t b = avail[r.next() % avail.size()];
            r.fr_canon(c);
            S.m[1].push(b, c);
            S.m[2].push(perm[x], one);
            avail.push_back(perm[x]);
        } else {
            S.m[1].push(0, one);
            S.m[2].push(a, (const uint64_t*)&S.m[0].val[32 * x]);
        }
    }
    S.z.resize(32 * n);
    circuit_witness(S, wseed, S.z.data());
}

static void gen_uniform(spx_synth& S, uint64_t seed) {
    const uint64_t n = S.n, mask = n - 1;
    Sm r{seed};
    std::vector<Fr> z(n);
    S.z.resize(32 * n);
    z[0] = Fr::one();
    uint64_t c[4] = {1, 0, 0, 0};
    memcpy(&S.z[0], c, 32);
    for (uint64_t i = 1; i < n; ++i) {
        do r.fr_canon(c);
        while (!(c[0] | c[1] | c[2] | c[3]));
        memcpy(&S.z[32 * i], c, 32);
        z[i] = Fr::from_canon(c);
    }
    std::vector<uint64_t> ai(n), bi(n), ci(n);
    std::vector<Fr> al(n), be(n);
    for (int k = 0; k < 3; ++k) {
        S.m[k].rp.assign(n + 1, 0);
        S.m[k].col.reserve(n);
        S.m[k].val.reserve(32 * n);
    }
    std::vector<Fr> zc(n);
    for (uint64_t x = 0; x < n; ++x) {
        ai[x] = r.next() & mask;
        r.fr_canon(c);
        S.m[0].push((uint32_t)ai[x], c);
        al[x] = Fr::from_canon(c);
        bi[x] = r.next() & mask;
        r.fr_canon(c);
        S.m[1].push((uint32_t)bi[x], c);
        be[x] = Fr::from_canon(c);
        ci[x] = r.next() & mask;
        zc[x] = z[ci[x]];
    }
    spx::host::batch_inverse(zc);
    for (uint64_t x = 0; x < n; ++x) {
        Fr g = al[x] * z[ai[x]] * be[x] * z[bi[x]] * zc[x];
        g.to_canon(c);
        S.m[2].push((uint32_t)ci[x], c);
        for (int k = 0; k < 3; ++k) S.m[k].rp[x + 1] = x + 1;
    }
}

static void push_lc(Mat& M, std::vector<uint64_t>& cols, uint64_t x) {
    std::sort(cols.begin(), cols.end());
    for (size_t i = 0; i < cols.size();) {
        size_t j = i;
        while (j < cols.size() && cols[j] == cols[i]) ++j;
        uint64_t c[4] = {(uint64_t)(j - i), 0, 0, 0};
        M.push((uint32_t)cols[i], c);
        i = j;
    }
    M.rp[x + 1] = M.col.size();
}

static void gen_ref(spx_synth& S, uint64_t seed, int density) {
    const uint64_t n = S.n, num_public = 1ull << S.log_v, num_private = n - num_public;
    if (num_public <= 3) throw std::invalid_argument("number of public variables should be greater to 3");
    Sm r{seed};
    std::vector<Fr> z(n, Fr::zero());
    z[0] = Fr::one();
    struct As {
        uint64_t var;
        Fr val;
    };
    std::vector<As> as;
    as.reserve(n + 4);
    uint64_t c[4];
    uint64_t ninst = 1, nwit = 0;
    r.fr_canon(c);
    Fr a_val = Fr::from_canon(c);
    uint64_t a_var = ninst++;
    z[a_var] = a_val;
    as.push_back({a_var, a_val});
    r.fr_canon(c);
    Fr b_val = Fr::from_canon(c);
    uint64_t b_var = ninst++;
    z[b_var] = b_val;
    as.push_back({a_var, a_val});  // sic: constraints.rs:47
    for (uint64_t i = 0; i + 3 < num_public; ++i) {
        r.fr_canon(c);
        Fr v = Fr::from_canon(c);
        uint64_t var = ninst++;
        z[var] = v;
        as.push_back({var, v});
    }
    for (int k = 0; k < 3; ++k) S.m[k].rp.assign(n + 1, 0);
    const uint64_t num_sparse = (num_private - 1) * (uint64_t)(510 - density) / 510;
    uint64_t x = 0;
    std::vector<uint64_t> cols;
    for (uint64_t i = 0; i < num_sparse; ++i, ++x) {
        uint64_t off_idx = 2 + r.next() % (num_public - 3);
        Fr off_val = as[off_idx].val;
        uint64_t off_var = as[off_idx].var;
        uint64_t c_var = num_public + nwit++;
        Fr c_val;
        if (i % 2 != 0) {
            c_val = a_val * (b_val + off_val);
            cols = {a_var};
            push_lc(S.m[0], cols, x);
            cols = {b_var, off_var};
            push_lc(S.m[1], cols, x);
        } else {
            c_val = a_val + b_val + off_val;
            cols = {a_var, b_var, off_var};
            push_lc(S.m[0], cols, x);
            cols = {0};
            push_lc(S.m[1], cols, x);
        }
        cols = {c_var};
        push_lc(S.m[2], cols, x);
        z[c_var] = c_val;
        as.push_back({c_var, c_val});
        a_val = b_val, a_var = b_var;
        b_val = c_val, b_var = c_var;
    }
    for (uint64_t i = num_sparse; i < num_private; ++i, ++x) {
        Fr cv = Fr::zero();
        for (auto& e : as) cv += e.val;
        cv = cv * cv;
        uint64_t c_var = num_public + nwit++;
        cols.clear();
        for (auto& e : as) cols.push_back(e.var);
        push_lc(S.m[0], cols, x);
        cols.clear();
        for (auto& e : as) cols.push_back(e.var);
        push_lc(S.m[1], cols, x);
        cols = {c_var};
        push_lc(S.m[2], cols, x);
        z[c_var] = cv;
    }
    for (; x < n; ++x)
        for (int k = 0; k < 3; ++k) S.m[k].rp[x + 1] = S.m[k].col.size();
    S.z.resize(32 * n);
    for (uint64_t i = 0; i < n; ++i) spx::host::fr_to_bytes(&S.z[32 * i], z[i]);
}

extern "C" {

int spx_synth_create(int kind, int log_n, int log_v, uint64_t seed, uint64_t param, spx_synth** out) {
    try {
        if (log_n < 1 || log_n > 28 || log_v < 0 || log_v > log_n) return SPX_INVALID_ARGUMENT;
        auto S = std::make_unique<spx_synth>();
        S->log_n = log_n;
        S->log_v = log_v;
        S->kind = kind;
        S->n = 1ull << log_n;
        if (kind == 0)
            gen_uniform(*S, seed);
        else if (kind == 1)
            gen_ref(*S, seed, (int)param);
        else if (kind == 3)
            gen_circuit(*S, seed, param);
        else
            return SPX_INVALID_ARGUMENT;
        *out = S.release();
        return SPX_OK;
    } catch (...) {
        return SPX_INVALID_ARGUMENT;
    }
}
uint64_t spx_synth_nnz(const spx_synth* s, int m) { return s->m[m].col.size(); }
int spx_synth_csr(const spx_synth* s, int m, spx_csr* out) {
    if (!s || m < 0 || m > 2 || !out) return SPX_INVALID_ARGUMENT;
    out->n = s->n;
    out->row_ptr = s->m[m].rp.data();
    out->col = s->m[m].col.data();
    out->val = s->m[m].val.data();
    return SPX_OK;
}
const uint8_t* spx_synth_z(const spx_synth* s) { return s->z.data(); }
int spx_synth_witnesses(const spx_synth* s, uint64_t wseed0, int count, uint8_t* z_out) {
    if (!s || s->kind != 3 || count < 0 || (count && !z_out)) return SPX_INVALID_ARGUMENT;
    const int nt = std::max(1, std::min<int>(count, (int)std::thread::hardware_concurrency()));
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t)
        th.emplace_back([=] {
            for (int i = t; i < count; i += nt) circuit_witness(*s, wseed0 + (uint64_t)i, z_out + 32 * s->n * (size_t)i);
        });
    for (auto& t : th) t.join();
    return SPX_OK;
}
int spx_synth_free(spx_synth* s) {
    delete s;
    return SPX_OK;
}

}  // extern "C"
