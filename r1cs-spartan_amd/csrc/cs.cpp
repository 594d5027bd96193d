// R1CS front-end: a constraint-system builder with ark-relations semantics, so a
// circuit can be stated directly against the C ABI instead of through Rust:
//   * variable 0 is the constant One (Variable::One / instance 0); inputs (Variable::Instance) are
//     numbered before witnesses (Variable::Witness) in z = v || w (ConstraintSystem::to_matrices);
//   * every linear combination is compactified when exported: terms sorted by variable, equal
//     variables merged, zero coefficients dropped (LinearCombination::compactify + inline_all_lcs);
//   * make_square pads exactly as test_utils.rs:81-102 (0 * 0 = 0 constraints, or dummy witnesses
//     of value one) and is_satisfied checks <A_i, z> <B_i, z> == <C_i, z> for every row.
// The exported CSR + z feed spx_index / spx_prove directly.
#include <algorithm>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "../../include/spartan_hip.h"
#include "host_ff.hpp"

using spx::host::Fr;

namespace {
constexpr uint64_t kWitness = 1ull << 63;
struct Term {
    Fr c;
    uint64_t var;
};
struct Cons {
    std::vector<Term> lc[3];
};
thread_local std::string g_cs_err;
}  // namespace

struct spx_cs {
    std::vector<Fr> inst{Fr::one()}, wit;
    std::vector<Cons> cons;
    // export cache
    bool fresh = false;
    std::vector<uint64_t> rp[3];
    std::vector<uint32_t> col[3];
    std::vector<uint8_t> val[3], v, w;
};

static int cs_fail(int code, const char* m) {
    g_cs_err = m;
    return code;
}

static uint64_t column(const spx_cs& cs, uint64_t var) {
    return (var & kWitness) ? cs.inst.size() + (var & ~kWitness) : var;
}

static bool read_lc(const spx_cs& cs, const spx_lc* lc, std::vector<Term>& out) {
    out.clear();
    if (!lc) return true;
    if (lc->len && (!lc->vars || !lc->coeffs)) return false;
    for (size_t i = 0; i < lc->len; ++i) {
        Term t;
        if (!spx::host::fr_from_bytes(t.c, lc->coeffs + 32 * i)) return false;
        t.var = lc->vars[i];
        const uint64_t k = t.var & ~kWitness;
        if ((t.var & kWitness) ? k >= cs.wit.size() : k >= cs.inst.size()) return false;
        out.push_back(t);
    }
    return true;
}

static void build(spx_cs& cs) {
    if (cs.fresh) return;
    const uint64_t nz = cs.inst.size() + cs.wit.size();
    for (int m = 0; m < 3; ++m) {
        cs.rp[m].assign(1, 0);
        cs.col[m].clear();
        cs.val[m].clear();
        for (const Cons& c : cs.cons) {
            std::map<uint64_t, Fr> acc;  // compactify: sorted by column, merged
            for (const Term& t : c.lc[m]) {
                auto it = acc.find(column(cs, t.var));
                if (it == acc.end())
                    acc.emplace(column(cs, t.var), t.c);
                else
                    it->second = it->second + t.c;
            }
            for (auto& kv : acc) {
                if (kv.second.is_zero()) continue;
                if (kv.first >= nz || kv.first > 0xffffffffull) throw std::runtime_error("column out of range");
                cs.col[m].push_back((uint32_t)kv.first);
                uint8_t b[32];
                spx::host::fr_to_bytes(b, kv.second);
                cs.val[m].insert(cs.val[m].end(), b, b + 32);
            }
            cs.rp[m].push_back(cs.col[m].size());
        }
    }
    cs.v.resize(32 * cs.inst.size());
    for (size_t i = 0; i < cs.inst.size(); ++i) spx::host::fr_to_bytes(&cs.v[32 * i], cs.inst[i]);
    cs.w.resize(32 * cs.wit.size());
    for (size_t i = 0; i < cs.wit.size(); ++i) spx::host::fr_to_bytes(&cs.w[32 * i], cs.wit[i]);
    cs.fresh = true;
}

extern "C" {

const char* spx_cs_last_error(void) { return g_cs_err.c_str(); }

int spx_cs_create(spx_cs** out) {
    if (!out) return cs_fail(SPX_INVALID_ARGUMENT, "null output");
    *out = new spx_cs();
    return SPX_OK;
}
int spx_cs_free(spx_cs* cs) {
    delete cs;
    return SPX_OK;
}
int spx_cs_new_input(spx_cs* cs, const uint8_t value[32], uint64_t* var) {
    Fr x;
    if (!cs || !var || !value || !spx::host::fr_from_bytes(x, value)) return cs_fail(SPX_INVALID_ARGUMENT, "bad input");
    cs->inst.push_back(x);
    cs->fresh = false;
    *var = cs->inst.size() - 1;
    return SPX_OK;
}
int spx_cs_new_witness(spx_cs* cs, const uint8_t value[32], uint64_t* var) {
    Fr x;
    if (!cs || !var || !value || !spx::host::fr_from_bytes(x, value)) return cs_fail(SPX_INVALID_ARGUMENT, "bad witness");
    cs->wit.push_back(x);
    cs->fresh = false;
    *var = kWitness | (cs->wit.size() - 1);
    return SPX_OK;
}
int spx_cs_enforce(spx_cs* cs, const spx_lc* a, const spx_lc* b, const spx_lc* c) {
    if (!cs) return cs_fail(SPX_INVALID_ARGUMENT, "null constraint system");
    Cons k;
    if (!read_lc(*cs, a, k.lc[0]) || !read_lc(*cs, b, k.lc[1]) || !read_lc(*cs, c, k.lc[2]))
        return cs_fail(SPX_INVALID_ARGUMENT, "bad linear combination (unknown variable or non-canonical coefficient)");
    cs->cons.push_back(std::move(k));
    cs->fresh = false;
    return SPX_OK;
}
int spx_cs_make_square(spx_cs* cs, uint64_t num_formatted_variables) {
    if (!cs) return cs_fail(SPX_INVALID_ARGUMENT, "null constraint system");
    const uint64_t nc = cs->cons.size();
    if (num_formatted_variables > nc)
        cs->cons.resize(num_formatted_variables);  // 0 * 0 == 0
    else
        for (uint64_t i = 0; i < nc - num_formatted_variables; ++i) cs->wit.push_back(Fr::one());
    cs->fresh = false;
    return SPX_OK;
}
int spx_cs_counts(const spx_cs* cs, uint64_t* constraints, uint64_t* instance, uint64_t* witness) {
    if (!cs) return cs_fail(SPX_INVALID_ARGUMENT, "null constraint system");
    if (constraints) *constraints = cs->cons.size();
    if (instance) *instance = cs->inst.size();
    if (witness) *witness = cs->wit.size();
    return SPX_OK;
}
int spx_cs_is_satisfied(spx_cs* cs, int* ok) {
    if (!cs || !ok) return cs_fail(SPX_INVALID_ARGUMENT, "null argument");
    auto eval = [&](const std::vector<Term>& lc) {
        Fr s = Fr::zero();
        for (const Term& t : lc) s = s + t.c * ((t.var & kWitness) ? cs->wit[t.var & ~kWitness] : cs->inst[t.var]);
        return s;
    };
    *ok = 1;
    for (const Cons& c : cs->cons)
        if (!(eval(c.lc[0]) * eval(c.lc[1]) == eval(c.lc[2]))) {
            *ok = 0;
            break;
        }
    return SPX_OK;
}
int spx_cs_matrices(spx_cs* cs, spx_csr* a, spx_csr* b, spx_csr* c, const uint8_t** v, const uint8_t** w) {
    if (!cs || !a || !b || !c) return cs_fail(SPX_INVALID_ARGUMENT, "null argument");
    try {
        build(*cs);
    } catch (const std::exception& e) {
        return cs_fail(SPX_INVALID_ARGUMENT, e.what());
    }
    spx_csr* o[3] = {a, b, c};
    for (int m = 0; m < 3; ++m) {
        o[m]->n = cs->cons.size();
        o[m]->row_ptr = cs->rp[m].data();
        o[m]->col = cs->col[m].data();
        o[m]->val = cs->val[m].data();
    }
    if (v) *v = cs->v.data();
    if (w) *w = cs->wit.empty() ? nullptr : cs->w.data();
    return SPX_OK;
}

}  // extern "C"
