"""Generates r1cs-spartan_amd/csrc/ff_asm.hpp: product-scanning (FIPS) Montgomery multiplication for
BLS12-381 Fr (8 x u32) and Fq (12 x u32) on gfx950. Every limb product is one v_mad_u64_u32 whose
64-bit carry-out lands in VCC and is absorbed by one v_addc_co_u32 into the third accumulator word
(2 instructions per product; the compiler's own lowering of the same C needs ~4). The column
bookkeeping (Montgomery quotient word, shifts) stays in C so the register allocator sees it.

Column k of the 2N-1 columns (Koc et al., FIPS):
  acc += sum_{i+j=k} a_i b_j + sum_{i+j=k, i<min(k,N)} m_i p_j        (asm mac chain)
  k <  N: m_k = lo(acc) * (-p^-1 mod 2^32); acc += m_k p_0            (low word becomes 0)
  k >= N: r_{k-N} = lo(acc)
  acc >>= 32
Result < 2p (spare top bits), one conditional subtraction.

fr_mul_x2_asm: two independent Fr products whose chains are interleaved instruction by instruction
(the second chain's carries in an SGPR pair instead of VCC), so one wave has two independent
multiply-accumulate chains in flight: the Fr kernels are bound by the dependent chain.
"""
import os

MODS = {
    "Fr": (8, 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001),
    "Fq": (12, 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB),
}


def limbs(x, n):
    return [(x >> (32 * i)) & 0xFFFFFFFF for i in range(n)]


def gen(name, N, p):
    P = limbs(p, N)
    inv = (-pow(p, -1, 1 << 32)) % (1 << 32)
    L = []
    L.append("// %s: N = %d limbs, p' = 0x%08x" % (name, N, inv))
    L.append("DEV void %s_mul_asm(Fe<%sCfg>& r, const Fe<%sCfg>& A, const Fe<%sCfg>& B) {" % (name.lower(), name, name, name))
    L.append("    const uint32_t* a = A.v;")
    L.append("    const uint32_t* b = B.v;")
    L.append("    uint32_t m[%d], t[%d];" % (N, N))
    L.append("    uint64_t acc = 0;")
    L.append("    uint32_t top;")
    for k in range(2 * N - 1):
        terms = []
        for i in range(max(0, k - N + 1), min(k, N - 1) + 1):
            terms.append(("a", i, "b", k - i))
        for i in range(max(0, k - N + 1), min(k - 1, N - 1) + 1):
            terms.append(("m", i, "p", k - i))
        L.append("    top = 0;")
        if terms:
            asm_lines = []
            ins = []
            for (x, i, y, j) in terms:
                xi = "%s%d" % (x, i)
                yj = "%s%d" % (y, j)
                asm_lines.append('"v_mad_u64_u32 %%[acc], vcc, %%[%s], %%[%s], %%[acc]\\n\\t"' % (xi, yj))
                asm_lines.append('"v_addc_co_u32 %[top], vcc, 0, %[top], vcc\\n\\t"')
                for nm in (xi, yj):
                    if nm not in [q[0] for q in ins]:
                        if nm[0] == "p":
                            ins.append((nm, '"s"(0x%08xu)' % P[int(nm[1:])]))
                        else:
                            ins.append((nm, '"v"(%s[%s])' % (nm[0], nm[1:])))
            L.append("    asm(" + "\n        ".join(asm_lines))
            L.append('        : [acc] "+v"(acc), [top] "+v"(top)')
            L.append("        : " + ", ".join("[%s] %s" % (nm, c) for nm, c in ins))
            L.append('        : "vcc");')
        if k < N and P[0] == 1 and inv == 0xFFFFFFFF:
            # Fr: m_k = -lo(acc), and lo(acc) + m_k * p_0 = 2^32 exactly when lo(acc) != 0, so the
            # shifted accumulator just takes that carry (no 64-bit add and compare)
            L.append("    m[%d] = 0u - (uint32_t)acc;" % k)
            L.append("    acc = (acc >> 32) + ((uint64_t)top << 32) + (uint64_t)((uint32_t)acc != 0u);")
            continue
        if k < N:
            L.append("    m[%d] = (uint32_t)acc * 0x%08xu;" % (k, inv))
            L.append("    {")
            L.append("        uint64_t s;")
            L.append("        top += __builtin_add_overflow(acc, (uint64_t)m[%d] * 0x%08xu, &s);" % (k, P[0]))
            L.append("        acc = s;")
            L.append("    }")
        else:
            L.append("    t[%d] = (uint32_t)acc;" % (k - N))
        L.append("    acc = (acc >> 32) | ((uint64_t)top << 32);")
    L.append("    t[%d] = (uint32_t)acc;" % (N - 1))
    L.append("    fe_reduce_once<%sCfg>(r, t);" % name)
    L.append("}")
    return "\n".join(L)


def gen_x2(name, N, p):
    P = limbs(p, N)
    inv = (-pow(p, -1, 1 << 32)) % (1 << 32)
    assert P[0] == 1 and inv == 0xFFFFFFFF  # Fr shortcut only
    L = []
    L.append("// %s: two independent products, their multiply-accumulate chains interleaved instruction by" % name)
    L.append("// instruction (carries in VCC and in an SGPR pair): twice the independent work per wave")
    L.append("DEV void %s_mul_x2_asm(Fe<%sCfg>& r0, const Fe<%sCfg>& A0, const Fe<%sCfg>& B0, Fe<%sCfg>& r1," % (name.lower(), name, name, name, name))
    L.append("                          const Fe<%sCfg>& A1, const Fe<%sCfg>& B1) {" % (name, name))
    L.append("    const uint32_t *a = A0.v, *b = B0.v, *c = A1.v, *d = B1.v;")
    L.append("    uint32_t m[%d], n[%d], t[%d], u[%d];" % (N, N, N, N))
    L.append("    uint64_t acc = 0, acd = 0, cs;")
    L.append("    uint32_t top, tpd;")
    for k in range(2 * N - 1):
        terms = []
        for i in range(max(0, k - N + 1), min(k, N - 1) + 1):
            terms.append(("ab", i, k - i))
        for i in range(max(0, k - N + 1), min(k - 1, N - 1) + 1):
            terms.append(("mp", i, k - i))
        L.append("    top = 0;")
        L.append("    tpd = 0;")
        if terms:
            lines = []
            ins = {}
            for (kind, i, j) in terms:
                if kind == "ab":
                    x0, y0, x1, y1 = "a%d" % i, "b%d" % j, "c%d" % i, "d%d" % j
                    ins[x0] = '"v"(a[%d])' % i; ins[y0] = '"v"(b[%d])' % j
                    ins[x1] = '"v"(c[%d])' % i; ins[y1] = '"v"(d[%d])' % j
                else:
                    x0, y0, x1, y1 = "m%d" % i, "p%d" % j, "n%d" % i, "p%d" % j
                    ins[x0] = '"v"(m[%d])' % i; ins[x1] = '"v"(n[%d])' % i
                    ins[y0] = '"s"(0x%08xu)' % P[j]
                lines.append('"v_mad_u64_u32 %%[acc], vcc, %%[%s], %%[%s], %%[acc]\\n\\t"' % (x0, y0))
                lines.append('"v_mad_u64_u32 %%[acd], %%[cs], %%[%s], %%[%s], %%[acd]\\n\\t"' % (x1, y1))
                lines.append('"v_addc_co_u32 %[top], vcc, 0, %[top], vcc\\n\\t"')
                lines.append('"v_addc_co_u32 %[tpd], %[cs], 0, %[tpd], %[cs]\\n\\t"')
            L.append("    asm(" + "\n        ".join(lines))
            L.append('        : [acc] "+v"(acc), [top] "+v"(top), [acd] "+v"(acd), [tpd] "+v"(tpd), [cs] "=&s"(cs)')
            L.append("        : " + ", ".join("[%s] %s" % (nm, cst) for nm, cst in ins.items()))
            L.append('        : "vcc");')
        if k < N:
            L.append("    m[%d] = 0u - (uint32_t)acc;" % k)
            L.append("    acc = (acc >> 32) + ((uint64_t)top << 32) + (uint64_t)((uint32_t)acc != 0u);")
            L.append("    n[%d] = 0u - (uint32_t)acd;" % k)
            L.append("    acd = (acd >> 32) + ((uint64_t)tpd << 32) + (uint64_t)((uint32_t)acd != 0u);")
            continue
        L.append("    t[%d] = (uint32_t)acc;" % (k - N))
        L.append("    acc = (acc >> 32) | ((uint64_t)top << 32);")
        L.append("    u[%d] = (uint32_t)acd;" % (k - N))
        L.append("    acd = (acd >> 32) | ((uint64_t)tpd << 32);")
    L.append("    t[%d] = (uint32_t)acc;" % (N - 1))
    L.append("    u[%d] = (uint32_t)acd;" % (N - 1))
    L.append("    fe_reduce_once<%sCfg>(r0, t);" % name)
    L.append("    fe_reduce_once<%sCfg>(r1, u);" % name)
    L.append("}")
    return "\n".join(L)


def main():
    out = [
        "// GENERATED by tools/gen_mont_asm.py — do not edit.",
        "// Product-scanning Montgomery multiplication with inline-asm multiply-accumulate chains",
        "// (v_mad_u64_u32 carry-out -> VCC -> v_addc_co_u32), see the generator's docstring.",
        "// Included by ff_dev.hpp after fe_reduce_once (inside namespace spx).",
        "#pragma once",
        "",
    ]
    for name, (N, p) in MODS.items():
        out.append(gen(name, N, p))
        out.append("")
    out.append(gen_x2("Fr", *MODS["Fr"]))
    out.append("")
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "r1cs-spartan_amd", "csrc", "ff_asm.hpp")
    open(path, "w").write("\n".join(out) + "\n")


if __name__ == "__main__":
    main()
