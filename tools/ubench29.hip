// Checks the radix-2^29 MSM arithmetic (ff29.hpp, curve29.hpp) against the 32-bit path
// (ff_dev.hpp, curve_dev.hpp) — same formulas, so results agree exactly on any inputs — and
// times both (MI355X).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include "../r1cs-spartan_amd/csrc/curve29.hpp"
using namespace spx;
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

template <class S> DEV void to29(typename R29<S>::T& r, const S& s) {
    typename R29<S>::T t; R29<S>::unpack(t, s); f29_map(r, t, Q29::FROM_R1);
}
template <class S> DEV void from29(S& s, const typename R29<S>::T& r) {
    typename R29<S>::T t; f29_map(t, r, Q29::TO_R1); R29<S>::pack(s, t);
}
template <class S> DEV bool same(const S& a, const S& b) {
    const uint32_t* x = (const uint32_t*)&a; const uint32_t* y = (const uint32_t*)&b; uint32_t acc = 0;
    for (int i = 0; i < (int)(sizeof(S) / 4); ++i) acc |= x[i] ^ y[i];
    return acc == 0;
}

// field ops
template <class S>
__global__ void k_field(const S* a, const S* b, int n, unsigned* bad) {
    int i = blockIdx.x * blockDim.x + threadIdx.x; if (i >= n) return;
    using T = typename R29<S>::T; using O = Ops29<T>;
    S x = a[i], y = b[i], r1, r2; T X, Y, Z;
    to29<S>(X, x); to29<S>(Y, y);
    FieldOps<S>::mul(r1, x, y); O::mul(Z, X, Y); from29<S>(r2, Z); if (!same(r1, r2)) atomicAdd(bad + 0, 1u);
    FieldOps<S>::sqr(r1, x); O::sqr(Z, X); from29<S>(r2, Z); if (!same(r1, r2)) atomicAdd(bad + 1, 1u);
    FieldOps<S>::sub(r1, x, y); O::template sub<2>(Z, X, Y); O::template reduce<4>(Z); from29<S>(r2, Z); if (!same(r1, r2)) atomicAdd(bad + 2, 1u);
    // chain of 16 dependent products with lazy adds in between
    S c1 = x; T C = X;
    for (int k = 0; k < 16; ++k) {
        FieldOps<S>::add(c1, c1, y); FieldOps<S>::mul(c1, c1, y);
        O::add(C, C, Y); O::mul(C, C, Y);
    }
    from29<S>(r2, C); if (!same(c1, r2)) atomicAdd(bad + 3, 1u);
}

// curve formulas: acc (XYZZ) += 32 affine points (some negated), then add/dbl
template <class S>
__global__ void k_curve(const Xyzz<S>* acc0, const Aff<S>* pts, int n, unsigned* bad) {
    int i = blockIdx.x * blockDim.x + threadIdx.x; if (i >= n) return;
    using T = typename R29<S>::T;
    Xyzz<S> a = acc0[i], q = acc0[(i + 7) % n];
    X29<T> A, Q;
    to29<S>(A.x, a.x); to29<S>(A.y, a.y); to29<S>(A.zz, a.zz); to29<S>(A.zzz, a.zzz);
    to29<S>(Q.x, q.x); to29<S>(Q.y, q.y); to29<S>(Q.zz, q.zz); to29<S>(Q.zzz, q.zzz);
    for (int k = 0; k < 32; ++k) {
        Aff<S> p = pts[(i * 31 + k * 977) % n];
        bool neg = (k % 3) == 1;
        xyzz_madd(a, p, neg);
        T px, py; to29<S>(px, p.x); to29<S>(py, p.y);
        x29_madd(A, px, py, neg);
    }
    { Xyzz<S> tmp; st29<S>(&tmp, A); ld29<S>(A, &tmp); }  // loose madd outputs survive the packed layout
    xyzz_add(a, q); x29_add(A, Q);
    xyzz_dbl(a, a); x29_dbl(A);
    Xyzz<S> b;
    from29<S>(b.x, A.x); from29<S>(b.y, A.y); from29<S>(b.zz, A.zz); from29<S>(b.zzz, A.zzz);
    if (!same(a, b)) atomicAdd(bad, 1u);
}

template <class S, int NEW>
__global__ __launch_bounds__(64) void k_madd_thr(Xyzz<S>* acc, const Aff<S>* pts, int npts, int iters) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (NEW) {
        using T = typename R29<S>::T;
        X29<T> A; ld29<S>(A, acc + i);
        for (int k = 0; k < iters; ++k) { A29<T> p; ld29<S>(p, pts + (i + k * 977) % npts); x29_madd(A, p.x, p.y, (k & 1) != 0); }
        st29<S>(acc + i, A);
    } else {
        Xyzz<S> a = acc[i];
        for (int k = 0; k < iters; ++k) { Aff<S> p = pts[(i + k * 977) % npts]; xyzz_madd(a, p, (k & 1) != 0); }
        acc[i] = a;
    }
}
// two waves per SIMD forced (<= 256 VGPRs)
template <class S>
__global__ __launch_bounds__(64, 2) void k_madd_thr_o2(Xyzz<S>* acc, const Aff<S>* pts, int npts, int iters) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    using T = typename R29<S>::T;
    X29<T> A; ld29<S>(A, acc + i);
    for (int k = 0; k < iters; ++k) { A29<T> p; ld29<S>(p, pts + (i + k * 977) % npts); x29_madd(A, p.x, p.y, (k & 1) != 0); }
    st29<S>(acc + i, A);
}
template <class S, int NEW>
__global__ __launch_bounds__(64) void k_add_lat(Xyzz<S>* acc, const Xyzz<S>* q, int iters) {
    if (NEW) {
        using T = typename R29<S>::T;
        X29<T> A; ld29<S>(A, acc + threadIdx.x);
        for (int k = 0; k < iters; ++k) { X29<T> B; ld29<S>(B, q + ((k + threadIdx.x) & 63)); x29_add(A, B); }
        st29<S>(acc + threadIdx.x, A);
    } else {
        Xyzz<S> a = acc[threadIdx.x];
        for (int k = 0; k < iters; ++k) xyzz_add(a, q[(k + threadIdx.x) & 63]);
        acc[threadIdx.x] = a;
    }
}
__global__ void k_fq_thr29(F29* out, const F29* in, int iters) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    F29 a = in[i], b = in[i + 1], c = in[i + 2], d = in[i + 3];
    for (int k = 0; k < iters; ++k) { f29_mul(a, a, b); f29_mul(c, c, d); }
    f29_add(a, a, c); out[i] = a;
}

static void fill_canon(void* p, size_t count, int words_per_fq) {  // 12-word Fq values < p (top word small)
    unsigned* h = (unsigned*)malloc(count * words_per_fq * 4);
    for (size_t i = 0; i < count * words_per_fq; ++i) h[i] = (unsigned)rand() * 2654435761u ^ (unsigned)rand();
    for (size_t i = 0; i < count; ++i) h[i * words_per_fq + 11] &= 0x0fffffffu;
    CHK(hipMemcpy(p, h, count * words_per_fq * 4, hipMemcpyHostToDevice));
    free(h);
}
static void fill29(void* p, size_t count) {  // 14-limb values < 2p-ish
    unsigned* h = (unsigned*)malloc(count * 56);
    for (size_t i = 0; i < count * 14; ++i) h[i] = ((unsigned)rand() * 2654435761u ^ (unsigned)rand()) & 0x1fffffffu;
    for (size_t i = 0; i < count; ++i) h[i * 14 + 13] &= 0x7;
    CHK(hipMemcpy(p, h, count * 56, hipMemcpyHostToDevice));
    free(h);
}
template <class F> static float timeit(F f) {
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    f(); CHK(hipDeviceSynchronize()); hipEventRecord(a); f(); hipEventRecord(b); CHK(hipEventSynchronize(b));
    float ms; hipEventElapsedTime(&ms, a, b); return ms;
}
int main() {
    const int n = 1 << 16;
    void *a, *b, *acc, *pts; unsigned* bad;
    CHK(hipMalloc(&a, (size_t)n * 96)); CHK(hipMalloc(&b, (size_t)n * 96)); CHK(hipMalloc(&bad, 64));
    CHK(hipMalloc(&acc, (size_t)n * sizeof(G2Xyzz))); CHK(hipMalloc(&pts, (size_t)n * sizeof(G2Aff)));
    unsigned hb[16];
    // Fq
    fill_canon(a, n, 12); fill_canon(b, n, 12); CHK(hipMemset(bad, 0, 64));
    hipLaunchKernelGGL(k_field<Fq>, dim3(n / 256), dim3(256), 0, 0, (const Fq*)a, (const Fq*)b, n, bad);
    CHK(hipMemcpy(hb, bad, 64, hipMemcpyDeviceToHost));
    printf("Fq  mul/sqr/sub/chain mismatches: %u %u %u %u\n", hb[0], hb[1], hb[2], hb[3]);
    fill_canon(a, 2 * n, 12); fill_canon(b, 2 * n, 12); CHK(hipMemset(bad, 0, 64));
    hipLaunchKernelGGL(k_field<Fq2>, dim3(n / 256), dim3(256), 0, 0, (const Fq2*)a, (const Fq2*)b, n, bad);
    CHK(hipMemcpy(hb, bad, 64, hipMemcpyDeviceToHost));
    printf("Fq2 mul/sqr/sub/chain mismatches: %u %u %u %u\n", hb[0], hb[1], hb[2], hb[3]);
    // curves (random coordinates: formulas are identical rational maps)
    fill_canon(acc, (size_t)n * 4, 12); fill_canon(pts, (size_t)n * 2, 12); CHK(hipMemset(bad, 0, 64));
    hipLaunchKernelGGL(k_curve<Fq>, dim3(n / 64), dim3(64), 0, 0, (const G1Xyzz*)acc, (const G1Aff*)pts, n, bad);
    CHK(hipMemcpy(hb, bad, 4, hipMemcpyDeviceToHost));
    printf("G1 madd x32 + add + dbl mismatches: %u / %d\n", hb[0], n);
    fill_canon(acc, (size_t)n * 8, 12); fill_canon(pts, (size_t)n * 4, 12); CHK(hipMemset(bad, 0, 64));
    hipLaunchKernelGGL(k_curve<Fq2>, dim3(n / 64), dim3(64), 0, 0, (const G2Xyzz*)acc, (const G2Aff*)pts, n, bad);
    CHK(hipMemcpy(hb, bad, 4, hipMemcpyDeviceToHost));
    printf("G2 madd x32 + add + dbl mismatches: %u / %d\n", hb[0], n);
    CHK(hipDeviceSynchronize());
    // throughput
    const int nth = 256 * 1024; const int npts = 1 << 16;
    void *tacc, *tpts, *fq;
    CHK(hipMalloc(&tacc, (size_t)nth * sizeof(G2Xyzz))); CHK(hipMalloc(&tpts, (size_t)npts * sizeof(G2Aff)));
    CHK(hipMalloc(&fq, (size_t)(nth + 16) * 56));
    fill_canon(tacc, (size_t)nth * 8, 12); fill_canon(tpts, (size_t)npts * 4, 12); fill29(fq, nth + 16);
    int it = 64; float t;
    t = timeit([&] { hipLaunchKernelGGL(k_fq_thr29, dim3(nth / 256), dim3(256), 0, 0, (F29*)fq, (const F29*)fq, it); });
    printf("Fq mul 29   : %.1f G/s\n", 2.0 * nth * it / t / 1e6);
    it = 32;
    t = timeit([&] { hipLaunchKernelGGL((k_madd_thr<Fq, 0>), dim3(nth / 64), dim3(64), 0, 0, (G1Xyzz*)tacc, (const G1Aff*)tpts, npts, it); });
    printf("G1 madd 32  : %.3f G/s\n", (double)nth * it / t / 1e6);
    t = timeit([&] { hipLaunchKernelGGL((k_madd_thr<Fq, 1>), dim3(nth / 64), dim3(64), 0, 0, (G1Xyzz*)tacc, (const G1Aff*)tpts, npts, it); });
    printf("G1 madd 29  : %.3f G/s\n", (double)nth * it / t / 1e6);
    t = timeit([&] { hipLaunchKernelGGL((k_madd_thr<Fq2, 0>), dim3(nth / 64), dim3(64), 0, 0, (G2Xyzz*)tacc, (const G2Aff*)tpts, npts, it); });
    printf("G2 madd 32  : %.3f G/s\n", (double)nth * it / t / 1e6);
    t = timeit([&] { hipLaunchKernelGGL((k_madd_thr<Fq2, 1>), dim3(nth / 64), dim3(64), 0, 0, (G2Xyzz*)tacc, (const G2Aff*)tpts, npts, it); });
    printf("G2 madd 29  : %.3f G/s\n", (double)nth * it / t / 1e6);
    t = timeit([&] { hipLaunchKernelGGL((k_madd_thr_o2<Fq2>), dim3(nth / 64), dim3(64), 0, 0, (G2Xyzz*)tacc, (const G2Aff*)tpts, npts, it); });
    printf("G2 madd 29 occ2: %.3f G/s\n", (double)nth * it / t / 1e6);
    it = 100;
    t = timeit([&] { hipLaunchKernelGGL((k_add_lat<Fq2, 0>), dim3(1), dim3(64), 0, 0, (G2Xyzz*)tacc, (const G2Xyzz*)tacc + 64, it); });
    printf("G2 add lat 32: %.1f us\n", t * 1e3 / it);
    t = timeit([&] { hipLaunchKernelGGL((k_add_lat<Fq2, 1>), dim3(1), dim3(64), 0, 0, (G2Xyzz*)tacc, (const G2Xyzz*)tacc + 64, it); });
    printf("G2 add lat 29: %.1f us\n", t * 1e3 / it);
    return 0;
}
