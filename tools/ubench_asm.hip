// Checks the asm Montgomery product against the portable CIOS form and times both (MI355X).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include "../r1cs-spartan_amd/csrc/curve_dev.hpp"
using namespace spx;
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

template <class C>
__global__ void k_check(const Fe<C>* a, const Fe<C>* b, int n, unsigned* bad) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Fe<C> x = a[i], y = b[i], r1, r2;
    fe_mul_cios(r1, x, y);
    fe_mul(r2, x, y);
    if (!fe_eq(r1, r2)) atomicAdd(bad, 1u);
    // chained: squares
    for (int k = 0; k < 8; ++k) { fe_mul_cios(r1, r1, y); fe_mul(r2, r2, y); }
    if (!fe_eq(r1, r2)) atomicAdd(bad + 1, 1u);
}
template <class C, int ASM>
__global__ __launch_bounds__(256) void k_thr(Fe<C>* out, const Fe<C>* in, int iters) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    Fe<C> a = in[i], b = in[i + 1], c = in[i + 2], d = in[i + 3];
    for (int k = 0; k < iters; ++k) {
        if (ASM) { fe_mul(a, a, b); fe_mul(c, c, d); }
        else { fe_mul_cios(a, a, b); fe_mul_cios(c, c, d); }
    }
    fe_add(a, a, c);
    out[i] = a;
}
template <class C, int ASM>
__global__ __launch_bounds__(64) void k_lat(Fe<C>* out, const Fe<C>* in, int iters) {
    Fe<C> a = in[threadIdx.x], b = in[threadIdx.x + 1];
    for (int k = 0; k < iters; ++k) {
        if (ASM) fe_mul(a, a, b); else fe_mul_cios(a, a, b);
    }
    out[threadIdx.x] = a;
}
__global__ __launch_bounds__(64) void k_g1madd(G1Xyzz* acc, const G1Aff* pts, int npts, int iters) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    G1Xyzz a = acc[i];
    for (int k = 0; k < iters; ++k) { G1Aff p = pts[(i + k * 977) % npts]; xyzz_madd(a, p, (k & 1) != 0); }
    acc[i] = a;
}
__global__ __launch_bounds__(64) void k_g2madd(G2Xyzz* acc, const G2Aff* pts, int npts, int iters) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    G2Xyzz a = acc[i];
    for (int k = 0; k < iters; ++k) { G2Aff p = pts[(i + k * 977) % npts]; xyzz_madd(a, p, (k & 1) != 0); }
    acc[i] = a;
}
__global__ __launch_bounds__(64) void k_g2add_lat(G2Xyzz* acc, const G2Xyzz* q, int iters) {
    G2Xyzz a = acc[0];
    for (int k = 0; k < iters; ++k) xyzz_add(a, q[k & 7]);
    acc[0] = a;
}
static void fill_mod(void* p, size_t count, int N, unsigned topmask) {
    unsigned* h = (unsigned*)malloc(count * N * 4);
    for (size_t i = 0; i < count * N; ++i) h[i] = (unsigned)rand() * 2654435761u ^ (unsigned)rand();
    for (size_t i = 0; i < count; ++i) h[i * N + N - 1] &= topmask;
    // a few all-ones-ish (just below modulus top) values
    CHK(hipMemcpy(p, h, count * N * 4, hipMemcpyHostToDevice));
    free(h);
}
template <class F>
static float timeit(F f) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    f(); CHK(hipDeviceSynchronize());
    hipEventRecord(a); f(); hipEventRecord(b);
    CHK(hipEventSynchronize(b));
    float ms; hipEventElapsedTime(&ms, a, b);
    return ms;
}
int main() {
    const int n = 1 << 20;
    void *a, *b, *o; unsigned* bad;
    CHK(hipMalloc(&a, (size_t)(n + 16) * 48)); CHK(hipMalloc(&b, (size_t)(n + 16) * 48)); CHK(hipMalloc(&o, (size_t)(n + 16) * 48));
    CHK(hipMalloc(&bad, 16));
    // Fr: top limb < 0x73eda753 -> value < r
    fill_mod(a, n + 16, 8, 0x73eda752u); fill_mod(b, n + 16, 8, 0x73eda752u);
    CHK(hipMemset(bad, 0, 16));
    hipLaunchKernelGGL(k_check<FrCfg>, dim3(n / 256), dim3(256), 0, 0, (const Fr*)a, (const Fr*)b, n, bad);
    unsigned hb[4]; CHK(hipMemcpy(hb, bad, 16, hipMemcpyDeviceToHost));
    printf("Fr check: %u / %u mismatches (single / chained)\n", hb[0], hb[1]);
    fill_mod(a, n + 16, 12, 0x1a0111e9u); fill_mod(b, n + 16, 12, 0x1a0111e9u);
    CHK(hipMemset(bad, 0, 16));
    hipLaunchKernelGGL(k_check<FqCfg>, dim3(n / 256), dim3(256), 0, 0, (const Fq*)a, (const Fq*)b, n, bad);
    CHK(hipMemcpy(hb, bad, 16, hipMemcpyDeviceToHost));
    printf("Fq check: %u / %u mismatches (single / chained)\n", hb[0], hb[1]);
    const int nth = 256 * 1024;
    int it = 64;
    float t;
    t = timeit([&] { hipLaunchKernelGGL((k_thr<FqCfg, 0>), dim3(nth / 256), dim3(256), 0, 0, (Fq*)o, (const Fq*)a, it); });
    printf("Fq mul cios : %.1f G/s\n", 2.0 * nth * it / t / 1e6);
    t = timeit([&] { hipLaunchKernelGGL((k_thr<FqCfg, 1>), dim3(nth / 256), dim3(256), 0, 0, (Fq*)o, (const Fq*)a, it); });
    printf("Fq mul asm  : %.1f G/s\n", 2.0 * nth * it / t / 1e6);
    t = timeit([&] { hipLaunchKernelGGL((k_thr<FrCfg, 0>), dim3(nth / 256), dim3(256), 0, 0, (Fr*)o, (const Fr*)a, it); });
    printf("Fr mul cios : %.1f G/s\n", 2.0 * nth * it / t / 1e6);
    t = timeit([&] { hipLaunchKernelGGL((k_thr<FrCfg, 1>), dim3(nth / 256), dim3(256), 0, 0, (Fr*)o, (const Fr*)a, it); });
    printf("Fr mul asm  : %.1f G/s\n", 2.0 * nth * it / t / 1e6);
    it = 1000;
    t = timeit([&] { hipLaunchKernelGGL((k_lat<FqCfg, 0>), dim3(1), dim3(64), 0, 0, (Fq*)o, (const Fq*)a, it); });
    printf("Fq mul lat cios: %.1f ns\n", t * 1e6 / it);
    t = timeit([&] { hipLaunchKernelGGL((k_lat<FqCfg, 1>), dim3(1), dim3(64), 0, 0, (Fq*)o, (const Fq*)a, it); });
    printf("Fq mul lat asm : %.1f ns\n", t * 1e6 / it);
    void *acc, *pts;
    const int npts = 1 << 20;
    CHK(hipMalloc(&acc, (size_t)nth * sizeof(G2Xyzz)));
    CHK(hipMalloc(&pts, (size_t)npts * sizeof(G2Aff)));
    fill_mod(acc, (size_t)nth * sizeof(G2Xyzz) / 48, 12, 0x1a0111e9u);
    fill_mod(pts, (size_t)npts * sizeof(G2Aff) / 48, 12, 0x1a0111e9u);
    it = 32;
    t = timeit([&] { hipLaunchKernelGGL(k_g1madd, dim3(nth / 64), dim3(64), 0, 0, (G1Xyzz*)acc, (const G1Aff*)pts, npts, it); });
    printf("G1 madd     : %.3f G/s\n", (double)nth * it / t / 1e6);
    t = timeit([&] { hipLaunchKernelGGL(k_g2madd, dim3(nth / 64), dim3(64), 0, 0, (G2Xyzz*)acc, (const G2Aff*)pts, npts, it); });
    printf("G2 madd     : %.3f G/s\n", (double)nth * it / t / 1e6);
    it = 200;
    t = timeit([&] { hipLaunchKernelGGL(k_g2add_lat, dim3(1), dim3(64), 0, 0, (G2Xyzz*)acc, (const G2Xyzz*)pts, it); });
    printf("G2 add lat (1 wave): %.1f us\n", t * 1e3 / it);
    return 0;
}
