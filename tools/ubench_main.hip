// Throughput / latency micro-benchmark of the big-integer primitives (MI355X).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include "../r1cs-spartan_amd/csrc/curve_dev.hpp"
using namespace spx;
#define K(name, ...) __global__ void name(__VA_ARGS__);
__global__ void k_g2madd_nl(G2Xyzz*, const G2Aff*, int, int);
__global__ void k_g2madd_in(G2Xyzz*, const G2Aff*, int, int);
__global__ void k_g2add_lat_nl(G2Xyzz*, const G2Xyzz*, int);
__global__ void k_g2add_lat_in(G2Xyzz*, const G2Xyzz*, int);
__global__ void k_g1madd_nl(G1Xyzz*, const G1Aff*, int, int);
__global__ void k_fqmul_nl(Fq*, const Fq*, int);
__global__ void k_frmul_nl(Fr*, const Fr*, int);
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
static void fill(void* p, size_t bytes) {  // random limbs, top limb small so values < modulus
    unsigned* h = (unsigned*)malloc(bytes);
    for (size_t i = 0; i < bytes / 4; ++i) h[i] = (unsigned)rand() * 2654435761u;
    for (size_t i = 11; i < bytes / 4; i += 12) h[i] &= 0x0fffffffu;
    CHK(hipMemcpy(p, h, bytes, hipMemcpyHostToDevice));
    free(h);
}
template <class F>
static float timeit(F f) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    f();
    CHK(hipDeviceSynchronize());
    hipEventRecord(a);
    f();
    hipEventRecord(b);
    CHK(hipEventSynchronize(b));
    float ms; hipEventElapsedTime(&ms, a, b);
    return ms;
}
int main() {
    const int nth = 256 * 1024, npts = 1 << 20;
    void *acc, *pts, *fq;
    CHK(hipMalloc(&acc, (size_t)nth * sizeof(G2Xyzz)));
    CHK(hipMalloc(&pts, (size_t)npts * sizeof(G2Aff)));
    CHK(hipMalloc(&fq, (size_t)(nth * 4 + 16) * sizeof(Fq)));
    fill(acc, (size_t)nth * sizeof(G2Xyzz));
    fill(pts, (size_t)npts * sizeof(G2Aff));
    fill(fq, (size_t)(nth * 4 + 16) * sizeof(Fq));
    int it = 64;
    float t;
    t = timeit([&] { hipLaunchKernelGGL(k_fqmul_nl, dim3(nth / 256), dim3(256), 0, 0, (Fq*)fq, (const Fq*)fq, it); });
    printf("Fq mul      : %.1f G/s\n", 2.0 * nth * it / t / 1e6);
    t = timeit([&] { hipLaunchKernelGGL(k_frmul_nl, dim3(nth / 256), dim3(256), 0, 0, (Fr*)fq, (const Fr*)fq, it); });
    printf("Fr mul      : %.1f G/s\n", 2.0 * nth * it / t / 1e6);
    it = 32;
    t = timeit([&] { hipLaunchKernelGGL(k_g1madd_nl, dim3(nth / 64), dim3(64), 0, 0, (G1Xyzz*)acc, (const G1Aff*)pts, npts, it); });
    printf("G1 madd     : %.3f G/s\n", (double)nth * it / t / 1e6);
    t = timeit([&] { hipLaunchKernelGGL(k_g2madd_nl, dim3(nth / 64), dim3(64), 0, 0, (G2Xyzz*)acc, (const G2Aff*)pts, npts, it); });
    printf("G2 madd (nl): %.3f G/s\n", (double)nth * it / t / 1e6);
    t = timeit([&] { hipLaunchKernelGGL(k_g2madd_in, dim3(nth / 64), dim3(64), 0, 0, (G2Xyzz*)acc, (const G2Aff*)pts, npts, it); });
    printf("G2 madd (in): %.3f G/s\n", (double)nth * it / t / 1e6);
    it = 200;
    t = timeit([&] { hipLaunchKernelGGL(k_g2add_lat_nl, dim3(1), dim3(64), 0, 0, (G2Xyzz*)acc, (const G2Xyzz*)pts, it); });
    printf("G2 add lat (nl, 1 wave): %.1f us\n", t * 1e3 / it);
    t = timeit([&] { hipLaunchKernelGGL(k_g2add_lat_in, dim3(1), dim3(64), 0, 0, (G2Xyzz*)acc, (const G2Xyzz*)pts, it); });
    printf("G2 add lat (in, 1 wave): %.1f us\n", t * 1e3 / it);
    return 0;
}
