// micro-benchmark kernels (compiled twice: inline / out-of-line Fq multiplication in Fq2)
#include "../r1cs-spartan_amd/csrc/curve_dev.hpp"
using namespace spx;
#ifndef SFX
#error SFX
#endif
#define CAT2(a, b) a##b
#define CAT(a, b) CAT2(a, b)
__global__ __launch_bounds__(64) void CAT(k_g2madd_, SFX)(G2Xyzz* acc, const G2Aff* pts, int npts, int iters) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    G2Xyzz a = acc[i];
    for (int k = 0; k < iters; ++k) {
        G2Aff p = pts[(i + k * 977) % npts];
        xyzz_madd(a, p, (k & 1) != 0);
    }
    acc[i] = a;
}
__global__ __launch_bounds__(64) void CAT(k_g2add_lat_, SFX)(G2Xyzz* acc, const G2Xyzz* q, int iters) {
    G2Xyzz a = acc[0];
    for (int k = 0; k < iters; ++k) xyzz_add(a, q[k & 7]);
    acc[0] = a;
}
__global__ __launch_bounds__(64) void CAT(k_g1madd_, SFX)(G1Xyzz* acc, const G1Aff* pts, int npts, int iters) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    G1Xyzz a = acc[i];
    for (int k = 0; k < iters; ++k) {
        G1Aff p = pts[(i + k * 977) % npts];
        xyzz_madd(a, p, (k & 1) != 0);
    }
    acc[i] = a;
}
__global__ __launch_bounds__(256) void CAT(k_fqmul_, SFX)(Fq* out, const Fq* in, int iters) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    Fq a = in[i], b = in[i + 1], c = in[i + 2], d = in[i + 3];
    for (int k = 0; k < iters; ++k) {
        fe_mul(a, a, b);
        fe_mul(c, c, d);
    }
    fe_add(a, a, c);
    out[i] = a;
}
__global__ __launch_bounds__(256) void CAT(k_frmul_, SFX)(Fr* out, const Fr* in, int iters) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    Fr a = in[i], b = in[i + 1], c = in[i + 2], d = in[i + 3];
    for (int k = 0; k < iters; ++k) {
        fe_mul(a, a, b);
        fe_mul(c, c, d);
    }
    fe_add(a, a, c);
    out[i] = a;
}
