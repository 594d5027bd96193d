// Calibration for rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950: one streaming read of exactly
// READ_BYTES (16 B per lane, coalesced) and one streaming write of exactly WRITE_BYTES.
#include <hip/hip_runtime.h>
#include <stdio.h>
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s\n", hipGetErrorString(e)); return 1; } } while (0)
__global__ void k_calib_read(const uint4* __restrict__ in, size_t n, unsigned* out) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x, st = (size_t)gridDim.x * blockDim.x;
    unsigned acc = 0;
    for (; i < n; i += st) {
        uint4 v = in[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}
__global__ void k_calib_write(uint4* __restrict__ o, size_t n) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x, st = (size_t)gridDim.x * blockDim.x;
    for (; i < n; i += st) o[i] = make_uint4((unsigned)i, 1, 2, 3);
}
int main() {
    const size_t bytes = 1ull << 30;  // 1 GiB: far past the 256 MiB Infinity Cache
    void *a, *b;
    unsigned* o;
    CHK(hipMalloc(&a, bytes));
    CHK(hipMalloc(&b, bytes));
    CHK(hipMalloc(&o, 4));
    CHK(hipMemset(a, 1, bytes));
    CHK(hipDeviceSynchronize());
    hipLaunchKernelGGL(k_calib_write, dim3(4096), dim3(256), 0, 0, (uint4*)b, bytes / 16);
    hipLaunchKernelGGL(k_calib_read, dim3(4096), dim3(256), 0, 0, (const uint4*)a, bytes / 16, o);
    CHK(hipDeviceSynchronize());
    printf("calib: read %zu B, write %zu B\n", bytes, bytes);
    return 0;
}
