// How many kernel launches per second can ONE process issue from many host threads, each on its own
// stream (the shape of spx_prove_many: one worker thread and stream per proof in flight)? Each thread
// launches `per` tiny kernels and waits for its stream after every `batch` launches (a proof's
// launches between host round trips). Run it alone and as two processes side by side: if two
// processes together issue about twice one process's rate, the per-process launch path is the limit.
//   hipcc -O2 --offload-arch=gfx950 tools/ubench_launch.hip -o tools/ubench_launch -lpthread
//   tools/ubench_launch THREADS LAUNCHES_PER_THREAD BATCH
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

__global__ void k_tiny(unsigned* p, unsigned v) {
    if (threadIdx.x == 0 && blockIdx.x == 0) p[0] = v;
}

#define CHK(x)                                                                      \
    do {                                                                            \
        hipError_t e = (x);                                                         \
        if (e != hipSuccess) {                                                      \
            fprintf(stderr, "HIP error %s at line %d\n", hipGetErrorString(e), __LINE__); \
            exit(1);                                                                \
        }                                                                           \
    } while (0)

int main(int argc, char** argv) {
    const int T = argc > 1 ? atoi(argv[1]) : 64;
    const int per = argc > 2 ? atoi(argv[2]) : 4000;
    const int batch = argc > 3 ? atoi(argv[3]) : 4;
    CHK(hipSetDeviceFlags(hipDeviceScheduleBlockingSync));
    CHK(hipSetDevice(0));
    std::vector<hipStream_t> st(T);
    std::vector<unsigned*> buf(T);
    for (int t = 0; t < T; ++t) {
        CHK(hipStreamCreateWithFlags(&st[t], hipStreamNonBlocking));
        CHK(hipMalloc(&buf[t], 256));
    }
    auto work = [&](int t, int n) {
        for (int i = 0; i < n; ++i) {
            hipLaunchKernelGGL(k_tiny, dim3(4), dim3(64), 0, st[t], buf[t], (unsigned)i);
            if ((i + 1) % batch == 0) CHK(hipStreamSynchronize(st[t]));
        }
        CHK(hipStreamSynchronize(st[t]));
    };
    {  // warm-up
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t) th.emplace_back(work, t, 64);
        for (auto& x : th) x.join();
    }
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t) th.emplace_back(work, t, per);
    for (auto& x : th) x.join();
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    printf("{\"threads\": %d, \"launches_per_thread\": %d, \"batch\": %d, \"seconds\": %.4f, \"launches_per_s\": %.0f}\n", T,
           per, batch, s, (double)T * per / s);
    return 0;
}
