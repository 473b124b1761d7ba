// Diagnostic (not shipped): aggregate kernel-dispatch rate of dependent kernel chains on N streams side by side.
// Each stream replays a captured graph of K dependent launches of a kernel with G workgroups of 512 threads that
// busy-waits `ns` nanoseconds on the 100 MHz constant clock (ns = 0: an empty kernel).  If N chains of short
// kernels stop scaling long before the GPU's CUs are full, the limit is the dispatch path, not the kernels.
// usage: dispatch_bench [G] [ns] [K] [reps]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));               \
            exit(1);                                                               \
        }                                                                          \
    } while (0)

__global__ __launch_bounds__(512) void k_spin(int ticks, float* sink) {
    if (ticks > 0) {
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)ticks) __builtin_amdgcn_s_sleep(1);
    }
    if (sink && threadIdx.x == 0 && blockIdx.x == 0) sink[0] = 1.f;   // vector store; never taken (sink = null)
}

int main(int argc, char** argv) {
    const int G = argc > 1 ? atoi(argv[1]) : 96;
    const int ns = argc > 2 ? atoi(argv[2]) : 0;
    const int K = argc > 3 ? atoi(argv[3]) : 1000;
    const int reps = argc > 4 ? atoi(argv[4]) : 5;
    const int ticks = ns / 10;
    const int NS[] = {1, 2, 3, 4, 6, 8};
    std::vector<hipStream_t> st(8);
    for (auto& s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    std::vector<hipGraphExec_t> ex(8);
    for (int i = 0; i < 8; ++i) {
        CK(hipStreamBeginCapture(st[i], hipStreamCaptureModeThreadLocal));
        for (int k = 0; k < K; ++k) hipLaunchKernelGGL(k_spin, dim3(G), dim3(512), 0, st[i], ticks, (float*)nullptr);
        hipGraph_t g;
        CK(hipStreamEndCapture(st[i], &g));
        CK(hipGraphInstantiate(&ex[i], g, nullptr, nullptr, 0));
        CK(hipGraphDestroy(g));
        CK(hipGraphLaunch(ex[i], st[i]));      // warm
    }
    CK(hipDeviceSynchronize());
    printf("G=%d workgroups x 512 threads, busy %d ns, chains of %d launches, %d replays\n", G, ns, K, reps);
    for (int n : NS) {
        const auto t0 = std::chrono::steady_clock::now();
        for (int r = 0; r < reps; ++r)
            for (int i = 0; i < n; ++i) CK(hipGraphLaunch(ex[i], st[i]));
        CK(hipDeviceSynchronize());
        const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        const double per = s / ((double)reps * K) * 1e6;
        printf("  %d chains: %8.1f ms, %6.2f us per launch per chain, %7.0f k launches/s aggregate\n", n, s * 1e3, per,
               n * reps * (double)K / s / 1e3);
    }
    return 0;
}
