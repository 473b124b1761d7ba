// Diagnostic microbenchmark (not part of liblbic.so): decode-shaped k_gemm launches with per-workgroup
// phase stamps (s_memtime) and back-to-back launch timing with HIP events.
//   build: make microbench      run: ./microbench
#define LBIC_PHASE_STAMPS 1
#include "kernels.hip"

#include <chrono>
#include <cstdio>
#include <vector>

namespace lbic {
int set_error(int code, const std::string& msg) { fprintf(stderr, "%s\n", msg.c_str()); return code; }
}
using namespace lbic;

__global__ void k_empty() {}

int main() {
    const int M = 32, K = 768, N = 768, nimg = 32, Hb = 96, Wb = 96, Cx = 192;
    float *act, *W, *bias, *out, *zpad;
    int4* blocks;
    unsigned long long* ph;
    (void)hipMalloc(&act, sizeof(float) * M * 1152);
    (void)hipMalloc(&W, sizeof(float) * 1152 * 1152);
    (void)hipMalloc(&bias, sizeof(float) * 1152);
    (void)hipMalloc(&out, sizeof(float) * M * 1152);
    (void)hipMalloc(&zpad, sizeof(float) * (size_t)nimg * (Hb + 2) * (Wb + 4) * Cx);
    (void)hipMalloc(&blocks, sizeof(int4) * M);
    (void)hipMalloc(&ph, 8 * 8 * 4096);
    (void)hipMemset(act, 0, sizeof(float) * M * 1152);
    (void)hipMemset(W, 0, sizeof(float) * 1152 * 1152);
    (void)hipMemset(bias, 0, sizeof(float) * 1152);
    (void)hipMemset(zpad, 0, sizeof(float) * (size_t)nimg * (Hb + 2) * (Wb + 4) * Cx);
    std::vector<int4> b(M);
    for (int i = 0; i < M; ++i) b[i] = make_int4(i, 10, 10, 0);
    (void)hipMemcpy(blocks, b.data(), sizeof(int4) * M, hipMemcpyHostToDevice);
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_phase), &ph, sizeof(ph));
    GemmArgs g{};
    g.M = M; g.N = N; g.K = K; g.P = 1; g.nseg = 1;
    g.seg[0] = Seg{act, SEG_DENSE, 1152, 0, 0, 0, K};
    g.blocks = blocks; g.W = W; g.NB16 = 1152 / 16; g.bias = bias; g.epi = EPI_BIAS; g.out = out; g.ldo = 1152;
    g.geo = Geo{zpad, Hb + 2, Wb + 4, Cx, act, Hb, Wb};
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int w = 0; w < 20; ++w) launch_gemm(g, nullptr);
    (void)hipDeviceSynchronize();
    const int R = 2000;
    for (int variant = 0; variant < 4; ++variant) {
        GemmArgs h = g;
        const char* name = "K768 N768";
        if (variant == 1) { h.K = 16; h.seg[0].k1 = 16; name = "K16 N768"; }
        if (variant == 2) { h.N = 192; name = "K768 N192"; }
        (void)hipEventRecord(e0, nullptr);
        if (variant == 3) { for (int i = 0; i < R; ++i) hipLaunchKernelGGL(k_empty, dim3(72), dim3(512), 0, nullptr); name = "empty 72x512"; }
        else for (int i = 0; i < R; ++i) launch_gemm(h, nullptr);
        (void)hipEventRecord(e1, nullptr);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        std::vector<unsigned long long> p(8 * 4096);
        (void)hipMemcpy(p.data(), ph, 8 * 8 * 4096, hipMemcpyDeviceToHost);
        const int nwg = ((h.N + 15) / 16) * ((h.M + 15) / 16);
        double acc[5] = {0, 0, 0, 0, 0};
        unsigned long long t0 = ~0ull, t1 = 0;
        for (int wg = 0; wg < nwg && variant != 3; ++wg) {
            const unsigned long long* q = p.data() + wg * 8;
            for (int i = 1; i < 5; ++i) acc[i] += (double)(q[i] - q[i - 1]);
            t0 = std::min(t0, q[0]);
            t1 = std::max(t1, q[4]);
        }
        printf("%-14s back-to-back %.2f us/launch", name, ms * 1e3 / R);
        if (variant != 3)
            printf(" | last launch, per-WG avg cycles: setup %.0f  kloop %.0f  lds %.0f  epi %.0f | span %llu cyc (%d WGs)",
                   acc[1] / nwg, acc[2] / nwg, acc[3] / nwg, acc[4] / nwg, t1 - t0, nwg);
        printf("\n");
    }
    // stream concurrency: R launches on one stream vs R/2 on each of two streams (eager), and as graphs
    {
        hipStream_t s1, s2;
        (void)hipStreamCreateWithFlags(&s1, hipStreamNonBlocking);
        (void)hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
        // separate output buffers so the two streams do not write the same memory
        float* out2;
        (void)hipMalloc(&out2, sizeof(float) * M * 1152);
        GemmArgs g2 = g;
        g2.out = out2;
        auto run = [&](int mode) {
            (void)hipDeviceSynchronize();
            auto t0 = std::chrono::high_resolution_clock::now();
            if (mode == 0) for (int i = 0; i < R; ++i) launch_gemm(g, s1);
            else for (int i = 0; i < R / 2; ++i) { launch_gemm(g, s1); launch_gemm(g2, s2); }
            (void)hipDeviceSynchronize();
            auto t1 = std::chrono::high_resolution_clock::now();
            return std::chrono::duration<double, std::micro>(t1 - t0).count() / R;
        };
        run(0);
        printf("eager: 1 stream %.2f us/launch, 2 streams %.2f us/launch\n", run(0), run(1));
        // graphs of 100 launches each
        auto mkgraph = [&](GemmArgs& gg, hipStream_t st) {
            hipGraph_t gr; hipGraphExec_t ex;
            (void)hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal);
            for (int i = 0; i < 100; ++i) launch_gemm(gg, st);
            (void)hipStreamEndCapture(st, &gr);
            (void)hipGraphInstantiate(&ex, gr, nullptr, nullptr, 0);
            return ex;
        };
        hipGraphExec_t ga = mkgraph(g, s1), gb = mkgraph(g2, s2);
        auto runq = [&](int mode) {
            (void)hipDeviceSynchronize();
            auto t0 = std::chrono::high_resolution_clock::now();
            for (int i = 0; i < R / 100; ++i) {
                if (mode == 0) { (void)hipGraphLaunch(ga, s1); }
                else if (i % 2 == 0) { (void)hipGraphLaunch(ga, s1); (void)hipGraphLaunch(gb, s2); }
            }
            (void)hipDeviceSynchronize();
            auto t1 = std::chrono::high_resolution_clock::now();
            return std::chrono::duration<double, std::micro>(t1 - t0).count() / R;
        };
        runq(0);
        printf("graphs: 1 stream %.2f us/launch, 2 streams %.2f us/launch\n", runq(0), runq(1));
    }
    // workgroup -> XCD placement over consecutive launches
    for (int rep = 0; rep < 4; ++rep) {
        launch_gemm(g, nullptr);
        (void)hipDeviceSynchronize();
        std::vector<unsigned long long> p(8 * 4096);
        (void)hipMemcpy(p.data(), ph, 8 * 8 * 4096, hipMemcpyDeviceToHost);
        printf("launch %d xcc of wg 0..23:", rep);
        for (int wg = 0; wg < 24; ++wg) printf(" %llu", p[wg * 8 + 7]);
        printf("\n");
    }
    return 0;
}
