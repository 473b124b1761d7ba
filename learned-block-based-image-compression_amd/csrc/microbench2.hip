// Diagnostic microbenchmark (not part of liblbic.so): the B8_lowrate decoder's per-step GEMM chain
// (11 layers, M = 32 rows, separate weights) as one captured graph, replayed; per-layer phase stamps.
//   build: make microbench2      run: ./build/microbench2
#define LBIC_PHASE_STAMPS 1
#include "kernels.hip"

#include <cstdio>
#include <vector>

namespace lbic {
int set_error(int code, const std::string& msg) { fprintf(stderr, "%s\n", msg.c_str()); return code; }
}
using namespace lbic;

int main(int argc, char** argv) {
    const int hot = argc > 1 ? atoi(argv[1]) : 0;   // 1: every WG reads the same few KB (L1/L2-hot)
    const int M = 32;
    struct L { int K, N, epi; const char* name; };
    const L layers[] = {{768, 1152, EPI_LEAKY, "ctx0"}, {1152, 960, EPI_LEAKY, "ctx1"}, {960, 768, EPI_LEAKY, "ctx2"},
                        {768, 192, EPI_BIAS, "ctx3"}, {864, 768, EPI_BIAS, "dec0"}, {768, 768, EPI_IGDN, "ig0"},
                        {768, 672, EPI_BIAS, "d1"}, {672, 672, EPI_IGDN, "ig1"}, {672, 576, EPI_BIAS, "d2"},
                        {576, 576, EPI_IGDN, "ig2"}, {576, 192, EPI_BIAS, "d3"}};
    const int NL = 11;
    float *act[2], *bias;
    int4* blocks;
    unsigned long long* ph;
    for (auto& a : act) { (void)hipMalloc(&a, sizeof(float) * M * 1152); (void)hipMemset(a, 0, sizeof(float) * M * 1152); }
    (void)hipMalloc(&bias, sizeof(float) * 1152);
    (void)hipMemset(bias, 0, sizeof(float) * 1152);
    (void)hipMalloc(&blocks, sizeof(int4) * M);
    (void)hipMemset(blocks, 0, sizeof(int4) * M);
    (void)hipMalloc(&ph, sizeof(unsigned long long) * 8 * 4096 * NL);
    (void)hipMemset(ph, 0, sizeof(unsigned long long) * 8 * 4096 * NL);
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_phase), &ph, sizeof(ph));
    std::vector<GemmArgs> gs(NL);
    for (int i = 0; i < NL; ++i) {
        float* W;
        const size_t nw = (size_t)layers[i].K * ((layers[i].N + 15) / 16 * 16);
        (void)hipMalloc(&W, sizeof(float) * nw);
        (void)hipMemset(W, 0, sizeof(float) * nw);
        GemmArgs g{};
        g.M = M; g.N = layers[i].N; g.K = layers[i].K; g.P = 1; g.nseg = 1;
        g.seg[0] = Seg{act[i & 1], SEG_DENSE, 1152, 0, 0, 0, g.K};
        g.blocks = blocks; g.W = W; g.NB16 = (g.N + 15) / 16; g.bias = bias; g.epi = layers[i].epi;
        g.out = act[(i + 1) & 1]; g.ldo = 1152; g.gx = act[i & 1]; g.ldx = 1152;
        g.ctr_stride = i;    // phase slot
        if (hot) { g.NB16 = 0; g.seg[0].ld = 0; }
        gs[i] = g;
    }
    hipStream_t s;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    hipGraph_t gr;
    hipGraphExec_t ex;
    const int CH = 10;   // steps per graph
    (void)hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
    for (int r = 0; r < CH; ++r)
        for (int i = 0; i < NL; ++i) launch_gemm(gs[i], s);
    (void)hipStreamEndCapture(s, &gr);
    (void)hipGraphInstantiate(&ex, gr, nullptr, nullptr, 0);
    for (int w = 0; w < 20; ++w) (void)hipGraphLaunch(ex, s);
    (void)hipStreamSynchronize(s);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int R = 200;
    (void)hipEventRecord(e0, s);
    for (int r = 0; r < R; ++r) (void)hipGraphLaunch(ex, s);
    (void)hipEventRecord(e1, s);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("chain of %d GEMMs (graph, %d steps per replay): %.2f us per step, %.2f us per launch\n", NL, CH,
           ms * 1e3 / R / CH, ms * 1e3 / R / CH / NL);
    std::vector<unsigned long long> p((size_t)8 * 4096 * NL);
    (void)hipMemcpy(p.data(), ph, p.size() * 8, hipMemcpyDeviceToHost);
    printf("per-WG average cycles (s_memtime) of the last replay: [0] start->offsets [1]->A issued [2]->MFMA done "
           "[3]->barrier [4]->epilogue done | span first start..last end\n");
    unsigned long long prev_end = 0;
    for (int i = 0; i < NL; ++i) {
        const int nwg = (((gs[i].N + 127) / 128) * 8) * ((M + 15) / 16);
        double acc[6] = {0, 0, 0, 0, 0, 0};
        unsigned long long t0 = ~0ull, t1 = 0;
        int live = 0;
        for (int wg = 0; wg < nwg; ++wg) {
            const unsigned long long* q = p.data() + ((size_t)i * 4096 + wg) * 8;
            if (q[0] == 0 || q[5] < q[0]) continue;
            ++live;
            for (int k = 1; k < 6; ++k) acc[k] += (double)(q[k] - q[k - 1]);
            t0 = std::min(t0, q[0]);
            t1 = std::max(t1, q[5]);
        }
        printf("%-5s K%5d N%5d %3d WGs: %6.0f %6.0f %6.0f %6.0f %6.0f | span %6llu  gap from prev end %lld\n", layers[i].name,
               gs[i].K, gs[i].N, live, acc[1] / live, acc[2] / live, acc[3] / live, acc[4] / live, acc[5] / live, t1 - t0,
               prev_end ? (long long)(t0 - prev_end) : 0LL);
        prev_end = t1;
    }
    return 0;
}
