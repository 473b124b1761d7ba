// Diagnostic microbenchmark (not shipped): k_rans_decode in isolation on synthetic streams.
#include "kernels.hip"
#include "entropy_host.cpp"

#include <chrono>
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

namespace lbic {
int set_error(int code, const std::string& msg) { fprintf(stderr, "%s\n", msg.c_str()); return code; }
}
using namespace lbic;

int main(int argc, char** argv) {
    const int n_img = argc > 1 ? atoi(argv[1]) : 32, M = argc > 2 ? atoi(argv[2]) : 96, steps = 64;
    // Gaussian tables exactly as GaussianConditional.update builds them (double erfc here; fine for a bench)
    EntropyTables t;
    t.n_tables = 64;
    for (int i = 0; i < 64; ++i) t.table.push_back((float)std::exp(std::log(0.11) + i * (std::log(256.0) - std::log(0.11)) / 63));
    const double mult = 6.1094;   // -Phi^-1(1e-9 / 2)
    int maxlen = 0;
    std::vector<std::vector<uint32_t>> cdfs;
    for (int i = 0; i < 64; ++i) {
        const int c = (int)std::ceil(t.table[i] * mult), len = 2 * c + 1;
        std::vector<float> pmf(len + 1);
        double lower0 = 0;
        for (int j = 0; j < len; ++j) {
            const double v = std::fabs(j - c);
            const double up = 0.5 * std::erfc(-(0.5 - v) / t.table[i] / std::sqrt(2.0));
            const double lo = 0.5 * std::erfc(-(-0.5 - v) / t.table[i] / std::sqrt(2.0));
            pmf[j] = (float)(up - lo);
            if (j == 0) lower0 = lo;
        }
        pmf[len] = (float)(2 * lower0);
        std::vector<uint32_t> q(len + 2);
        pmf_to_quantized_cdf(pmf.data(), len + 1, 16, q.data());
        cdfs.push_back(q);
        t.length.push_back(len + 2);
        t.offset.push_back(-c);
        maxlen = std::max(maxlen, len + 2);
    }
    t.stride = maxlen;
    t.cdf.assign((size_t)64 * maxlen, 0);
    for (int i = 0; i < 64; ++i)
        for (size_t j = 0; j < cdfs[i].size(); ++j) t.cdf[(size_t)i * maxlen + j] = (int32_t)cdfs[i][j];
    std::vector<uint16_t> c16;
    std::vector<int> meta;
    if (build_rans_gpu_tables(t, c16, meta)) return 1;
    const int total16 = (int)c16.size();
    const int lo_idx = argc > 3 ? atoi(argv[3]) : 0, hi_idx = argc > 4 ? atoi(argv[4]) : 63;
    const int sparse = argc > 5 ? atoi(argv[5]) : 0;            // 1: k_rans_decode_sparse
    const float spread = argc > 6 ? (float)atof(argv[6]) : 1.2f;   // value ~ N(0, spread sigma): 0.1 = low rate
    // symbols: index uniform over the table, value ~ N(0, spread sigma)
    std::mt19937 rng(1);
    std::vector<int32_t> idx((size_t)n_img * steps * M), sym(idx.size());
    for (size_t i = 0; i < idx.size(); ++i) {
        idx[i] = lo_idx + (int)(rng() % (hi_idx - lo_idx + 1));
        std::normal_distribution<float> nd(0.f, t.table[idx[i]] * spread);
        sym[i] = (int)std::lrint(nd(rng));
    }
    std::vector<uint32_t> words;
    std::vector<long long> base(n_img);
    std::vector<int> cnt(n_img), ptr(n_img, 2);
    std::vector<unsigned long long> x0(n_img);
    for (int im = 0; im < n_img; ++im) {
        std::vector<uint8_t> b;
        rans_encode(t, sym.data() + (size_t)im * steps * M, idx.data() + (size_t)im * steps * M, (size_t)steps * M, b);
        base[im] = (long long)words.size();
        cnt[im] = (int)(b.size() / 4);
        const uint32_t* w = reinterpret_cast<const uint32_t*>(b.data());
        words.insert(words.end(), w, w + b.size() / 4);
        x0[im] = (unsigned long long)w[0] | ((unsigned long long)w[1] << 32);
    }
    // device
    auto up = [](const void* src, size_t n) { void* p; (void)hipMalloc(&p, n); (void)hipMemcpy(p, src, n, hipMemcpyHostToDevice); return p; };
    std::vector<int32_t> idx_step((size_t)steps * n_img * M);     // [step][img][M]
    for (int st = 0; st < steps; ++st)
        for (int im = 0; im < n_img; ++im)
            for (int k = 0; k < M; ++k) idx_step[((size_t)st * n_img + im) * M + k] = idx[((size_t)im * steps + st) * M + k];
    std::vector<int4> blocks(n_img);
    for (int im = 0; im < n_img; ++im) blocks[im] = make_int4(im, 0, 0, 0);
    RansArgs a{};
    a.cdf16 = (const uint16_t*)up(c16.data(), c16.size() * 2);
    a.tmeta = (const int*)up(meta.data(), meta.size() * 4);
    a.total16 = total16;
    a.words = (const uint32_t*)up(words.data(), words.size() * 4);
    a.word_base = (const long long*)up(base.data(), base.size() * 8);
    a.word_count = (const int*)up(cnt.data(), cnt.size() * 4);
    a.state_x = (unsigned long long*)up(x0.data(), x0.size() * 8);
    a.state_ptr = (int*)up(ptr.data(), ptr.size() * 4);
    std::vector<int> zero(n_img, 0);
    a.status = (int*)up(zero.data(), zero.size() * 4);
    int32_t* idx_d = (int32_t*)up(idx_step.data(), idx_step.size() * 4);
    std::vector<float> ksi((size_t)n_img * 2 * M, 0.f);
    a.ksi = (const float*)up(ksi.data(), ksi.size() * 4);
    a.ldk = 2 * M; a.Mlat = M; a.ldy = M; a.rows = n_img;
    a.sparse = sparse;
    size_t nbytes = words.size() * 4;
    float* yq; (void)hipMalloc(&yq, sizeof(float) * n_img * M * steps);
    a.blocks = (const int4*)up(blocks.data(), blocks.size() * sizeof(int4));
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
#ifdef LBIC_RANS_STAMPS
    unsigned long long* dbg; (void)hipMalloc(&dbg, 8 * 4 * n_img); (void)hipMemset(dbg, 0, 8 * 4 * n_img);
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_rdbg), &dbg, sizeof(dbg));
#endif
    (void)hipEventRecord(e0, nullptr);
    for (int st = 0; st < steps; ++st) {
        a.idx = idx_d + (size_t)st * n_img * M;
        a.yq = yq + (size_t)st * n_img * M;
        launch_rans_decode(a, nullptr);
    }
    (void)hipEventRecord(e1, nullptr);
    (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    std::vector<float> out((size_t)n_img * M * steps);
    (void)hipMemcpy(out.data(), yq, out.size() * 4, hipMemcpyDeviceToHost);
    long bad = 0;
    for (int st = 0; st < steps; ++st)
        for (int im = 0; im < n_img; ++im)
            for (int k = 0; k < M; ++k)
                bad += (int)out[((size_t)st * n_img + im) * M + k] != sym[((size_t)im * steps + st) * M + k];
#ifdef LBIC_RANS_STAMPS
    {   // last step: mean over waves of prologue / symbol loop / epilogue (s_memtime = shader clock)
        std::vector<unsigned long long> d(4 * n_img);
        (void)hipMemcpy(d.data(), dbg, 8 * 4 * n_img, hipMemcpyDeviceToHost);
        double t[3] = {0, 0, 0};
        for (int im = 0; im < n_img; ++im) for (int k = 0; k < 3; ++k) t[k] += (double)(d[im * 4 + k + 1] - d[im * 4 + k]) / n_img;
        printf("cycles (s_memtime): prologue %.0f, loop %.0f (%.0f / symbol), epilogue %.0f\n", t[0], t[1], t[1] / M, t[2]);
    }
#endif
    printf("rans decode (%s): %d images x %d symbols, tables %d..%d, %.3f bits/symbol: %.2f us/step, %.0f ns/symbol, "
           "mismatches %ld\n", sparse ? "sparse" : "lds", n_img, M, lo_idx, hi_idx, 8.0 * nbytes / idx.size(),
           ms * 1e3 / steps, ms * 1e6 / steps / M, bad);
    return 0;
}
