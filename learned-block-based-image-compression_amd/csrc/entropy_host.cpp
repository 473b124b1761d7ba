// Host-side entropy coding for liblbic.so: pmf -> 16-bit quantized CDF, and the rANS encoder/decoder
// in the reference's bitstream format.
//
// Replaces CompressAI's C++ (`compressai._CXX.pmf_to_quantized_cdf`, reached from
// graphs/layers/entropy_layers_cai.py:61-64, and `compressai.ans.BufferedRansEncoder / RansDecoder`,
// reached from graphs/models/BlockBasedImgCompLossy_net.py:328,359-360,409-410,439).  The format is
// CompressAI's: a 64-bit rANS state (ryg_rans "rans64"), 32-bit renormalisation words emitted back to
// front, 16-bit frequencies, a per-table escape symbol (index cdf_length-2) followed by 4-bit "bypass"
// chunks for values outside the table.  CompressAI is not available offline, so byte-level parity with
// it is unpinned; tests pin this coder against oracle/rans_oracle.c and by round trips.
#include "lbic_internal.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <numeric>

namespace lbic {

static constexpr int kPrec = 16;
static constexpr int kBypassBits = 4;
static constexpr uint32_t kBypassMax = (1u << kBypassBits) - 1;
static constexpr uint64_t kRansL = 1ull << 31;

int pmf_to_quantized_cdf(const float* pmf, int n, int precision, uint32_t* cdf) {
    if (n <= 0 || precision <= 0 || precision > 16) return LBC_E_ARG;
    for (int i = 0; i < n; ++i)
        if (!(pmf[i] >= 0.f) || !std::isfinite(pmf[i])) return set_error(LBC_E_ARG, "invalid pmf value");
    const uint32_t one = 1u << precision;
    cdf[0] = 0;
    uint64_t total = 0;
    for (int i = 0; i < n; ++i) {
        cdf[i + 1] = (uint32_t)std::round(pmf[i] * (float)one);   // float product, then round (ops.cpp)
        total += cdf[i + 1];
    }
    if (total == 0) return set_error(LBC_E_ARG, "pmf has no mass");
    for (int i = 0; i <= n; ++i) cdf[i] = (uint32_t)(((uint64_t)one * cdf[i]) / total);
    for (int i = 1; i <= n; ++i) cdf[i] += cdf[i - 1];
    cdf[n] = one;
    // every symbol needs a non-zero frequency: steal one count from the smallest frequency > 1
    for (int i = 0; i < n; ++i) {
        if (cdf[i] != cdf[i + 1]) continue;
        uint32_t best = ~0u;
        int steal = -1;
        for (int j = 0; j < n; ++j) {
            const uint32_t f = cdf[j + 1] - cdf[j];
            if (f > 1 && f < best) { best = f; steal = j; }
        }
        if (steal < 0) return set_error(LBC_E_ARG, "cannot make cdf strictly increasing");
        if (steal < i) { for (int j = steal + 1; j <= i; ++j) cdf[j]--; }
        else { for (int j = i + 1; j <= steal; ++j) cdf[j]++; }
    }
    return LBC_OK;
}

namespace {
struct Sym {
    uint16_t start, range;
    bool bypass;
};
}  // namespace

int rans_encode(const EntropyTables& t, const int32_t* symbols, const int32_t* indexes, size_t n,
                std::vector<uint8_t>& out) {
    std::vector<Sym> syms;
    syms.reserve(n + 16);
    for (size_t i = 0; i < n; ++i) {
        const int32_t ci = indexes[i];
        if (ci < 0 || ci >= t.n_tables) return set_error(LBC_E_ARG, "scale index out of range");
        const int32_t* cdf = t.cdf.data() + (size_t)ci * t.stride;
        const int32_t maxv = t.length[ci] - 2;
        int32_t v = symbols[i] - t.offset[ci];
        uint32_t raw = 0;
        if (v < 0) { raw = (uint32_t)(-2 * v - 1); v = maxv; }
        else if (v >= maxv) { raw = (uint32_t)(2 * (v - maxv)); v = maxv; }
        syms.push_back({(uint16_t)cdf[v], (uint16_t)(cdf[v + 1] - cdf[v]), false});
        if (v == maxv) {
            uint32_t nb = 0;
            while (nb < 8 && (raw >> (nb * kBypassBits)) != 0) ++nb;
            uint32_t c = nb;
            for (; c >= kBypassMax; c -= kBypassMax) syms.push_back({(uint16_t)kBypassMax, (uint16_t)(kBypassMax + 1), true});
            syms.push_back({(uint16_t)c, (uint16_t)(c + 1), true});
            for (uint32_t j = 0; j < nb; ++j) {
                const uint32_t chunk = (raw >> (j * kBypassBits)) & kBypassMax;
                syms.push_back({(uint16_t)chunk, (uint16_t)(chunk + 1), true});
            }
        }
    }
    std::vector<uint32_t> words(syms.size() + 2);
    uint32_t* ptr = words.data() + words.size();
    uint64_t x = kRansL;
    for (size_t k = syms.size(); k-- > 0;) {
        const Sym s = syms[k];
        if (!s.bypass) {
            const uint64_t x_max = ((kRansL >> kPrec) << 32) * s.range;
            if (x >= x_max) { *--ptr = (uint32_t)x; x >>= 32; }
            x = ((x / s.range) << kPrec) + (x % s.range) + s.start;
        } else {
            const uint64_t x_max = ((kRansL >> 16) << 32) * (1u << (16 - kBypassBits));
            if (x >= x_max) { *--ptr = (uint32_t)x; x >>= 32; }
            x = (x << kBypassBits) | s.start;
        }
    }
    ptr -= 2;
    ptr[0] = (uint32_t)x;
    ptr[1] = (uint32_t)(x >> 32);
    const size_t nbytes = (size_t)(words.data() + words.size() - ptr) * 4;
    out.resize(nbytes);
    std::memcpy(out.data(), ptr, nbytes);
    return LBC_OK;
}

int rans_decode_host(const EntropyTables& t, const uint8_t* data, size_t len, const int32_t* indexes, size_t n,
                     int32_t* out) {
    if (len < 8 || (len & 3)) return set_error(LBC_E_STREAM, "bitstream length must be a multiple of 4, >= 8");
    const uint32_t* w = reinterpret_cast<const uint32_t*>(data);
    const size_t nw = len / 4;
    size_t p = 2;
    uint64_t x = (uint64_t)w[0] | ((uint64_t)w[1] << 32);
    auto next = [&]() -> uint32_t { return p < nw ? w[p++] : 0u; };
    auto bits = [&](uint32_t nbits) -> uint32_t {
        const uint32_t v = (uint32_t)(x & ((1u << nbits) - 1));
        x >>= nbits;
        if (x < kRansL) x = (x << 32) | next();
        return v;
    };
    for (size_t i = 0; i < n; ++i) {
        const int32_t ci = indexes[i];
        if (ci < 0 || ci >= t.n_tables) return set_error(LBC_E_ARG, "scale index out of range");
        const int32_t* cdf = t.cdf.data() + (size_t)ci * t.stride;
        const int32_t len_i = t.length[ci];
        const uint32_t cum = (uint32_t)(x & 0xffff);
        // first entry > cum, minus one (upper_bound on the strictly increasing prefix)
        const int32_t s = (int32_t)(std::upper_bound(cdf, cdf + len_i, (int32_t)cum) - cdf) - 1;
        const uint32_t start = (uint32_t)cdf[s], freq = (uint32_t)(cdf[s + 1] - cdf[s]);
        x = freq * (x >> kPrec) + (x & 0xffff) - start;
        if (x < kRansL) x = (x << 32) | next();
        int32_t v = s;
        if (v == len_i - 2) {
            uint32_t c = bits(kBypassBits), nb = c;
            while (c == kBypassMax) { c = bits(kBypassBits); nb += c; }
            uint32_t raw = 0;
            for (uint32_t j = 0; j < nb; ++j) raw |= bits(kBypassBits) << (j * kBypassBits);
            v = (int32_t)(raw >> 1);
            v = (raw & 1) ? -v - 1 : v + len_i - 2;
        }
        out[i] = v + t.offset[ci];
    }
    return LBC_OK;
}

// LDS image of the GPU decoder's tables (k_rans_decode, kernels.hip).  Every CDF entry c is stored as the
// 16-bit e = c - 1 (mod 2^16): c <= cum  <=>  e < cum for every c >= 1, the only c = 0 entry (index 0)
// becomes 0xFFFF and is never counted (the decoder counts lane 0 of a window itself), and the implicit
// final 2^16 is also 0xFFFF (and e + 1 = 2^16 recovers it).
//   coarse [n_tables][64]  lane l of table t: e[min(l * S_t, len_t - 1)], 0xFFFF past the table
//   fine   per table: e[0 .. len_t - 2], then 64 x 0xFFFF (so a 64-wide window never leaves the table)
// S_t = ceil((len_t - 1) / 64) symbols per coarse segment; a table with len_t <= 64 is "short": its coarse
// row is its whole CDF (S = 1).
// meta [8][64]: fine row start (bytes), S (in bytes: 2 S), len - 2 (the escape symbol), coarse row start (bytes),
// offset (-pmf_center), then the intervals lo | freq << 16 of the symbols of value 0, -1 and +1 (the sparse
// decoder's compare-only paths).
int build_rans_gpu_tables(const EntropyTables& t, std::vector<uint16_t>& img, std::vector<int>& meta) {
    const int nt = t.n_tables;
    if (nt < 1 || nt > 64) return set_error(LBC_E_ARG, "GPU rANS decoder supports 1..64 tables");
    img.assign((size_t)nt * 64, 0xFFFF);
    meta.assign(8 * 64, 0);
    for (int i = 0; i < nt; ++i) {
        const int len = t.length[i];
        if (len < 3 || len > t.stride) return set_error(LBC_E_ARG, "bad cdf length");
        if (len - 1 > 63 * 64) return set_error(LBC_E_ARG, "cdf longer than the GPU decoder's 2-level search");
        const int32_t* cdf = t.cdf.data() + (size_t)i * t.stride;
        if (cdf[0] != 0 || cdf[len - 1] != 65536) return set_error(LBC_E_ARG, "cdf must span [0, 2^16]");
        for (int j = 0; j + 1 < len; ++j)
            if (cdf[j + 1] <= cdf[j]) return set_error(LBC_E_ARG, "cdf must be strictly increasing");
        const size_t fbase = img.size();
        for (int j = 0; j < len - 1; ++j) img.push_back((uint16_t)((cdf[j] - 1) & 0xFFFF));
        for (int j = 0; j < 64; ++j) img.push_back(0xFFFF);
        const bool shrt = len <= 64;
        const int S = shrt ? 1 : (len - 1 + 63) / 64;
        for (int l = 0; l < 64; ++l) img[(size_t)i * 64 + l] = img[fbase + std::min(l * S, len - 1)];
        meta[i] = (int)fbase * 2;
        meta[64 + i] = S * 2;
        meta[128 + i] = len - 2;
        meta[192 + i] = i * 128;
        meta[256 + i] = t.offset[i];
        // the most probable symbol (value 0, index -offset): its interval [lo, lo + freq) packed lo | freq << 16
        // (freq < 2^16: the escape symbol always keeps a share), the sparse decoder's one-compare fast path
        const int c0 = -t.offset[i];
        if (c0 < 0 || c0 + 1 >= len - 1) return set_error(LBC_E_ARG, "cdf offset outside the table");
        for (int d = 0; d < 3; ++d) {     // value 0, -1, +1: index c0, c0 - 1, c0 + 1
            const int c = d == 0 ? c0 : d == 1 ? c0 - 1 : c0 + 1;
            if (c < 0 || c >= len - 2) continue;   // no such symbol, or the escape: freq 0 never matches
            const int lo = cdf[c], fr = cdf[c + 1] - cdf[c];
            if (lo > 0xFFFF || fr > 0xFFFF) return set_error(LBC_E_ARG, "bad centre interval");
            meta[(5 + d) * 64 + i] = lo | (fr << 16);
        }
    }
    while (img.size() & 7) img.push_back(0xFFFF);   // 16-byte granules for the LDS staging loads
    if (img.size() * 2 > 150 * 1024) return set_error(LBC_E_ARG, "cdf tables exceed the LDS budget");
    return LBC_OK;
}

}  // namespace lbic
