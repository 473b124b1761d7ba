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

// For the GPU decoder: per table, the symbol index whose interval contains cum = 256*q (q = 0..255),
// i.e. the largest s with cdf[s] <= 256*q.  A symbol with cum in bucket q lies in [lut[q], lut[q+1]].
// Start-index LUT of the GPU decoder: for each table whose CDF has more than 64 entries, 256 buckets of
// cum (cum >> 8) -> the last symbol s with cdf[s] <= 256*bucket (the 64-entry window search starts there).
// Short tables need none (their whole CDF fits one window): lut_off[i] = -1.  Keeping only the long
// tables' rows halves the decoder's LDS footprint (87 -> 71 KB for the 64 Gaussian tables).
void build_start_lut(const EntropyTables& t, std::vector<uint16_t>& lut, std::vector<int>& lut_off) {
    lut.clear();
    lut_off.assign(t.n_tables, -1);
    for (int i = 0; i < t.n_tables; ++i) {
        if (t.length[i] - 1 <= 64) continue;
        lut_off[i] = (int)lut.size();
        const int32_t* cdf = t.cdf.data() + (size_t)i * t.stride;
        int s = 0;
        for (int q = 0; q < 256; ++q) {
            const int32_t c = 256 * q;
            while (s + 1 <= t.length[i] - 2 && cdf[s + 1] <= c) ++s;
            lut.push_back((uint16_t)s);
        }
    }
}

}  // namespace lbic
