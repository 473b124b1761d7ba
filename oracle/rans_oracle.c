/* Oracle (TEST INFRASTRUCTURE ONLY -- never linked into the product or measured as it).
 *
 * Plain-C restatement of the two native pieces of CompressAI that the reference calls on the hot path:
 *   - compressai._CXX.pmf_to_quantized_cdf   (called at graphs/layers/entropy_layers_cai.py:61-64,181)
 *   - compressai.ans.BufferedRansEncoder / RansDecoder (called at
 *     graphs/models/BlockBasedImgCompLossy_net.py:328,359-360 (encode) and :409-410,439 (decode)).
 * CompressAI is absent from the container and not vendored in /root/reference; its version is unpinned
 * (README installs git HEAD).  This follows CompressAI's published algorithm (cpp_exts/ops/ops.cpp and
 * cpp_exts/rans/rans_interface.cpp over ryg_rans' rans64.h): 64-bit rANS state, 32-bit renormalisation
 * words written back to front, 16-bit CDF precision, and the 4-bit "bypass" escape for symbols that fall
 * outside a table.  PARITY UNPINNED for bitstream bytes: no reference fixture holds a CompressAI stream.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>

#define PREC 16
#define BYPASS_PREC 4
#define MAX_BYPASS ((1 << BYPASS_PREC) - 1)
#define RANS_L (1ull << 31)

/* ---------------------------------------------------------------- pmf -> quantized cdf (ops.cpp) */
int oracle_pmf_to_quantized_cdf(const float *pmf, int n, int precision, uint32_t *cdf /* n+1 */) {
    for (int i = 0; i < n; ++i)
        if (pmf[i] < 0 || !isfinite(pmf[i])) return -1;
    cdf[0] = 0;
    for (int i = 0; i < n; ++i) cdf[i + 1] = (uint32_t)roundf(pmf[i] * (float)(1 << precision));
    uint32_t total = 0;
    for (int i = 0; i <= n; ++i) total += cdf[i];
    if (total == 0) return -2;
    for (int i = 0; i <= n; ++i) cdf[i] = (uint32_t)(((uint64_t)(1u << precision) * cdf[i]) / total);
    for (int i = 1; i <= n; ++i) cdf[i] += cdf[i - 1];
    cdf[n] = 1u << precision;
    for (int i = 0; i < n; ++i) {
        if (cdf[i] == cdf[i + 1]) {
            uint32_t best_freq = ~0u;
            int best_steal = -1;
            for (int j = 0; j < n; ++j) {
                uint32_t freq = cdf[j + 1] - cdf[j];
                if (freq > 1 && freq < best_freq) { best_freq = freq; best_steal = j; }
            }
            if (best_steal < 0) return -3;
            if (best_steal < i) {
                for (int j = best_steal + 1; j <= i; ++j) cdf[j]--;
            } else {
                for (int j = i + 1; j <= best_steal; ++j) cdf[j]++;
            }
        }
    }
    return 0;
}

/* ---------------------------------------------------------------- encoder (BufferedRansEncoder) */
typedef struct { uint16_t start, range; uint8_t bypass; } sym_t;

/* cdfs: [n_tables][cdf_stride] int32 (the reference's _quantized_cdf rows), sizes = _cdf_length,
 * offsets = _offset.  Returns the byte count written to out (a multiple of 4) or <0 on error. */
long oracle_rans_encode(const int32_t *symbols, const int32_t *indexes, long n, const int32_t *cdfs,
                        int cdf_stride, const int32_t *sizes, const int32_t *offsets, int n_tables,
                        uint8_t *out, long out_cap) {
    long cap = 16 + n * 4;
    sym_t *syms = (sym_t *)malloc(sizeof(sym_t) * (size_t)cap);
    long ns = 0;
    for (long i = 0; i < n; ++i) {
        int32_t ci = indexes[i];
        if (ci < 0 || ci >= n_tables) { free(syms); return -1; }
        const int32_t *cdf = cdfs + (long)ci * cdf_stride;
        int32_t max_value = sizes[ci] - 2;
        int32_t value = symbols[i] - offsets[ci];
        uint32_t raw = 0;
        if (value < 0) { raw = (uint32_t)(-2 * value - 1); value = max_value; }
        else if (value >= max_value) { raw = (uint32_t)(2 * (value - max_value)); value = max_value; }
        if (ns + 40 >= cap) { cap *= 2; syms = (sym_t *)realloc(syms, sizeof(sym_t) * (size_t)cap); }
        syms[ns].start = (uint16_t)cdf[value];
        syms[ns].range = (uint16_t)(cdf[value + 1] - cdf[value]);
        syms[ns].bypass = 0; ns++;
        if (value == max_value) {
            int32_t nb = 0;
            while ((raw >> (nb * BYPASS_PREC)) != 0) ++nb;
            int32_t val = nb;
            while (val >= MAX_BYPASS) {
                syms[ns].start = MAX_BYPASS; syms[ns].range = MAX_BYPASS + 1; syms[ns].bypass = 1; ns++;
                val -= MAX_BYPASS;
            }
            syms[ns].start = (uint16_t)val; syms[ns].range = (uint16_t)(val + 1); syms[ns].bypass = 1; ns++;
            for (int32_t j = 0; j < nb; ++j) {
                int32_t v = (raw >> (j * BYPASS_PREC)) & MAX_BYPASS;
                syms[ns].start = (uint16_t)v; syms[ns].range = (uint16_t)(v + 1); syms[ns].bypass = 1; ns++;
            }
        }
    }
    /* flush: encode in reverse, words written back to front */
    long nwords = ns + 2;
    uint32_t *buf = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)nwords);
    uint32_t *ptr = buf + nwords;
    uint64_t x = RANS_L;
    for (long k = ns - 1; k >= 0; --k) {
        const sym_t s = syms[k];
        if (!s.bypass) {
            uint64_t x_max = ((RANS_L >> PREC) << 32) * s.range;
            if (x >= x_max) { *--ptr = (uint32_t)x; x >>= 32; }
            x = ((x / s.range) << PREC) + (x % s.range) + s.start;
        } else {
            uint32_t freq = 1u << (16 - BYPASS_PREC);
            uint64_t x_max = ((RANS_L >> 16) << 32) * freq;
            if (x >= x_max) { *--ptr = (uint32_t)x; x >>= 32; }
            x = (x << BYPASS_PREC) | s.start;
        }
    }
    ptr -= 2;
    ptr[0] = (uint32_t)(x >> 0);
    ptr[1] = (uint32_t)(x >> 32);
    long nbytes = (long)((buf + nwords) - ptr) * 4;
    free(syms);
    if (nbytes > out_cap) { free(buf); return -2; }
    memcpy(out, ptr, (size_t)nbytes);
    free(buf);
    return nbytes;
}

/* ---------------------------------------------------------------- decoder (RansDecoder) */
typedef struct { uint64_t x; const uint32_t *ptr, *end; } dec_t;

void *oracle_dec_new(const uint8_t *data, long len) {
    dec_t *d = (dec_t *)calloc(1, sizeof(dec_t));
    d->ptr = (const uint32_t *)data;
    d->end = (const uint32_t *)(data + len);
    d->x = (uint64_t)d->ptr[0] | ((uint64_t)d->ptr[1] << 32);
    d->ptr += 2;
    return d;
}

void oracle_dec_free(void *d) { free(d); }

static inline uint32_t rd_word(dec_t *d) { return d->ptr < d->end ? *d->ptr++ : 0u; }

static inline uint32_t get_bits(dec_t *d, uint32_t nbits) {
    uint64_t x = d->x;
    uint32_t val = (uint32_t)(x & ((1u << nbits) - 1));
    x >>= nbits;
    if (x < RANS_L) x = (x << 32) | rd_word(d);
    d->x = x;
    return val;
}

/* decode_stream: n symbols with the given table indexes (graphs/models/...:439). */
int oracle_dec_decode(void *dv, const int32_t *indexes, long n, const int32_t *cdfs, int cdf_stride,
                      const int32_t *sizes, const int32_t *offsets, int n_tables, int32_t *out) {
    dec_t *d = (dec_t *)dv;
    for (long i = 0; i < n; ++i) {
        int32_t ci = indexes[i];
        if (ci < 0 || ci >= n_tables) return -1;
        const int32_t *cdf = cdfs + (long)ci * cdf_stride;
        int32_t max_value = sizes[ci] - 2;
        int32_t offset = offsets[ci];
        uint32_t cum = (uint32_t)(d->x & ((1u << PREC) - 1));
        int32_t s = 0;
        while (s + 1 < sizes[ci] && (uint32_t)cdf[s + 1] <= cum) ++s;   /* first cdf[j] > cum, minus one */
        uint32_t start = (uint32_t)cdf[s], freq = (uint32_t)(cdf[s + 1] - cdf[s]);
        uint64_t x = d->x;
        x = (uint64_t)freq * (x >> PREC) + (x & ((1u << PREC) - 1)) - start;
        if (x < RANS_L) x = (x << 32) | rd_word(d);
        d->x = x;
        int32_t value = s;
        if (value == max_value) {
            int32_t val = (int32_t)get_bits(d, BYPASS_PREC);
            int32_t nb = val;
            while (val == MAX_BYPASS) { val = (int32_t)get_bits(d, BYPASS_PREC); nb += val; }
            int32_t raw = 0;
            for (int32_t j = 0; j < nb; ++j) {
                val = (int32_t)get_bits(d, BYPASS_PREC);
                raw |= val << (j * BYPASS_PREC);
            }
            value = raw >> 1;
            if (raw & 1) value = -value - 1;
            else value += max_value;
        }
        out[i] = value + offset;
    }
    return 0;
}
