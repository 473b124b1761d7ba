// HIP kernels for gfx950 (MI355X): the per-step GEMM chain of the block codec and the GPU rANS decoder.
//
// k_gemm: out[rows, N] = epilogue( A[rows, K] . W[K, N] ), fp32 in / fp32 accumulate on
// v_mfma_f32_16x16x4_f32 (exact f32 fma chains, MI355X_MICROARCH.md "Matrix cores").  The A operand is
// gathered on the fly from up to 6 K-segments (dense activations, a reconstructed neighbour block of the
// padded zhat, or the block's own pixels x), so the masked 3x3 'A' convolutions of the reference
// (masked_conv2d.py:9-21, used at net:380-397) are a single GEMM over the 4 live taps with no im2col
// buffer; GDN's C x C contraction (gdn_compressai.py:71) is the same GEMM with A squared on load and a
// x*rsqrt / x*sqrt epilogue; the quantize / scale-index / likelihood step (entropy_layers_cai.py:126-151,
// 615-654) is the epilogue of the last encoder layer; the clamp + write-back of the reconstruction
// (net:357) is the epilogue of the last decoder layer.
//
// Tiles: BM rows x BN columns per workgroup, NW waves.  K is cut into KSPLIT = 8 fixed slices (by
// 16-wide k-blocks); wave w accumulates slices w, w+NW, ... in separate registers, partials meet in LDS
// and are summed in slice order.  The per-element arithmetic is therefore the same for every (BM, BN,
// NW), which is what keeps the encoder's wavefront steps and the decoder's raster steps bit-identical
// (the rANS decoder needs exactly the encoder's scale indexes).
#include "kernels.h"

#include <cmath>

#include "lbic_internal.h"

namespace lbic {

typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int scale_index(float s, const float* table) {
    // build_indexes (entropy_layers_cai.py:649-654): idx = 63 - #{k < 63 : max(s, .11) <= table[k]}
    s = fmaxf(s, 0.11f);
    int idx = 63;
#pragma unroll 8
    for (int k = 0; k < 63; ++k) idx -= (s <= table[k]) ? 1 : 0;
    return idx;
}

__device__ __forceinline__ float std_cum(float x) {
    // _standardized_cumulative (entropy_layers_cai.py:569-573)
    return 0.5f * erfcf(-0.70710677f * x);
}

template <int BM, int BN, int NW>
__global__ __launch_bounds__(NW * 64) void k_gemm(const GemmArgs g) {
    constexpr int MS = BM / 16, NS = BN / 16, SPW = KSPLIT / NW;
    extern __shared__ __attribute__((aligned(16))) float red[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int n0 = blockIdx.x * BN, m0 = blockIdx.y * BM;
    const int q4 = (lane >> 4) * 4;

    // per-lane source offsets of the rows this lane feeds (row = lane&15 of each 16-row subtile)
    long zoff[MS], xoff[MS];
    int drow[MS];
#pragma unroll
    for (int s = 0; s < MS; ++s) {
        const int r = min(m0 + 16 * s + (lane & 15), g.M - 1);
        drow[s] = r;
        const int m = r / g.P, p = r - m * g.P;
        const int4 b = g.blocks[m];
        const int vv = b.y + 2 + g.pos_dy[p], hh = b.z + 2 + g.pos_dx[p];
        zoff[s] = ((long)(b.x * g.geo.Hp + vv) * g.geo.Wp + hh) * g.geo.Cx;
        xoff[s] = ((long)(b.x * g.geo.Hb + b.y) * g.geo.Wb + b.z) * g.geo.Cx;
    }

    f4 acc[SPW][MS][NS];
#pragma unroll
    for (int q = 0; q < SPW; ++q)
#pragma unroll
        for (int s = 0; s < MS; ++s)
#pragma unroll
            for (int j = 0; j < NS; ++j) acc[q][s][j] = f4{0.f, 0.f, 0.f, 0.f};

    const int nkb = g.K >> 4;
    const f4* Wt = reinterpret_cast<const f4*>(g.W) + lane;
    const int nb0 = n0 >> 4;
#pragma unroll
    for (int q = 0; q < SPW; ++q) {
        const int slice = wave + q * NW;
        const int kb0 = slice * nkb / KSPLIT, kb1 = (slice + 1) * nkb / KSPLIT;
        int si = 0;
        for (int kb = kb0; kb < kb1; ++kb) {
            const int k = kb << 4;
            while (k >= g.seg[si].k1) ++si;     // wave-uniform
            const Seg& sg = g.seg[si];
            const int kk = k - sg.k0 + q4;
            f4 a[MS];
#pragma unroll
            for (int s = 0; s < MS; ++s) {
                const float* src;
                if (sg.kind == SEG_DENSE) src = sg.base + (long)drow[s] * sg.ld;
                else if (sg.kind == SEG_ZTAP) src = g.geo.zpad + zoff[s] + (long)(sg.dy * g.geo.Wp + sg.dx) * g.geo.Cx;
                else src = g.geo.x + xoff[s];
                a[s] = *reinterpret_cast<const f4*>(src + kk);
                if (g.square_a) a[s] = a[s] * a[s];
            }
            f4 w[NS];
#pragma unroll
            for (int j = 0; j < NS; ++j) w[j] = Wt[((long)kb * g.NB16 + nb0 + j) * 64];
#pragma unroll
            for (int e = 0; e < 4; ++e)
#pragma unroll
                for (int s = 0; s < MS; ++s)
#pragma unroll
                    for (int j = 0; j < NS; ++j)
                        acc[q][s][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s][e], w[j][e], acc[q][s][j], 0, 0, 0);
        }
    }

    // partials -> LDS [slice][((s*NS + j)*4 + r)*64 + lane]
    constexpr int TE = BM * BN;
#pragma unroll
    for (int q = 0; q < SPW; ++q) {
        float* dst = red + (wave + q * NW) * TE;
#pragma unroll
        for (int s = 0; s < MS; ++s)
#pragma unroll
            for (int j = 0; j < NS; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) dst[((s * NS + j) * 4 + r) * 64 + lane] = acc[q][s][j][r];
    }
    __syncthreads();

    for (int e = threadIdx.x; e < TE; e += NW * 64) {
        float v = red[e];
#pragma unroll
        for (int i = 1; i < KSPLIT; ++i) v += red[i * TE + e];
        const int l = e & 63, r = (e >> 6) & 3, sj = e >> 8;
        const int row = m0 + (sj / NS) * 16 + (l >> 4) * 4 + r;
        const int col = n0 + (sj % NS) * 16 + (l & 15);
        if (row >= g.M || col >= g.N) continue;
        switch (g.epi) {
            case EPI_BIAS:
                g.out[(long)row * g.ldo + col] = v + g.bias[col];
                break;
            case EPI_LEAKY: {
                const float t = v + g.bias[col];
                g.out[(long)row * g.ldo + col] = t > 0.f ? t : t * 0.01f;
                break;
            }
            case EPI_GDN:
            case EPI_IGDN: {
                const float norm = v + g.bias[col];
                const float xv = g.gx[(long)row * g.ldx + col];
                const float sq = __fsqrt_rn(norm);
                g.out[(long)row * g.ldo + col] = g.epi == EPI_GDN ? xv * __fdiv_rn(1.0f, sq) : xv * sq;
                break;
            }
            case EPI_QUANT: {
                const float y = v + g.bias[col];
                const float scale = g.ksi[(long)row * g.ldk + col];
                const float mean = g.ksi[(long)row * g.ldk + g.Mlat + col];
                const float d = y - mean;
                const int sym = (int)rintf(d);               // torch.round: half to even
                const float yq = (float)sym + mean;
                g.out[(long)row * g.ldo + col] = yq;
                const int4 b = g.blocks[row];
                const long pos = ((long)b.x * g.HW + (long)b.y * g.geo.Wb + b.z) * g.Mlat + col;
                g.sym[pos] = sym;
                g.idx[pos] = scale_index(scale, g.table);
                if (g.bits) {
                    const float av = fabsf(yq - mean), sb = fmaxf(scale, 0.11f);
                    const float lik = std_cum((0.5f - av) / sb) - std_cum((-0.5f - av) / sb);
                    g.bits[pos] = -log2f(fmaxf(lik, 1e-9f));
                }
                break;
            }
            case EPI_CTXIDX: {
                const float t = v + g.bias[col];
                g.out[(long)row * g.ldo + col] = t;
                if (col < g.Mlat) g.idx[(long)row * g.Mlat + col] = scale_index(t, g.table);
                break;
            }
            case EPI_CLAMPZ: {
                const float t = fminf(fmaxf(v + g.bias[col], -0.5f), 0.5f);
                const int4 b = g.blocks[row];
                g.geo.zpad[((long)(b.x * g.geo.Hp + b.y + 2) * g.geo.Wp + b.z + 2) * g.geo.Cx + col] = t;
                break;
            }
        }
    }
}

template <int BM, int BN, int NW>
static int launch_cfg(const GemmArgs& g, hipStream_t s) {
    const size_t lds = (size_t)KSPLIT * BM * BN * sizeof(float);
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_gemm<BM, BN, NW>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        attr = true;
    }
    dim3 grid((g.N + BN - 1) / BN, (g.M + BM - 1) / BM);
    hipLaunchKernelGGL((k_gemm<BM, BN, NW>), grid, dim3(NW * 64), lds, s, g);
    return hipGetLastError() == hipSuccess ? LBC_OK : set_error(LBC_E_HIP, "k_gemm launch failed");
}

int launch_gemm(const GemmArgs& g, hipStream_t s, int* cfg_id) {
    if (g.M <= 0) return LBC_OK;
    if (g.K % 16 || g.K < 16) return set_error(LBC_E_ARG, "GEMM K must be a positive multiple of 16");
    if (g.M <= 64) {
        if (cfg_id) *cfg_id = 0;
        return launch_cfg<32, 16, 8>(g, s);
    }
    if (cfg_id) *cfg_id = 1;
    return launch_cfg<64, 32, 4>(g, s);
}

// ----------------------------------------------------------------------------------------- rANS decode
// One 64-lane wave per image decodes that image's Mlat symbols of the current block (RansDecoder::
// decode_stream, called per block at net:439), entirely on the GPU: the CDF tables live in LDS as
// 16-bit entries, each symbol's search is one wave-wide window compare (ballot + popcount) around the
// table centre, the 64-bit state stays wave-uniform.  Output: y_qnt = sym + mean (dequantize,
// entropy_layers_cai.py:159-168, net:440-442) for the decoder's first layer.
__global__ __launch_bounds__(64) void k_rans_decode(const RansArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint16_t lcdf[];
    const int lane = threadIdx.x;
    {
        const uint32_t* src = reinterpret_cast<const uint32_t*>(a.cdf16);
        uint32_t* dst = reinterpret_cast<uint32_t*>(lcdf);
        for (int i = lane; i < a.total16 / 2; i += 64) dst[i] = src[i];
    }
    __syncthreads();
    const int row = blockIdx.x;
    const int img = a.blocks[row].x;
    unsigned long long x = a.state_x[img];
    int p = a.state_ptr[img];
    const uint32_t* w = a.words + a.word_base[img];
    const int nw = a.word_count[img];
    int bad = 0;
    auto next_word = [&]() -> uint32_t {
        uint32_t v = 0;
        if (p < nw) v = w[p]; else bad = 1;
        ++p;
        return v;
    };
    auto get_bits = [&](int nb) -> uint32_t {
        const uint32_t v = (uint32_t)(x & ((1u << nb) - 1));
        x >>= nb;
        if (x < (1ull << 31)) x = (x << 32) | next_word();
        return v;
    };
    for (int i = 0; i < a.Mlat; ++i) {
        const int ci = a.idx[(long)row * a.Mlat + i];
        if (ci < 0 || ci > 63) { bad = 2; break; }
        const int base = a.tmeta[ci], len = a.tmeta[64 + ci], off = a.tmeta[128 + ci];
        const uint32_t cum = (uint32_t)(x & 0xffff);
        int lo = max(0, -off - 31);
        int s;
        for (;;) {
            const int j = lo + lane;
            const uint32_t c = j < len - 1 ? (uint32_t)lcdf[base + j] : 65536u;
            const unsigned long long m = __ballot(c <= cum);
            const int cnt = __popcll(m);
            if (cnt == 0) { lo = max(0, lo - 63); continue; }
            if (cnt == 64) { lo += 63; continue; }
            s = lo + cnt - 1;
            break;
        }
        const uint32_t start = lcdf[base + s];
        const uint32_t nxt = (s + 1 >= len - 1) ? 65536u : (uint32_t)lcdf[base + s + 1];
        x = (unsigned long long)(nxt - start) * (x >> 16) + (x & 0xffff) - start;
        if (x < (1ull << 31)) x = (x << 32) | next_word();
        int v = s;
        if (v == len - 2) {   // escape: value coded in 4-bit bypass chunks
            uint32_t c = get_bits(4), nb = c;
            while (c == 15u) { c = get_bits(4); nb += c; }
            if (nb > 8) { bad = 3; break; }
            uint32_t raw = 0;
            for (uint32_t jj = 0; jj < nb; ++jj) raw |= get_bits(4) << (jj * 4);
            v = (int)(raw >> 1);
            v = (raw & 1) ? -v - 1 : v + len - 2;
        }
        if (lane == 0) {
            const float mean = a.ksi[(long)row * a.ldk + a.Mlat + i];
            a.yq[(long)row * a.ldy + i] = (float)(v + off) + mean;
        }
    }
    if (lane == 0) {
        a.state_x[img] = x;
        a.state_ptr[img] = p;
        if (bad) a.status[img] = bad;
    }
}

int launch_rans_decode(const RansArgs& a, hipStream_t s) {
    const size_t lds = (size_t)a.total16 * sizeof(uint16_t);
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_rans_decode), hipFuncAttributeMaxDynamicSharedMemorySize,
                            160 * 1024);
        attr = true;
    }
    hipLaunchKernelGGL(k_rans_decode, dim3(a.rows), dim3(64), lds, s, a);
    return hipGetLastError() == hipSuccess ? LBC_OK : set_error(LBC_E_HIP, "k_rans_decode launch failed");
}

__global__ void k_copy_interior(const float* __restrict__ zpad, float* __restrict__ zout, int n_img, int Hb, int Wb,
                                int Cx) {
    const long total = (long)n_img * Hb * Wb * Cx / 4;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const long e = i * 4;
        const int c = (int)(e % Cx);
        long t = e / Cx;
        const int h = (int)(t % Wb);
        t /= Wb;
        const int v = (int)(t % Hb);
        const int img = (int)(t / Hb);
        const long src = ((long)(img * (Hb + 2) + v + 2) * (Wb + 4) + h + 2) * Cx + c;
        *reinterpret_cast<f4*>(zout + e) = *reinterpret_cast<const f4*>(zpad + src);
    }
}

int launch_copy_interior(const float* zpad, float* zout, int n_img, int Hb, int Wb, int Cx, hipStream_t s) {
    const long total = (long)n_img * Hb * Wb * Cx / 4;
    const int blocks = (int)std::min<long>((total + 255) / 256, 4096);
    hipLaunchKernelGGL(k_copy_interior, dim3(blocks), dim3(256), 0, s, zpad, zout, n_img, Hb, Wb, Cx);
    return hipGetLastError() == hipSuccess ? LBC_OK : set_error(LBC_E_HIP, "copy launch failed");
}

}  // namespace lbic
