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
#include "kernels_dev.h"

namespace lbic {

// CH k-blocks per chunk: all their loads are issued together, and chunk c+1 is in flight while chunk c
// is multiplied, so a slice of K costs about one memory round trip instead of one per k-block.
// OCC: minimum waves per SIMD the register allocation must allow (1 = no constraint).  The team decoder keeps
// 256 of each SIMD's 512 VGPRs while it runs, so the encoder's residency beside it is (512 - 256) / its VGPRs.
// ONE: A is a single dense segment (every layer but the first of each transform and of the context net): each
// k-block's fragments are buffer loads at a per-lane row address plus a scalar k-block offset (weights likewise: lane *
// 16 plus the fragment's scalar offset), with no per-k-block segment selection and no 64-bit address arithmetic -- the
// k-loop issues its loads and MFMAs and little else (the encoder's GEMMs wait on instruction issue, round-3 PMC).
template <int BM, int BN, int NW, int CH, int OCC = 1, bool ONE = false>
__global__ __launch_bounds__(NW * 64, OCC) void k_gemm(const GemmArgs g) {
    constexpr int MS = BM / 16, NS = BN / 16, SPW = KSPLIT / NW;
    extern __shared__ __attribute__((aligned(16))) float red[];
    warm_kernargs<10>();
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // uniform: keeps the k-loop scalar
    const int bid = blockIdx.y * gridDim.x + blockIdx.x;
    const int n0 = (bid % gridDim.x) * BN;
    const int m0 = (bid / gridDim.x) * BM;
    const int q4 = (lane >> 4) * 4;

    stamp_start(g.ts);
    PHASE(0);
    const int4* blocks = g.ctr ? g.blocks + (long)(*g.ctr) * g.ctr_stride : g.blocks;
    // per-lane, per-segment element offsets of the rows this lane feeds (row = lane&15 of each subtile)
    Rows<MS> R;
#pragma unroll
    for (int s = 0; s < MS; ++s) {
        const int r = min(m0 + 16 * s + (lane & 15), g.M - 1);
        const int m = r / g.P, p = r - m * g.P;
        const int4 b = g.need_blocks ? blocks[m] : make_int4(0, 0, 0, 0);   // dense-only GEMMs skip this load
        const long cell = ((long)b.x * g.geo.Hp + b.y + 2 + g.pos_dy[p]) * g.geo.Wp + b.z + 2 + g.pos_dx[p];
        const long xrow = (((long)b.x * g.geo.Hb + b.y) * g.geo.Wb + b.z) * g.geo.Cx;
#pragma unroll
        for (int t = 0; t < MAXSEG; ++t) {
            const Seg& sg = g.seg[t];
            const long o = (long)r * sg.ld + sg.zs * cell + (sg.xs ? xrow : 0l) + sg.tap;
            R.off[t][s] = (unsigned)(o >> 2);
        }
    }

    f4 acc[SPW][MS][NS];
#pragma unroll
    for (int q = 0; q < SPW; ++q)
#pragma unroll
        for (int s = 0; s < MS; ++s)
#pragma unroll
            for (int j = 0; j < NS; ++j) acc[q][s][j] = f4{0.f, 0.f, 0.f, 0.f};
    PHASE(1);

    const int nkb = g.K >> 4;
    const int nb0 = n0 >> 4;
    // ONE: buffer resources of the A segment and the weights, per-lane byte addresses of this lane's A rows
    const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(g.seg[0].base), 0, -1, 0x00020000);
    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(g.W), 0, -1, 0x00020000);
    unsigned va[MS];
#pragma unroll
    for (int s = 0; s < MS; ++s) va[s] = (R.off[0][s] << 4) + (unsigned)(q4 << 2);
#pragma unroll
    for (int q = 0; q < SPW; ++q) {
        const int slice = wave + q * NW;
        const int kb0 = slice * nkb / KSPLIT, kb1 = (slice + 1) * nkb / KSPLIT;
        if (kb0 >= kb1) continue;
        Frag<MS, NS> fa[CH], fb[CH];
        // out-of-range k-blocks of the last chunk re-load the slice's last block (valid address) and
        // skip their MFMAs, so the summation order is the plain k order for every CH
        auto load_chunk = [&](int base, Frag<MS, NS>(&f)[CH]) {
#pragma unroll
            for (int c = 0; c < CH; ++c) {
                const int kb = min(base + c, kb1 - 1);
                if constexpr (ONE) {
#pragma unroll
                    for (int s = 0; s < MS; ++s)
                        f[c].a[s] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(ra, va[s], (unsigned)kb << 6, 0));
#pragma unroll
                    for (int j = 0; j < NS; ++j)
                        f[c].w[j] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(
                                                               rw, (unsigned)lane << 4, (unsigned)(kb * g.NB16 + nb0 + j) << 10, 0));
                } else {
                    load_kb<MS, NS>(g, kb, nb0, R, q4, lane, f[c]);
                }
            }
        };
        auto mma_chunk = [&](int base, Frag<MS, NS>(&f)[CH]) {
#pragma unroll
            for (int c = 0; c < CH; ++c)
                if (base + c < kb1) mma_kb<MS, NS>(g, f[c], acc[q]);
        };
        int kb = kb0;
        load_chunk(kb, fa);
        while (kb < kb1) {               // two named buffers, statically indexed (no scratch)
            if (kb + CH < kb1) load_chunk(kb + CH, fb);
            mma_chunk(kb, fa);
            kb += CH;
            if (kb >= kb1) break;
            if (kb + CH < kb1) load_chunk(kb + CH, fa);
            mma_chunk(kb, fb);
            kb += CH;
        }
    }

    PHASE(2);
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
    PHASE(3);

    for (int e = threadIdx.x; e < TE; e += NW * 64) {
        float v = red[e];
#pragma unroll
        for (int i = 1; i < KSPLIT; ++i) v += red[i * TE + e];
        const int l = e & 63, r = (e >> 6) & 3, sj = e >> 8;
        const int row = m0 + (sj / NS) * 16 + (l >> 4) * 4 + r;
        const int col = n0 + (sj % NS) * 16 + (l & 15);
        if (row >= g.M || col >= g.N) continue;
        const bool gdn = g.epi == EPI_GDN || g.epi == EPI_IGDN;
        epilogue(g, v, row, col, BlkSrc{blocks, 0, 0, 0, 0}, g.bias[col], gdn ? g.gx[(long)row * g.ldx + col] : 0.f);
    }
    PHASE(4);
    stamp_end(g.ts);
}

// k-blocks [kb0, kb0 + n) of this wave's slice onto acc; n in {L, L+1} (the 8 slices of nkb k-blocks
// differ by at most one).  The (L+1)-th block is always loaded and multiplied into a side accumulator,
// selected afterwards, so every load feeds an unconditional MFMA and none is sunk behind a branch.
template <int L, bool RASTER, bool EXACT = false>
__device__ __forceinline__ f4 small_slice(const GemmArgs& g, int kb0, int n, int nt, int m0, int lane, const BlkSrc& blocks,
                                          f4 acc) {
    constexpr int LL = EXACT ? L : L + 1;     // EXACT: every slice has exactly L k-blocks (K/16 divisible by 8)
    const int nkb = g.K >> 4;
    const f4* Wt = reinterpret_cast<const f4*>(g.W) + lane;
    f4 w[LL], a[LL];
    const SBlk bk = small_blk<RASTER>(g, m0, lane, blocks);   // issued first: the A addresses wait for it
    if constexpr (RASTER) {
        // the block is computed, not loaded: every address is known now, so each k-block's weight and
        // activation fragments are requested together and the MFMA chain starts as soon as the first pair lands
        SRow rw;
        small_offsets(g, bk, lane, rw);
#pragma unroll
        for (int c = 0; c < LL; ++c) {
            const int kb = min(kb0 + c, nkb - 1);
            w[c] = Wt[((long)kb * g.NB16 + nt) * 64];
            a[c] = small_a(rw, kb);
        }
        PHASE(1);
    } else {
#pragma unroll
        for (int c = 0; c < LL; ++c) w[c] = Wt[((long)min(kb0 + c, nkb - 1) * g.NB16 + nt) * 64];
        SRow rw;
        small_offsets(g, bk, lane, rw);
        PHASE(1);
#pragma unroll
        for (int c = 0; c < LL; ++c) a[c] = small_a(rw, min(kb0 + c, nkb - 1));
    }
    // keep every load above the MFMAs (the scheduler would otherwise sink each one next to its first use
    // and wait for it there: one memory round trip per k-block)
    __builtin_amdgcn_sched_barrier(0);
    PHASE(2);
#pragma unroll
    for (int c = 0; c < LL; ++c) {
        f4 av = a[c];
        if (g.square_a) av = av * av;
        f4 t = acc;
#pragma unroll
        for (int e = 0; e < 4; ++e) t = __builtin_amdgcn_mfma_f32_16x16x4f32(av[e], w[c][e], t, 0, 0, 0);
        acc = c < n ? t : acc;
    }
    return acc;
}

// L = (K/16) / 8 k-blocks per slice (each slice L or L+1); L > 12: chunks of 12
template <int L, bool RASTER, bool EXACT>
__global__ __launch_bounds__(512) void k_gemm_s(const GemmArgs g) {
    __shared__ __attribute__((aligned(16))) float red[KSPLIT * 256];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nt = blockIdx.x;
    const int n0 = nt * 16, m0 = blockIdx.y * 16;
    warm_kernargs<10>();
    unsigned long long dph0_ = 0;
    (void)dph0_;
    DPH(0);
    stamp_start(g.ts);
    PHASE(0);
    // epilogue operands of this thread's output element (threads 0..255; the rest load a duplicate)
    const int el = threadIdx.x & 63, er = (threadIdx.x >> 6) & 3;
    const int erow = min(m0 + (el >> 4) * 4 + er, g.M - 1), ecol = min(n0 + (el & 15), g.N - 1);
    const float bcol = g.bias[ecol];
    const float xv = (g.epi == EPI_GDN || g.epi == EPI_IGDN) ? g.gx[(long)erow * g.ldx + ecol] : 0.f;

    const int nkb = g.K >> 4;
    const int kb0 = wave * nkb / KSPLIT, kb1 = (wave + 1) * nkb / KSPLIT;
    BlkSrc blocks{g.blocks, RASTER ? 1 : 0, g.raster_img0, 0, g.raster_h};
    if (g.need_blocks && g.ctr) {
        // scalar load: stays out of the vector-memory counter, so no weight load waits behind it
        int c;
        asm volatile("s_load_dword %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(c) : "s"(g.ctr) : "memory");
        if constexpr (RASTER) blocks.v = c;
        else blocks.p += (long)c * g.ctr_stride;
    }
    f4 acc = f4{0.f, 0.f, 0.f, 0.f};
    DPH(1);
    if constexpr (L <= 12) {
        acc = small_slice<L, RASTER, EXACT>(g, kb0, kb1 - kb0, nt, m0, lane, blocks, acc);
    } else {
        for (int c0 = kb0; c0 < kb1; c0 += 12)
            acc = small_slice<11, RASTER>(g, c0, min(12, kb1 - c0), nt, m0, lane, blocks, acc);
    }
    PHASE(3);
    DPH(2);
#pragma unroll
    for (int i = 0; i < 4; ++i) red[wave * 256 + i * 64 + lane] = acc[i];
    __syncthreads();
    DPH(3);
    PHASE(4);
    if (threadIdx.x < 256) {
        const int e = threadIdx.x;
        float v = red[e];
#pragma unroll
        for (int i = 1; i < KSPLIT; ++i) v += red[i * 256 + e];
        const int row = m0 + (el >> 4) * 4 + er, col = n0 + (el & 15);
        if (row < g.M && col < g.N) epilogue(g, v, row, col, blocks, bcol, xv);
    }
    PHASE(5);
    DPH(4);
    stamp_end(g.ts);
}

// largest M for the small-M kernel: the wavefront's ramp steps; a decoder raster step stays on it up to 1024 rows
// (ganged raster passes of up to 32 batches of 32 images: a raster step's latency barely grows with its rows)
constexpr int SMALL_MAX = 64, DEC_SMALL_MAX = 1024;

// 0 = k_gemm_s (latency-shaped, any M; the decoder's raster steps stay on it when several batches are decoded
// together: a raster step's latency barely grows with its rows), 1 = k_gemm (the encoder's wavefront steps)
int gemm_class(const GemmArgs& g) {
    static const int small_max = [] {      // experiment hook: LBIC_ENC_SMALL = largest M on k_gemm_s
        const char* e = getenv("LBIC_ENC_SMALL");
        return e ? atoi(e) : SMALL_MAX;
    }();
    return (g.M <= small_max || (g.raster && g.M <= DEC_SMALL_MAX)) ? 0 : 1;
}
template <int BM, int BN, int NW, int CH, int OCC = 1>
static int launch_cfg(const GemmArgs& g, hipStream_t s) {
    const size_t lds = std::max<size_t>((size_t)KSPLIT * BM * BN * sizeof(float), (size_t)std::max(g.lds_floor, 0));
    if (lds > 160 * 1024) return set_error(LBC_E_ARG, "LDS request above 160 KB");
    static const bool attr = [] {     // once per instantiation (thread-safe static initialisation)
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_gemm<BM, BN, NW, CH, OCC>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_gemm<BM, BN, NW, CH, OCC, true>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        return true;
    }();
    (void)attr;
    dim3 grid((g.N + BN - 1) / BN, (g.M + BM - 1) / BM);
    // the single-dense-segment instance where its 32-bit buffer offsets reach every A row and weight fragment
    const double a_end = ((double)(((g.M + BM - 1) / BM) * BM) * g.seg[0].ld + g.K) * 4.0;
    const double w_end = (double)(g.K / 16) * g.NB16 * 1024.0;
    if (g.nseg == 1 && g.seg[0].kind == SEG_DENSE && a_end < 4294967296.0 && w_end < 4294967296.0)
        hipLaunchKernelGGL((k_gemm<BM, BN, NW, CH, OCC, true>), grid, dim3(NW * 64), lds, s, g);
    else
        hipLaunchKernelGGL((k_gemm<BM, BN, NW, CH, OCC>), grid, dim3(NW * 64), lds, s, g);
    return launch_status("k_gemm");
}

int prepare_gemm(GemmArgs& g) {
    g.need_blocks = g.epi == EPI_QUANT || g.epi == EPI_CLAMPZ || g.epi == EPI_SCATTER || g.epi == EPI_LEAKY_L0 || g.zero_oob;
    for (int t = 0; t < g.nseg && t < MAXSEG; ++t) g.need_blocks |= g.seg[t].kind != SEG_DENSE;
    if (g.M <= 0) return LBC_OK;
    if (g.K % 16 || g.K < 16) return set_error(LBC_E_ARG, "GEMM K must be a positive multiple of 16");
    // host-side checks of what the kernel assumes: contiguous 16-aligned segments with real bases
    if (g.nseg < 1 || g.nseg > MAXSEG || g.seg[0].k0 != 0 || g.seg[g.nseg - 1].k1 < g.K)
        return set_error(LBC_E_ARG, "GEMM segments must cover [0, K)");
    for (int t = 0; t < g.nseg; ++t) {
        const Seg& sg = g.seg[t];
        if (!sg.base || (sg.k0 & 15) || (t && sg.k0 != g.seg[t - 1].k1) || (sg.kind == SEG_L0TAP && (sg.ld & 15)))
            return set_error(LBC_E_ARG, "bad GEMM segment");
    }
    if (!g.W || !g.bias || !g.blocks || g.P < 1 || g.P > 5) return set_error(LBC_E_ARG, "bad GEMM arguments");
    for (int t = 0; t < g.nseg; ++t) {            // branch-free row offset: r*ld + zs*zrow + xs*xrow + tap
        Seg& sg = g.seg[t];
        sg.zs = sg.kind == SEG_ZTAP ? g.geo.Cx : sg.kind == SEG_L0TAP ? sg.ld : 0;
        sg.xs = sg.kind == SEG_X;
        sg.tap = sg.zs * (sg.dy * g.geo.Wp + sg.dx);
        if (sg.kind != SEG_DENSE) sg.ld = 0;
    }
    for (int t = g.nseg; t < MAXSEG; ++t) {       // unused segments: never selected (k0 past every k)
        g.seg[t] = g.seg[0];
        g.seg[t].k0 = g.seg[t].k1 = 1 << 30;
    }
    return LBC_OK;
}

int launch_gemm(const GemmArgs& g0, hipStream_t s, int* cfg_id) {
    GemmArgs g = g0;
    if (g.M <= 0) return LBC_OK;
    int rc = prepare_gemm(g);
    if (rc) return rc;
    if (gemm_class(g) == 0) {      // small M (the decoder's per-step batch, wavefront ramps): latency-shaped kernel
        if (cfg_id) *cfg_id = 0;
        dim3 grid((g.N + 15) / 16, (g.M + 15) / 16);
        // the computed-block (RASTER) variant also serves every dense-only GEMM: its A rows need no block, and the
        // block-list variant would make their addresses wait for a block-index load (one memory round trip)
        const bool raster = (g.raster && g.ctr && g.need_blocks) || !g.need_blocks;
        if (g.raster && !g.ctr) return set_error(LBC_E_ARG, "raster GEMM needs the row counter");
        // every slice exactly L k-blocks: no (L+1)-th block to load (loads are what a launch waits for)
        const bool exact = ((g.K >> 4) % KSPLIT) == 0;
        const int sel = (raster ? 1 : 0) + (exact ? 2 : 0);
        switch ((g.K >> 4) / KSPLIT) {
#define LBIC_V(L, R, E) hipLaunchKernelGGL((k_gemm_s<L, R, E>), grid, dim3(512), 0, s, g)
#define LBIC_L(L)                                                                                  \
    case L:                                                                                        \
        switch (sel) {                                                                             \
            case 0: LBIC_V(L, false, false); break;                                                \
            case 1: LBIC_V(L, true, false); break;                                                 \
            case 2: LBIC_V(L, false, true); break;                                                 \
            default: LBIC_V(L, true, true); break;                                                 \
        }                                                                                          \
        break;
            case 0:
                if (raster) LBIC_V(0, true, false);
                else LBIC_V(0, false, false);
                break;
            LBIC_L(1) LBIC_L(2) LBIC_L(3) LBIC_L(4) LBIC_L(5) LBIC_L(6)
            LBIC_L(7) LBIC_L(8) LBIC_L(9) LBIC_L(10) LBIC_L(11) LBIC_L(12)
#undef LBIC_L
            default:
                if (raster) LBIC_V(13, true, false);
                else LBIC_V(13, false, false);
#undef LBIC_V
        }
        return launch_status("k_gemm_s");
    }
    if (cfg_id) *cfg_id = 1;
    // Encoder wavefront steps (n_img images x up to 48 blocks): many small tiles beat few large ones; the per-tile K
    // loop is latency-bound, so the step wants workgroups and waves.  Measured encode time per 32-frame 768x768
    // batch, encoder alone (tools/enc_exp.py, profiles/r02_exp/encoder_occupancy.txt), every shape bit-identical:
    // 16x32 / 8 waves / one k-block per chunk (56 VGPRs: 8 waves per SIMD) 98.7 ms; 16x32 / 4 waves / 2-block
    // chunks 108.2 (round 2's earlier default, 86 VGPRs: 5 waves per SIMD, 2 beside the team decoder's 256 VGPRs);
    // 16x32 / 4 / 1 capped at 70 VGPRs 105.7; 32x32 / 8 / 1 107.5; 16x64 / 8 / 1 112.0; 16x16 / 4 / 1 122.3;
    // register caps that spill (64 / 80 VGPRs) 116.7 / 115.8.  Beside the team decoder (bench.py --steps 20):
    // 84.9 Mpix/s against 79.7 for the earlier default.  (Other tiles, XCD-aware and 2-D XCD tile orders: measured
    // in rounds 2-3 and removed)
    static const int tile = [] {       // experiment hook: LBIC_ENC_TILE=1 -> 32 x 32 tiles (round 6, 128-frame passes)
        const char* e = getenv("LBIC_ENC_TILE");
        return e ? atoi(e) : 0;
    }();
    if (tile == 1) return launch_cfg<32, 32, 8, 1>(g, s);
    if (tile == 2) return launch_cfg<16, 64, 8, 1>(g, s);
    return launch_cfg<16, 32, 8, 1>(g, s);
}


__global__ __launch_bounds__(RANS_WPB * 64) void k_rans_decode(const RansArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint16_t lcdf[];
    warm_kernargs<3>();
    stamp_start(a.ts);
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * RANS_WPB + (threadIdx.x >> 6);
    rans_row(a, lcdf, row, lane);
    stamp_end(a.ts);
}

// one wave per stream, one stream per workgroup: no LDS shared between waves, so nothing to wait for but
// the wave's own loads
__global__ __launch_bounds__(64) void k_rans_decode_sparse(const RansArgs a) {
    __shared__ __attribute__((aligned(16))) uint32_t lwin[RANS_WIN];
    warm_kernargs<3>();
    stamp_start(a.ts);
    rans_row_sparse(a, lwin, blockIdx.x, threadIdx.x);
    stamp_end(a.ts);
}

int launch_rans_decode(const RansArgs& a, hipStream_t s) {
    if (a.rows <= 0) return LBC_OK;     // an empty wavefront step (e.g. odd steps of a one-column frame)
    if (a.Mlat > RANS_MAXLAT) return set_error(LBC_E_ARG, "M > 256 not supported by the GPU rANS decoder");
    if (a.total16 % 8) return set_error(LBC_E_ARG, "cdf16 tables must be padded to 16 bytes");
    if (a.sparse) {
        hipLaunchKernelGGL(k_rans_decode_sparse, dim3(a.rows), dim3(64), 0, s, a);
        return launch_status("k_rans_decode_sparse");
    }
    const size_t lds = (size_t)a.total16 * sizeof(uint16_t) + (size_t)RANS_WPB * RANS_WIN * sizeof(uint32_t);
    static const bool attr = [] {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_rans_decode),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        return true;
    }();
    (void)attr;
    const int wpb = a.rows < RANS_WPB ? a.rows : RANS_WPB;
    hipLaunchKernelGGL(k_rans_decode, dim3((a.rows + RANS_WPB - 1) / RANS_WPB), dim3(wpb * 64), lds, s, a);
    return launch_status("k_rans_decode");
}

__global__ void k_ctr_add(int* c, int d) { *c += d; }

// zeroes n 64-bit words (the timing-slot range at the head of a sampled graph: a captured memset node
// there wrote a stale 16-byte fill pattern into the range when several threads replayed graphs)
__global__ void k_zero_u64(unsigned long long* p, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = 0ull;
}

int launch_zero_u64(unsigned long long* p, int n, hipStream_t s) {
    if (n <= 0) return LBC_OK;
    hipLaunchKernelGGL(k_zero_u64, dim3((n + 255) / 256), dim3(256), 0, s, p, n);
    return launch_status("zero");
}

int launch_ctr_add(int* ctr, int d, hipStream_t s) {
    hipLaunchKernelGGL(k_ctr_add, dim3(1), dim3(1), 0, s, ctr, d);
    return launch_status("ctr");
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

__global__ void k_fill_interior(const float* __restrict__ zin, float* __restrict__ zpad, int n_img, int Hb, int Wb,
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
        const long dst = ((long)(img * (Hb + 2) + v + 2) * (Wb + 4) + h + 2) * Cx + c;
        *reinterpret_cast<f4*>(zpad + dst) = *reinterpret_cast<const f4*>(zin + e);
    }
}

// Layer-0 map cache (KS[1] = 3, codec.hip) before a closed loop: every channel of the cells of block row -1 (columns
// -1 .. Wb) and of columns -1 and Wb of every block row set to LeakyReLU(bias) (compress(): layer 0 of the
// zero-padded window, net:342-351, where every tap is zero) or to 0 (bias = null: forward()'s frame padding).  The
// GEMM computes such a cell as (slice sums of zeros) + bias -> LeakyReLU, i.e. the same value.  Columns -1 / Wb
// of rows >= 0 hold data-dependent values under compress(): the closed loops compute them before they are read.
__global__ void k_l0_border(float* __restrict__ l0, int n_img, int Hb, int Wb, int C, const float* __restrict__ bias) {
    const int per_img = (Wb + 2) + 2 * Hb;            // top row, then (left, right) of each block row
    const long total = (long)n_img * per_img * C;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const int c = (int)(i % C);
        const long t = i / C;
        const int img = (int)(t / per_img), k = (int)(t % per_img);
        int v, h;
        if (k < Wb + 2) { v = -1; h = k - 1; }
        else { v = (k - (Wb + 2)) >> 1; h = ((k - (Wb + 2)) & 1) ? Wb : -1; }
        float val = 0.f;
        if (bias) {
            const float b = bias[c];
            val = b > 0.f ? b : b * 0.01f;
        }
        l0[(((long)img * (Hb + 2) + v + 2) * (Wb + 4) + h + 2) * C + c] = val;
    }
}

int launch_l0_border(float* l0, int n_img, int Hb, int Wb, int C, const float* bias, hipStream_t s) {
    const long total = (long)n_img * ((Wb + 2) + 2 * Hb) * C;
    const int blocks = (int)std::min<long>((total + 255) / 256, 4096);
    hipLaunchKernelGGL(k_l0_border, dim3(blocks), dim3(256), 0, s, l0, n_img, Hb, Wb, C, bias);
    return launch_status("l0 border");
}

int launch_fill_interior(const float* zin, float* zpad, int n_img, int Hb, int Wb, int Cx, hipStream_t s) {
    const long total = (long)n_img * Hb * Wb * Cx / 4;
    const int blocks = (int)std::min<long>((total + 255) / 256, 4096);
    hipLaunchKernelGGL(k_fill_interior, dim3(blocks), dim3(256), 0, s, zin, zpad, n_img, Hb, Wb, Cx);
    return launch_status("fill");
}

int launch_copy_interior(const float* zpad, float* zout, int n_img, int Hb, int Wb, int Cx, hipStream_t s) {
    const long total = (long)n_img * Hb * Wb * Cx / 4;
    const int blocks = (int)std::min<long>((total + 255) / 256, 4096);
    hipLaunchKernelGGL(k_copy_interior, dim3(blocks), dim3(256), 0, s, zpad, zout, n_img, Hb, Wb, Cx);
    return launch_status("copy");
}

}  // namespace lbic
