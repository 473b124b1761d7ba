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
template <int BM, int BN, int NW, int CH, int OCC = 1>
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
            for (int c = 0; c < CH; ++c) load_kb<MS, NS>(g, min(base + c, kb1 - 1), nb0, R, q4, lane, f[c]);
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

// ----------------------------------------------------------------------------------------- k_gemm_t
// The encoder's wavefront GEMMs for N >= TG_MIN_N, LDS-staged: one 64 x 64 output tile per 512-thread workgroup.
// Eight waves = two K groups x four spatial waves (each a 32 x 32 quarter, 2 x 2 MFMA subtiles): group 0 takes K
// slices 0-3, group 1 slices 4-7.  Every operand fragment is brought into LDS once per group by LDS-DMA
// (global_load_lds_dwordx4: one wave instruction = one 1-KB fragment in the MFMA operand layout, lane l's 16 bytes at
// lane offset l, so the consumer's ds_read_b128 is lane-contiguous and conflict-free) and read by the two waves of the
// group that share its row or column subtile: 16 FLOP per byte taken in by the CU, three times k_gemm's 16 x 32 tile,
// whose waves each load their own fragments (5.3 FLOP/B: the CU's intake, not the MFMA pipe, bounded it).
// Why two K groups: a tile is 204 of the ~256 workgroups of a typical wavefront step (1,031 rows x N = 768), so one
// workgroup per CU; with four waves (one per SIMD) a wave's per-k-block overhead (the barrier, the DMA issue, the LDS
// reads) cannot overlap its own MFMAs (in-order issue) -- measured 158-167 ms per batch against k_gemm's 94.  Two
// groups put two waves on each SIMD and halve the serial k walk of a tile.
// Arithmetic: each wave walks its group's K slices in k order; slice s's chain runs in `acc`
// (v_mfma_f32_16x16x4_f32 on the same fragments, in the same order, as every other GEMM kernel).  Group 0 folds its
// slices as it goes (F = p0, F += p1, p2, p3); group 1 keeps p4..p7; at the end F crosses to group 1 through LDS, which
// folds ((((F + p4) + p5) + p6) + p7) -- the slice-ordered left fold the other kernels do through LDS (an empty slice
// adds +0 there and here).  Results are therefore bit-identical to k_gemm / k_gemm_s / k_dec_team / k_dec_one.
// Pipeline, per group: a ring of R one-k-block stages (8 fragments, 8 KB); every wave DMAs its row subtile's A fragment
// and its column subtile's W fragment of each k-block (incremental source addresses; the A segment is looked up only
// where one ends); per k-block: wait for its own DMAs (counted vmcnt), one s_barrier (everyone's landed, everyone done
// reading the slot the next DMA overwrites), issue the k-block R - 1 ahead, read and multiply.  LDS reads are inline
// asm: the compiler would otherwise drain every LDS-DMA in flight (vmcnt(0)) before any LDS read it can see.
constexpr int TG_FRAG = 64;         // f4 per fragment (1 KB)
constexpr int TG_R_DEFAULT = 4;     // k-block stages per group ring (R - 1 in flight): 2 x 32 KB of LDS
constexpr int TG_MIN_N = 256;       // narrower GEMMs (N = 96 / 192: 2-3 column tiles, too few workgroups) stay on k_gemm

__device__ __forceinline__ unsigned lds_addr(const void* p) {
    return (unsigned)(size_t)(const __attribute__((address_space(3))) void*)p;
}

// s_waitcnt vmcnt(2 n) for a wave-uniform n in [0, R - 2]: all but this wave's n youngest k-blocks landed
template <int TG_R>
__device__ __forceinline__ void tg_vmwait(int n) {
    static_assert(TG_R - 2 <= 6, "vmcnt range");
    switch (n) {
#define LBIC_W(s)                                                                                          \
    case s:                                                                                                \
        if constexpr (s <= TG_R - 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * s) : "memory");          \
        break;
        LBIC_W(1) LBIC_W(2) LBIC_W(3) LBIC_W(4) LBIC_W(5) LBIC_W(6)
#undef LBIC_W
        default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    }
}

template <bool SQ, int TG_R>
__global__ __launch_bounds__(512) void k_gemm_t(const GemmArgs g) {
    extern __shared__ __attribute__((aligned(16))) f4 tl[];   // [2 groups][TG_R][8 fragments: A 0-3, W 4-7][64]
    warm_kernargs<10>();
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int grp = wave >> 2, wq = wave & 3;
    const int wm = wq >> 1, wn = wq & 1;
    const int n0 = blockIdx.x * 64, m0 = blockIdx.y * 64;
    stamp_start(g.ts);
    const int4* bl = g.ctr ? g.blocks + (long)(*g.ctr) * g.ctr_stride : g.blocks;
    const BlkSrc blocks{bl, 0, 0, 0, 0};
    // this lane's DMA sources: A row m0 + 16 wq + lane % 16 (clamped), W column tile n0 / 16 + wq (clamped)
    SRow rw;
    {
        const SBlk bk = small_blk<false>(g, m0 + 16 * wq, lane, blocks);
        small_offsets(g, bk, lane, rw);
    }
    const int nkb = g.K >> 4;
    const int kmid = 4 * nkb / KSPLIT;                         // group 0: k-blocks [0, kmid), group 1: [kmid, nkb)
    const int kbA = grp ? kmid : 0, len = grp ? nkb - kmid : kmid;
    const int L = max(kmid, nkb - kmid);                       // both groups meet at every barrier
    const long wstep = (long)g.NB16 * TG_FRAG;
    const f4* wp = reinterpret_cast<const f4*>(g.W) + (long)min((n0 >> 4) + wq, g.NB16 - 1) * TG_FRAG + lane +
                   (long)kbA * wstep;
    const f4* ap = nullptr;
    int seg_end = -1;      // the first k-block past ap's segment (the A source is re-resolved there)
    f4* ring = tl + grp * TG_R * 8 * TG_FRAG;
    typedef __attribute__((address_space(3))) void* lds_vp;
    auto issue = [&](int j) {         // k-block kbA + j into slot j % R (j ascending, one call per j)
        const int kb = kbA + j;
        if (kb >= seg_end) {
            ap = small_a_ptr(rw, kb);
            int e = nkb;
#pragma unroll
            for (int t = 1; t < MAXSEG; ++t) {
                const int b = rw.k0[t] >> 4;
                e = (b > kb && b < e) ? b : e;
            }
            seg_end = e;
        }
        f4* d = ring + (j % TG_R) * 8 * TG_FRAG;
        __builtin_amdgcn_global_load_lds((const void*)ap, (lds_vp)(d + wq * TG_FRAG), 16, 0, 0);
        __builtin_amdgcn_global_load_lds((const void*)wp, (lds_vp)(d + (4 + wq) * TG_FRAG), 16, 0, 0);
        ap += 4;
        wp += wstep;
    };
    const int pro = min(TG_R - 1, len);
    for (int j = 0; j < pro; ++j) issue(j);

    const unsigned lb = lds_addr(ring) + (unsigned)lane * 16;
    const unsigned oa0 = (unsigned)(2 * wm) * 1024, oa1 = oa0 + 1024;
    const unsigned ow0 = (unsigned)(4 + 2 * wn) * 1024, ow1 = ow0 + 1024;
    // part[0]: group 0's running fold F; group 1: p4..p6 in part[0..2], p7 stays in acc
    f4 part[3][2][2], acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
            acc[i][jj] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int q = 0; q < 3; ++q) part[q][i][jj] = f4{0.f, 0.f, 0.f, 0.f};
        }
    int s = grp * 4;                       // the slice acc is accumulating
    const int s_end = s + 4;
    // close every slice of this group that ends at or before k-block `done`
    auto close = [&](int done) {
        while (s < s_end - grp && (s + 1) * nkb / KSPLIT <= done) {     // (group 1: slice 7 stays in acc)
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int jj = 0; jj < 2; ++jj) {
                    if (grp == 0) {
                        part[0][i][jj] = s == 0 ? acc[i][jj] : part[0][i][jj] + acc[i][jj];
                    } else {
#pragma unroll
                        for (int q = 0; q < 3; ++q)
                            if (s - 4 == q) part[q][i][jj] = acc[i][jj];
                    }
                    acc[i][jj] = f4{0.f, 0.f, 0.f, 0.f};
                }
            ++s;
        }
    };
    close(kbA);
    for (int j = 0; j < L; ++j) {
        tg_vmwait<TG_R>(j < len ? min(len - 1 - j, TG_R - 2) : 0);
        __builtin_amdgcn_s_barrier();
        if (j + TG_R - 1 < len) issue(j + TG_R - 1);
        if (j < len) {
            const unsigned fb = lb + (unsigned)((j % TG_R) * 8 * 1024);
            f4 a0, a1, w0, w1;
            asm volatile(
                "ds_read_b128 %0, %4\n\t"
                "ds_read_b128 %1, %5\n\t"
                "ds_read_b128 %2, %6\n\t"
                "ds_read_b128 %3, %7\n\t"
                "s_waitcnt lgkmcnt(0)"
                : "=&v"(a0), "=&v"(a1), "=&v"(w0), "=&v"(w1)
                : "v"(fb + oa0), "v"(fb + oa1), "v"(fb + ow0), "v"(fb + ow1)
                : "memory");
            if constexpr (SQ) {
                a0 = a0 * a0;
                a1 = a1 * a1;
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[e], w0[e], acc[0][0], 0, 0, 0);
                acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[e], w1[e], acc[0][1], 0, 0, 0);
                acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[e], w0[e], acc[1][0], 0, 0, 0);
                acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[e], w1[e], acc[1][1], 0, 0, 0);
            }
            close(kbA + j + 1);
        }
    }
    close(nkb);
    // F (group 0) -> group 1 through LDS (the rings are free once every wave passed the first barrier below); group 1
    // folds in slice order and leaves the sums there; then all eight waves run the epilogue, eight elements a thread
    float* xf = reinterpret_cast<float*>(tl);
    __builtin_amdgcn_s_barrier();
    const int xo = wq * 1024 + lane;       // element (i, jj, r) of this lane's quarter at xo + ((i 2 + jj) 4 + r) 64
    if (grp == 0) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int jj = 0; jj < 2; ++jj)
#pragma unroll
                for (int r = 0; r < 4; ++r) xf[xo + ((i * 2 + jj) * 4 + r) * 64] = part[0][i][jj][r];
    }
    __syncthreads();
    if (grp == 1) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int jj = 0; jj < 2; ++jj)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    float v = xf[xo + ((i * 2 + jj) * 4 + r) * 64];
#pragma unroll
                    for (int q = 0; q < 3; ++q) v += part[q][i][jj][r];
                    xf[xo + ((i * 2 + jj) * 4 + r) * 64] = v + acc[i][jj][r];
                }
    }
    __syncthreads();
    const bool gdn = g.epi == EPI_GDN || g.epi == EPI_IGDN;
    for (int e = threadIdx.x; e < 4096; e += 512) {
        const int l = e & 63, q = e >> 6;
        const int r = q & 3, i = (q >> 3) & 1, jj = (q >> 2) & 1, qw = q >> 4;
        const int row = m0 + 32 * (qw >> 1) + 16 * i + (l >> 4) * 4 + r;
        const int col = n0 + 32 * (qw & 1) + 16 * jj + (l & 15);
        if (row >= g.M || col >= g.N) continue;
        epilogue(g, xf[e], row, col, blocks, g.bias[col], gdn ? g.gx[(long)row * g.ldx + col] : 0.f);
    }
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
    return (g.M <= SMALL_MAX || (g.raster && g.M <= DEC_SMALL_MAX)) ? 0 : 1;
}
// the encoder's wavefront GEMM kernel: k_gemm_t with a ring of R k-block stages (default), or k_gemm (0)
static int enc_tiled() {
    static const int tiled = [] {
        const char* e = getenv("LBIC_ENC_TILED");     // A/B switch: 0 = k_gemm; 4, 5, 6: k_gemm_t's ring depth
        const int r = e ? atoi(e) : 0;   // (k_gemm_t is opt-in until it measures faster)
        return r == 0 || r == 4 || r == 5 || r == 6 ? r : TG_R_DEFAULT;
    }();
    return tiled;
}
const char* encoder_gemm_name() { return enc_tiled() ? "k_gemm_t" : "k_gemm"; }

template <int BM, int BN, int NW, int CH, int OCC = 1>
static int launch_cfg(const GemmArgs& g, hipStream_t s) {
    const size_t lds = std::max<size_t>((size_t)KSPLIT * BM * BN * sizeof(float), (size_t)std::max(g.lds_floor, 0));
    if (lds > 160 * 1024) return set_error(LBC_E_ARG, "LDS request above 160 KB");
    static const bool attr = [] {     // once per instantiation (thread-safe static initialisation)
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_gemm<BM, BN, NW, CH, OCC>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        return true;
    }();
    (void)attr;
    dim3 grid((g.N + BN - 1) / BN, (g.M + BM - 1) / BM);
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
    const int tiled = enc_tiled();
    if (tiled && g.N >= TG_MIN_N) {
        static const bool attr = [] {
            for (const void* f : {reinterpret_cast<const void*>(&k_gemm_t<false, 4>), reinterpret_cast<const void*>(&k_gemm_t<true, 4>),
                                  reinterpret_cast<const void*>(&k_gemm_t<false, 5>), reinterpret_cast<const void*>(&k_gemm_t<true, 5>),
                                  reinterpret_cast<const void*>(&k_gemm_t<false, 6>), reinterpret_cast<const void*>(&k_gemm_t<true, 6>)})
                (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
            return true;
        }();
        (void)attr;
        const size_t lds = std::max<size_t>((size_t)2 * tiled * 8 * TG_FRAG * 16, (size_t)std::max(g.lds_floor, 0));
        if (lds > 160 * 1024) return set_error(LBC_E_ARG, "LDS request above 160 KB");
        dim3 grid((g.N + 63) / 64, (g.M + 63) / 64);
#define LBIC_T(R)                                                                                  \
    case R:                                                                                        \
        if (g.square_a) hipLaunchKernelGGL((k_gemm_t<true, R>), grid, dim3(512), lds, s, g);       \
        else hipLaunchKernelGGL((k_gemm_t<false, R>), grid, dim3(512), lds, s, g);                 \
        break;
        switch (tiled) { LBIC_T(5) LBIC_T(6) default: LBIC_T(4) }
#undef LBIC_T
        return launch_status("k_gemm_t");
    }
    // Encoder wavefront steps (n_img images x up to 48 blocks): many small tiles beat few large ones; the per-tile K
    // loop is latency-bound, so the step wants workgroups and waves.  Measured encode time per 32-frame 768x768
    // batch, encoder alone (tools/enc_exp.py, profiles/r02_exp/encoder_occupancy.txt), every shape bit-identical:
    // 16x32 / 8 waves / one k-block per chunk (56 VGPRs: 8 waves per SIMD) 98.7 ms; 16x32 / 4 waves / 2-block
    // chunks 108.2 (round 2's earlier default, 86 VGPRs: 5 waves per SIMD, 2 beside the team decoder's 256 VGPRs);
    // 16x32 / 4 / 1 capped at 70 VGPRs 105.7; 32x32 / 8 / 1 107.5; 16x64 / 8 / 1 112.0; 16x16 / 4 / 1 122.3;
    // register caps that spill (64 / 80 VGPRs) 116.7 / 115.8.  Beside the team decoder (bench.py --steps 20):
    // 84.9 Mpix/s against 79.7 for the earlier default.  (Other tiles, XCD-aware and 2-D XCD tile orders: measured
    // in rounds 2-3 and removed)
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
