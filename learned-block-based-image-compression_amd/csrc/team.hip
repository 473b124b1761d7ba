// Team decoder (gfx950): lbc_decode_team's persistent raster decode of several batches in one launch.
#include "kernels_dev.h"

namespace lbic {

constexpr int RC_WORDS = 576;   // rans_row_sparse's persistent coder-state cache (see kernels_dev.h)
constexpr int CTL_WORDS = 32;   // LDS control words (word 18: the barrier verdict team_sync broadcasts)

// ----------------------------------------------------------------------------------------- team decoder
// k_dec_team: the reference-format raster decodes of T <= 8 batches in ONE persistent launch.  Team t = the S
// workgroups with blockIdx % 8 == t decodes batch t (a team's workgroups share one XCD under the observed round-robin
// placement: speed, and plain hand-off stores once the census below has confirmed it; nothing else depends on it).  A team runs its batch's raster steps with
// the operations the graph decoder launches -- context net x 4, rANS, decoder x 7, recorded by the host as
// prepared GemmArgs / RansArgs -- and a team barrier between operations instead of a kernel boundary: a raster
// step of 12 dependent launches pays 12 barriers (one agent-scope arrival per workgroup, one polling lane) in
// place of 12 launch boundaries, and T chains run side by side in one launch instead of one per hardware queue
// (at most four overlap: DESIGN.md §5).
// Hand-offs follow cdna_hip_programming.md §6 Guideline 16, R1: every value a workgroup writes for the others
// (activations, scale indexes, y_qnt, the reconstruction and the layer-0 cache) is stored sc1 (write-through),
// every storing wave drains (vmcnt(0)) before its workgroup's single arrival, and every load of such a value is an
// sc1 load (buffer_load ... sc1 for the GEMM A operand, global sc1 loads for the GDN inputs and the rANS inputs);
// weights, biases and the tables are read-only.  Every spin is bounded (TeamArgs::tmo): a workgroup that gives up
// sets the failure word, which every other waiter reads, so the whole grid drains and the host reports an error.
// GEMM arithmetic per output element is k_gemm_s's (KSPLIT slices, the same MFMA chains, the slice-ordered sum,
// the shared epilogue): results are bit-identical to the graph decoder's.

// A fragment of k-block kb through an sc1 (L1-bypassing) buffer load; byte offsets < 4 GB (host-checked)
__device__ __forceinline__ f4 small_a_sc1(const SRow& rw, int kb) {
    const int k = kb << 4;
    gfloat_p base = rw.base[0];
    unsigned o = rw.off[0];
#pragma unroll
    for (int t = 1; t < MAXSEG; ++t) {
        const bool in = k >= rw.k0[t];
        base = in ? rw.base[t] : base;
        o = in ? rw.off[t] : o;
    }
    const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, -1, 0x00020000);
    return __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs, (o + (unsigned)(k >> 2)) << 4, 0, 16));
}

// the workgroup's barrier between the partial stores to LDS and the reduction
__device__ __forceinline__ void wg_bar() {
    __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0)
    __builtin_amdgcn_s_barrier();
}

// K beyond the fast path (or more than two row tiles): each output tile (row tile mt, column tile nt) = item
// i = nt * MT + mt, items rank, rank + S, ...; each item's slice in chunks of CH k-blocks, double-buffered: chunk c + 1's
// fragments are requested before chunk c's MFMAs (the KS3311 context layer 1, K = 5 C1, streams 8-67 k-blocks per slice)
__device__ __forceinline__ void team_gemm_long(const GemmArgs& g, int v, int h, int rank, int S, int nt0, int ntn, float* red,
                                               bool wt) {
    constexpr int CH = 4;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nkb = g.K >> 4;
    const int kb0 = wave * nkb / KSPLIT, kb1 = (wave + 1) * nkb / KSPLIT;
    const int MT = (g.M + 15) >> 4, items = MT * ntn;
    const BlkSrc blocks{nullptr, 1, 0, v, h};
    const bool gdn = g.epi == EPI_GDN || g.epi == EPI_IGDN;
    const f4* Wt = reinterpret_cast<const f4*>(g.W) + lane;
    const int el = threadIdx.x & 63, er = (threadIdx.x >> 6) & 3;
    int buf = 0;
    for (int it = rank; it < items; it += S) {
        const int mt = it % MT, nt = nt0 + it / MT;
        const int erow = min(mt * 16 + (el >> 4) * 4 + er, g.M - 1), ecol = min(nt * 16 + (el & 15), g.N - 1);
        const float bb = g.bias[ecol];
        const float xx = gdn ? ld<true>(g.gx + (long)erow * g.ldx + ecol) : 0.f;
        const SBlk bk = small_blk<true>(g, mt * 16, lane, blocks);
        SRow rw;
        small_offsets(g, bk, lane, rw);
        f4 acc = f4{0.f, 0.f, 0.f, 0.f};
        f4 a0[CH], w0[CH], a1[CH], w1[CH];
        // clamped, unconditional loads (a block past the slice re-reads a valid one; its MFMAs are discarded below)
        auto load = [&](int c0, f4 (&a)[CH], f4 (&w)[CH]) {
#pragma unroll
            for (int c = 0; c < CH; ++c) {
                const int kb = min(c0 + c, nkb - 1);
                w[c] = Wt[((long)kb * g.NB16 + nt) * 64];
                a[c] = small_a_sc1(rw, kb);
            }
        };
        auto mma = [&](int c0, f4 (&a)[CH], f4 (&w)[CH]) {
            __builtin_amdgcn_sched_barrier(0);   // the next chunk's requests stay above this chunk's MFMAs
#pragma unroll
            for (int c = 0; c < CH; ++c) {
                f4 av = a[c];
                if (g.square_a) av = av * av;
                f4 t = acc;
#pragma unroll
                for (int e = 0; e < 4; ++e) t = __builtin_amdgcn_mfma_f32_16x16x4f32(av[e], w[c][e], t, 0, 0, 0);
                acc = c0 + c < kb1 ? t : acc;
            }
        };
        int c0 = kb0;
        load(c0, a0, w0);
        for (;;) {
            load(c0 + CH, a1, w1);
            mma(c0, a0, w0);
            c0 += CH;
            if (c0 >= kb1) break;
            load(c0 + CH, a0, w0);
            mma(c0, a1, w1);
            c0 += CH;
            if (c0 >= kb1) break;
        }
        float* rb = red + buf * (KSPLIT * 256);
        buf ^= 1;
#pragma unroll
        for (int i = 0; i < 4; ++i) rb[wave * 256 + i * 64 + lane] = acc[i];
        wg_bar();
        if (threadIdx.x < 256) {
            const int e = threadIdx.x;
            float vv = rb[e];
#pragma unroll
            for (int i = 1; i < KSPLIT; ++i) vv += rb[i * 256 + e];
            const int row = mt * 16 + (el >> 4) * 4 + er, col = nt * 16 + (el & 15);
            if (row < g.M && col < g.N) epilogue<true, true>(g, vv, row, col, blocks, bb, xx, wt);
        }
    }
}

// The common case: ni <= TEAM_NI_MAX output tiles per workgroup (item i = nt * MT + mt; items rank, rank + S, ...;
// with S % MT == 0 every item of a workgroup has the same row tile, so its A rows are loaded once).  Item j + 1's
// weight fragments are requested before item j's chain (two register buffers; one where a slice holds more than 7
// k-blocks, to stay within 128 VGPRs), unconditionally (the last request repeats the last item) so that no load sits
// behind a branch (the compiler's wait after such a join counts conservatively and serialises the prefetch); the
// chains run back to back, and their partials meet in LDS behind ONE workgroup barrier; then every thread sums and
// finishes its output elements.
// ph: 0 the whole GEMM; 1 (beside the rANS decode) only the waves w < wy, whose K slices read no y_qnt, compute
// their chains and leave the partials in LDS; 2 the remaining waves, then the reduction.
// dts (sampled raster step, team rank 0; LBIC_TEAM_DIAG builds): wave 0's s_memtime at entry, loads issued, first
// chain done, all chains done, outputs written.
__device__ __forceinline__ void dstamp(unsigned long long* dts, int p, float dep, bool every_wave = false) {
#ifndef LBIC_TEAM_DIAG
    (void)dts; (void)p; (void)dep; (void)every_wave;   // diagnostic build only (make team_diag)
#else
    if (dts && (every_wave ? (threadIdx.x & 63) == 0 : threadIdx.x == 0)) {
        unsigned long long t;
        float d;       // the v_mov reads `dep` (an MFMA result): the stamp follows its chain
        asm volatile("v_mov_b32 %1, %2\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t), "=v"(d) : "v"(dep) : "memory");
        dts[p] = t;
    }
#endif
}

// Buffer resource of a read-only or hand-off operand: 32-bit byte offsets (host-checked: < 4 GB)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t team_rsrc(const void* base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, -1, 0x00020000);
}

// ONESEG: A is one segment (every decoder GEMM but the two whose K spans the z-taps): its k-blocks are plain offsets
// from one per-lane row address (a scalar offset per k-block), no per-k-block segment selection.  The prologue of an
// operation -- epilogue operands, weight and A addressing -- is kept to scalar arithmetic and a few vector
// instructions: it is issue-bound (the two waves of a SIMD run it one after the other before their chains start), so
// every instruction there delays the slower wave of each SIMD and, through the workgroup barrier, the whole operation.
template <int L, bool EXACT, bool ONESEG>
__device__ __forceinline__ void team_gemm_items(const GemmArgs& g, int v, int h, int rank, int S, int nt0, int ni,
                                                float* red, bool wt, int ph, int wy, unsigned long long* dts,
                                                const int4& tq) {
    constexpr int NPRE = 3;                      // output elements per thread (ni * 256 over 512 threads) whose epilogue
                                                 // operands are requested before the chains: every one up to 6 tiles
    constexpr int LL = EXACT ? L : L + 1;
    constexpr bool PF = LL <= 7;                 // prefetch the next item's fragments (128-VGPR budget)
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nkb = g.K >> 4;
    const int kb0 = wave * nkb / KSPLIT, n = (wave + 1) * nkb / KSPLIT - kb0;
    const int MT = (g.M + 15) >> 4;
    // (S % MT == 0 on the fast path) item j of this workgroup: row tile mt, column tile ntb + j nts; the quotients
    // precomputed once per launch for the step's usual row-tile count (tq: {MT, rank / MT, rank % MT, S / MT})
    const bool pre = MT == tq.x;
    const int mt = pre ? tq.z : (int)((unsigned)rank % (unsigned)MT);
    const int ntb = nt0 + (pre ? tq.y : (int)((unsigned)rank / (unsigned)MT));
    const int nts = pre ? tq.w : (int)((unsigned)S / (unsigned)MT);
    const BlkSrc blocks{nullptr, 1, 0, v, h};
    const bool gdn = g.epi == EPI_GDN || g.epi == EPI_IGDN;
    const bool act = ph == 0 || (ph == 1 ? wave < wy : wave >= wy);
    const int nout = ni * 256;
    // this thread's output elements o = threadIdx.x + 512 q: item j = (threadIdx.x >> 8) + 2 q, one row for all q
    const int ol = threadIdx.x & 63, orr = (threadIdx.x >> 6) & 3, jt = threadIdx.x >> 8;
    const int erow = min(mt * 16 + (ol >> 4) * 4 + orr, g.M - 1);
    // the GDN input row (other layers: the bias row again, read and not used): branch-free operand loads
    const float* xr = gdn ? g.gx + (long)erow * g.ldx : g.bias;
    auto operands = [&](int q0, float (&b)[NPRE], float (&x)[NPRE]) {
#pragma unroll
        for (int q = 0; q < NPRE; ++q) {
            const int j = min(jt + 2 * (q0 + q), ni - 1);     // clamped: every thread loads NPRE
            const int ecol = min((ntb + j * nts) * 16 + (ol & 15), g.N - 1);
            b[q] = g.bias[ecol];
            x[q] = ld<true>(xr + ecol);
        }
    };
    f4 a[LL], w0[LL], w1[LL];
    dstamp(dts, 0, 0.f);
    float bb[NPRE], xx[NPRE];
    if (ph != 1) operands(0, bb, xx);
    dstamp(dts, 5, 0.f);
    if (act) {      // loads and chains in one branch: no join between a load and its use
        // weights: one buffer resource, this lane's 16 bytes of a fragment at lane * 16, the fragment's start in the
        // scalar offset ((k-block * NB16 + column tile) KB)
        const __amdgpu_buffer_rsrc_t wr = team_rsrc(g.W);
        const unsigned lo16 = (unsigned)lane << 4;
        auto issue = [&](int j, f4 (&w)[LL]) {
            const int nt = ntb + j * nts;
#pragma unroll
            for (int c = 0; c < LL; ++c)
                w[c] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(
                                                  wr, lo16, (unsigned)(min(kb0 + c, nkb - 1) * g.NB16 + nt) << 10, 0));
        };
        auto chain = [&](int j, f4 (&w)[LL]) {
            __builtin_amdgcn_sched_barrier(0);   // the requests above this item's chain
            f4 acc = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int c = 0; c < LL; ++c) {
                const f4 av = a[c];
                f4 t = acc;
#pragma unroll
                for (int e = 0; e < 4; ++e) t = __builtin_amdgcn_mfma_f32_16x16x4f32(av[e], w[c][e], t, 0, 0, 0);
                // (a select on every k-block, not only the (L+1)-th: the chain with a VALU select and its wait states
                // between k-blocks runs faster than a back-to-back dependent MFMA chain -- measured, r06 call 5)
                acc = c < n ? t : acc;
            }
            // partials -> LDS [item][slice][256]
#pragma unroll
            for (int i = 0; i < 4; ++i) red[(j * KSPLIT + wave) * 256 + i * 64 + lane] = acc[i];
            if (j == 0) dstamp(dts, 2, acc[0]);
            if (j == ni - 1) dstamp(dts, 3, acc[0]);
            if (j == 0) dstamp(dts, 24 + wave, acc[0], true);
            if (j == ni - 1) dstamp(dts, 16 + wave, acc[0], true);
        };
        issue(0, w0);
        dstamp(dts, 6, 0.f);
        {
            const SBlk bk = small_blk<true>(g, mt * 16, lane, blocks);
            if constexpr (ONESEG) {
                // this lane's row of the single segment; k-block kb at + kb * 64 bytes (scalar offset)
                const Seg& sg = g.seg[0];
                const long cell = ((long)bk.b.x * g.geo.Hp + bk.b.y + 2 + bk.dy) * g.geo.Wp + bk.b.z + 2 + bk.dx;
                const unsigned ro = (unsigned)(((long)bk.r * sg.ld + sg.zs * cell + sg.tap + ((lane >> 4) << 2)) << 2);
                const __amdgpu_buffer_rsrc_t ar = team_rsrc(sg.base);
                dstamp(dts, 7, 0.f);
#pragma unroll
                for (int c = 0; c < LL; ++c)
                    a[c] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(
                                                      ar, ro, (unsigned)min(kb0 + c, nkb - 1) << 6, 16));
            } else {
                SRow rw;
                small_offsets(g, bk, lane, rw);
                dstamp(dts, 7, 0.f);
#pragma unroll
                for (int c = 0; c < LL; ++c) a[c] = small_a_sc1(rw, min(kb0 + c, nkb - 1));
            }
        }
        dstamp(dts, 1, 0.f);
        dstamp(dts, 32 + wave, 0.f, true);
        dstamp(dts, 40 + wave, a[0][0], true);     // (waits for the first A fragment)
        // GDN (g.square_a): A squared once, in place, for every item (the same f32 products the chains used to form per
        // item; a runtime choice, so one instance per slice length serves GDN and plain GEMMs -- fewer instances, less
        // code for a raster step to fetch).  The next item's fragments are requested first, unconditionally (the last
        // request repeats the last item: an L2 hit) so that no load sits behind a branch
        auto square = [&]() {
            if (g.square_a) {
#pragma unroll
                for (int c = 0; c < LL; ++c) a[c] = a[c] * a[c];
            }
        };
        if constexpr (PF) {
            issue(min(1, ni - 1), w1);
            square();
            for (int j = 0;;) {
                chain(j, w0);
                if (++j >= ni) break;
                issue(min(j + 1, ni - 1), w0);
                chain(j, w1);
                if (++j >= ni) break;
                issue(min(j + 1, ni - 1), w1);
            }
        } else {
            square();
            for (int j = 0;;) {
                chain(j, w0);
                if (++j >= ni) break;
                issue(j, w0);
            }
        }
    }
    if (ph == 1) return;
    // the second round's epilogue operands (more than six tiles per workgroup) requested before the workgroup barrier:
    // their latency hides behind the wait for the other waves' chains
    static_assert(TEAM_NI_MAX * 256 <= 2 * NPRE * 512, "at most two epilogue rounds");
    float bb1[NPRE], xx1[NPRE];
    if ((int)threadIdx.x + 512 * NPRE < nout) operands(NPRE, bb1, xx1);
    wg_bar();
    dstamp(dts, 8, 0.f);
    // output o = threadIdx.x + 512 (NPRE r + q), round r: item j = o >> 8; its K slices' partials summed in slice order,
    // then the epilogue.  Round 0's operands came before the chains, round 1's before the barrier.  Both loops rolled:
    // one copy of the (decoder-only) epilogue serves every output of an instance
    const int row = mt * 16 + (ol >> 4) * 4 + orr;
#pragma unroll 1
    for (int r = 0; (int)threadIdx.x + 512 * NPRE * r < nout; ++r) {
        if (r > 0) {
#pragma unroll
            for (int q = 0; q < NPRE; ++q) {
                bb[q] = bb1[q];
                xx[q] = xx1[q];
            }
        }
#pragma unroll 1
        for (int q = 0; q < NPRE; ++q) {      // rolled: one copy of the epilogue per instance
            const int o = threadIdx.x + 512 * (NPRE * r + q);
            if (o >= nout) break;
            const int j = o >> 8, ee = o & 255;
            float vv = red[j * KSPLIT * 256 + ee];
#pragma unroll
            for (int i = 1; i < KSPLIT; ++i) vv += red[(j * KSPLIT + i) * 256 + ee];
            const int col = (ntb + j * nts) * 16 + (ol & 15);
            const float b_ = q == 0 ? bb[0] : q == 1 ? bb[1] : bb[2];
            const float x_ = q == 0 ? xx[0] : q == 1 ? xx[1] : xx[2];
            if (row < g.M && col < g.N) epilogue<true, true>(g, vv, row, col, blocks, b_, x_, wt);
        }
        if (r == 0) dstamp(dts, 9, 0.f);
    }
    dstamp(dts, 4, 0.f);
}

// The output tiles of g this workgroup computes: rank `rank` of the team's S workgroups
__device__ __forceinline__ void team_gemm_any(const GemmArgs& g, int v, int h, int rank, int S, float* red, bool wt,
                                              int ph, int wy, unsigned long long* dts, const int4& tq) {
    const int nt0 = 0, ntn = (g.N + 15) >> 4;
    const int nkb = g.K >> 4;
    const int L = nkb / KSPLIT;
    const bool exact = (nkb % KSPLIT) == 0;
    const int MT = (g.M + 15) >> 4, items = MT * ntn;
    const int ni = rank < items ? (items - rank + S - 1) / S : 0;
    if (ni == 0) return;
    if (team_fast_path(g, S)) {
        switch (L * 2 + (exact ? 1 : 0)) {
#define LBIC_N(L_)                                                                                            \
    case L_ * 2 + 1:                                                                                          \
        if (g.nseg == 1) team_gemm_items<L_, true, true>(g, v, h, rank, S, nt0, ni, red, wt, ph, wy, dts, tq);   \
        else team_gemm_items<L_, true, false>(g, v, h, rank, S, nt0, ni, red, wt, ph, wy, dts, tq);              \
        return;                                                                                               \
    case L_ * 2:                                                                                              \
        if (g.nseg == 1) team_gemm_items<L_, false, true>(g, v, h, rank, S, nt0, ni, red, wt, ph, wy, dts, tq);  \
        else team_gemm_items<L_, false, false>(g, v, h, rank, S, nt0, ni, red, wt, ph, wy, dts, tq);             \
        return;
            LBIC_N(1) LBIC_N(2) LBIC_N(3) LBIC_N(4) LBIC_N(5) LBIC_N(6) LBIC_N(7) LBIC_N(8) LBIC_N(9)
#undef LBIC_N
            default: break;
        }
    }
    if (ph == 1) return;     // (the host splits a GEMM only where every workgroup takes the path above)
    team_gemm_long(g, v, h, rank, S, nt0, ntn, red, wt);
}

// the rANS decode of one wave of the team kernel: rows r0, r0 + nrw S, ... of the team's batch, in LDS area I (per
// wave: [window RANS_WIN words][coder-state cache RC_WORDS words][centre intervals 256 words], from the LDS base).
// Not inlined: the coder gets a register allocation of its own (inlined beside the GEMM instances, the sparse
// kernel spilled 25-30 VGPRs to scratch, reloaded in every GEMM epilogue).  A call's arguments travel in VGPRs: each
// is made uniform again (readfirstlane) so the recorded RansArgs come in by scalar loads from the constant address
// space; the LDS is the kernel's dynamic array, declared here again (LDS instructions, not flat ones).
constexpr int TEAM_RW = RANS_WIN + RC_WORDS + 256;
typedef const __attribute__((address_space(4))) RansArgs* crans_p;
template <bool DENSE, int I>
__device__ __attribute__((noinline)) void team_rans(unsigned long long rp, int r0, int S, int nrw, int wt, int tab_off) {
    extern __shared__ __attribute__((aligned(16))) uint32_t team_lds[];
    const unsigned rlo = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)rp);
    const unsigned rhi = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(rp >> 32));
    const RansArgs& R = *(const RansArgs*)(crans_p)(((unsigned long long)rhi << 32) | rlo);
    r0 = __builtin_amdgcn_readfirstlane(r0);
    S = __builtin_amdgcn_readfirstlane(S);
    nrw = __builtin_amdgcn_readfirstlane(nrw);
    const bool w = __builtin_amdgcn_readfirstlane(wt) != 0;
    const int lane = threadIdx.x & 63;
    uint32_t* lwin = team_lds + I * TEAM_RW;
    uint32_t* llf = lwin + RANS_WIN + RC_WORDS;
    if (!DENSE && r0 < R.rows && r0 + nrw * S >= R.rows) {
        // one image per wave, the same one at every step: the coder state stays in LDS
        rans_row_sparse<true, true>(R, lwin, r0, lane, w, nullptr, lwin + RANS_WIN, nullptr, nullptr, nullptr, nullptr,
                                    llf);
    } else {
        uint16_t* tab = reinterpret_cast<uint16_t*>(team_lds + __builtin_amdgcn_readfirstlane(tab_off));
        for (int r = r0; r < R.rows; r += nrw * S) {
            if constexpr (DENSE) rans_row<true>(R, tab, r, lane, lwin, w);
            else rans_row_sparse<true>(R, lwin, r, lane, w, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, llf);
        }
    }
}

// team barrier: every wave's stores drained, one arrival per workgroup, one lane polls (relaxed, s_sleep between
// polls, bounded); false: the launch failed (timeout here or anywhere else)
__device__ __forceinline__ bool team_sync(unsigned* ctr, unsigned target, unsigned* fail, unsigned long long tmo,
                                          int* sflag) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // EVERY storing wave (R1)
    __syncthreads();
    if (threadIdx.x == 0)
        __hip_atomic_fetch_add((gptr<unsigned>)ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (threadIdx.x == 0) {
        int f = 0;
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        // the failure word only every 16th poll: each poll is then one round trip to the team's L2, not two
        for (int it = 0; __hip_atomic_load((gptr<unsigned>)ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target; ++it) {
            if ((it & 15) == 15 && __hip_atomic_load((gptr<unsigned>)fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                f = 1;
                break;
            }
            if (__builtin_amdgcn_s_memrealtime() - t0 > tmo) {
                __hip_atomic_store((gptr<unsigned>)fail, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                f = 1;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        *sflag = f;
    }
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // no instruction: keeps the loads below the poll
    return *sflag == 0;
}

// ta.plain: the team's workgroups were checked (below) to share one XCD, so its L2 is the coherence point for every
// hand-off: values are stored plain (they stay in that L2) and still loaded sc1 (past the reading CU's L1).  If
// any team of the launch spans XCDs the launch stops before its first operation with failure word 2 and the host
// relaunches with plain = 0 (every hand-off write-through): results never depend on placement.
// 128 VGPRs at most (4 waves per SIMD): the encoder's kernels keep room beside the persistent launch.
// DENSE (TeamArgs::dense): the high-rate instance, tables staged in LDS and rans_row<true>; a separate instance so the
// low-rate one keeps its register allocation.
template <bool DENSE>
__global__ __launch_bounds__(512, 4) void k_dec_team(const TeamArgs ta) {
    // dynamic LDS, sized by the host (team_lds_bytes), per rANS wave i < nrw: [rANS window RANS_WIN words]
    // [rANS cache RC_WORDS words][rANS centre intervals 256 words]; then [control CTL_WORDS words]
    // [GEMM partials ni_max x KSPLIT x 256 floats][dense rANS only: the table image, total16 16-bit entries]
    extern __shared__ __attribute__((aligned(16))) uint32_t team_lds[];
    const int nrw = ta.nrw;
    uint32_t* ctl = team_lds + nrw * TEAM_RW;
    int& sflag = *reinterpret_cast<int*>(ctl + 18);
    float* red = reinterpret_cast<float*>(ctl + CTL_WORDS);
    if (threadIdx.x < 2 && (int)threadIdx.x < nrw)     // no cached coder state yet (ordered by the barriers below)
        team_lds[threadIdx.x * TEAM_RW + RANS_WIN + 4] = 0u;
    const int T = ta.T, S = ta.S;
    // grid = 8 x S (x sub): team t = the workgroups with blockIdx % 8 == t (t < T; one XCD each under round-robin
    // placement, whatever T is); the others leave at once
    // spread P = 2, 4, 8 (at most 8 / P teams): team t = the workgroups of slots P t .. P t + P - 1 (P XCDs), ranks
    // interleaved over them
    // sub = 2 (more than 8 teams): two teams per slot, team slot + 8 q = the slot's workgroups q S .. q S + S - 1
    const int slot = blockIdx.x & 7;
    const int kk = (int)(blockIdx.x >> 3);
    const int team = ta.sub > 1 ? slot + TEAM_SLOTS * (kk / S) : slot / ta.spread;
    const int rank = ta.sub > 1 ? kk % S : kk * ta.spread + slot % ta.spread;
    if (team >= T || rank >= S) return;
    unsigned* ctr = ta.sync + team * 32;
    unsigned* fail = ta.sync + T * 32;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint16_t* tab = reinterpret_cast<uint16_t*>(red + ta.ni_max * KSPLIT * 256);
    // the recorded operations are read-only for the launch: constant address space, so their fields come in by
    // scalar loads into SGPRs like kernel arguments (the scalar cache only reads)
    typedef const __attribute__((address_space(4))) GemmArgs* cgemm_p;
    const cgemm_p G = (cgemm_p)(ta.gemm) + (long)team * 3 * ta.NG;
    const RansArgs& R = *(const RansArgs*)((crans_p)(ta.rans) + team);
    unsigned long long* ts = ta.ts && rank == 0 ? ta.ts + team * TEAM_TS_WORDS : nullptr;
    unsigned long long* tsr = ta.ts ? ta.ts + team * TEAM_TS_WORDS : nullptr;   // every rank: [160 + rank] rANS done, [192 + rank]
                                                                       // the GEMM waves beside it done (sampled step)
    if (ts && threadIdx.x == 0) ts[62] = __builtin_amdgcn_s_memrealtime();
    if constexpr (DENSE) {     // the rANS tables, once per launch (read-only: no hand-off)
        const uint4* src = reinterpret_cast<const uint4*>(R.cdf16);
        uint4* dst = reinterpret_cast<uint4*>(tab);
        for (int i = threadIdx.x; i < R.total16 / 8; i += blockDim.x) dst[i] = src[i];
    }
    __syncthreads();
    unsigned target = 0;
    const bool wt = !ta.plain;
    // the quotients of this rank by the usual row-tile count (the batch's images: ceil(M / 16) of every GEMM but the
    // KS3311 context layer 0 at border columns), once per launch
    int4 tq;
    {
        const unsigned mt0 = (unsigned)((ta.rows0 + 15) >> 4);
        tq = make_int4((int)mt0, (int)((unsigned)rank / mt0), (int)((unsigned)rank % mt0), (int)((unsigned)S / mt0));
    }
    if (ta.plain) {
        // placement census: every workgroup ORs its XCD into its team's word [1], then a barrier over the whole
        // grid (counter [T * 32 + 1]); any team on more than one XCD -> every workgroup leaves
        if (threadIdx.x == 0)
            __hip_atomic_fetch_or((gptr<unsigned>)(ta.sync + team * 32 + 1), 1u << xcc_id(), __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);
        if (!team_sync(ta.sync + T * 32 + 1, (unsigned)(T * S), fail, ta.tmo, &sflag)) return;
        bool local = true;
        for (int t = 0; t < T; ++t)
            local &= __popc(__hip_atomic_load((gptr<unsigned>)(ta.sync + t * 32 + 1), __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT)) == 1;
        if (!local) {
            if (threadIdx.x == 0) __hip_atomic_store((gptr<unsigned>)fail, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return;
        }
    }
    for (int v = 0; v < ta.Hb; ++v) {
        for (int h = 0; h < ta.Wb; ++h) {
            const int cls = h == 0 ? 0 : h == ta.Wb - 1 ? 2 : 1;
            const bool samp = ts && v == ta.sv && h == ta.sh;
            for (int op = 0; op < ta.nops; ++op) {
                const int k = ta.opk[op];
                if (k >= 0) {
                    const GemmArgs& g = *(const GemmArgs*)(G + cls * ta.NG + k);
                    team_gemm_any(g, v, h, rank, S, red, wt, op == ta.split_op ? 2 : 0, ta.split_wy,
                                  samp ? ts + 256 + op * 64 : nullptr, tq);
                } else {
                    // the rANS decode on the last nrw waves (wave i: rows rank + i S, rank + (i + nrw) S, ...); beside
                    // it the first split_wy <= KSPLIT - nrw waves compute the K slices of the next GEMM (the decoder's
                    // first layer) that do not read y_qnt
                    const bool sstep = tsr && v == ta.sv && h == ta.sh && rank < 32;
                    const int rw0 = ta.split_op >= 0 ? KSPLIT - nrw : 0;
                    if (wave >= rw0 && wave < rw0 + nrw) {
                        // wave i's LDS area at a compile-time offset (two call sites): a runtime base costs registers
                        // in the coder's loop
                        const unsigned long long rp = (unsigned long long)((crans_p)(ta.rans) + team);
                        const int toff = (int)(reinterpret_cast<uint32_t*>(tab) - team_lds);
                        if (wave == rw0) team_rans<DENSE, 0>(rp, rank, S, nrw, wt ? 1 : 0, toff);
                        else team_rans<DENSE, 1>(rp, rank + S, S, nrw, wt ? 1 : 0, toff);
                        if (sstep && lane == 0 && wave == rw0) tsr[160 + rank] = __builtin_amdgcn_s_memrealtime();
                    } else if (ta.split_op >= 0) {
                        const GemmArgs& g = *(const GemmArgs*)(G + cls * ta.NG + ta.opk[ta.split_op]);
                        team_gemm_any(g, v, h, rank, S, red, wt, 1, ta.split_wy, nullptr, tq);
                        if (sstep && threadIdx.x == 0) tsr[192 + rank] = __builtin_amdgcn_s_memrealtime();
                    }
                }
                if (samp && threadIdx.x == 0) ts[32 + op] = __builtin_amdgcn_s_memrealtime();
                target += S;
                if (!team_sync(ctr, target, fail, ta.tmo, &sflag)) return;
                if (samp && threadIdx.x == 0) ts[op] = __builtin_amdgcn_s_memrealtime();
            }
            if (samp && threadIdx.x == 0) ts[61] = __builtin_amdgcn_s_memrealtime();
            if (ts && v == ta.sv && h == ta.sh - 1 && threadIdx.x == 0) ts[60] = __builtin_amdgcn_s_memrealtime();
        }
    }
    if (ts && threadIdx.x == 0) ts[63] = __builtin_amdgcn_s_memrealtime();
}

static const void* team_instance(int dense) {
    return dense ? reinterpret_cast<const void*>(&k_dec_team<true>) : reinterpret_cast<const void*>(&k_dec_team<false>);
}

int team_blocks_per_cu(int dense, size_t lds) {
    int nb = 0;
    const void* f = team_instance(dense);
    (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, f, 512, lds) != hipSuccess) return 0;
    return nb;
}

size_t team_lds_bytes(const TeamArgs& a) {
    return (size_t)((RANS_WIN + RC_WORDS + 256) * a.nrw + CTL_WORDS) * 4 + (size_t)a.ni_max * KSPLIT * 256 * 4 +
           (size_t)(a.dense ? 1 : 0) * a.tab16 * 2;
}

int launch_dec_team(const TeamArgs& a, hipStream_t s) {
    if (a.T < 1 || a.T > TEAM_MAX || a.S < 1 || a.nops < 1 || a.nops > TEAM_MAXOPS || !a.gemm || !a.rans || !a.sync)
        return set_error(LBC_E_ARG, "bad team decoder arguments");
    if (a.ni_max < 1 || a.ni_max > TEAM_NI_MAX) return set_error(LBC_E_ARG, "bad team decoder tile count");
    if (a.nrw < 1 || a.nrw > 2 || (a.split_op >= 0 && (a.split_wy < 1 || a.split_wy > KSPLIT - a.nrw)))
        return set_error(LBC_E_ARG, "bad team decoder rANS wave count");
    static const bool attr = [] {
        for (int d = 0; d < 2; ++d)
            (void)hipFuncSetAttribute(team_instance(d), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        return true;
    }();
    (void)attr;
    const size_t lds = team_lds_bytes(a);
    if (lds > 160 * 1024) return set_error(LBC_E_ARG, "team decoder: LDS image too large");
    if ((a.spread != 1 && a.spread != 2 && a.spread != 4 && a.spread != 8) ||
        (a.spread > 1 && (a.T > TEAM_SLOTS / a.spread || a.S % a.spread || a.plain)))
        return set_error(LBC_E_ARG, "bad team spread");
    if ((a.sub != 1 && a.sub != 2) || (a.sub == 2 && a.spread != 1) || a.T > TEAM_SLOTS * a.sub)
        return set_error(LBC_E_ARG, "bad team count per XCD slot");
    const dim3 grid(TEAM_SLOTS * a.S * a.sub / a.spread);
    if (a.dense) hipLaunchKernelGGL((k_dec_team<true>), grid, dim3(512), lds, s, a);
    else hipLaunchKernelGGL((k_dec_team<false>), grid, dim3(512), lds, s, a);
    return launch_status("k_dec_team");
}

}  // namespace lbic
