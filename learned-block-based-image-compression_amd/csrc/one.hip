// Single-image decoder (gfx950): the reference-format raster decode of ONE image (decompress, net:400-452; the batch-1
// path of eval_model, agents/blkbsdimgcomp_agent.py:591-599) as one persistent launch over every CU.
//
// Why a kernel of its own: at batch 1 a raster step is a chain of 12 dependent operations on ONE row; the graph decoder
// pays a launch boundary per operation and streams every weight tile from the Infinity Cache every step (25.6 MB per
// step at B8_lowrate), the team kernel pays a barrier over all its workgroups and the same stream.  Here the weights
// never move: every column tile of every GEMM of the step (K x 16 fp32, 48-72 KB) is copied ONCE into the LDS of one
// workgroup (25.6 MB over 256 CUs x ~143 KB of LDS), and an operation is computed by the workgroups holding its tiles
// as soon as its inputs are there.  Hand-offs are data-tagged granules (MI355X_MICROARCH.md "handoff-1to1"): every
// output element is stored as one 8-byte {float bits, step + 1} word, write-through (sc1); a consumer polls the
// granules it needs with sc1 loads until every tag reads the current step, so data and flag arrive together and only the
// producers and the consumers of an edge take part (no barrier).  The reconstruction goes to zpad as well (write-through,
// drained before the d3 granules are published), where later steps read their window taps.
//
// Arithmetic per output element is k_gemm_s's: the same KSPLIT = 8 K slices, each a k-ordered chain of
// v_mfma_f32_16x16x4_f32 on the same fragments (row 0 of the 16-row tile carries the image; rows 1-15 are zero), the
// slice-ordered sum and the same epilogue formulas: bit-identical to lbc_decode's graph decoder
// (tests/test_one_gpu.py).  The rANS decode is rans_row_sparse on one wave of a workgroup that holds no weights, its
// coder state persistent in LDS.
#include "kernels_dev.h"

namespace lbic {

namespace {

constexpr int ONE_RC_WORDS = 576;    // rans_row_sparse's persistent coder-state cache
constexpr int ONE_SCR = 256;         // floats of A scratch per wave (>= ONE_LL_MAX x 16)

typedef const __attribute__((address_space(4))) OneOp* cop_p;

__device__ __forceinline__ uint4 ld16_sc1(const void* base, unsigned byte_off) {
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, -1, 0x00020000);
    return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, byte_off, 0, 16));   // aux 16: sc1
}
__device__ __forceinline__ void st_gran(unsigned long long* p, float v, unsigned tag) {
    const unsigned long long w = ((unsigned long long)tag << 32) | __float_as_uint(v);
    __hip_atomic_store((gptr<unsigned long long>)p, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// the epilogue value of k_gemm_s / k_dec_team (kernels_dev.h epilogue) for one output element: the same float operations
__device__ __forceinline__ float one_epi(int epi, float v, float b, float xv) {
    switch (epi) {
        case EPI_LEAKY: {
            const float t = v + b;
            return t > 0.f ? t : t * 0.01f;
        }
        case EPI_GDN: {
            const float sq = __fsqrt_rn(v + b);
            return xv * __fdiv_rn(1.0f, sq);
        }
        case EPI_IGDN: {
            const float sq = __fsqrt_rn(v + b);
            return xv * sq;
        }
        case EPI_CLAMPZ:
            return fminf(fmaxf(v + b, -0.5f), 0.5f);
        default:   // EPI_BIAS, EPI_CTXIDX (the value; the caller turns the scale columns into scale indexes)
            return v + b;
    }
}

struct OneCtl {
    unsigned* fail;
    unsigned long long tmo;
};

// Wait until granules [g0, g0 + cnt) of `gran` carry `tag`, then leave their values in scr[0, cnt) (LDS).  One wave;
// pairs of granules per lane (g0 even).  Returns false when the launch failed (timeout here or elsewhere).
// ge: every tag >= `tag` (a visibility proxy: granules are only ever overwritten by later steps), no values kept
// NQ = 4: up to 512 granules in one poll (the half-tile operations' long K slices)
template <int NQ = 2>
__device__ __forceinline__ bool wave_wait_gran(const unsigned long long* gran, int g0, int cnt, unsigned tag, float* scr,
                                               const OneCtl& c, bool ge = false) {
    const int lane = threadIdx.x & 63;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0;; ++it) {
        bool ok = true;
        uint4 q[NQ];
        // only the granules asked for (a poll is a memory-side round trip of every polling wave on the chip)
#pragma unroll
        for (int p = 0; p < NQ; ++p) {
            q[p] = uint4{0u, 0u, 0u, 0u};
            if ((p == 0 || cnt > p * 128) && p * 128 + lane * 2 < cnt)
                q[p] = ld16_sc1(gran, (unsigned)(g0 + p * 128 + lane * 2) * 8u);
        }
#pragma unroll
        for (int p = 0; p < NQ; ++p) {
            const int j = (p * 64 + lane) * 2;
            if (j < cnt)
                ok &= ge ? (q[p].y >= tag && (j + 1 >= cnt || q[p].w >= tag)) : (q[p].y == tag && (j + 1 >= cnt || q[p].w == tag));
        }
        if (__ballot(!ok) == 0ull) {
            if (ge) return true;
#pragma unroll
            for (int p = 0; p < NQ; ++p) {
                const int j = (p * 64 + lane) * 2;
                if (j < cnt) scr[j] = __uint_as_float(q[p].x);
                if (j + 1 < cnt) scr[j + 1] = __uint_as_float(q[p].z);
            }
            return true;
        }
        // the failure word only every 16th poll: a poll is one memory round trip, not two
        if ((it & 15) == 15 &&
            __hip_atomic_load((gptr<unsigned>)c.fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
            return false;
        if (__builtin_amdgcn_s_memrealtime() - t0 > c.tmo) {
            if (lane == 0) __hip_atomic_store((gptr<unsigned>)c.fail, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return false;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

// every tag of granules [g0, g0 + cnt) >= tag (any count; no values kept)
__device__ __forceinline__ bool wave_wait_ge(const unsigned long long* gran, int g0, int cnt, unsigned tag,
                                             const OneCtl& c) {
    bool ok = true;
    for (int k = 0; k < cnt && ok; k += 512)
        ok = wave_wait_gran<4>(gran, g0 + k, min(512, cnt - k), tag, nullptr, c, true);
    return ok;
}

// my[i] without dynamic indexing into a register array (which would put the array in scratch)
__device__ __forceinline__ int4 pick(const int4 (&my)[ONE_NT_MAX], int i) {
    int x = my[0].x, y = my[0].y, z = my[0].z;
#pragma unroll
    for (int j = 1; j < ONE_NT_MAX; ++j) {
        x = i == j ? my[j].x : x;
        y = i == j ? my[j].y : y;
        z = i == j ? my[j].z : z;
    }
    return make_int4(x, y, z, 0);
}

__device__ __forceinline__ int4 pick4(const int4 (&my)[ONE_NT_MAX], int i) {   // all four fields
    int4 r = my[0];
#pragma unroll
    for (int j = 1; j < ONE_NT_MAX; ++j) {
        r.x = i == j ? my[j].x : r.x;
        r.y = i == j ? my[j].y : r.y;
        r.z = i == j ? my[j].z : r.z;
        r.w = i == j ? my[j].w : r.w;
    }
    return r;
}

__device__ __forceinline__ float pick_f(const float (&v)[ONE_NT_MAX], int i) {
    float r = v[0];
#pragma unroll
    for (int j = 1; j < ONE_NT_MAX; ++j) r = i == j ? v[j] : r;
    return r;
}

// the segment of k-block kb (uniform)
__device__ __forceinline__ int seg_of(const OneOp& op, int kb) {
    const int k = kb << 4;
    int s = 0;
#pragma unroll
    for (int i = 1; i < ONE_MAXSEG; ++i) s = (i < op.nseg && k >= op.seg[i].k0) ? i : s;
    return s;
}

// A run of layer-0 cache taps (k-blocks [kb, kb + nk) of segment sg, KS[1] = 3): wait until the cells it reads are
// written.  The cache's producer (op sg.src, the context net's layer 0) stores a cell's channels, drains them, then
// publishes the same columns' granules, tagged step + 1 and overwritten only by later steps, so a tag >= s + 1 on a
// column means every cell that column's producer wrote up to step s is visible.  Every tap reads a cell of an earlier
// step (tag >= step: the previous step's layer 0 published) but two, which a row end computes in THIS step's layer 0:
// (v, -1) at h = 0 (tap (0, -1)) and (v - 1, Wb) at h = Wb - 1 (tap (-1, +1)) -- tag >= step + 1 there.
__device__ __forceinline__ bool l0_wait(const OneArgs& a, const OneSeg& sg, int kb, int nk, int h, unsigned tag,
                                        const OneCtl& c) {
    const bool now = (sg.dy == 0 && sg.dx == -1 && h == 0) || (sg.dy == -1 && sg.dx == 1 && h == a.Wb - 1);
    const unsigned need = now ? tag : tag - 1;
    if (need == 0) return true;
    const OneOp& src = *(const OneOp*)((cop_p)a.ops + sg.src);
    return wave_wait_ge(src.gran, sg.c0 + (kb << 4) - sg.k0, nk * 16, need, c);
}

// One GEMM operation: the tiles of `op` this workgroup holds (my[]), for block (v, h) at step tag - 1.  Every thread
// returns the same value (false: the launch failed).
// L0: the operation touches the layer-0 cache (the layer-0 op itself, or cache taps in K): a separate instance, so the
// KS[1] = 1 operations keep the code (and the instruction-cache footprint) they had without it
template <int LL, bool L0>
__device__ __forceinline__ bool one_gemm(const OneArgs& a, const OneOp& op, int o, const int4 (&my)[ONE_NT_MAX], int v,
                                         int h, unsigned tag, const f4* wl, float* red, float* scr_all, int* sflag,
                                         const OneCtl& c, unsigned long long* lst, const float* ltab) {
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nkb = op.K >> 4;
    const int kb0 = wave * nkb / KSPLIT, n = (wave + 1) * nkb / KSPLIT - kb0;
    float* scr = scr_all + wave * ONE_SCR;
    bool ok = true;
    const OneOp& last = *(const OneOp*)((cop_p)a.ops + (a.nops - 1));    // d3: the reconstruction of every step
    const int t = (int)tag - 1;
    // (stamps only, step ts_step) times kept in registers, then in this workgroup's LDS stamp slot of the op (written to
    // memory after the last step: no stamp store or atomic may sit in a memory queue that a wait drains)
    const bool st_on = a.ts && t == a.ts_step;
    unsigned long long s_in = 0, s_rdy = 0, s_regs = 0, s_chain = 0, s_red = 0, s_st = 0;
    if (st_on) s_in = __builtin_amdgcn_s_memrealtime();
    // the epilogue operands of this op's tiles (bias, read-only), requested before anything waits
    float bb[ONE_NT_MAX];
#pragma unroll
    for (int i = 0; i < ONE_NT_MAX; ++i) {
        const int4 ti = my[i];
        bb[i] = ti.x == o ? op.bias[min(ti.y * 16 + (lane & 15), op.N - 1)] : 0.f;
    }
    // inputs of this wave's K slice, run by run of k-blocks of one segment:
    //  * granules of an earlier op of this step (tag): values into the wave's scratch;
    //  * the left window tap (0, -1) for h >= 1: the previous step's d3 granules (tag - 1) ARE that block -- values into
    //    the scratch, no zpad round trip;
    //  * the taps of the row above: zpad, visible once d3's granules have reached the producing step t' (+ 1, or + 2
    //    with lazy drains: a d3 producer drains its zpad store of step t' only before publishing step t' + 1)
    unsigned zneed = 0;
    // (uniform) the common shape: the whole of K is one granule segment of one source op from its column c0
    const bool gran1 = op.nseg == 1 && op.seg[0].kind == ONE_GRAN;
    // otherwise: each fragment's source resolved before the waits (the per-k-block segment lookup is a chain of scalar
    // loads): bit cc of zmask (uniform) = a zpad tap at byte offset zo[cc] (or, bit cc of lmask, a layer-0 cache cell),
    // else the wave's scratch
    const int q4 = (lane >> 4) * 4;
    const long cell = ((long)(v + 2) * a.Wp + (h + 2));
    // the layer-0 op (l0out) at a row end: positions 1 (and 2) in MFMA rows 1 (2), the graph decoder's raster positions
    // (codec.hip run_ctx): h = 0 adds (v, -1), h = Wb - 1 adds (v - 1, Wb)
    const int P = L0 && op.l0out ? 1 + (h == 0 ? 1 : 0) + (h == a.Wb - 1 ? 1 : 0) : 1;
    const long cell1 = h == 0 ? cell - 1 : cell - a.Wp + 1, cell2 = cell - a.Wp + 1;
    const int prow = lane & 15;
    // this lane's zpad byte shift from the block's own cell to its row's position (rows past P: none)
    const unsigned zdl = prow == 1 && P > 1 ? (unsigned)((cell1 - cell) * a.Cx * 4)
                         : prow == 2 && P > 2 ? (unsigned)((cell2 - cell) * a.Cx * 4) : 0u;
    unsigned zmask = 0, lmask = 0;
    unsigned zo[LL];
    if (!gran1) {
#pragma unroll
        for (int cc = 0; cc < LL; ++cc) {
            const int ci = max(min(cc, n - 1), 0);      // (an empty slice, n = 0, loads k-block kb0 and adds nothing)
            const int kb = kb0 + ci;
            const OneSeg& sg = op.seg[seg_of(op, kb)];
            const bool z = sg.kind == ONE_ZTAP && !(sg.dy == 0 && sg.dx == -1 && h >= 1);
            const bool l = L0 && sg.kind == ONE_L0TAP;
            zmask |= z ? 1u << cc : 0u;
            lmask |= l ? 1u << cc : 0u;
            zo[cc] = (unsigned)((cell + (long)sg.dy * a.Wp + sg.dx) * (l ? a.C1P : a.Cx) + (kb << 4) - sg.k0 + q4) * 4u;
        }
    }
    if (gran1) {
        if (n > 0) {
            const OneOp& src = *(const OneOp*)((cop_p)a.ops + op.seg[0].src);
            ok = wave_wait_gran(src.gran, op.seg[0].c0 + (kb0 << 4), n * 16, tag, scr, c);
        }
    } else
    for (int cb = 0; cb < n && ok;) {
        const int s = seg_of(op, kb0 + cb);
        const OneSeg& sg = op.seg[s];
        int ce = cb + 1;
        while (ce < n && seg_of(op, kb0 + ce) == s) ++ce;
        if (sg.kind == ONE_GRAN) {
            const OneOp& src = *(const OneOp*)((cop_p)a.ops + sg.src);
            const int g0 = sg.c0 + ((kb0 + cb) << 4) - sg.k0;
            ok = wave_wait_gran(src.gran, g0, (ce - cb) * 16, tag, scr + cb * 16, c);
        } else if (L0 && sg.kind == ONE_L0TAP) {
            ok = l0_wait(a, sg, kb0 + cb, ce - cb, h, tag, c);
        } else if (sg.dy == 0 && sg.dx == -1) {
            if (h >= 1) ok = wave_wait_gran(last.gran, ((kb0 + cb) << 4) - sg.k0, (ce - cb) * 16, tag - 1, scr + cb * 16, c);
        } else {
            const int vv = v + sg.dy, hh = h + sg.dx;
            if (vv >= 0 && vv < a.Hb && hh >= 0 && hh < a.Wb)
                zneed = max(zneed, (unsigned)(vv * a.Wb + hh) + (a.lazy_z ? 2u : 1u));
        }
        // the layer-0 op's row-end positions (MFMA rows 1, 2) read every tap from zpad: their in-frame taps too (at
        // Wb = 1 the left tap of (v - 1, Wb) is zhat(v - 1, 0) of the previous step, which no row-0 tap orders)
        if (L0 && sg.kind == ONE_ZTAP)
            for (int p = 1; p < P; ++p) {
                const int vv = (p == 1 && h == 0 ? v : v - 1) + sg.dy, hh = (p == 1 && h == 0 ? -1 : a.Wb) + sg.dx;
                if (vv >= 0 && vv < a.Hb && hh >= 0 && hh < a.Wb)
                    zneed = max(zneed, (unsigned)(vv * a.Wb + hh) + (a.lazy_z ? 2u : 1u));
            }
        cb = ce;
    }
    // a row start (h = 0): the context net's first op has no left tap, so nothing above orders it after the previous
    // step.  Wait for d3 of step t - 1 (every op of step t - 1 done, so every reader of a granule has read it) before
    // this step's granules overwrite any: without it the new row's ops could republish while a slow
    // consumer of step t - 1 still polls for the old tag -- correct values, but a stall until the timeout
    if (o == 0 && h == 0 && t >= 1 && wave == 0) zneed = max(zneed, (unsigned)t);
    if (zneed && ok) {
        for (int g0 = 0; g0 < last.gw && ok; g0 += 256)
            ok = wave_wait_gran(last.gran, g0, min(256, last.gw - g0), zneed, scr + 240, c, true);
    }
    if (st_on) s_rdy = __builtin_amdgcn_s_memrealtime();     // (this wave's inputs are there)
    // A fragments (row 0 = lanes 0, 16, 32, 48: k = kb 16 + 4 (lane >> 4) + 0..3; the other rows are zero)
    __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): this wave's scratch stores are done
    __builtin_amdgcn_wave_barrier();
    f4 av[LL];
    const bool row0 = (lane & 15) == 0;
    if (gran1) {      // every fragment from the wave's scratch: no per-k-block segment lookup
#pragma unroll
        for (int cc = 0; cc < LL; ++cc) {
            const int ci = max(min(cc, n - 1), 0);
            f4 x = *reinterpret_cast<const f4*>(scr + ci * 16 + q4);
            x = row0 ? x : f4{0.f, 0.f, 0.f, 0.f};
            if (op.sq) x = x * x;
            av[cc] = x;
        }
    } else if (L0 && P > 1) {     // (the layer-0 op at a row end) rows 1 .. P - 1: every tap from zpad at their positions
#pragma unroll
        for (int cc = 0; cc < LL; ++cc) {
            const int ci = max(min(cc, n - 1), 0);
            const f4 u = __builtin_bit_cast(f4, ld16_sc1(a.zpad, zo[cc] + zdl));
            const f4 sv = *reinterpret_cast<const f4*>(scr + ci * 16 + q4);
            f4 x = row0 ? (((zmask >> cc) & 1u) ? u : sv) : prow < P ? u : f4{0.f, 0.f, 0.f, 0.f};
            if (op.sq) x = x * x;
            av[cc] = x;
        }
    } else
#pragma unroll
    for (int cc = 0; cc < LL; ++cc) {
        const int ci = max(min(cc, n - 1), 0);
        f4 x = f4{0.f, 0.f, 0.f, 0.f};
        if (((zmask | lmask) >> cc) & 1u) {
            const uint4 u = ld16_sc1(L0 && ((lmask >> cc) & 1u) ? (const void*)a.l0 : (const void*)a.zpad, zo[cc]);
            x = row0 ? __builtin_bit_cast(f4, u) : x;
        } else {
            const f4 u = *reinterpret_cast<const f4*>(scr + ci * 16 + q4);
            x = row0 ? u : x;
        }
        if (op.sq) x = x * x;
        av[cc] = x;
    }
    // every tile of this op the workgroup holds: chain, partials, slice-ordered sum, epilogue, publish
    const int N = op.N, gw = op.gw;
    for (int i = 0; i < ONE_NT_MAX; ++i) {
        const int4 ti = pick(my, i);
        if (ti.x != o) continue;
        const int nt = ti.y;
        const f4* wt = wl + ti.z + lane;
        f4 acc = f4{0.f, 0.f, 0.f, 0.f};
        f4 wv[LL];
#pragma unroll
        for (int cc = 0; cc < LL; ++cc) wv[cc] = wt[(kb0 + max(min(cc, n - 1), 0)) * 64];
        if (st_on && s_regs == 0) {
            __builtin_amdgcn_s_waitcnt(0xC07F);
            s_regs = __builtin_amdgcn_s_memrealtime();
        }
#pragma unroll
        for (int cc = 0; cc < LL; ++cc) {
            f4 t = acc;
#pragma unroll
            for (int e = 0; e < 4; ++e) t = __builtin_amdgcn_mfma_f32_16x16x4f32(av[cc][e], wv[cc][e], t, 0, 0, 0);
            acc = (cc < LL - 1 || cc < n) ? t : acc;    // n >= LL - 1: only the last fragment can be discarded
        }
        if (lane < 16) {
            red[wave * 16 + lane] = acc[0];     // row 0, column lane
            if (L0 && P > 1) red[(KSPLIT + wave) * 16 + lane] = acc[1];
            if (L0 && P > 2) red[(2 * KSPLIT + wave) * 16 + lane] = acc[2];
        }
        if (st_on && s_chain == 0)    // (after the chain's result)
            s_chain = __builtin_amdgcn_s_memrealtime() + (__builtin_amdgcn_readfirstlane(__float_as_int(acc[0])) == 1 ? 1 : 0);
        __syncthreads();
        if (st_on && s_red == 0) s_red = __builtin_amdgcn_s_memrealtime();
        if (threadIdx.x < 16) {
            const int e = threadIdx.x, col = nt * 16 + e;
            float vv = red[e];
#pragma unroll
            for (int s = 1; s < KSPLIT; ++s) vv += red[s * 16 + e];
            float out = 0.f;
            if (col < N) {
                float xv = 0.f;
                if (op.epi == EPI_GDN || op.epi == EPI_IGDN) {
                    // the layer input x = this op's A operand (one granule segment from k = 0): the values the wave that
                    // owns column col's k-block left in its scratch
                    const int kbc = col >> 4;
                    int w = 0;
#pragma unroll
                    for (int q = 1; q < KSPLIT; ++q) w = q * nkb / KSPLIT <= kbc ? q : w;
                    xv = scr_all[w * ONE_SCR + col - (w * nkb / KSPLIT) * 16];
                }
                out = one_epi(op.epi, vv, pick_f(bb, i), xv);
                if (L0 && op.l0out) {
                    // the layer-0 cache cells of every position (write-through), drained before the granule: a reader
                    // of a cell orders itself by these granules' tags (l0_wait)
                    st<true>(a.l0 + cell * a.C1P + col, out, true);
                    for (int p = 1; p < P; ++p) {
                        float vp = red[p * KSPLIT * 16 + e];
#pragma unroll
                        for (int s = 1; s < KSPLIT; ++s) vp += red[(p * KSPLIT + s) * 16 + e];
                        st<true>(a.l0 + (p == 1 ? cell1 : cell2) * a.C1P + col, one_epi(op.epi, vp, pick_f(bb, i), 0.f),
                                 true);
                    }
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
                if (op.epi == EPI_CLAMPZ) {
                    // lazy: this thread's previous zpad store (step t - 1) drained now, the current one by step t + 1
                    if (a.lazy_z) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    st<true>(a.zpad + cell * a.Cx + col, out, true);
                    if (!a.lazy_z) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the tap data before the granule
                }
            }
            // the context net's scale columns go out as their scale indexes (build_indexes, the int in the float's
            // bits): the rANS workgroup decodes from them directly, the search done here by 16 lanes per tile
            if (op.epi == EPI_CTXIDX && col < a.Mlat) out = __int_as_float(scale_index(out, ltab));
            if (col < gw) st_gran(op.gran + col, out, tag);
            if (st_on && s_st == 0) s_st = __builtin_amdgcn_s_memrealtime();
        }
        __syncthreads();
    }
    if (st_on) {
        int sl = 0;
#pragma unroll
        for (int i = ONE_NT_MAX - 1; i >= 0; --i) sl = my[i].x == o ? i : sl;
        unsigned long long* d = lst + sl * ONE_TS_PER_OP;
        if (lane == 0) {
            d[1 + wave] = s_rdy;
            d[1 + KSPLIT + wave] = s_regs;
            d[1 + 2 * KSPLIT + wave] = s_chain;
        }
        if (threadIdx.x == 0) {
            d[0] = s_in;
            d[1 + 3 * KSPLIT] = s_red;
            d[2 + 3 * KSPLIT] = __builtin_amdgcn_s_memrealtime();
            d[3 + 3 * KSPLIT] = s_st;
        }
    }
    // a uniform verdict for the whole workgroup
    if (!ok && lane == 0) *sflag = 1;
    __syncthreads();
    const bool good = *sflag == 0;
    __syncthreads();
    return good;
}

// A half-tile operation (OneOp::half: a column tile's weights -- K x 16 fp32 -- do not fit one workgroup's LDS, e.g. the
// KS3311 context layer 1 of B4_highrate, K = 5 x 768): this workgroup holds half `hh` of column tile ti.y, the k-blocks
// of K slices 4 hh .. 4 hh + 3, and its waves 0-3 run those four slices' chains (the same k-ordered MFMA chains as
// one_gemm, weights from LDS).  A slice's fragments are its layer-0 cache taps (the host puts every cache segment before
// the granule segment) and then this step's granules, so its chain runs in two phases: the cache part as soon as the
// cells are written -- normally a whole raster step before this one's layer 0 publishes -- with its A fragments in
// registers (chunks of C, the next chunk requested before this one's MFMAs); then, once the granules are there, the rest
// from the LDS scratch.  The critical path after layer 0 is then one poll plus the granule part of the chain.  Half 0
// hands its four partials over as granules (pgran, by step parity: half 0 of step t + 2 can only start after layer 0
// of step t + 1, i.e. after this step's whole chain -- the half-1 reader included -- has finished); half 1's wave 4
// collects them while its waves 0-3 compute, then the eight partials are summed in slice order and the shared epilogue
// publishes the column tile.  Bit-identical to a whole-tile operation.
template <int LLH>
__device__ __forceinline__ bool one_gemm_half(const OneArgs& a, const OneOp& op, int4 ti, int v, int h, unsigned tag,
                                              const f4* wl, float* red, float* scr_all, int* sflag, const OneCtl& c) {
    constexpr int C = 8, NC = (LLH + C - 1) / C;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nkb = op.K >> 4;
    const int hh = ti.w - 1;
    const int kbl = (4 * hh) * nkb / KSPLIT;            // the first k-block this half holds
    const bool cw = wave < 4;                            // (uniform) a chain wave
    const int sl = 4 * hh + (wave & 3);
    const int kb0 = sl * nkb / KSPLIT, n = cw ? (sl + 1) * nkb / KSPLIT - kb0 : 0;
    float* scr = scr_all + (wave & 3) * 2 * ONE_SCR;     // (a chain wave's slice: up to 2 ONE_SCR floats)
    const int t = (int)tag - 1;
    const int q4 = (lane >> 4) * 4;
    const long cell = ((long)(v + 2) * a.Wp + (h + 2));
    const int NT = op.gw >> 4;
    const float bb = op.bias[min(ti.y * 16 + (lane & 15), op.N - 1)];
    unsigned long long* pg = op.pgran + ((long)(t & 1) * NT + ti.y) * 64;
    bool ok = true;
    f4 acc = f4{0.f, 0.f, 0.f, 0.f};
    if (cw) {
        const bool row0 = (lane & 15) == 0;
        const f4* wt = wl + ti.z + lane;
        // nl: the slice's leading cache fragments (the first granule segment's k0 bounds them)
        int kg = op.K;
        for (int i = 0; i < op.nseg; ++i) kg = op.seg[i].kind == ONE_GRAN ? min(kg, op.seg[i].k0) : kg;
        const int nl = min(max((kg >> 4) - kb0, 0), n);
        // ---- phase 1: the cache taps
        for (int cb = 0; cb < nl && ok;) {
            const int sx = seg_of(op, kb0 + cb);
            int ce = cb + 1;
            while (ce < nl && seg_of(op, kb0 + ce) == sx) ++ce;
            ok = l0_wait(a, op.seg[sx], kb0 + cb, ce - cb, h, tag, c);
            cb = ce;
        }
        if (ok && nl > 0) {
            // fragment cc through one buffer load: the lane's part is its 4 k (q4), the rest the uniform scalar offset
            const auto lr = __builtin_amdgcn_make_buffer_rsrc(a.l0, 0, -1, 0x00020000);
            const unsigned lq = (unsigned)q4 * 4u;
            f4 ab[2][C];
            auto aload = [&](int k, f4 (&A)[C]) {
#pragma unroll
                for (int j = 0; j < C; ++j) {
                    const int kb = kb0 + min(k * C + j, nl - 1);
                    const OneSeg& sg = op.seg[seg_of(op, kb)];
                    const unsigned so = (unsigned)(((cell + (long)sg.dy * a.Wp + sg.dx) * a.C1P + (kb << 4) - sg.k0) * 4);
                    A[j] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(lr, lq, so, 16));
                }
            };
            aload(0, ab[0]);
            if (NC > 1) aload(1, ab[1]);
#pragma unroll
            for (int k = 0; k < NC; ++k) {
                f4 w[C];
#pragma unroll
                for (int j = 0; j < C; ++j) w[j] = wt[(kb0 + min(k * C + j, nl - 1) - kbl) * 64];
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int j = 0; j < C; ++j) {
                    const int cc = k * C + j;
                    if (cc < LLH) {
                        f4 x = row0 ? ab[k & 1][j] : f4{0.f, 0.f, 0.f, 0.f};
                        if (op.sq) x = x * x;
                        f4 tt = acc;
#pragma unroll
                        for (int e = 0; e < 4; ++e) tt = __builtin_amdgcn_mfma_f32_16x16x4f32(x[e], w[j][e], tt, 0, 0, 0);
                        acc = cc < nl ? tt : acc;
                    }
                }
                __builtin_amdgcn_sched_barrier(0);
                if (k + 2 < NC) aload(k + 2, ab[k & 1]);
            }
        }
        // ---- phase 2: this step's granules (values into the scratch at their slice positions), then their chain
        for (int cb = nl; cb < n && ok;) {
            const int sx = seg_of(op, kb0 + cb);
            const OneSeg& sg = op.seg[sx];
            int ce = cb + 1;
            while (ce < n && seg_of(op, kb0 + ce) == sx) ++ce;
            const OneOp& src = *(const OneOp*)((cop_p)a.ops + sg.src);
            ok = wave_wait_gran<4>(src.gran, sg.c0 + ((kb0 + cb) << 4) - sg.k0, (ce - cb) * 16, tag, scr + cb * 16, c);
            cb = ce;
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_wave_barrier();
        if (ok) {
            for (int cb = nl; cb < n; cb += C) {          // (A and weights from LDS: runtime positions)
                f4 x[C], w[C];
#pragma unroll
                for (int j = 0; j < C; ++j) {
                    const int ci = min(cb + j, n - 1);
                    x[j] = *reinterpret_cast<const f4*>(scr + ci * 16 + q4);
                    w[j] = wt[(kb0 + ci - kbl) * 64];
                }
#pragma unroll
                for (int j = 0; j < C; ++j) {
                    f4 xx = row0 ? x[j] : f4{0.f, 0.f, 0.f, 0.f};
                    if (op.sq) xx = xx * xx;
                    f4 tt = acc;
#pragma unroll
                    for (int e = 0; e < 4; ++e) tt = __builtin_amdgcn_mfma_f32_16x16x4f32(xx[e], w[j][e], tt, 0, 0, 0);
                    acc = cb + j < n ? tt : acc;
                }
            }
        }
        if (lane < 16) red[sl * 16 + lane] = acc[0];
    } else if (wave == 4 && hh == 1) {
        ok = wave_wait_gran(pg, 0, 64, tag, red, c);       // half 0's partials -> red[0 .. 63] (slices 0-3)
    }
    if (!ok && lane == 0) *sflag = 1;
    __syncthreads();
    const bool good = *sflag == 0;     // (a uniform verdict: no output from a failed wait)
    if (good) {
        if (hh == 0) {
            if (threadIdx.x < 64) st_gran(pg + threadIdx.x, red[threadIdx.x], tag);
        } else if (threadIdx.x < 16) {
            const int e = threadIdx.x, col = ti.y * 16 + e;
            float vv = red[e];
#pragma unroll
            for (int s = 1; s < KSPLIT; ++s) vv += red[s * 16 + e];
            const float out = col < op.N ? one_epi(op.epi, vv, bb, 0.f) : 0.f;
            if (col < op.gw) st_gran(op.gran + col, out, tag);
        }
    }
    __syncthreads();
    return good;
}

// LL = fragments per wave: L = (K / 16) / 8 k-blocks per slice, L + 1 when the slices differ in length (the extra
// fragment's MFMAs are discarded), L when every slice has exactly L (nothing to discard: a shorter chain)
// KL0: the kernel instance under the layer-0 cache (k_dec_one<true>); the other instance compiles no cache code at all
template <bool KL0>
__device__ __forceinline__ bool one_gemm_any(const OneArgs& a, const OneOp& op, int o, const int4 (&my)[ONE_NT_MAX], int v, int h,
                             unsigned tag, const f4* wl, float* red, float* scr, int* sflag, const OneCtl& c,
                             unsigned long long* lst, const float* ltab) {
    const int nkb = op.K >> 4;
    const bool l0 = KL0 && (op.l0out || op.l0seg);
    int key = (nkb / KSPLIT) * 2 + (nkb % KSPLIT == 0 ? 1 : 0);
    if constexpr (KL0) {     // the layer-0-cache kernel (B4_highrate: K = 384 / 512 / 640): exact slices of 3-5
                             // k-blocks, no discarded fragment (only this kernel carries the instances)
        if (!l0) switch (key) {
            case 7: return one_gemm<3, false>(a, op, o, my, v, h, tag, wl, red, scr, sflag, c, lst, ltab);
            case 9: return one_gemm<4, false>(a, op, o, my, v, h, tag, wl, red, scr, sflag, c, lst, ltab);
            case 11: return one_gemm<5, false>(a, op, o, my, v, h, tag, wl, red, scr, sflag, c, lst, ltab);
            default: break;
        }
    }
#ifndef LBIC_ONE_EXACT_ALL
    if ((key & 1) && key != 13 && key != 19) key &= ~1;     // exact slices without an instance: the L + 1 form
#endif
    switch (key) {
#define LBIC_ONE(L_) \
    case L_ * 2: return l0 ? one_gemm<L_ + 1, KL0>(a, op, o, my, v, h, tag, wl, red, scr, sflag, c, lst, ltab) \
                           : one_gemm<L_ + 1, false>(a, op, o, my, v, h, tag, wl, red, scr, sflag, c, lst, ltab);
#define LBIC_ONE_EX(L_) \
    case L_ * 2 + 1: return l0 ? one_gemm<L_, KL0>(a, op, o, my, v, h, tag, wl, red, scr, sflag, c, lst, ltab) \
                               : one_gemm<L_, false>(a, op, o, my, v, h, tag, wl, red, scr, sflag, c, lst, ltab);
        LBIC_ONE(0) LBIC_ONE(1) LBIC_ONE(2) LBIC_ONE(3) LBIC_ONE(4) LBIC_ONE(5) LBIC_ONE(6) LBIC_ONE(7) LBIC_ONE(8)
        LBIC_ONE(9) LBIC_ONE(10) LBIC_ONE(11)
#ifdef LBIC_ONE_EXACT_ALL
        LBIC_ONE_EX(1) LBIC_ONE_EX(2) LBIC_ONE_EX(3) LBIC_ONE_EX(4) LBIC_ONE_EX(5) LBIC_ONE_EX(7) LBIC_ONE_EX(8)
        LBIC_ONE_EX(10) LBIC_ONE_EX(11) LBIC_ONE_EX(12)
#endif
        LBIC_ONE_EX(6) LBIC_ONE_EX(9)   // K = 768, 1152 (the B8 context / decoder widths)
#undef LBIC_ONE
#undef LBIC_ONE_EX
        default: return false;   // (the host admits K <= 1536 only)
    }
}

}  // namespace

// dynamic LDS: [weight tiles wlds_f4 float4s][partials red_rows (1; 3 under the layer-0 cache) x KSPLIT x 16][A scratch 8 x ONE_SCR][rANS window RANS_WIN words]
// [rANS state cache ONE_RC_WORDS][scale indexes | means 512][yq 256][flag 4 words][stamp slots ONE_NT_MAX x ONE_TS_PER_OP
// u64][scale table 64][rANS centre intervals 256]
size_t one_lds_bytes(int wlds_f4, int red_rows) {
    return (size_t)wlds_f4 * 16 + (size_t)(red_rows * KSPLIT * 16 + KSPLIT * ONE_SCR) * 4 +
           (size_t)(RANS_WIN + ONE_RC_WORDS + 512 + 256 + 4) * 4 + (size_t)ONE_NT_MAX * ONE_TS_PER_OP * 8 + 64 * 4 +
           256 * 4;
}

// L0: KS[1] = 3 (the layer-0 cache, half-tile operations); L0 = false is the KS[1] = 1 kernel without any of that code
template <bool L0>
__global__ __launch_bounds__(512, 1) void k_dec_one(const OneArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t one_lds[];
    f4* wl = reinterpret_cast<f4*>(one_lds);
    float* red = reinterpret_cast<float*>(wl + a.wlds_f4);
    float* scr = red + a.red_rows * KSPLIT * 16;
    uint32_t* lwin = reinterpret_cast<uint32_t*>(scr + KSPLIT * ONE_SCR);
    uint32_t* rcache = lwin + RANS_WIN;
    float* l_ksi = reinterpret_cast<float*>(rcache + ONE_RC_WORDS);
    float* l_yq = l_ksi + 512;
    int* sflag = reinterpret_cast<int*>(l_yq + 256);
    unsigned long long* lst = reinterpret_cast<unsigned long long*>(sflag + 4);    // (8-byte aligned)
    float* ltab_s = reinterpret_cast<float*>(lst + ONE_NT_MAX * ONE_TS_PER_OP);   // the scale table (scale_index)
    uint32_t* l_lf = reinterpret_cast<uint32_t*>(ltab_s + 64);                     // the rANS wave's centre intervals
    const int rank = blockIdx.x;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const OneCtl c{a.fail, a.tmo};
    int4 my[ONE_NT_MAX];
#pragma unroll
    for (int i = 0; i < ONE_NT_MAX; ++i) my[i] = a.tiles[rank * ONE_NT_MAX + i];
    // this workgroup's weight tiles into LDS, once (read-only for the launch)
    for (int i = 0; i < ONE_NT_MAX; ++i) {
        const int4 ti = pick4(my, i);      // (no dynamic index into the register array)
        if (ti.x < 0) continue;
        const OneOp& op = *(const OneOp*)((cop_p)a.ops + ti.x);
        const f4* src = reinterpret_cast<const f4*>(op.W);
        const int nkb = op.K >> 4;
        // (a half-tile piece: k-blocks [0, 4 nkb / 8) or [4 nkb / 8, nkb))
        const int kb_lo = ti.w == 2 ? 4 * nkb / KSPLIT : 0, kb_hi = ti.w == 1 ? 4 * nkb / KSPLIT : nkb;
        for (int j = threadIdx.x; j < (kb_hi - kb_lo) * 64; j += blockDim.x) {
            const int kb = kb_lo + (j >> 6), l = j & 63;
            wl[ti.z + j] = src[((long)kb * op.NB16 + ti.y) * 64 + l];
        }
    }
    if (threadIdx.x == 0) {
        rcache[4] = 0u;    // no cached coder state yet
        *sflag = 0;
    }
    if (a.ts)
        for (int i = threadIdx.x; i < ONE_NT_MAX * ONE_TS_PER_OP; i += blockDim.x) lst[i] = 0ull;
    if (threadIdx.x < 64) ltab_s[threadIdx.x] = a.table[threadIdx.x];
    const RansArgs& R = *(const RansArgs*)((const __attribute__((address_space(4))) RansArgs*)a.rans);
    // the stream's workgroup holds no weights: its LDS takes a copy of the table image, so the rare symbols off the
    // centre intervals are searched in LDS instead of global memory (two dependent loads each)
    const uint16_t* ltab = nullptr;
    if (rank == a.rans_wg && a.rans_lds_tab) {
        const uint4* src = reinterpret_cast<const uint4*>(R.cdf16);
        uint4* dst = reinterpret_cast<uint4*>(wl);
        for (int i = threadIdx.x; i < R.total16 / 8; i += blockDim.x) dst[i] = src[i];
        ltab = reinterpret_cast<const uint16_t*>(wl);
    }
    __syncthreads();
    for (int t = 0; t < a.Hb * a.Wb; ++t) {
        const int v = t / a.Wb, h = t - v * a.Wb;
        const unsigned tag = (unsigned)t + 1u;
        for (int o = 0; o < a.nops; ++o) {
            if (o == a.rans_op) {
                if (rank != a.rans_wg) continue;
                bool ok = true;
                const bool stamp = a.ts && t == a.ts_step;
                unsigned long long r_in = 0, r_rdy = 0, r_coded = 0, r_pub = 0, c_rdy = 0, c_coded = 0;
                if (stamp) r_in = __builtin_amdgcn_s_memrealtime();
                if (wave == 0) {
                    // scale indexes | means of the context net (2 Mlat granules: ctx3's epilogue turned the scales into
                    // their indexes) into LDS
                    const OneOp& ctx = *(const OneOp*)((cop_p)a.ops + (o - 1));
                    const int M = a.Mlat;
                    for (int g0 = 0; g0 < 2 * M && ok; g0 += 256)
                        ok = wave_wait_gran(ctx.gran, g0, min(256, 2 * M - g0), tag, l_ksi + g0, c);
                    __builtin_amdgcn_s_waitcnt(0xC07F);
                    __builtin_amdgcn_wave_barrier();
                    if (stamp) {
                        r_rdy = __builtin_amdgcn_s_memrealtime();
                        c_rdy = __builtin_amdgcn_s_memtime();    // (the shader clock)
                    }
                    if (ok) {
                        rans_row_sparse<false, true, true>(R, lwin, 0, lane, false, ltab, rcache,
                                                           reinterpret_cast<const int32_t*>(l_ksi), l_ksi, l_yq,
                                                           stamp ? lst + 8 : nullptr, l_lf);
                        __builtin_amdgcn_s_waitcnt(0xC07F);
                        __builtin_amdgcn_wave_barrier();
                        if (stamp) {
                            r_coded = __builtin_amdgcn_s_memrealtime();
                            c_coded = __builtin_amdgcn_s_memtime();
                        }
                        const OneOp& yo = *(const OneOp*)((cop_p)a.ops + o);
                        for (int i = lane; i < yo.gw; i += 64) st_gran(yo.gran + i, i < M ? l_yq[i] : 0.f, tag);
                        if (stamp) r_pub = __builtin_amdgcn_s_memrealtime();
                    }
                    if (stamp && lane == 0) {
                        lst[0] = r_in;
                        lst[1] = r_coded;
                        lst[2] = r_pub;
                        lst[3] = r_rdy;
                        lst[4] = c_rdy;
                        lst[5] = c_coded;
                    }
                    if (!ok && lane == 0) *sflag = 1;
                }
                __syncthreads();
                const bool good = *sflag == 0;
                __syncthreads();
                if (!good) return;
                continue;
            }
            bool mine = false;
#pragma unroll
            for (int i = 0; i < ONE_NT_MAX; ++i) mine |= my[i].x == o;
            if (!mine) continue;
            const OneOp& op = *(const OneOp*)((cop_p)a.ops + o);
            if (L0 && op.half) {     // (one piece of a half-tile op per workgroup: host-checked)
                int sl = 0;
#pragma unroll
                for (int i = ONE_NT_MAX - 1; i >= 1; --i) sl = my[i].x == o ? i : sl;
                const int4 ti = pick4(my, sl);
                const int key = ((op.K >> 4) + KSPLIT - 1) / KSPLIT;
                const bool good = key == 30 ? one_gemm_half<30>(a, op, ti, v, h, tag, wl, red, scr, sflag, c)
                                            : one_gemm_half<ONE_LLH_MAX>(a, op, ti, v, h, tag, wl, red, scr, sflag, c);
                if (!good) return;
                continue;
            }
            if (!one_gemm_any<L0>(a, op, o, my, v, h, tag, wl, red, scr, sflag, c, lst, ltab_s)) return;
        }
    }
    // the stamps of step ts_step, from LDS to memory after the last step
    if (a.ts) {
        __syncthreads();
        if (rank == a.rans_wg) {
            if (threadIdx.x == 0) {
                const int o = a.rans_op;
                a.ts[o * 4] = lst[0];
                a.ts[o * 4 + 1] = lst[1];
                a.ts[o * 4 + 2] = lst[2];
                a.ts[o * 4 + 3] = lst[3];
                a.ts[ONE_MAXOPS * 4] = lst[3];
                a.ts[ONE_MAXOPS * 4 + 1] = lst[1];
                a.ts[ONE_MAXOPS * 4 + 2] = lst[4];
                a.ts[ONE_MAXOPS * 4 + 3] = lst[5];
                for (int k = 0; k < 5; ++k) a.ts[ONE_TS_DETAIL + o * ONE_TS_PER_OP + k] = lst[8 + k];
            }
        } else if (threadIdx.x < ONE_NT_MAX) {
            const int i = threadIdx.x;
            const int4 ti = pick(my, i);
            const int o = ti.x;
            bool first = o >= 0;
#pragma unroll
            for (int j = 0; j < ONE_NT_MAX; ++j) first &= !(j < i && my[j].x == o);
            if (first) {
                const unsigned long long* d = lst + i * ONE_TS_PER_OP;
                unsigned long long r = 0;
                for (int w = 0; w < KSPLIT; ++w) r = d[1 + w] > r ? d[1 + w] : r;
                atomicMin(a.ts + o * 4, d[0]);
                atomicMax(a.ts + o * 4 + 1, d[1 + 3 * KSPLIT]);
                atomicMax(a.ts + o * 4 + 2, d[2 + 3 * KSPLIT]);
                atomicMax(a.ts + o * 4 + 3, r);
                if (ti.y == 0)
                    for (int k = 0; k < ONE_TS_PER_OP; ++k) a.ts[ONE_TS_DETAIL + o * ONE_TS_PER_OP + k] = d[k];
            }
        }
    }
}

static const void* one_instance(bool l0) {
    return l0 ? reinterpret_cast<const void*>(&k_dec_one<true>) : reinterpret_cast<const void*>(&k_dec_one<false>);
}

int one_blocks_per_cu(size_t lds, bool l0) {
    int nb = 0;
    (void)hipFuncSetAttribute(one_instance(l0), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, one_instance(l0), 512, lds) != hipSuccess) return 0;
    return nb;
}

int launch_dec_one(const OneArgs& a, int grid, hipStream_t s) {
    if (!a.ops || !a.tiles || !a.rans || !a.fail || !a.zpad || a.nops < 2 || a.nops > ONE_MAXOPS || grid < 2 ||
        a.rans_wg < 0 || a.rans_wg >= grid || a.rans_op < 1 || a.rans_op >= a.nops || a.Mlat > 256 || a.Mlat < 1 ||
        (a.l0 && a.C1P % 16))
        return set_error(LBC_E_ARG, "bad single-image decoder arguments");
    if (a.red_rows != (a.l0 ? 3 : 1)) return set_error(LBC_E_ARG, "single-image decoder: partial rows");
    const size_t lds = one_lds_bytes(a.wlds_f4, a.red_rows);
    if (lds > 160 * 1024) return set_error(LBC_E_ARG, "single-image decoder: LDS image too large");
    static const bool attr = [] {
        for (int l = 0; l < 2; ++l)
            (void)hipFuncSetAttribute(one_instance(l != 0), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        return true;
    }();
    (void)attr;
    if (a.l0) hipLaunchKernelGGL(k_dec_one<true>, dim3(grid), dim3(512), lds, s, a);
    else hipLaunchKernelGGL(k_dec_one<false>, dim3(grid), dim3(512), lds, s, a);
    return launch_status("k_dec_one");
}

}  // namespace lbic
