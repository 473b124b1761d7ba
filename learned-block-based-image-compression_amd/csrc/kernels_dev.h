// Device-side building blocks shared by kernels.hip and team.hip (gfx950): kernel-argument warm-up, timing
// stamps, the GEMM epilogue, the small-M A-operand addressing, and the sparse rANS row decoder.
#pragma once
#include <type_traits>

#include "kernels.h"

#include <cmath>
#include <string>

#include "lbic_internal.h"

namespace lbic {

typedef float f4 __attribute__((ext_vector_type(4)));

// Kernel arguments are read with scalar loads through the scalar cache.  hipcc fetches the large argument
// blocks field by field at first use, in several dependent rounds (a branch on one argument, then the loads
// it guards, then a wait...), each an L2 round trip.  One asm statement touching every 64-byte line of the
// block up front turns that into one round trip: the later, compiler-placed loads hit the scalar cache.
// (Scalar LOADS only: nothing is written through the scalar cache.)
template <int NLINES>
__device__ __forceinline__ void warm_kernargs() {
    static_assert(NLINES >= 1 && NLINES <= 10, "kernarg lines");
    const auto kp = __builtin_amdgcn_kernarg_segment_ptr();
    uint32_t d0, d1, d2, d3, d4, d5, d6, d7, d8, d9;
    if constexpr (NLINES <= 3) {
        asm volatile("s_load_dword %0, %3, 0x0\n\ts_load_dword %1, %3, 0x40\n\ts_load_dword %2, %3, 0x80\n\t"
                     "s_waitcnt lgkmcnt(0)"
                     : "=&s"(d0), "=&s"(d1), "=&s"(d2) : "s"(kp) : "memory");
    } else {
        asm volatile("s_load_dword %0, %10, 0x0\n\ts_load_dword %1, %10, 0x40\n\ts_load_dword %2, %10, 0x80\n\t"
                     "s_load_dword %3, %10, 0xc0\n\ts_load_dword %4, %10, 0x100\n\ts_load_dword %5, %10, 0x140\n\t"
                     "s_load_dword %6, %10, 0x180\n\ts_load_dword %7, %10, 0x1c0\n\ts_load_dword %8, %10, 0x200\n\t"
                     "s_load_dword %9, %10, 0x230\n\ts_waitcnt lgkmcnt(0)"
                     : "=&s"(d0), "=&s"(d1), "=&s"(d2), "=&s"(d3), "=&s"(d4), "=&s"(d5), "=&s"(d6), "=&s"(d7), "=&s"(d8), "=&s"(d9)
                     : "s"(kp) : "memory");
    }
}
static_assert(sizeof(GemmArgs) <= 0x240 && sizeof(GemmArgs) > 0x230, "warm_kernargs<10> covers GemmArgs");
static_assert(sizeof(RansArgs) <= 0xC0, "warm_kernargs<3> covers RansArgs");

static int launch_status(const char* what) {
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? LBC_OK : set_error(LBC_E_HIP, std::string(what) + " launch failed: " + hipGetErrorString(e));
}

// Launch-span stamps for sampled launches (bench.py's per-kernel roofline).  HIP events cannot be
// recorded inside a captured graph on ROCm 7.2, so the kernels stamp themselves on the constant 100 MHz
// clock: per XCD (the counters of different XCDs need not agree) the earliest workgroup start and the
// latest workgroup end, slot = 8 x {max(~start), max(end)}; slots are zeroed at every graph replay.
__device__ __forceinline__ int xcc_id() {
    int v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
    return v & 7;
}
__device__ __forceinline__ void stamp_start(unsigned long long* ts) {
    if (ts && threadIdx.x == 0)
        atomicMax(ts + 2 * xcc_id(), ~0ull - (unsigned long long)__builtin_amdgcn_s_memrealtime());
}
__device__ __forceinline__ void stamp_end(unsigned long long* ts) {
    if (ts) {
        __syncthreads();
        if (threadIdx.x == 0) atomicMax(ts + 2 * xcc_id() + 1, (unsigned long long)__builtin_amdgcn_s_memrealtime());
    }
}

#ifdef LBIC_PHASE_STAMPS
// diagnostic build only (csrc/microbench.hip): per-workgroup s_memtime at phase boundaries
__device__ unsigned long long* g_phase;
// (launch slot = g.ctr_stride, which the microbenchmark's dense-only launches do not otherwise use)
#define PHASE(i)                                                                                  \
    do {                                                                                          \
        const long ph_ = ((long)g.ctr_stride * 4096 + blockIdx.y * gridDim.x + blockIdx.x) * 8;   \
        if (threadIdx.x == 0) g_phase[ph_ + (i)] = __builtin_amdgcn_s_memtime();                   \
        if (threadIdx.x == 0 && (i) == 0) g_phase[ph_ + 7] = xcc_id();                            \
    } while (0)
#else
#define PHASE(i) do {} while (0)
#endif

#ifdef LBIC_PHASE_DIAG
// diagnostic library build only (make diag -> liblbic_diag.so, LBIC_LIB_VARIANT=diag): sampled k_gemm_s launches
// record, per phase boundary i = 1..4, the max and the sum over workgroups of (s_memtime at i - at kernel start)
// in slot words 16 + i / 24 + i, and the workgroup count in word 31 (lbc_profile_end prints them)
#define DPH(i)                                                                                    \
    do {                                                                                          \
        if (g.ts && threadIdx.x == 0) {                                                           \
            const unsigned long long t_ = __builtin_amdgcn_s_memtime();                           \
            if ((i) == 0) dph0_ = t_;                                                             \
            else {                                                                                \
                atomicMax(g.ts + 16 + (i), t_ - dph0_);                                           \
                atomicAdd(g.ts + 24 + (i), t_ - dph0_);                                           \
                if ((i) == 4) atomicAdd(g.ts + 31, 1ull);                                         \
            }                                                                                     \
        }                                                                                         \
    } while (0)
#else
#define DPH(i) do {} while (0)
#endif

__device__ __forceinline__ int scale_index(float s, const float* table) {
    // build_indexes (entropy_layers_cai.py:649-654): idx = 63 - #{k < 63 : max(s, .11) <= table[k]}
    //   = #{k < 63 : table[k] < s} for an increasing table (the compares are the same float compares).
    // The table is get_scale_table()'s geometric grid, so s's position on it (approximate: a log) leaves the count in a
    // window of four entries, which exact compares settle; the two outer compares prove the window holds the count, and
    // any other table (or a position off by more than one) takes the full count.  One round of 4 (L1-resident) loads
    // instead of 63 loads in 8 rounds.
    s = fmaxf(s, 0.11f);
    const float t0 = table[0], t62 = table[62];
    const float u = __logf(s / t0) / __logf(t62 / t0) * 62.f;
    const int k = (int)floorf(fminf(fmaxf(u, 0.f), 62.f));
    const float tm = table[max(k - 1, 0)], tk = table[k], tp = table[min(k + 1, 62)], tq = table[min(k + 2, 62)];
    if ((k == 0 || tm < s) && (k + 2 > 62 || !(tq < s))) return k + (tk < s ? 1 : 0) + (k + 1 <= 62 && tp < s ? 1 : 0);
    int idx = 63;
#pragma unroll 8
    for (int j = 0; j < 63; ++j) idx -= (s <= table[j]) ? 1 : 0;
    return idx;
}

__device__ __forceinline__ float std_cum(float x) {
    // _standardized_cumulative (entropy_layers_cai.py:569-573)
    return 0.5f * erfcf(-0.70710677f * x);
}

// Plain, or write-through (sc1) / L1-bypassing (sc1) global accesses: the team decoder (k_dec_team) hands every
// value it writes to other workgroups of the same launch (cdna_hip_programming.md §6 Guideline 16, R1).
template <typename T>
using gptr = __attribute__((address_space(1))) T*;
template <bool SC1, typename T>
__device__ __forceinline__ void st(T* p, T v, bool wt = true) {   // wt: (uniform) write through when SC1
    if constexpr (SC1) {
        if (wt) __hip_atomic_store((gptr<T>)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else *(gptr<T>)p = v;
    } else {
        *p = v;
    }
}
template <bool SC1, typename T>
__device__ __forceinline__ T ld(const T* p) {
    if constexpr (SC1) return __hip_atomic_load((gptr<T>)const_cast<T*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else return *p;
}

// Block (img, v, h) of A-row block m: from the block list, or computed for a decoder raster step
// (GemmArgs::raster: img = img0 + m, v = the graph's row counter, h fixed), which saves the kernel one
// dependent global load before its first activation load.
struct BlkSrc {
    const int4* p;
    int raster, img0, v, h;
    __device__ __forceinline__ int4 at(int m) const { return raster ? make_int4(img0 + m, v, h, 0) : p[m]; }
};

// Output element (row, col) of a GEMM from its slice-ordered sum v: bias + the layer's epilogue.  Shared by
// both GEMM kernels so that they compute bit-identical values.
// bcol = bias[col]; xv = the GDN input x[row][col] (GDN / IGDN only), both loaded by the caller.
// DEC: only the decoder's epilogues (the team kernel's instance: EPI_QUANT and EPI_SCATTER compiled out, so the code
// every raster-step operation runs stays small -- the host records decoder GEMMs only and checks it)
template <bool SC1 = false, bool DEC = false>
__device__ __forceinline__ void epilogue(const GemmArgs& g, float v, int row, int col, const BlkSrc& blocks, float bcol,
                                         float xv, bool wt = true) {
    switch (g.epi) {
        case EPI_BIAS:
            st<SC1>(g.out + (long)row * g.ldo + col, v + bcol, wt);
            break;
        case EPI_LEAKY: {
            const float t = v + bcol;
            float o = t > 0.f ? t : t * 0.01f;
            if (g.zero_oob) {    // row = block * P + position; position outside the frame -> 0
                const int m = row / g.P, p = row - m * g.P;
                int dy = 0, dx = 0;
#pragma unroll
                for (int q = 0; q < 5; ++q) {
                    dy = p == q ? g.pos_dy[q] : dy;
                    dx = p == q ? g.pos_dx[q] : dx;
                }
                const int4 b = blocks.at(m);
                const int vv = b.y + dy, hh = b.z + dx;
                if (vv < 0 || vv >= g.geo.Hb || hh < 0 || hh >= g.geo.Wb) o = 0.f;
            }
            st<SC1>(g.out + (long)row * g.ldo + col, o, wt);
            break;
        }
        case EPI_LEAKY_L0: {   // row = block * P + position -> the layer-0 cache cell of that position
            const float t = v + bcol;
            float o = t > 0.f ? t : t * 0.01f;
            const int m = row / g.P, p = row - m * g.P;
            int dy = 0, dx = 0;
#pragma unroll
            for (int q = 0; q < 5; ++q) {
                dy = p == q ? g.pos_dy[q] : dy;
                dx = p == q ? g.pos_dx[q] : dx;
            }
            const int4 b = blocks.at(m);
            const int vv = b.y + dy, hh = b.z + dx;
            if (g.zero_oob && (vv < 0 || vv >= g.geo.Hb || hh < 0 || hh >= g.geo.Wb)) o = 0.f;
            st<SC1>(g.out + (((long)b.x * g.geo.Hp + vv + 2) * g.geo.Wp + hh + 2) * g.ldo + col, o, wt);
            break;
        }
        case EPI_GDN:
        case EPI_IGDN: {
            const float norm = v + bcol;
            const float sq = __fsqrt_rn(norm);
            st<SC1>(g.out + (long)row * g.ldo + col, g.epi == EPI_GDN ? xv * __fdiv_rn(1.0f, sq) : xv * sq, wt);
            break;
        }
        case EPI_QUANT: {
            if constexpr (DEC) break;
            const float y = v + bcol;
            const float scale = g.ksi[(long)row * g.ldk + col];
            const float mean = g.ksi[(long)row * g.ldk + g.Mlat + col];
            const float d = y - mean;
            const int sym = (int)rintf(d);               // torch.round: half to even
            const float yq = (float)sym + mean;
            st<SC1>(g.out + (long)row * g.ldo + col, yq, wt);
            const int4 b = blocks.at(row);
            const long pos = ((long)b.x * g.HW + (long)b.y * g.geo.Wb + b.z) * g.Mlat + col;
            st<SC1>(g.sym + pos, (int32_t)sym, wt);
            st<SC1>(g.idx + pos, (int32_t)(g.table ? scale_index(scale, g.table) : 0), wt);   // no table: forward()/validation before update()
            if (g.bits) {
                const float av = fabsf(yq - mean), sb = fmaxf(scale, 0.11f);
                const float lik = std_cum((0.5f - av) / sb) - std_cum((-0.5f - av) / sb);
                st<SC1>(g.bits + pos, -log2f(fmaxf(lik, 1e-9f)), wt);
            }
            break;
        }
        case EPI_CTXIDX: {
            const float t = v + bcol;
            st<SC1>(g.out + (long)row * g.ldo + col, t, wt);
            if (col < g.Mlat) st<SC1>(g.idx + (long)row * g.Mlat + col, (int32_t)scale_index(t, g.table), wt);
            break;
        }
        case EPI_SCATTER: {   // output row of block (img, v, h) -> out[img][v][h][col] (forward()'s xhat)
            if constexpr (DEC) break;
            const int4 b = blocks.at(row);
            st<SC1>(g.out + ((long)b.x * g.HW + (long)b.y * g.geo.Wb + b.z) * g.ldo + col, v + bcol, wt);
            break;
        }
        case EPI_CLAMPZ: {
            const float t = fminf(fmaxf(v + bcol, -0.5f), 0.5f);
            const int4 b = blocks.at(row);
            st<SC1>(g.geo.zpad + ((long)(b.x * g.geo.Hp + b.y + 2) * g.geo.Wp + b.z + 2) * g.geo.Cx + col, t, wt);
            break;
        }
    }
}

// A / W fragments of one 16-wide k-block for this lane (operand maps: the packing comment in codec.hip)
template <int MS, int NS>
struct Frag {
    f4 a[MS];
    f4 w[NS];
};

constexpr int MAXSEG = 6;

// Source addressing without branches in the k-loop: every lane precomputes, per segment t and row
// subtile s, a 32-bit offset from that segment's base pointer; a k-block then selects its segment with
// uniform compares (SALU) and the offset with v_cndmask, so the compiler never branches around a load (a
// branch per load makes hipcc drain vmcnt(0) each time: cdna_hip_programming.md §5, "Three .s-level traps",
// (c)).  Offsets count float4s (every row offset, tap offset and k-block start is a multiple of 4 floats:
// widths and 3B^2 are padded to 16) and are unsigned: computed in 64 bits, they address 2^32 float4s (64 GB)
// from a base, so a ganged decoder workspace of more than 2^31 floats stays in range at no cost per load.
template <int MS>
struct Rows {
    unsigned off[MAXSEG][MS];
};

template <int MS, int NS>
__device__ __forceinline__ void load_kb(const GemmArgs& g, int kb, int nb0, const Rows<MS>& R, int q4, int lane,
                                        Frag<MS, NS>& f) {
    const int k = kb << 4;
    const float* base = g.seg[0].base;
    int k0 = g.seg[0].k0;
    unsigned o[MS];
#pragma unroll
    for (int s = 0; s < MS; ++s) o[s] = R.off[0][s];
#pragma unroll
    for (int t = 1; t < MAXSEG; ++t) {
        const bool in = k >= g.seg[t].k0;     // wave-uniform (unused segments: k0 past K)
        base = in ? g.seg[t].base : base;
        k0 = in ? g.seg[t].k0 : k0;
#pragma unroll
        for (int s = 0; s < MS; ++s) o[s] = in ? R.off[t][s] : o[s];
    }
    const unsigned kk4 = (unsigned)(k - k0 + q4) >> 2;
#pragma unroll
    for (int s = 0; s < MS; ++s) f.a[s] = reinterpret_cast<const f4*>(base)[o[s] + kk4];
    const f4* Wt = reinterpret_cast<const f4*>(g.W) + lane;
#pragma unroll
    for (int j = 0; j < NS; ++j) f.w[j] = Wt[((long)kb * g.NB16 + nb0 + j) * 64];
}

template <int MS, int NS>
__device__ __forceinline__ void mma_kb(const GemmArgs& g, Frag<MS, NS>& f, f4 (&acc)[MS][NS]) {
    if (g.square_a) {
#pragma unroll
        for (int s = 0; s < MS; ++s) f.a[s] = f.a[s] * f.a[s];
    }
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int s = 0; s < MS; ++s)
#pragma unroll
            for (int j = 0; j < NS; ++j)
                acc[s][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(f.a[s][e], f.w[j][e], acc[s][j], 0, 0, 0);
}

// Small-M GEMM (the decoder's per-step batch, M = n_img rows, and the wavefront's ramp steps): one
// 16 x 16 output tile per workgroup, 8 waves = the 8 K slices, one slice per wave.  Latency-shaped:
// every weight and activation fragment of a slice is requested before the first MFMA (the weights
// first: they need nothing but the kernel arguments), and bias / GDN input of the epilogue at the start
// too, so a launch costs about one memory round trip plus the slice's dependent MFMA chain.  The slice
// length L (k-blocks) is dispatched to a fully unrolled body, so no load sits behind a branch.  Slices,
// chain order and the slice-ordered sum are those of k_gemm: results are bit-identical to it.
typedef const float __attribute__((address_space(1)))* gfloat_p;   // global (not flat) loads

struct SRow {            // per-lane A addressing of every segment, computed once per launch
    gfloat_p base[MAXSEG];
    int k0[MAXSEG];
    unsigned off[MAXSEG];   // float4 offset of this lane's row in segment t, minus k0 (plus q4), mod 2^32 (Rows)
};

// this lane's A row: the row, its block (img, v, h) when a segment or the epilogue needs it, and its
// context position; the block load is issued here and waited for only in small_offsets
struct SBlk {
    int r, dy, dx;
    int4 b;
};

template <bool RASTER>
__device__ __forceinline__ SBlk small_blk(const GemmArgs& g, int m0, int lane, const BlkSrc& blocks) {
    SBlk s;
    s.r = min(m0 + (lane & 15), g.M - 1);
    int m = s.r;
    s.dy = s.dx = 0;
    if (g.P > 1) {
        m = s.r / g.P;
        const int p = s.r - m * g.P;
#pragma unroll
        for (int q = 0; q < 5; ++q) {         // static indices only (a per-lane index would copy g to scratch)
            s.dy = p == q ? g.pos_dy[q] : s.dy;
            s.dx = p == q ? g.pos_dx[q] : s.dx;
        }
    }
    if constexpr (RASTER) s.b = make_int4(blocks.img0 + m, blocks.v, blocks.h, 0);
    else s.b = blocks.p[m];   // unconditional (a branch here costs a full vmcnt drain); unused by dense-only GEMMs
    return s;
}

__device__ __forceinline__ void small_offsets(const GemmArgs& g, const SBlk& k, int lane, SRow& s) {
    const int4 b = k.b;
    const long cell = ((long)b.x * g.geo.Hp + b.y + 2 + k.dy) * g.geo.Wp + b.z + 2 + k.dx;
    const long xrow = (((long)b.x * g.geo.Hb + b.y) * g.geo.Wb + b.z) * g.geo.Cx;
    const int q4 = (lane >> 4) * 4;
#pragma unroll
    for (int t = 0; t < MAXSEG; ++t) {
        const Seg& sg = g.seg[t];
        s.base[t] = (gfloat_p)sg.base;
        s.k0[t] = sg.k0;
        // opaque from here on: the per-k-block selects pick values, not kernel-argument addresses
        // (a selected address would become one dependent scalar load per k-block)
        asm volatile("" : "+s"(s.base[t]), "+s"(s.k0[t]));
        const long o = (long)k.r * sg.ld + sg.zs * cell + (sg.xs ? xrow : 0l) + sg.tap - sg.k0 + q4;
        s.off[t] = (unsigned)(o >> 2);     // may wrap below zero: + k / 4 in small_a lands in range
    }
}

// A fragment of k-block kb (elements kb*16 + q4 .. +3 of this lane's row)
__device__ __forceinline__ f4 small_a(const SRow& rw, int kb) {
    const int k = kb << 4;
    gfloat_p base = rw.base[0];
    unsigned o = rw.off[0];
#pragma unroll
    for (int t = 1; t < MAXSEG; ++t) {
        const bool in = k >= rw.k0[t];     // wave-uniform; unused segments have k0 past K
        base = in ? rw.base[t] : base;
        o = in ? rw.off[t] : o;
    }
    return reinterpret_cast<const f4 __attribute__((address_space(1)))*>(base)[o + (unsigned)(k >> 2)];
}

#ifndef LBIC_RANS_WPB
#define LBIC_RANS_WPB 4   // one wave per SIMD: a lone wave issues its latency-bound chain ~13 % faster than two
#endif
constexpr int RANS_WPB = LBIC_RANS_WPB;   // waves (streams) per workgroup
constexpr int RANS_MAXLAT = 256;          // Mlat <= 4 * 64
constexpr int RANS_WIN = 512;             // stream words staged in LDS per wave and launch (>= 52/32 * MAXLAT)
constexpr int RANS_FILL = 8192 / (RANS_WPB * 64);   // 16-byte table loads per thread in flight (128 KB per pass)

__device__ __forceinline__ uint32_t rdlane(uint32_t v, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, l); }
__device__ __forceinline__ int rdlane_i(int v, int l) { return __builtin_amdgcn_readlane(v, l); }

__device__ __forceinline__ unsigned long long uni64(unsigned long long v) {   // keep a uniform value in SGPRs
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v), hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
    return ((unsigned long long)hi << 32) | lo;
}

#ifdef LBIC_RANS_STAMPS
__device__ unsigned long long* g_rdbg;   // diagnostic build (rans_bench): per wave s_memtime at 4 points
#define RSTAMP(k)                                                                                    \
    do {                                                                                             \
        __builtin_amdgcn_sched_barrier(0);                                                           \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();                                  \
        if (lane == 0 && row_in < a.rows) g_rdbg[row_in * 4 + (k)] = t_;                             \
        __builtin_amdgcn_sched_barrier(0);                                                           \
    } while (0)
#else
#define RSTAMP(k) do {} while (0)
#endif
// ----------------------------------------------------------------------------------------- rANS decode
// One 64-lane wave per stream (reference format: one per image) decodes the Mlat symbols of the current
// block (RansDecoder::decode_stream, called per block at net:439), entirely on the GPU.  Up to 8 streams
// share a workgroup and one LDS copy of the tables (build_rans_gpu_tables: CDF entries stored as c - 1,
// a 64-entry coarse row per table, fine rows padded with 0xFFFF).  The 64-bit state is wave-uniform
// (SGPRs); one wave issues about one instruction per 4 cycles, so the per-symbol body is kept short and
// everything that does not depend on the state is done a symbol ahead:
//   * before the loop, every lane gathers the table metadata of "its" symbols (lane i of chunk kb =
//     symbol 64 kb + i); per symbol the next symbol's metadata is a v_readlane and its coarse row an
//     LDS read issued while the current symbol waits for its own fine read;
//   * level 1: cum against the prefetched coarse row (one compare + popcount) picks a segment of S
//     symbols; level 2: one 64-wide LDS window read from that segment start, compare + popcount gives
//     the symbol, two v_readlanes its interval (a short table, <= 64 entries, has S = 1);
//   * the block's stream words are staged in LDS with the tables; renormalisation takes the next word
//     from there, requested as soon as the previous one is consumed.
// Output: y_qnt = sym + mean (dequantize, entropy_layers_cai.py:159-168, net:440-442).
// Called by every wave of the workgroup (rows past a.rows only help fill the LDS tables): the wave's
// stream state and indexes are requested first, the workgroup then copies the tables into LDS while those
// loads are in flight.
// TEAM (k_dec_team, high rates): the workgroup staged the tables into `lds` once at launch start; only the calling
// wave runs (no table fill, no workgroup barrier), its stream words go to `twin`, the indexes and means come in by
// sc1 loads and y_qnt goes out by st<true> (cdna_hip_programming.md Guideline 16, as rans_row_sparse<true>).
template <bool TEAM = false>
__device__ __forceinline__ void rans_row(const RansArgs& a, uint16_t* lds, int row_in, int lane, uint32_t* twin = nullptr,
                                         bool wt = true) {
    RSTAMP(0);
    const bool valid = row_in < a.rows;
    const int row = valid ? row_in : a.rows - 1;
    // stream / state of this row: the image's (reference format: row = image) or the block row's
    // (sub-stream format, via the block list)
    int img = row;
    if (a.streams_per_img > 1) {
        const int4* blocks = a.ctr ? a.blocks + (long)(*a.ctr) * a.ctr_stride : a.blocks;
        const int4 blk = blocks[row];
        img = blk.x * a.streams_per_img + blk.y;
    }
    img = __builtin_amdgcn_readfirstlane(img);
    const int Mlat = a.Mlat;
    // per-table metadata, lane t holds table t
    const int t_fb = a.tmeta[lane], t_S = a.tmeta[64 + lane], t_lm2 = a.tmeta[128 + lane];
    const int t_ca = a.tmeta[192 + lane], t_off = a.tmeta[256 + lane];
    const unsigned long long x_in = a.state_x[img];
    const int p_in = a.state_ptr[img];
    const long long wb = a.word_base[img];
    const int nw_in = a.word_count[img];
    // table of symbol i (ti) and of symbol i + 1 (tn: the next symbol's metadata is read a symbol ahead)
    int ti[4], tn[4];
    float mv[4];         // the means, requested with the indexes (not after the decode: one round trip less per block)
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
        const int i = kb * 64 + lane;
        // clamped, unconditional loads (indexes are 0..63 by construction; entries past Mlat are unused)
        ti[kb] = ld<TEAM>(a.idx + (long)row * Mlat + min(i, Mlat - 1)) & 63;
        tn[kb] = ld<TEAM>(a.idx + (long)row * Mlat + min(i + 1, Mlat - 1)) & 63;
        mv[kb] = a.sym_out ? 0.f : ld<TEAM>(a.ksi + (long)row * a.ldk + Mlat + min(i, Mlat - 1));
    }
    // LDS staging: the tables (one image built on the host) and this wave's stream words p0 .. p0 +
    // RANS_WIN - 1 (0 past the stream's end; a block never needs more: <= 52 bits per symbol incl. a
    // bypass escape), so renormalisation reads LDS at a uniform address instead of global memory.  The
    // first table chunk is requested before anything waits (it depends on nothing), the words as soon as
    // the stream position has arrived; loads are clamped and unconditional and all issued before the
    // first LDS store (a guarded load, or a load -> store pair per iteration, waits for each in turn).
    const uint4* tsrc = reinterpret_cast<const uint4*>(a.cdf16);
    uint4* tdst = reinterpret_cast<uint4*>(lds);
    const int n16 = a.total16 / 8, bd = blockDim.x;
    uint4 r[TEAM ? 1 : RANS_FILL];
    if constexpr (!TEAM) {
#pragma unroll
        for (int k = 0; k < RANS_FILL; ++k) r[k] = tsrc[min((int)threadIdx.x + k * bd, n16 - 1)];
    }
    unsigned long long x = uni64(x_in);
    int p = __builtin_amdgcn_readfirstlane(p_in);
    const uint32_t* w = a.words + wb;
    const int nw = __builtin_amdgcn_readfirstlane(nw_in);
    const int p0 = p;
    {
        uint32_t* win = TEAM ? twin : reinterpret_cast<uint32_t*>(lds + a.total16) + (threadIdx.x >> 6) * RANS_WIN;
        uint32_t wv[RANS_WIN / 64];
#pragma unroll
        for (int k = 0; k < RANS_WIN / 64; ++k) wv[k] = w[min(p0 + k * 64 + lane, max(nw - 1, 0))];
        if constexpr (!TEAM) {
#pragma unroll
            for (int k = 0; k < RANS_FILL; ++k) tdst[min((int)threadIdx.x + k * bd, n16 - 1)] = r[k];   // past the end: a duplicate
            for (int i0 = threadIdx.x + RANS_FILL * bd; i0 < n16; i0 += RANS_FILL * bd) {   // tables > RANS_FILL chunks
#pragma unroll
                for (int k = 0; k < RANS_FILL; ++k) r[k] = tsrc[min(i0 + k * bd, n16 - 1)];
#pragma unroll
                for (int k = 0; k < RANS_FILL; ++k) tdst[min(i0 + k * bd, n16 - 1)] = r[k];
            }
        }
#pragma unroll
        for (int k = 0; k < RANS_WIN / 64; ++k) win[k * 64 + lane] = p0 + k * 64 + lane < nw ? wv[k] : 0u;
    }
    // symbol-major metadata (gathered from the table lanes): lane i of chunk kb = symbol 64 kb + i + 1
    // (fine row start, S, escape symbol, coarse row start); the offset of symbol 64 kb + i itself
    int nfbv[4], nSv[4], nlmv[4], ncav[4], moff[4], symv[4];
    int fb, S, lm2, ca0;
    {
        const int sel0 = __builtin_amdgcn_readfirstlane(ti[0]);
        fb = rdlane_i(t_fb, sel0); S = rdlane_i(t_S, sel0); lm2 = rdlane_i(t_lm2, sel0); ca0 = rdlane_i(t_ca, sel0);
    }
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
        const int sel = tn[kb] << 2;
        nfbv[kb] = __builtin_amdgcn_ds_bpermute(sel, t_fb);
        nSv[kb] = __builtin_amdgcn_ds_bpermute(sel, t_S);
        nlmv[kb] = __builtin_amdgcn_ds_bpermute(sel, t_lm2);
        ncav[kb] = __builtin_amdgcn_ds_bpermute(sel, t_ca);
        moff[kb] = __builtin_amdgcn_ds_bpermute(ti[kb] << 2, t_off);
        symv[kb] = 0;
    }
    if constexpr (TEAM) {
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the window is in LDS (this wave's own writes)
        __builtin_amdgcn_wave_barrier();
    } else {
        __syncthreads();
    }
    if (!valid) return;
    RSTAMP(1);
    int bad = 0;
    const uint32_t* win = TEAM ? twin : reinterpret_cast<const uint32_t*>(lds + a.total16) + (threadIdx.x >> 6) * RANS_WIN;
    // words q0 .. q0 + 63 of the LDS window lane-distributed in a register; wn = the word renormalisation
    // takes next (a v_readlane, prepared as soon as the previous word is consumed)
    int q0 = 0;
    uint32_t wbuf = win[lane];
    uint32_t wn = rdlane(wbuf, 0);
    auto renorm = [&]() {
        uint32_t t = (uint32_t)(x >> 32) | ((uint32_t)x >> 31);   // 0 <=> x < RANS64_L = 2^31
        asm("" : "+s"(t));               // keep the test on the scalar unit (not a 64-bit VALU compare)
        if (t == 0) {
            x = (x << 32) | wn;
            ++p;
            if (p - p0 - q0 >= 64) {     // next 64 words (rare: a stall of one LDS read)
                q0 = min(q0 + 64, RANS_WIN - 64);
                wbuf = win[q0 + lane];
            }
            wn = rdlane(wbuf, min(p - p0 - q0, 63));
        }
        x = uni64(x);
    };
    const char* lb = reinterpret_cast<const char*>(lds);
    const int lane2 = lane * 2;
    uint32_t cv = *reinterpret_cast<const uint16_t*>(lb + ca0 + lane2);   // coarse row of symbol 0
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
        const int cnt_i = __builtin_amdgcn_readfirstlane(min(64, Mlat - kb * 64));
        if (cnt_i <= 0) break;
        for (int ii = 0; ii < cnt_i; ++ii) {
            const uint32_t cum = (uint32_t)x & 0xffffu;
            // level 1: segment j (coarse lane 0 is never counted: j = #entries <= cum, minus one)
            const int j = __popcll(__ballot(cv < cum));
            const int sbb = j * S;                  // segment start (bytes; fb and S are in bytes)
            const uint32_t fine = *reinterpret_cast<const uint16_t*>(lb + fb + sbb + lane2);
            // next symbol's metadata and coarse row, in the shadow of the fine read
            const int nfb = rdlane_i(nfbv[kb], ii), nS = rdlane_i(nSv[kb], ii);
            const int nlm2 = rdlane_i(nlmv[kb], ii), nca = rdlane_i(ncav[kb], ii);
            const uint32_t cvn = *reinterpret_cast<const uint16_t*>(lb + nca + lane2);
            __builtin_amdgcn_sched_barrier(0);   // both LDS reads issued before the fine read is waited for
            // level 2: the window from the segment start (lane 0 is <= cum by construction; a short
            // table has S = 1, so its window always answers kk = 0)
            const int kk = __popcll(__ballot(fine < cum) | 1ull) - 1;
            const int s = (sbb >> 1) + kk;
            const uint32_t start = (rdlane(fine, kk) + 1u) & 0xffffu;   // e + 1 = c (the c = 0 entry wraps)
            const uint32_t nxt = rdlane(fine, kk + 1) + 1u;
            x = (unsigned long long)(nxt - start) * (x >> 16) + (cum - start);
            renorm();
            int v = s;
            if (__builtin_expect(s == lm2, 0)) {   // escape: value coded in 4-bit bypass chunks
                auto get_bits = [&]() -> uint32_t {
                    const uint32_t b = (uint32_t)(x & 15u);
                    x >>= 4;
                    renorm();
                    return b;
                };
                uint32_t cc = get_bits(), nb = cc;
                while (cc == 15u && nb <= 8) { cc = get_bits(); nb += cc; }
                if (nb > 8) { bad |= 4; nb = 0; }
                uint32_t raw = 0;
                for (uint32_t jj = 0; jj < nb; ++jj) raw |= get_bits() << (jj * 4);
                v = (int)(raw >> 1);
                v = (raw & 1) ? -v - 1 : v + lm2;
            }
            symv[kb] = lane == ii ? v : symv[kb];
            fb = nfb; S = nS; lm2 = nlm2; cv = cvn;
        }
    }
    RSTAMP(2);
    bad |= p > nw;                       // consumed words past the end of the stream
    bad |= (p - p0 > RANS_WIN) ? 8 : 0;  // (cannot happen: <= 52 bits per symbol)
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
        const int i = kb * 64 + lane;
        if (i < Mlat) {
            if (a.sym_out) a.sym_out[(long)row * Mlat + i] = symv[kb] + moff[kb];
            else st<TEAM>(a.yq + (long)row * a.ldy + i, (float)(symv[kb] + moff[kb]) + mv[kb], wt);
        }
    }
    if (lane == 0) {
        a.state_x[img] = x;
        a.state_ptr[img] = p;
        if (bad) a.status[img] = bad;
    }
    RSTAMP(3);
}

// Sparse variant (low rates: almost every symbol is the most probable one, value 0).  No table image in LDS:
// per symbol ONE compare of cum against the centre interval [lo, lo + freq) of the symbol's table (tmeta row
// 5, gathered into a lane-per-symbol register in the prologue) decides; a hit costs the 64-bit state update
// and nothing else.  A miss compares against the intervals of values -1 and +1 (rows 6 and 7, SALU only), then
// runs the two-level search of rans_row on the table image in global memory (the 70 KB image stays L2-resident:
// every launch of every decoder reads it).  The prologue therefore needs only
// the stream state, the block's indexes and the stream words -- no 70 KB LDS fill and no workgroup barrier
// for it -- and each wave is independent.  Bit-identical to rans_row (same coder, same tables).
// SC1: inside k_dec_team (indexes and means from the context net's workgroups by sc1 loads, y_qnt to the decoder's
// workgroups by sc1 stores, plain ones when wt is false: the whole team shares one L2)
// PERSIST (k_dec_team, a workgroup that decodes the same single image at every raster step): the coder state (x, p),
// the window base, the stream's word range and the table metadata stay in an LDS cache `lc` ([0..1] x, [2] p, [3] the
// window's first word, [4] valid, [5..6] word base, [7] word count, [64..575] tmeta) between the raster steps, and the
// window is refilled from global memory only when fewer words than one block can consume remain in it: the step's
// only global reads are then the block's scale indexes (written by the context net this step).
// LOCAL (k_dec_one): the scale indexes, the context output (scales | means, stride 2 Mlat) and y_qnt are the caller's LDS
// arrays lidx / lksi / lyq of ONE row instead of a.idx / a.ksi / a.yq
template <bool SC1 = false, bool PERSIST = false, bool LOCAL = false>
__device__ __forceinline__ void rans_row_sparse(const RansArgs& a, uint32_t* lwin, int row_in, int lane, bool wt = true,
                                                const uint16_t* tab = nullptr, uint32_t* lc = nullptr,
                                                const int32_t* lidx = nullptr, const float* lksi = nullptr,
                                                float* lyq = nullptr, unsigned long long* rts = nullptr,
                                                uint32_t* llf = nullptr) {
    RSTAMP(0);
    unsigned long long rt1 = 0, rt2 = 0;     // (rts: prologue done, symbols done; written at the end)
    uint32_t n_brk = 0, n_pm1 = 0, n_srch = 0;   // (rts: speculation breaks, +-1 symbols, searched symbols)
    const bool valid = row_in < a.rows;
    const int row = valid ? row_in : a.rows - 1;
    int img = row;
    if (a.streams_per_img > 1) {
        const int4* blocks = a.ctr ? a.blocks + (long)(*a.ctr) * a.ctr_stride : a.blocks;
        const int4 blk = blocks[row];
        img = blk.x * a.streams_per_img + blk.y;
    }
    img = __builtin_amdgcn_readfirstlane(img);
    const int Mlat = a.Mlat;
    int ti[4];
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
        ti[kb] = (LOCAL ? lidx[min(kb * 64 + lane, Mlat - 1)] : ld<SC1>(a.idx + (long)row * Mlat + min(kb * 64 + lane, Mlat - 1))) & 63;
    // the means (y_qnt = symbol + mean) requested with the indexes, not after the decode: the context net wrote both
    // in the same epilogue, and a load issued at the end would add a memory round trip to every block
    float mv[4];
    if (LOCAL || !a.sym_out) {
#pragma unroll
        for (int kb = 0; kb < 4; ++kb) {
            const int i = min(kb * 64 + lane, Mlat - 1);
            mv[kb] = LOCAL ? lksi[Mlat + i] : ld<SC1>(a.ksi + (long)row * a.ldk + Mlat + i);
        }
    } else {
#pragma unroll
        for (int kb = 0; kb < 4; ++kb) mv[kb] = 0.f;
    }
    int t_fb, t_S, t_lm2, t_ca, t_off, t_lf, t_lfm, t_lfp;
    unsigned long long x;
    int p, nw, p0;
    long long wb;
    bool have = false;
    if constexpr (PERSIST) have = __builtin_amdgcn_readfirstlane((int)lc[4]) == 1;
    if (have) {
        t_fb = (int)lc[64 + lane]; t_S = (int)lc[128 + lane]; t_lm2 = (int)lc[192 + lane]; t_ca = (int)lc[256 + lane];
        t_off = (int)lc[320 + lane]; t_lf = (int)lc[384 + lane]; t_lfm = (int)lc[448 + lane]; t_lfp = (int)lc[512 + lane];
        x = uni64(((unsigned long long)lc[1] << 32) | lc[0]);
        p = __builtin_amdgcn_readfirstlane((int)lc[2]);
        p0 = __builtin_amdgcn_readfirstlane((int)lc[3]);
        wb = (long long)(((unsigned long long)(uint32_t)__builtin_amdgcn_readfirstlane((int)lc[6]) << 32) |
                         (uint32_t)__builtin_amdgcn_readfirstlane((int)lc[5]));
        nw = __builtin_amdgcn_readfirstlane((int)lc[7]);
    } else {
        t_fb = a.tmeta[lane]; t_S = a.tmeta[64 + lane]; t_lm2 = a.tmeta[128 + lane];
        t_ca = a.tmeta[192 + lane]; t_off = a.tmeta[256 + lane]; t_lf = a.tmeta[320 + lane];
        t_lfm = a.tmeta[384 + lane]; t_lfp = a.tmeta[448 + lane];
        const unsigned long long x_in = a.state_x[img];
        const int p_in = a.state_ptr[img];
        wb = a.word_base[img];
        const int nw_in = a.word_count[img];
        x = uni64(x_in);
        p = __builtin_amdgcn_readfirstlane(p_in);
        nw = __builtin_amdgcn_readfirstlane(nw_in);
        p0 = p;
    }
    const uint32_t* w = a.words + wb;
    // (re)fill the window from p: always without the cache, with it once fewer words remain than a block can take
    // (<= 52 bits per symbol incl. a bypass escape)
    if (!have || p - p0 > RANS_WIN - (52 * Mlat + 31) / 32 - 2) {
        p0 = p;
        uint32_t wv[RANS_WIN / 64];
#pragma unroll
        for (int k = 0; k < RANS_WIN / 64; ++k) wv[k] = w[min(p0 + k * 64 + lane, max(nw - 1, 0))];
#pragma unroll
        for (int k = 0; k < RANS_WIN / 64; ++k) lwin[k * 64 + lane] = p0 + k * 64 + lane < nw ? wv[k] : 0u;
    }
    // lane i of chunk kb = symbol 64 kb + i: its centre interval (lo, freq), table metadata and offset
    int lov[4], frv[4], ivm[4], ivp[4], sfb[4], sS[4], slm[4], sca[4], moff[4], symv[4];
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
        if (kb * 64 >= Mlat) {           // (uniform) no symbols in this chunk: skip its nine gathers
            lov[kb] = frv[kb] = ivm[kb] = ivp[kb] = sfb[kb] = sS[kb] = slm[kb] = sca[kb] = moff[kb] = symv[kb] = 0;
            continue;
        }
        const int sel = ti[kb] << 2;
        const int lf = __builtin_amdgcn_ds_bpermute(sel, t_lf);
        if (llf) llf[kb * 64 + lane] = (uint32_t)lf;     // (symbol-ordered centre intervals for the vector runs)
        lov[kb] = lf & 0xffff;
        frv[kb] = (int)((uint32_t)lf >> 16);
        ivm[kb] = __builtin_amdgcn_ds_bpermute(sel, t_lfm);
        ivp[kb] = __builtin_amdgcn_ds_bpermute(sel, t_lfp);
        sfb[kb] = __builtin_amdgcn_ds_bpermute(sel, t_fb);
        sS[kb] = __builtin_amdgcn_ds_bpermute(sel, t_S);
        slm[kb] = __builtin_amdgcn_ds_bpermute(sel, t_lm2);
        sca[kb] = __builtin_amdgcn_ds_bpermute(sel, t_ca);
        moff[kb] = __builtin_amdgcn_ds_bpermute(sel, t_off);
        symv[kb] = -moff[kb];            // the centre symbol's index (value 0)
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the window is in LDS (this wave's own writes)
    __builtin_amdgcn_wave_barrier();
    if (!valid) return;
    RSTAMP(1);
    if (rts) rt1 = __builtin_amdgcn_s_memrealtime();
    // every table's centre frequency <= 65534 (a table with a single-value pmf has 65535: then every step is tested).
    // Measured (round 4, profiles/r04_onecheck.txt): rANS operation 9.5-9.7 -> 9.2-9.4 us, decode alone -1.4 %.
    const bool one_check = __ballot(((uint32_t)t_lf >> 16) > 65534u) == 0ull;
    int bad = 0;
    // the 64-word chunk of the window that holds word p (p0: the window's first word)
    int q0 = min((p - p0) & ~63, RANS_WIN - 64);
    uint32_t wbuf = lwin[q0 + lane];
    uint32_t wn = rdlane(wbuf, min(p - p0 - q0, 63));
    auto renorm_slow = [&]() {           // x < 2^31: shift in the next stream word
        x = (x << 32) | wn;
        ++p;
        if (p - p0 - q0 >= 64) {
            q0 = min(q0 + 64, RANS_WIN - 64);
            wbuf = lwin[q0 + lane];
        }
        wn = rdlane(wbuf, min(p - p0 - q0, 63));
    };
    auto renorm = [&]() {
        uint32_t t = (uint32_t)(x >> 32) | ((uint32_t)x >> 31);   // 0 <=> x < RANS64_L = 2^31
        asm("" : "+s"(t));
        if (t == 0) renorm_slow();
        x = uni64(x);
    };
    const uint16_t* img16 = tab ? tab : a.cdf16;     // tab: a copy of the table image in LDS (k_dec_team<2>)
    const int lane2 = lane * 2;
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
        const int cnt_i = __builtin_amdgcn_readfirstlane(min(64, Mlat - kb * 64));
        if (cnt_i <= 0) break;
        // one most-probable symbol: a compare, the 64-bit state update, a (rare) renormalisation
        auto fast = [&](uint32_t lo, uint32_t fr) -> bool {
            const uint32_t d = ((uint32_t)x & 0xffffu) - lo;
            if (d >= fr) return false;
            x = (unsigned long long)fr * (x >> 16) + d;
            const uint32_t t = (uint32_t)(x >> 32) | ((uint32_t)x >> 31);
            if (__builtin_expect(t == 0, 0)) renorm_slow();
            return true;
        };
        // one centre step of the state, no test: the caller checks d < fr and the renormalisation bound afterwards
        auto step = [](unsigned long long xv, uint32_t lo, uint32_t fr, uint32_t& bad) -> unsigned long long {
            const uint32_t d = ((uint32_t)xv & 0xffffu) - lo;
            bad |= d >= fr ? 1u : 0u;
            const unsigned long long xn = (unsigned long long)fr * (xv >> 16) + d;
            bad |= ((uint32_t)(xn >> 32) | ((uint32_t)xn >> 31)) == 0u ? 1u : 0u;   // x < 2^31: renormalise
            return xn;
        };
        // the same without the renormalisation test (one_check: the caller tests the last of four states)
        auto step_nr = [](unsigned long long xv, uint32_t lo, uint32_t fr, uint32_t& bad) -> unsigned long long {
            const uint32_t d = ((uint32_t)xv & 0xffffu) - lo;
            bad |= d >= fr ? 1u : 0u;
            return (unsigned long long)fr * (xv >> 16) + d;
        };
        int ii = 0;
        while (ii < cnt_i) {
            // runs of most-probable symbols, 4 per iteration, speculatively: the 8 interval reads (v_readlane,
            // independent of the state) first, then 4 state updates with no branch between them, one test at the end
            // (a symbol outside its centre interval or a renormalisation anywhere in the four); on a hit the four are
            // committed, otherwise the state is restored and the careful loop below decodes them one by one.
            // one_check: no centre frequency above 65534, so a state that falls below 2^31 stays below it through
            // further centre steps (fr (x >> 16) + d < 65534 * 2^15 + 65534 < 2^31): testing the fourth state covers all
            // four renormalisation conditions
            auto spec = [&](auto one_tag) {
                constexpr bool ONE = decltype(one_tag)::value;
                while (ii + 4 <= cnt_i) {
                    const uint32_t l0 = rdlane((uint32_t)lov[kb], ii), f0 = rdlane((uint32_t)frv[kb], ii);
                    const uint32_t l1 = rdlane((uint32_t)lov[kb], ii + 1), f1 = rdlane((uint32_t)frv[kb], ii + 1);
                    const uint32_t l2 = rdlane((uint32_t)lov[kb], ii + 2), f2 = rdlane((uint32_t)frv[kb], ii + 2);
                    const uint32_t l3 = rdlane((uint32_t)lov[kb], ii + 3), f3 = rdlane((uint32_t)frv[kb], ii + 3);
                    uint32_t bad = 0;
                    unsigned long long xv;
                    if constexpr (ONE) {
                        xv = step_nr(x, l0, f0, bad);
                        xv = step_nr(xv, l1, f1, bad);
                        xv = step_nr(xv, l2, f2, bad);
                        xv = step_nr(xv, l3, f3, bad);
                        bad |= ((uint32_t)(xv >> 32) | ((uint32_t)xv >> 31)) == 0u ? 1u : 0u;
                    } else {
                        xv = step(x, l0, f0, bad);
                        xv = step(xv, l1, f1, bad);
                        xv = step(xv, l2, f2, bad);
                        xv = step(xv, l3, f3, bad);
                    }
                    if (__builtin_amdgcn_readfirstlane(bad)) {
                        if (rts) ++n_brk;
                        break;
                    }
                    x = uni64(xv);
                    ii += 4;
                }
            };
            // llf (k_dec_one) and one_check: the same runs with the state in a VGPR (every lane the same value) and the
            // four intervals as broadcast LDS reads, a group ahead -- the state chain then runs on the vector ALU
            // (v_mad_u64_u32) instead of a 16-instruction scalar sequence per symbol, and no v_readlane waits
            if (llf && one_check) {
                if (ii + 4 <= cnt_i) {
                    unsigned long long xv = x;
                    asm volatile("" : "+v"(xv));
                    const uint32_t* lb = llf + kb * 64;
                    uint32_t q0 = lb[ii], q1 = lb[ii + 1], q2 = lb[ii + 2], q3 = lb[ii + 3];
                    while (true) {
                        const int nx = min(ii + 4, 60);
                        uint32_t n0 = lb[nx], n1 = lb[nx + 1], n2 = lb[nx + 2], n3 = lb[nx + 3];
                        asm volatile("" : "+v"(q0), "+v"(q1), "+v"(q2), "+v"(q3));
                        uint32_t bad = 0;
                        unsigned long long y = step_nr(xv, q0 & 0xffffu, q0 >> 16, bad);
                        y = step_nr(y, q1 & 0xffffu, q1 >> 16, bad);
                        y = step_nr(y, q2 & 0xffffu, q2 >> 16, bad);
                        y = step_nr(y, q3 & 0xffffu, q3 >> 16, bad);
                        bad |= ((uint32_t)(y >> 32) | ((uint32_t)y >> 31)) == 0u ? 1u : 0u;
                        if (__ballot(bad != 0u) != 0ull) {
                            if (rts) ++n_brk;
                            break;
                        }
                        xv = y;
                        ii += 4;
                        if (ii + 4 > cnt_i) break;
                        q0 = n0; q1 = n1; q2 = n2; q3 = n3;
                    }
                    x = uni64(((unsigned long long)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(xv >> 32)) << 32) |
                              (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)xv));
                }
            } else if (one_check) spec(std::true_type{});
            else spec(std::false_type{});
            while (ii < cnt_i && fast(rdlane((uint32_t)lov[kb], ii), rdlane((uint32_t)frv[kb], ii))) ++ii;
            if (ii >= cnt_i) break;
            const uint32_t cum = (uint32_t)x & 0xffffu;
            // value -1 or +1 (most of the misses): two more interval compares, no memory access
            {
                const uint32_t im = rdlane((uint32_t)ivm[kb], ii), ip = rdlane((uint32_t)ivp[kb], ii);
                const uint32_t dm = cum - (im & 0xffffu), dp = cum - (ip & 0xffffu);
                const bool hm = dm < (im >> 16), hp = dp < (ip >> 16);
                if (hm || hp) {
                    if (rts) ++n_pm1;
                    const uint32_t fr = hm ? im >> 16 : ip >> 16, d = hm ? dm : dp;
                    x = (unsigned long long)fr * (x >> 16) + d;
                    renorm();
                    symv[kb] = lane == ii ? symv[kb] + (hm ? -1 : 1) : symv[kb];
                    ++ii;
                    continue;
                }
            }
            // another symbol: the two-level search of rans_row on the table image in global memory
            if (rts) ++n_srch;
            const int fb = rdlane_i(sfb[kb], ii), S = rdlane_i(sS[kb], ii);
            const int lm2 = rdlane_i(slm[kb], ii), ca = rdlane_i(sca[kb], ii);
            const uint32_t cv = *reinterpret_cast<const uint16_t*>(reinterpret_cast<const char*>(img16) + ca + lane2);
            const int j = __popcll(__ballot(cv < cum));
            const int sbb = j * S;
            const uint32_t fine = *reinterpret_cast<const uint16_t*>(reinterpret_cast<const char*>(img16) + fb + sbb + lane2);
            const int kk = __popcll(__ballot(fine < cum) | 1ull) - 1;
            const int sidx = (sbb >> 1) + kk;
            const uint32_t start = (rdlane(fine, kk) + 1u) & 0xffffu;
            const uint32_t nxt = rdlane(fine, kk + 1) + 1u;
            x = (unsigned long long)(nxt - start) * (x >> 16) + (cum - start);
            renorm();
            int v = sidx;
            if (__builtin_expect(sidx == lm2, 0)) {   // escape: value coded in 4-bit bypass chunks
                auto get_bits = [&]() -> uint32_t {
                    const uint32_t b = (uint32_t)(x & 15u);
                    x >>= 4;
                    renorm();
                    return b;
                };
                uint32_t cc = get_bits(), nb = cc;
                while (cc == 15u && nb <= 8) { cc = get_bits(); nb += cc; }
                if (nb > 8) { bad |= 4; nb = 0; }
                uint32_t raw = 0;
                for (uint32_t jj = 0; jj < nb; ++jj) raw |= get_bits() << (jj * 4);
                v = (int)(raw >> 1);
                v = (raw & 1) ? -v - 1 : v + lm2;
            }
            symv[kb] = lane == ii ? v : symv[kb];
            ++ii;
        }
    }
    RSTAMP(2);
    if (rts) rt2 = __builtin_amdgcn_s_memrealtime();
    bad |= p > nw;
    bad |= (p - p0 > RANS_WIN) ? 8 : 0;
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
        const int i = kb * 64 + lane;
        if (i < Mlat) {
            if constexpr (LOCAL) lyq[i] = (float)(symv[kb] + moff[kb]) + mv[kb];
            else if (a.sym_out) a.sym_out[(long)row * Mlat + i] = symv[kb] + moff[kb];
            else st<SC1>(a.yq + (long)row * a.ldy + i, (float)(symv[kb] + moff[kb]) + mv[kb], wt);
        }
    }
    if (lane == 0) {
        a.state_x[img] = x;
        a.state_ptr[img] = p;
        if (bad) a.status[img] = bad;
    }
    if constexpr (PERSIST) {
        if (!have) {
            lc[64 + lane] = (uint32_t)t_fb; lc[128 + lane] = (uint32_t)t_S; lc[192 + lane] = (uint32_t)t_lm2;
            lc[256 + lane] = (uint32_t)t_ca; lc[320 + lane] = (uint32_t)t_off; lc[384 + lane] = (uint32_t)t_lf;
            lc[448 + lane] = (uint32_t)t_lfm; lc[512 + lane] = (uint32_t)t_lfp;
            if (lane == 0) {
                lc[5] = (uint32_t)wb;
                lc[6] = (uint32_t)((unsigned long long)wb >> 32);
                lc[7] = (uint32_t)nw;
            }
        }
        if (lane == 0) {
            lc[0] = (uint32_t)x;
            lc[1] = (uint32_t)(x >> 32);
            lc[2] = (uint32_t)p;
            lc[3] = (uint32_t)p0;
            lc[4] = 1u;
        }
    }
    if (rts && lane == 0) {
        rts[0] = rt1;
        rts[1] = rt2;
        rts[2] = n_brk;
        rts[3] = n_pm1;
        rts[4] = n_srch;
    }
    RSTAMP(3);
}


}  // namespace lbic
