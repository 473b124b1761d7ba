// Kernel argument blocks and launchers (kernels.hip).  Device-side data layout:
//   x     [n_img][Hb][Wb][Cx]            fp32, block-major (Cx = 3 B^2)
//   zpad  [n_img][Hb+2][Wb+4][Cx]        fp32 reconstruction with a zero border: block (v,h) at
//                                        [v+2][h+2]; rows -2,-1 and columns -2,-1,Wb,Wb+1 stay zero, so
//                                        every window gather of the reference (zero pad outside the
//                                        frame, net:342-351) is a plain load.
//   W     [K/16][N/16][4][16][4]         packed fp32 weights of one GEMM (see pack_weights in codec.hip)
//   acts  [rows][width]                  per-step activations, row = block (or block x position)
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace lbic {

constexpr int KSPLIT = 8;   // every GEMM output = ((s0 + s1) + ... + s7) + bias, s_i = k-ordered fma chain
                            // over the i-th eighth of K: identical for every tile shape, so the encoder
                            // (large wavefront M) and the decoder (M = n_img) compute bit-identical values.

// SEG_L0TAP: a cell of the context net's layer-0 map cache (KS[1] = 3; codec.hip, "layer-0 map cache"), laid
// out like zpad ([n_img][Hb+2][Wb+4] cells) with the layer-0 width per cell
enum SegKind : int { SEG_DENSE = 0, SEG_ZTAP = 1, SEG_X = 2, SEG_L0TAP = 3 };
// EPI_LEAKY_L0: LeakyReLU, written to the layer-0 map cache cell of the row's (block, position) instead of row-major
enum Epi : int { EPI_BIAS = 0, EPI_LEAKY, EPI_GDN, EPI_IGDN, EPI_QUANT, EPI_CTXIDX, EPI_CLAMPZ, EPI_SCATTER, EPI_LEAKY_L0 };

struct Seg {                 // one K-range of the A operand: K columns [k0, k1)
    const float* base;       // SEG_DENSE: activations base
    int kind;
    int ld;                  // SEG_DENSE row stride; SEG_L0TAP cell width (floats)
    int dy, dx;              // SEG_ZTAP / SEG_L0TAP: tap offset relative to the output position
    int k0, k1;
    int zs, xs, tap;         // set by launch_gemm: row offset = r*ld + zs*cell + xs*xrow + tap (no branches), cell =
                             // the zpad-geometry cell index of the row's position, zs = that segment's cell width
};

struct Geo {
    float* zpad;
    int Hp, Wp, Cx;
    const float* x;
    int Hb, Wb;
};

struct GemmArgs {
    int M, N, K, P;          // P: A rows per block (context layer 0 positions); rows = blocks * P
    int nseg;
    Seg seg[6];
    int pos_dy[5], pos_dx[5];
    const int4* blocks;      // per block (img, v, h, 0); row r belongs to block r / P
    const int* ctr;          // optional device counter: blocks += *ctr * ctr_stride (graph replays per row)
    int ctr_stride;
    int reserved0;           // (unused; keeps the argument block's layout)
    int raster;              // decoder raster step (needs ctr): the block of row r is (raster_img0 + r / P,
    int raster_img0, raster_h;   // *ctr, raster_h), computed instead of loaded from `blocks`
    unsigned long long* ts;  // optional timing slot {max(~start), max(end)} in s_memrealtime ticks (100 MHz)
    const float* W;
    int NB16;                // N padded / 16
    const float* bias;       // bias (beta for GDN)
    int epi, square_a;
    int need_blocks;         // set by launch_gemm: a z-tap / x segment or a scattering epilogue
    float* out;
    int ldo;
    const float* gx;         // GDN: the layer input x (epilogue x * rsqrt(norm))
    int ldx;
    const float* ksi;        // EPI_QUANT: context output [rows][2*Mlat] (scales | means)
    int ldk, Mlat;
    const float* table;      // scale table (64)
    int32_t* sym;            // EPI_QUANT: [n_img][HW*Mlat]; EPI_CTXIDX: idx_ws [rows][Mlat] in `idx`
    int32_t* idx;
    float* bits;
    int HW;
    Geo geo;
    int lds_floor;           // k_gemm: LDS bytes to reserve per workgroup (caps residency, lbc_set_option)
    int zero_oob;            // EPI_LEAKY: rows whose context position lies outside the frame are written as 0
                             // (forward()'s zero padding of the layer-0 map, KS[1] = 3)
};

struct RansArgs {
    const uint16_t* cdf16;   // LDS image of the tables (build_rans_gpu_tables: coarse rows, then padded
                             // fine rows, entries stored as cdf - 1)
    const int* tmeta;        // [8][64] per table: fine row start, 2 S (S = symbols per coarse lane), cdf_length - 2,
                             // coarse row start (starts in bytes of the image), offset (-pmf_center), intervals
                             // of the value 0, -1, +1 symbols packed lo | freq << 16
    int total16;             // entries in cdf16 (multiple of 8)
    const uint32_t* words;   // concatenated streams
    const long long* word_base;
    const int* word_count;
    unsigned long long* state_x;
    int* state_ptr;
    int* status;             // non-zero: stream overrun / bad index (per image)
    const int32_t* idx;      // [rows][Mlat]
    const float* ksi;
    int ldk, Mlat;
    float* yq;
    int ldy;
    int32_t* sym_out;        // non-null: write the decoded symbols [rows][Mlat] instead of y_qnt
    const int4* blocks;
    const int* ctr;
    int ctr_stride;
    unsigned long long* ts;
    int rows;
    int streams_per_img;     // 1: one stream per image (reference format); Hb: one per block row (sub-stream format)
    int sparse;              // 1: k_rans_decode_sparse (centre-interval fast path, tables read from global memory)
};

// Team decoder (k_dec_team, team.hip): the raster decodes of T <= 8 batches in ONE persistent launch, S workgroups
// per batch ("team", the workgroups of one blockIdx % 8 slot), team barriers between the recorded operations of a raster step instead of kernel boundaries
constexpr int TEAM_SLOTS = 8;      // XCD slots of a launch (blockIdx % 8: one XCD each under round-robin placement)
constexpr int TEAM_MAX = 16;       // teams per launch: up to two per slot (TeamArgs::sub)
constexpr int TEAM_MAXOPS = 24;    // operations per raster step
constexpr int TEAM_TS_WORDS = 1024;   // stamp words per team (TeamArgs::ts)
constexpr int TEAM_NI_MAX = 10;    // output tiles per workgroup and GEMM on the team kernel's fast path (64 images per
                                   // team: the context net's N = 1,152 layer deals 9 to a workgroup)
struct TeamArgs {
    const GemmArgs* gemm;    // [T][3][NG] prepared GEMMs of one raster step, per team and column class
                             // (0: h = 0, 1: 0 < h < Wb - 1, 2: h = Wb - 1); block rows / columns set in-kernel
    const RansArgs* rans;    // [T] (one stream per image)
    int opk[TEAM_MAXOPS];    // the step: >= 0 a GEMM index, -1 the rANS decode
    int nops, NG, T, S, Hb, Wb;
    unsigned* sync;          // [T][32]: per team [0] arrival counter, [1] XCD census (one 128-byte line each), then
                             // [T * 32] the failure word (1 timeout, 2 a team spans XCDs) and [T * 32 + 1] the
                             // census barrier; zeroed before every launch
    int plain;               // 1: plain hand-off stores (needs every team on one XCD: checked in-kernel)
    int ni_max;              // most output tiles one workgroup computes in one GEMM of the step (LDS for partials)
    int split_op, split_wy;  // split_op >= 0: the GEMM after the rANS decode; its K slices w < split_wy (no y_qnt)
                             // run beside the rANS decode, the rest after it
    unsigned long long tmo;  // s_memrealtime ticks (100 MHz) one barrier waits before the launch gives up
    unsigned long long* ts;  // optional [T][TEAM_TS_WORDS]: s_memrealtime after every barrier of raster step (sv, sh), then
                             // [256 + 64 op + p] s_memtime inside its GEMMs (team_gemm_items, rank 0)
    int sv, sh;
    int dense;               // 1: the streams average >= 1 bit per symbol (high rates): every workgroup stages the
                             // rANS tables in its LDS once at launch start and the rANS operation runs rans_row<true>
                             // on them; 0: rans_row_sparse (centre intervals, tables from global memory)
    int tab16;               // entries of the table image (RansArgs::total16; the dense variant's LDS)
    int spread;              // XCD slots per team P: 1, 2, 4 or 8 (T <= 8 / P: team t = the workgroups on slots P t ..
                             // P t + P - 1, S ranks over P XCDs; P > 1: hand-offs write-through, plain = 0)
    int sub;                 // teams per XCD slot (1, or 2 when T > 8: team slot + 8 q = the slot's workgroups
                             // q S .. q S + S - 1 in launch order; spread = 1)
    int nrw;                 // rANS waves per workgroup (1 or 2: images per team up to S or 2 S decode side by side,
                             // wave i the rows rank + i S, rank + (i + nrw) S, ...)
    int rows0;               // A rows of the step's usual GEMM (the images of a team): its row-tile quotients are
                             // computed once per launch
};
// the team kernel's fast GEMM path (team_gemm_items) covers g for a team of S workgroups: what a split GEMM needs
__host__ __device__ inline bool team_fast_path(const GemmArgs& g, int S) {
    const int nkb = g.K >> 4, L = nkb / KSPLIT, MT = (g.M + 15) >> 4;
    const int items = MT * ((g.N + 15) >> 4);
    const int ni = (items + S - 1) / S;
    return S % MT == 0 && L >= 1 && L <= 9 && ni <= TEAM_NI_MAX;
}

// Single-image decoder (k_dec_one, one.hip): the reference-format raster decode of ONE image in one persistent launch
// over every CU, each weight column tile of the step's GEMMs resident in the LDS of one workgroup for the whole launch,
// operations handed over as data-tagged 8-byte granules {value, step + 1} (no barriers)
constexpr int ONE_MAXOPS = 12;     // operations of a raster step: context net x 4, rANS, decoder x 7
constexpr int ONE_MAXSEG = 6;
constexpr int ONE_NT_MAX = 4;      // weight tiles one workgroup holds
constexpr int ONE_LL_MAX = 12;     // k-blocks of one K slice (K <= 1536)
constexpr int ONE_LLH_MAX = 32;    // k-blocks of one K slice of a half-tile operation (OneOp::half: K <= 4096)
enum OneSrc : int { ONE_GRAN = 0, ONE_ZTAP = 1, ONE_L0TAP = 2 };
struct OneSeg {
    int kind;                // ONE_GRAN: columns [k0, k1) of K are columns [c0, c0 + k1 - k0) of op `src`'s granules;
    int src, c0;             // ONE_ZTAP: the zpad tap (dy, dx) of the current block, channels [k - k0];
    int dy, dx;              // ONE_L0TAP (KS[1] = 3): the layer-0 cache cell (v + dy, h + dx), channels [k - k0],
    int k0, k1;              //   ordered by op `src`'s granules (the cache's producer, the context net's layer 0)
};
struct OneOp {             // (the epilogue's fields first: one scalar-cache line)
    const float* W;          // packed [K/16][NB16][4][16][4] (GEMMs; null for the rANS operation)
    const float* bias;
    int K, N, NB16, epi, sq; // epi: EPI_BIAS / EPI_LEAKY / EPI_IGDN / EPI_GDN / EPI_CTXIDX (value only) / EPI_CLAMPZ
    int l0out;               // 1: the context net's layer 0 under the layer-0 cache (KS[1] = 3): every output also goes
                             // to the cache cell of its position, and at a row end a second position (h = 0: (v, -1);
                             // h = Wb - 1: (v - 1, Wb)) rides in MFMA row 1 (and 2 when Wb = 1) -- the graph decoder's
                             // raster positions (codec.hip run_ctx)
    int half;                // 1: every column tile is held as two halves (K slices 0-3 / 4-7) by two workgroups (a
                             // whole tile would not fit one workgroup's LDS); half 0 hands its four slice partials over
                             // as granules `pgran` [2 step parities][N / 16][4][16], half 1 sums all eight in slice order
    int gw;                  // granule width (N padded to 16)
    unsigned long long* gran;   // this op's output granules [gw] {float bits, step + 1}
    int l0seg;               // 1: layer-0 cache taps (ONE_L0TAP) among the segments
    int nseg;
    int gx_src;              // GDN / IGDN: the op whose granules hold the layer input x
    OneSeg seg[ONE_MAXSEG];
    unsigned long long* pgran;
};
struct OneArgs {
    const OneOp* ops;        // [nops] device, read-only for the launch
    int nops, rans_op, rans_wg;
    const int4* tiles;       // [grid][ONE_NT_MAX] {op, column tile, LDS offset in float4s, piece}; op -1: none; piece
                             // 0 the whole tile, 1 / 2 its half 0 / 1 (OneOp::half)
    int wlds_f4;             // float4s of weight tiles per workgroup (dynamic LDS)
    float* zpad;
    int Hp, Wp, Cx, Hb, Wb;
    float* l0;               // the layer-0 map cache [Hb + 2][Wb + 4][C1P] (KS[1] = 3; zpad geometry), else null
    int C1P;
    int red_rows;            // MFMA rows of the partials area: 3 with the layer-0 cache (row-end positions), else 1
    const RansArgs* rans;    // device: the stream's coder state / tables (idx, ksi, yq unused: LDS copies)
    int Mlat;
    const float* table;      // scale table (64)
    unsigned* fail;          // failure word (1: a wait timed out), zeroed before the launch
    unsigned long long tmo;  // s_memrealtime ticks one wait may take
    int lazy_z;              // 1 (Wb >= 3): a d3 producer drains its zpad store of step t only before publishing step t + 1
    int rans_lds_tab;        // 1: the rANS workgroup copies the table image into its (weight-free) LDS
    int ts_step;             // the sampled raster step of `ts`
    unsigned long long* ts;  // optional [ONE_MAXOPS][4] s_memrealtime of step ts_step (kept in registers and LDS, written
                             // after the last step): [0] first workgroup in, [1] last workgroup's partials reduced, [2]
                             // last one published, [3] the last wave's inputs all there; then [ONE_MAXOPS * 4] the
                             // rANS op's decode started (inputs in LDS), [+ 1] its symbols decoded, [+ 2], [+ 3]
                             // s_memtime (shader clock) at those two points; then [ONE_TS_DETAIL + ONE_TS_PER_OP o] the
                             // workgroup holding column tile 0 of op o: [0] in, [1 + w] wave w's inputs there, [9 + w]
                             // its A and weights in registers, [17 + w] its chain done, [25] partials reduced,
                             // [26] published (the tile loop's barrier passed), [27] thread 0's granule store issued;
                             // for the rANS op: [0] coder prologue done, [1] symbols decoded, [2] speculation breaks,
                             // [3] +-1 symbols, [4] searched symbols
};
constexpr int ONE_TS_DETAIL = ONE_MAXOPS * 4 + 4;
constexpr int ONE_TS_PER_OP = 32;
constexpr int ONE_TS_WORDS = ONE_TS_DETAIL + ONE_MAXOPS * ONE_TS_PER_OP;
size_t one_lds_bytes(int wlds_f4, int red_rows);
int one_blocks_per_cu(size_t lds, bool l0);
int launch_dec_one(const OneArgs& a, int grid, hipStream_t s);

int prepare_gemm(GemmArgs& g);     // launch_gemm's host-side checks and segment set-up, without the launch
size_t team_lds_bytes(const TeamArgs& a);   // k_dec_team's dynamic LDS for a launch
int launch_dec_team(const TeamArgs& a, hipStream_t s);
int team_blocks_per_cu(int dense, size_t lds);   // k_dec_team workgroups one CU holds at `lds` bytes of dynamic LDS
                                                 // (occupancy query; 0 on error)
int launch_gemm(const GemmArgs& g, hipStream_t s, int* cfg_id = nullptr);   // cfg_id: 0 = k_gemm_s, 1 = k_gemm
int gemm_class(const GemmArgs& g);   // the kernel launch_gemm picks: 0 = k_gemm_s, 1 = k_gemm
int launch_rans_decode(const RansArgs& a, hipStream_t s);
int launch_ctr_add(int* ctr, int d, hipStream_t s);
int launch_zero_u64(unsigned long long* p, int n, hipStream_t s);
int launch_copy_interior(const float* zpad, float* zout, int n_img, int Hb, int Wb, int Cx, hipStream_t s);
int launch_fill_interior(const float* zin, float* zpad, int n_img, int Hb, int Wb, int Cx, hipStream_t s);
int launch_l0_border(float* l0, int n_img, int Hb, int Wb, int C, const float* bias, hipStream_t s);

}  // namespace lbic
