// liblbic.so host side: model handle, state-dict loader and weight packing, wavefront / raster step
// scheduler, and the C ABI declared in include/lbic.h.
//
// Encode (compress, net:319-361): the raster closed loop is replayed as a skewed anti-diagonal
// wavefront.  Block (v, h) needs the reconstructions of (v-1, h-1..h+1), (v, h-1) (and, for KS[1] = 3,
// of (v-2, h-2..h+2), (v-1, h-2), (v, h-2)), so every block with h + 2v = t depends only on steps < t
// and all of them -- across every image of the batch -- are coded in one step of 18 GEMM launches.
// Decode (decompress, net:400-452) keeps the reference's single raster-ordered rANS stream per image:
// each raster step decodes the same block position of every image (ctx GEMMs -> GPU rANS -> decoder
// GEMMs).  Both phases run the same k_gemm arithmetic, so decoder scale indexes equal the encoder's.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "kernels.h"
#include "lbic_internal.h"

namespace lbic {

static thread_local std::string g_err;
// graph captures of different handles are serialised (one-off cost): concurrent first-time captures from
// several host threads failed a kernel launch under rocprofv3's tracer
static std::mutex g_capture_mu;

int set_error(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define HIPCHK(x)                                                                                   \
    do {                                                                                            \
        hipError_t e_ = (x);                                                                        \
        if (e_ != hipSuccess) return set_error(LBC_E_HIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
    } while (0)

static int hip_rc(hipError_t e) {   // for code that must not return early (inside a stream capture)
    return e == hipSuccess ? LBC_OK : set_error(LBC_E_HIP, hipGetErrorString(e));
}

// Encoder graph fork: each wavefront step's context net (4 GEMMs) and the transform's first six GEMMs are independent
// (only the quantising GEMM reads the means / scales), so they are captured as two branches joined before it.
// Encoder alone 98.7 -> 95.0 ms per 32-frame batch, bit-identical; beside the team decoder within noise (+0.3..0.9 %;
// profiles/r02_exp/encoder_fork_team.txt).  Only for passes whose largest wavefront step has at most ENC_FORK_MAX_ROWS
// rows: a 128-frame pass's launches fill the chip for several rounds each, and two branches then only compete (bench,
// four batches per pass: 136.0 / 133.3 Mpix/s with one chain vs 132.9 / 131.5 forked, profiles/r06/exp/fs_*).
// LBIC_ENC_FORK=0 / 1 forces it (with four busy streams, the workers schedule, the branch's extra hardware queue cost
// 5 %: profiles/r02_exp/encoder_fork.txt).
// (LBC_OPT_ENC_FORK: -1 this rule, 0 / 1 forced)
constexpr int ENC_FORK_MAX_ROWS = 2048;
static bool enc_fork_on(int mmax, int opt) {
    const char* e = getenv("LBIC_ENC_FORK");
    if (e) return atoi(e) != 0;
    return opt >= 0 ? opt != 0 : mmax <= ENC_FORK_MAX_ROWS;
}

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    ~DevBuf() { release(); }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
    int alloc(size_t b) {
        if (b <= bytes && p) return LBC_OK;
        release();
        if (hipMalloc(&p, std::max<size_t>(b, 16)) != hipSuccess) {
            p = nullptr;
            return set_error(LBC_E_HIP, "hipMalloc failed");
        }
        bytes = b;
        return LBC_OK;
    }
    template <class T>
    T* as() const { return reinterpret_cast<T*>(p); }
};

struct Layer {
    DevBuf W, bias;
    int K = 0, N = 0, NB16 = 0;
};

// sampled per-kernel timing (lbc_profile_begin / lbc_profile_end): sampled launches stamp their span
// into a device slot {max(~start), max(end)}; one slot range per graph, zeroed at every replay
constexpr int kSlotsPerRange = 4096;
#ifdef LBIC_PHASE_DIAG
constexpr int kSlotU64 = 32;      // + per-phase max / sum / workgroup count (diagnostic build)
#else
constexpr int kSlotU64 = 16;      // 8 XCDs x {max(~start), max(end)}
#endif
constexpr int kRanges = 6;        // 0 encoder graph, 1..4 raster decoder lanes, 5 wavefront decoder graph
// kernel classes of the profile: gemm_class() (0 k_gemm_s, 1 k_gemm), 2 rANS, 3 copies
constexpr int kNClass = 4;
struct Prof {
    int sample_every = 0;
    bool active = false;          // current step is sampled
    // prev: slot of the launch before this one in the same sampled step of the same stream chain (-1: none),
    // so lbc_profile_end can also report the launch-to-launch period end(prev) -> end(this)
    struct Rec { int cls; int slot; double flops, bytes; int prev; };
    std::vector<Rec> recs;
    int last_slot = -1;
    unsigned long long* slots = nullptr;   // device, kRanges ranges
    int range = 0, next = 0;               // slot allocation inside the range being captured
    long long per_replay[8][kNClass] = {};       // launches of each kernel class per replay of each range's graph
    double work_replay[8][kNClass][2] = {};      // their algorithmic FLOPs and bytes per replay (every launch, sampled or not)
    long long replays[8] = {};             // replays of each range's graph since lbc_profile_begin
    bool nochain = false;                  // capturing a forked graph: no launch-to-launch period (two chains)
    // the encoder graph's slot range (0) copied to the host after EVERY replay since lbc_profile_begin (its stamps are
    // zeroed at the head of each replay): lbc_profile_end averages over all of them, not only the last replay
    int used0 = 0;                         // slots of range 0 the captured encoder graph uses
    unsigned long long* snap = nullptr;    // pinned host ring: kSnaps x kSlotsPerRange x kSlotU64 words
    int nsnap = 0;
    static constexpr int kSnaps = 64;
    unsigned long long* take() {
        if (!slots || next >= kSlotsPerRange) return nullptr;
        return slots + kSlotU64 * ((size_t)range * kSlotsPerRange + next++);
    }
    void step(bool on) {          // a new wavefront / raster step starts (sampled or not)
        active = on;
        last_slot = -1;
    }
    void add(int cls, const unsigned long long* ts, double flops, double bytes) {
        const int slot = (int)((ts - slots) / kSlotU64);
        recs.push_back({cls, slot, flops, bytes, nochain ? -1 : last_slot});
        last_slot = slot;
    }
};
static const char* kKernelNames[kNClass] = {"k_gemm_s", "k_gemm", "k_rans_decode", "k_copy_interior"};
static thread_local Prof* g_prof = nullptr;

struct HostT {
    std::vector<float> v;
    std::vector<int64_t> shape;
};

inline int pad16(int x) { return (x + 15) & ~15; }

// A "lane" = one HIP stream + its own step workspace.  The encoder runs on lane 0 (the caller's
// stream); the decoder splits the images into kLanes groups whose raster chains run concurrently.
constexpr int kLanes = 4;
struct Work {
    int rows = 0;
    DevBuf ctx0, ctx1, ctx2, ksi, e0, e1, yq, d0, d1, idx;
};

// The packed device weights of one finalized state dict: shared (read-only) by every handle made from it with
// lbc_create_sibling, so several handles decoding side by side keep one copy in the Infinity Cache.  gen: a
// process-unique id of this packed set (recorded programs key on it: a new set may reuse freed addresses)
struct Net {
    Layer ctx0, ctx1, ctx2, ctx3, enc0, g0, e1, g1, e2, g2, e3, dec0, ig0, d1, ig1, d2, ig2, d3;
    long long gen = next_gen();
    static long long next_gen() {
        static std::atomic<long long> g{0};
        return ++g;
    }
};

static const int TAPS_A[4][2] = {{-1, -1}, {-1, 0}, {-1, 1}, {0, -1}};       // masked_conv2d.py:9-17 'A'
static const int TAPS_B[5][2] = {{-1, -1}, {-1, 0}, {-1, 1}, {0, -1}, {0, 0}};  // 'B' adds the centre

}  // namespace lbic

using namespace lbic;

struct lbc_model {
    lbc_config cfg{};
    int B = 0, Cx = 0, N = 0, M = 0, N7 = 0, N6 = 0, C1 = 0, C2 = 0, C3 = 0, C4 = 0, P = 1;
    int NP = 0, C1P = 0, C2P = 0, C3P = 0;   // widths padded to 16 (activation row strides)
    std::map<std::string, HostT> host;
    bool finalized = false;
    std::shared_ptr<Net> net = std::make_shared<Net>();
    EntropyTables tabs;
    bool tabs_set = false;
    DevBuf table_dev, cdf16_dev, tmeta_dev;
    int total16 = 0;
    std::vector<uint16_t> c16_host;
    std::vector<int> meta_host;
    bool tabs_dirty = false;
    // per-shape workspace
    int ws_n = 0, ws_Hb = 0, ws_Wb = 0, Mmax = 0;
    DevBuf zpad, blocks_enc, blocks_dec;
    // layer-0 map cache of the context net (KS[1] = 3): cell (img, v, h) = LeakyReLU(layer 0) at block position
    // (v, h), zpad geometry [n_img][Hb+2][Wb+4][C1P]; cells_enc = the cells each wavefront step computes
    bool l0_on = false;
    DevBuf l0, cells_enc;
    std::vector<int> cell_off, cell_cnt;
    int enc_lds_floor = 0;      // LBC_OPT_ENC_LDS_FLOOR
    int enc_fork = -1;          // LBC_OPT_ENC_FORK
    int team_wpc = 1;           // LBC_OPT_TEAM_WG_PER_CU
    int team_size = 0;          // LBC_OPT_TEAM_SIZE (0: CUs / 8)
    Work lane[kLanes];
    hipStream_t lstream[kLanes] = {nullptr, nullptr, nullptr, nullptr};
    hipEvent_t lev[kLanes + 1] = {nullptr, nullptr, nullptr, nullptr, nullptr};
    std::vector<int> step_off, step_cnt;
    DevBuf words, word_base, word_count, st_x, st_ptr, st_status;
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    bool enc_timed = false, dec_timed = false;
    Prof prof;
    // HIP graphs: the whole encoder wavefront (one replay per call) and, per decoder lane, one block row
    // (replayed Hb times; kernels take the row from a device counter)
    hipGraphExec_t enc_exec = nullptr, wf_exec = nullptr;
    std::vector<hipGraphExec_t> dec_exec;
    std::vector<long long> enc_key, dec_key, wf_key;
    DevBuf x_in, sym_buf, idx_buf, bits_buf, ctr;
    hipStream_t cap = nullptr;
    // encoder graph fork (LBIC_ENC_FORK=1): each wavefront step's context net is captured on cap2, beside the
    // encoder transform's first six GEMMs on cap; the quantising GEMM joins both
    hipStream_t cap2 = nullptr;
    hipEvent_t fev[2] = {nullptr, nullptr};
    // workspace set-up (ws_zero / dev_upload with a handle): a private non-blocking stream ordered after the caller's stream by
    // an event, never the legacy stream
    hipStream_t aux = nullptr;
    hipEvent_t aux_ev = nullptr;
    // band pipeline (lbc_band_*): this handle codes block rows [band_v0, band_v0 + ws_Hb) of taller frames;
    // one captured graph per range of global wavefront steps
    int band_v0 = -1;
    std::map<std::pair<int, int>, hipGraphExec_t> band_exec;
    std::vector<long long> band_key;
    // team decoder (lbc_decode_team, held by the first handle of a call): the recorded raster step of every
    // team, the barrier words, and the stamps of the last launch
    DevBuf team_prog, team_sync, team_ts;
    std::vector<long long> team_key;
    TeamArgs team_args{};
    std::vector<unsigned long long> team_ts_host;
    int team_fallbacks = 0, team_plain_last = -1;   // launches rerun write-through; mode of the last launch
    int team_timeouts = 0;    // team launches that timed out at a barrier and were decoded through lbc_decode instead
    bool no_one = false;      // lbc_decode skips k_dec_one (set by team_fallback after a residency timeout)
    int team_mode_last = 0;   // the last lbc_decode_team call: 0 lbc_decode per batch (a fallback), 1 team + sparse rANS,
                              // 2 team + dense, one batch of one image through lbc_decode: 3 its single-image decoder
                              // (k_dec_one), 4 its row graphs
    double team_step_bytes = 0, team_step_flops = 0;  // algorithmic work of one team's raster step (inner column)
    double team_launch_bytes = 0, team_launch_flops = 0;
    // single-image decoder (k_dec_one, one.hip; lbc_decode of one image): the step's operations, the weight-tile
    // placement over the grid, the granule buffers and the failure word
    DevBuf one_ops, one_tiles, one_gran, one_fail, one_rans, one_ts;
    std::vector<unsigned long long> one_ts_host;
    std::vector<long long> one_key;
    OneArgs one_args{};
    int one_grid = 0;
    int one_ok = 0;             // the placement fits (0: lbc_decode keeps the graph decoder for single images)
    int dec_path_last = 0;      // the last lbc_decode: 0 the row graphs, 1 k_dec_one
    int one_timeouts = 0;       // k_dec_one launches that timed out and were decoded by the row graphs instead
};

namespace {

// workspace set-up stream of handle m, ordered after the caller's stream s (an event recorded on s, waited for by the
// handle's private non-blocking stream): a legacy-stream memset / copy fails while another thread of the process
// captures a graph (decoder handles sizing their workspaces beside each other's captures), and a plain non-blocking
// stream without the event raced the handle's previous encode still running on s (round 5, test_batch_equals_single)
hipStream_t ws_stream(lbc_model* m, hipStream_t s) {
    if (!m->aux) return nullptr;
    if (hipEventRecord(m->aux_ev, s) != hipSuccess || hipStreamWaitEvent(m->aux, m->aux_ev, 0) != hipSuccess) {
        set_error(LBC_E_HIP, "workspace stream ordering failed");
        return nullptr;
    }
    return m->aux;
}

int dev_upload(DevBuf& d, const void* src, size_t bytes, lbc_model* m = nullptr, hipStream_t s = nullptr) {
    int rc = d.alloc(bytes);
    if (rc) return rc;
    if (!m) {
        HIPCHK(hipMemcpy(d.p, src, bytes, hipMemcpyHostToDevice));
        return LBC_OK;
    }
    // on the handle's set-up stream (after the caller's earlier work on s), then waited for
    hipStream_t q = ws_stream(m, s);
    if (!q) return set_error(LBC_E_HIP, "workspace stream unavailable");
    HIPCHK(hipMemcpyAsync(d.p, src, bytes, hipMemcpyHostToDevice, q));
    HIPCHK(hipStreamSynchronize(q));
    return LBC_OK;
}

// Pack W[k][n] (row-major K x N, N padded to 16) into [K/16][N/16][4][16][4]: the float4 lane l of
// a wave loads for a 16x16 k-n tile holds W[4*(l>>4) + e][l&15], e = 0..3 -- the A/B operand of four
// v_mfma_f32_16x16x4_f32 (operand maps: cdna_hip_programming.md §3).
int upload_layer(Layer& L, const std::vector<float>& wkn, const std::vector<float>& bias, int K, int N) {
    if (K % 16) return set_error(LBC_E_ARG, "layer K not a multiple of 16");
    const int NB = ((N + 31) / 32) * 2;   // whole 32-column tiles: the widest BN never reads past the end
    std::vector<float> pk((size_t)K * NB * 16, 0.f);
    for (int kb = 0; kb < K / 16; ++kb)
        for (int nb = 0; nb < NB; ++nb)
            for (int l = 0; l < 64; ++l)
                for (int e = 0; e < 4; ++e) {
                    const int k = kb * 16 + 4 * (l >> 4) + e, n = nb * 16 + (l & 15);
                    pk[(((size_t)kb * NB + nb) * 64 + l) * 4 + e] = n < N ? wkn[(size_t)k * N + n] : 0.f;
                }
    std::vector<float> b(NB * 16, 0.f);
    std::copy(bias.begin(), bias.end(), b.begin());
    L.K = K;
    L.N = N;
    L.NB16 = NB;
    int rc = dev_upload(L.W, pk.data(), pk.size() * 4);
    if (rc) return rc;
    return dev_upload(L.bias, b.data(), b.size() * 4);
}

const HostT* get(lbc_model* m, const std::string& n) {
    auto it = m->host.find(n);
    return it == m->host.end() ? nullptr : &it->second;
}

// conv weight [cout][cin][k][k] -> W[k = slot*cin + ci][n] for the listed taps (a 1x1 conv is one slot)
// slot = K stride between taps (>= cin; padded columns keep zero weights)
int conv_to_kn(lbc_model* m, const std::string& name, int cin, int cout, const int (*taps)[2], int ntaps,
               std::vector<float>& wkn, int k_base, int slot, std::vector<float>* bias_acc) {
    const HostT* w = get(m, name + ".weight");
    const HostT* b = get(m, name + ".bias");
    if (!w || !b) return set_error(LBC_E_STATE, "missing tensor " + name);
    const int ks = (int)w->shape[2];
    if ((int)w->shape[0] != cout || (int)w->shape[1] != cin || (int)b->v.size() != cout)
        return set_error(LBC_E_ARG, "bad shape for " + name);
    for (int t = 0; t < ntaps; ++t) {
        const int ky = ks == 1 ? 0 : 1 + taps[t][0], kx = ks == 1 ? 0 : 1 + taps[t][1];
        for (int ci = 0; ci < cin; ++ci)
            for (int co = 0; co < cout; ++co)
                wkn[(size_t)(k_base + t * slot + ci) * cout + co] = w->v[(((size_t)co * cin + ci) * ks + ky) * ks + kx];
    }
    if (bias_acc) {
        if (bias_acc->empty()) bias_acc->assign(b->v.begin(), b->v.end());
        else for (int co = 0; co < cout; ++co) (*bias_acc)[co] += b->v[co];
    }
    return LBC_OK;
}

int pack_conv(lbc_model* m, Layer& L, const std::string& name, int cin, int cout, int ntaps, const int (*taps)[2]) {
    const int slot = pad16(cin);
    std::vector<float> wkn((size_t)ntaps * slot * cout, 0.f), bias;
    int rc = conv_to_kn(m, name, cin, cout, taps, ntaps, wkn, 0, slot, &bias);
    if (rc) return rc;
    return upload_layer(L, wkn, bias, ntaps * slot, cout);
}

// first layer of the encoder / decoder transform: 4 masked taps of prtr_*2 on zhat + the 1x1 prtr_*1
// on x (or y_qnt), one GEMM (K = 4*Cx + cin1); bias = b1 + b2 (net:379-387: out_x + out_zhat).
int pack_first(lbc_model* m, Layer& L, const std::string& n2, const std::string& n1, int cin1) {
    const int K = 4 * m->Cx + cin1;
    std::vector<float> wkn((size_t)K * m->N), bias;
    int rc = conv_to_kn(m, n2, m->Cx, m->N, TAPS_A, 4, wkn, 0, m->Cx, &bias);
    if (rc) return rc;
    static const int one[1][2] = {{0, 0}};
    rc = conv_to_kn(m, n1, cin1, m->N, one, 1, wkn, 4 * m->Cx, cin1, &bias);
    if (rc) return rc;
    return upload_layer(L, wkn, bias, K, m->N);
}

// GDN: norm_i = beta_i + sum_j gamma_ij x_j^2 with the reparametrisation of
// utils/parametrizers.py:45-47: v -> max(v, bound)^2 - pedestal, pedestal = 2^-36,
// bound = sqrt(minimum + pedestal) (beta_min = 1e-6, gdn_compressai.py:43-56).
int pack_gdn(lbc_model* m, Layer& L, const std::string& name, int C) {
    const HostT* be = get(m, name + ".beta");
    const HostT* ga = get(m, name + ".gamma");
    if (!be || !ga) return set_error(LBC_E_STATE, "missing tensor " + name);
    if ((int)be->v.size() != C || (int)ga->v.size() != C * C) return set_error(LBC_E_ARG, "bad GDN shape " + name);
    const float ped = (float)std::pow(2.0, -36.0);
    const float bb = (float)std::sqrt(1e-6 + std::pow(2.0, -36.0));
    const float gb = (float)std::sqrt(0.0 + std::pow(2.0, -36.0));
    std::vector<float> beta(C), wkn((size_t)pad16(C) * C, 0.f);
    for (int i = 0; i < C; ++i) {
        const float t = std::max(be->v[i], bb);
        beta[i] = t * t - ped;
    }
    for (int i = 0; i < C; ++i)
        for (int j = 0; j < C; ++j) {
            const float t = std::max(ga->v[(size_t)i * C + j], gb);
            wkn[(size_t)j * C + i] = t * t - ped;       // W[k = j][n = i]
        }
    return upload_layer(L, wkn, beta, pad16(C), C);
}

// zero a fresh workspace buffer on the handle's set-up stream (ordered after the caller's earlier work on s, ws_stream)
// and wait for it
static int ws_zero(lbc_model* m, hipStream_t s, void* p, size_t b) {
    hipStream_t q = ws_stream(m, s);
    if (!q) return set_error(LBC_E_HIP, "workspace stream unavailable");
    HIPCHK(hipMemsetAsync(p, 0, b, q));
    HIPCHK(hipStreamSynchronize(q));
    return LBC_OK;
}

int ensure_workspace(lbc_model* m, int n_img, int Hb, int Wb, hipStream_t s) {
    if (m->ws_n == n_img && m->ws_Hb == Hb && m->ws_Wb == Wb) return LBC_OK;
    const int T = (Wb - 1) + 2 * (Hb - 1) + 1;
    std::vector<int4> enc;
    m->step_off.assign(T, 0);
    m->step_cnt.assign(T, 0);
    int mmax = n_img;
    for (int t = 0; t < T; ++t) {
        m->step_off[t] = (int)enc.size();
        for (int img = 0; img < n_img; ++img)
            for (int v = 0; v < Hb; ++v) {
                const int h = t - 2 * v;
                if (h >= 0 && h < Wb) enc.push_back(make_int4(img, v, h, 0));
            }
        m->step_cnt[t] = (int)enc.size() - m->step_off[t];
        mmax = std::max(mmax, m->step_cnt[t]);
    }
    std::vector<int4> dec((size_t)Hb * Wb * n_img);
    for (int s = 0; s < Hb * Wb; ++s)
        for (int img = 0; img < n_img; ++img) dec[(size_t)s * n_img + img] = make_int4(img, s / Wb, s % Wb, 0);
    // the GEMM kernels address A rows with unsigned 32-bit float4 offsets from a segment base (kernels.hip, Rows):
    // up to 2^34 floats (64 GB) per buffer
    const double lim = 17179869184.0;
    if ((double)n_img * (Hb + 2) * (Wb + 4) * m->Cx >= lim || (double)n_img * Hb * Wb * m->Cx >= lim ||
        (double)mmax * m->P * std::max({m->C1P, m->NP, m->C2P}) * 5 >= lim)
        return set_error(LBC_E_ARG, "frame batch too large (a workspace buffer above 64 GB); split the batch");
    // Layer-0 map cache (KS[1] = 3).  The context net's second layer reads layer 0 at the five positions (v-1, h-1..h+1),
    // (v, h-1), (v, h) (a 3x3 'B' mask); the value at a position depends only on reconstructions coded
    // before that position's own block (the 'A' taps), so it is computed once -- at its own block's step, position
    // (0,0) -- and read from the cache afterwards, instead of at five positions in every step.  Border cells under
    // compress() (the zero-padded window, net:342-351): row -1 is constant (k_l0_border); column -1 of row v depends
    // on zhat(v-1, 0) and is computed at block (v, 0)'s step, column Wb of row v-1 on zhat(v-2 .. v-1, Wb-1) and is
    // computed at block (v, Wb-1)'s step, the only step that reads it.
    std::vector<int4> cells;
    if (m->l0_on) {
        m->cell_off.assign(T, 0);
        m->cell_cnt.assign(T, 0);
        for (int t = 0; t < T; ++t) {
            m->cell_off[t] = (int)cells.size();
            for (int img = 0; img < n_img; ++img)
                for (int v = 0; v < Hb; ++v) {
                    const int h = t - 2 * v;
                    if (h < 0 || h >= Wb) continue;
                    cells.push_back(make_int4(img, v, h, 0));
                    if (h == 0) cells.push_back(make_int4(img, v, -1, 0));
                    if (h == Wb - 1) cells.push_back(make_int4(img, v - 1, Wb, 0));
                }
            m->cell_cnt[t] = (int)cells.size() - m->cell_off[t];
        }
        if ((double)n_img * (Hb + 2) * (Wb + 4) * m->C1P >= lim)
            return set_error(LBC_E_ARG, "frame batch too large (layer-0 cache above 64 GB); split the batch");
    }
    int rc;
    if ((rc = dev_upload(m->blocks_enc, enc.data(), enc.size() * sizeof(int4), m, s))) return rc;
    if ((rc = dev_upload(m->blocks_dec, dec.data(), dec.size() * sizeof(int4), m, s))) return rc;
    if (m->l0_on) {
        if ((rc = dev_upload(m->cells_enc, cells.data(), cells.size() * sizeof(int4), m, s))) return rc;
        const size_t b = (size_t)n_img * (Hb + 2) * (Wb + 4) * m->C1P * sizeof(float);
        if ((rc = m->l0.alloc(b))) return rc;
        if ((rc = ws_zero(m, s, m->l0.p, b))) return rc;   // pad channels stay 0 (never written; A x 0-weight meets no NaN)
    }
    const size_t F = sizeof(float);
    if ((rc = m->zpad.alloc((size_t)n_img * (Hb + 2) * (Wb + 4) * m->Cx * F))) return rc;
    const int gmax = n_img;      // a decoder lane may get every image (lane count is chosen per call)
    for (int l = 0; l < kLanes; ++l) {
        Work& w = m->lane[l];
        const size_t rows = (size_t)(l == 0 ? mmax : gmax);
        w.rows = (int)rows;
        // activation widths are padded to 16 columns; the pad columns are zeroed once and never
        // written, so GEMMs can run K over whole 16-wide k-blocks (their weights are zero there too)
        DevBuf* bufs[] = {&w.ctx0, &w.ctx1, &w.ctx2, &w.ksi, &w.e0, &w.e1, &w.d0, &w.d1, &w.yq, &w.idx};
        const size_t widths[] = {(size_t)m->P * m->C1P, (size_t)m->C2P, (size_t)m->C3P, (size_t)m->C4, (size_t)m->NP,
                                 (size_t)m->NP, (size_t)m->NP, (size_t)m->NP, (size_t)m->M, (size_t)m->M};
        for (int i = 0; i < 10; ++i) {
            if (l > 0 && (i == 4 || i == 5)) continue;   // encoder-only buffers
            if ((rc = bufs[i]->alloc(rows * widths[i] * F))) return rc;
            if ((rc = ws_zero(m, s, bufs[i]->p, rows * widths[i] * F))) return rc;
        }
    }
    m->Mmax = mmax;
    m->ws_n = n_img;
    m->ws_Hb = Hb;
    m->ws_Wb = Wb;
    return LBC_OK;
}

// first device use: events and the entropy tables (host copies made by lbc_set_entropy_tables)
int prepare_device(lbc_model* m) {
    HIPCHK(hipSetDevice(m->cfg.device));
    if (!m->ev[0]) {
        for (auto& e : m->ev) HIPCHK(hipEventCreate(&e));
        for (auto& e : m->lev) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        // (lane streams are created only when a decode uses several lanes: every stream a process creates
        // takes a turn on its few hardware queues, and two busy streams on one queue serialise)
        HIPCHK(hipStreamCreateWithFlags(&m->cap, hipStreamNonBlocking));
        HIPCHK(hipStreamCreateWithFlags(&m->cap2, hipStreamNonBlocking));
        for (auto& e : m->fev) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        HIPCHK(hipStreamCreateWithFlags(&m->aux, hipStreamNonBlocking));
        HIPCHK(hipEventCreateWithFlags(&m->aux_ev, hipEventDisableTiming));
    }
    if (m->tabs_dirty) {
        int rc;
        if ((rc = dev_upload(m->table_dev, m->tabs.table.data(), 64 * sizeof(float)))) return rc;
        if ((rc = dev_upload(m->cdf16_dev, m->c16_host.data(), m->c16_host.size() * 2))) return rc;
        if ((rc = dev_upload(m->tmeta_dev, m->meta_host.data(), m->meta_host.size() * sizeof(int)))) return rc;
        m->tabs_dirty = false;
    }
    return LBC_OK;
}

void drop_recs(Prof& p, int r) {
    std::vector<Prof::Rec> keep;
    for (const auto& x : p.recs)
        if (x.slot / kSlotsPerRange != r) keep.push_back(x);
    p.recs.swap(keep);
}

// start capturing sampled launches into slot range r: the range is zeroed by the graph's first node
int prof_range_begin(Prof* p, int r, hipStream_t s) {
    p->range = r;
    p->next = 0;
    for (auto& c : p->per_replay[r]) c = 0;
    for (auto& c : p->work_replay[r]) c[0] = c[1] = 0;
    if (p->sample_every && p->slots)
        return launch_zero_u64(p->slots + kSlotU64 * (size_t)r * kSlotsPerRange, kSlotU64 * kSlotsPerRange, s);
    return LBC_OK;
}

// Recording mode (lbc_decode_team): gemm() prepares the arguments as launch_gemm would and appends them to the
// program instead of launching; the team kernel replays them for every raster step.
struct Recorder {
    std::vector<GemmArgs> gemms;
    std::vector<int> ops;     // >= 0: GEMM index, -1: the rANS decode
};
static thread_local Recorder* g_rec = nullptr;

// launch a GEMM; in a sampled step give it a timing slot and record its algorithmic work
static void gemm_work(const GemmArgs& g, int k_live, double& flops, double& bytes) {
    const double K = k_live > 0 ? k_live : g.K;
    flops = 2.0 * g.M * K * g.N;
    bytes = 4.0 * (K * g.N + (double)g.M * K + (double)g.M * g.N * (g.square_a ? 2 : 1));
}

int gemm(const GemmArgs& g0, hipStream_t s, int k_live = -1) {
    if (g_rec) {
        GemmArgs g = g0;
        if (g.M <= 0) return set_error(LBC_E_ARG, "empty GEMM in a recorded step");
        const int rc = prepare_gemm(g);
        if (rc) return rc;
        g_rec->ops.push_back((int)g_rec->gemms.size());
        g_rec->gemms.push_back(g);
        return LBC_OK;
    }
    Prof* p = g_prof;
    if (p) {
        const int c = gemm_class(g0);       // the class launch_gemm will pick
        double f, b;
        gemm_work(g0, k_live, f, b);
        p->per_replay[p->range][c] += 1;
        p->work_replay[p->range][c][0] += f;
        p->work_replay[p->range][c][1] += b;
    }
    if (!p || !p->active) return launch_gemm(g0, s);
    GemmArgs g = g0;
    g.ts = p->take();
    if (!g.ts) return launch_gemm(g0, s);
    int cls = 0;
    int rc = launch_gemm(g, s, &cls);
    if (rc) return rc;
    double flops, bytes;
    gemm_work(g, k_live, flops, bytes);
    p->add(cls, g.ts, flops, bytes);
    return LBC_OK;
}

RansArgs rans_args(lbc_model* m) {
    RansArgs r{};
    r.cdf16 = m->cdf16_dev.as<uint16_t>();
    r.tmeta = m->tmeta_dev.as<int>();
    r.total16 = m->total16;
    r.words = m->words.as<uint32_t>();
    r.word_base = m->word_base.as<long long>();
    r.word_count = m->word_count.as<int>();
    r.state_x = m->st_x.as<unsigned long long>();
    r.state_ptr = m->st_ptr.as<int>();
    r.status = m->st_status.as<int>();
    r.ldk = m->C4;
    r.Mlat = m->M;
    r.ldy = m->M;
    r.streams_per_img = 1;
    return r;
}

// Upload rANS (sub-)streams: concatenated words, per-stream base / count, and the initial state of each
// (Rans64DecInit: the first two words).  The word buffer is baked into the decoder graphs, so it grows
// with headroom to stay put across calls.
int upload_streams(lbc_model* m, const std::vector<std::pair<const uint8_t*, size_t>>& subs, hipStream_t s) {
    const size_t n = subs.size();
    std::vector<long long> base(n);
    std::vector<int> cnt(n), ptr(n, 2);
    std::vector<unsigned long long> x0(n);
    size_t total = 0;
    for (size_t i = 0; i < n; ++i) {
        if (!subs[i].first || subs[i].second < 8 || (subs[i].second & 3)) return set_error(LBC_E_STREAM, "invalid bitstream");
        if (subs[i].second / 4 > 0x7fffffff) return set_error(LBC_E_STREAM, "bitstream too long");
        base[i] = (long long)(total / 4);
        cnt[i] = (int)(subs[i].second / 4);
        total += subs[i].second;
        uint32_t w[2];
        std::memcpy(w, subs[i].first, 8);
        x0[i] = (unsigned long long)w[0] | ((unsigned long long)w[1] << 32);
    }
    int rc;
    // every allocation before the first queued copy: an error return below must not leave copies in flight
    // that read the local host arrays or the caller's borrowed buffers
    if (total > m->words.bytes && (rc = m->words.alloc(total + total / 2 + (1 << 20)))) return rc;
    // per-stream arrays: sized by the stream count, pointers kept stable for the graphs
    const size_t cap = std::max<size_t>(n, 64);
    if ((rc = m->word_base.alloc(cap * sizeof(long long))) || (rc = m->word_count.alloc(cap * sizeof(int))) ||
        (rc = m->st_x.alloc(cap * sizeof(unsigned long long))) || (rc = m->st_ptr.alloc(cap * sizeof(int))) ||
        (rc = m->st_status.alloc(cap * sizeof(int))))
        return rc;
    // each stream straight from the caller's buffer to its word offset (no host-side concatenation),
    // stream-ordered on the decoder's stream: the words are rewritten only after that stream's previous
    // graph (which reads them) has drained, whatever the stream's blocking flags.  The local arrays and the
    // borrowed buffers stay alive until the synchronisation below, on the error path as well.
    hipError_t e = hipSuccess;
    for (size_t i = 0; i < n && e == hipSuccess; ++i)
        e = hipMemcpyAsync(static_cast<uint8_t*>(m->words.p) + (size_t)base[i] * 4, subs[i].first, subs[i].second,
                           hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipMemcpyAsync(m->word_base.p, base.data(), n * sizeof(long long), hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipMemcpyAsync(m->word_count.p, cnt.data(), n * sizeof(int), hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipMemcpyAsync(m->st_x.p, x0.data(), n * sizeof(unsigned long long), hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipMemcpyAsync(m->st_ptr.p, ptr.data(), n * sizeof(int), hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipMemsetAsync(m->st_status.p, 0, n * sizeof(int), s);
    const hipError_t es = hipStreamSynchronize(s);      // always: drains whatever was queued
    if (e != hipSuccess) return set_error(LBC_E_HIP, std::string("bitstream upload: ") + hipGetErrorString(e));
    if (es != hipSuccess) return set_error(LBC_E_HIP, std::string("bitstream upload sync: ") + hipGetErrorString(es));
    return LBC_OK;
}

int rans_sparse_choice(const size_t* lens, int n, double symbols) {
    if (const char* e = getenv("LBIC_RANS_SPARSE")) return atoi(e) ? 1 : 0;
    static const double thr = [] {
        const char* e = getenv("LBIC_RANS_SPARSE_BPS");
        return e ? atof(e) : 1.0;
    }();
    double bytes = 0;
    for (int i = 0; i < n; ++i) bytes += (double)lens[i];
    return symbols > 0 && 8.0 * bytes / symbols < thr ? 1 : 0;
}

// full: the decode consumed every block of every stream, so each rANS stream must end where its encoder began: state
// RANS64_L = 2^31 (Rans64EncInit; the decoder retraces the encoder's states in reverse).  A truncated stream overruns
// (status); a corrupted one ends in another state with near certainty -- both raise.  Words past the last one read
// (trailing padding) are ignored, as CompressAI's RansDecoder ignores them (lbic.h, lbc_decode).
int check_status(lbc_model* m, size_t n, hipStream_t s, bool full) {
    std::vector<int> status(n), ptr(full ? n : 0), cnt(full ? n : 0);
    std::vector<unsigned long long> x(full ? n : 0);
    HIPCHK(hipMemcpyAsync(status.data(), m->st_status.p, n * sizeof(int), hipMemcpyDeviceToHost, s));
    if (full) {
        HIPCHK(hipMemcpyAsync(x.data(), m->st_x.p, n * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(ptr.data(), m->st_ptr.p, n * sizeof(int), hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(cnt.data(), m->word_count.p, n * sizeof(int), hipMemcpyDeviceToHost, s));
    }
    HIPCHK(hipStreamSynchronize(s));
    for (size_t i = 0; i < n; ++i) {
        if (status[i]) return set_error(LBC_E_STREAM, "corrupt bitstream (stream " + std::to_string(i) + ")");
        if (full && (x[i] != (1ull << 31) || ptr[i] > cnt[i]))
            return set_error(LBC_E_STREAM, "corrupt bitstream (stream " + std::to_string(i) +
                                               ": the decode does not end in the encoder's initial state)");
    }
    return LBC_OK;
}

GemmArgs base_args(lbc_model* m, const int4* blocks, int rows, const float* x, int n_img, int Hb, int Wb) {
    GemmArgs g{};
    g.M = rows;
    g.P = 1;
    g.blocks = blocks;
    g.pos_dy[0] = g.pos_dx[0] = 0;
    g.geo.zpad = m->zpad.as<float>();
    g.geo.Hp = Hb + 2;
    g.geo.Wp = Wb + 4;
    g.geo.Cx = m->Cx;
    g.geo.x = x;
    g.geo.Hb = Hb;
    g.geo.Wb = Wb;
    g.table = m->table_dev.as<float>();
    g.Mlat = m->M;
    g.HW = Hb * Wb;
    g.lds_floor = m->enc_lds_floor;
    (void)n_img;
    return g;
}

void set_layer(GemmArgs& g, const Layer& L, int epi, float* out, int ldo) {
    g.W = L.W.as<float>();
    g.bias = L.bias.as<float>();
    g.NB16 = L.NB16;
    g.K = L.K;
    g.N = L.N;
    g.epi = epi;
    g.out = out;
    g.ldo = ldo;
}

void seg_dense(GemmArgs& g, const float* base, int ld, int k0, int k1) {
    Seg& s = g.seg[g.nseg++];
    s = Seg{base, SEG_DENSE, ld, 0, 0, k0, k1};
}

void segs_ztaps(GemmArgs& g, int Cx) {
    for (int t = 0; t < 4; ++t) {
        Seg& s = g.seg[g.nseg++];
        s = Seg{g.geo.zpad, SEG_ZTAP, 0, TAPS_A[t][0], TAPS_A[t][1], t * Cx, (t + 1) * Cx};
    }
}

int run_dense(GemmArgs g, const Layer& L, const float* in, int ld_in, int epi, float* out, int ldo, hipStream_t s) {
    g.nseg = 0;
    g.square_a = 0;
    set_layer(g, L, epi, out, ldo);
    seg_dense(g, in, ld_in, 0, L.K);
    return gemm(g, s);
}

// ld: row stride of `in` and `out` (the padded activation width)
int run_gdn(GemmArgs g, const Layer& L, const float* in, int ld, bool inverse, float* out, hipStream_t s) {
    g.nseg = 0;
    set_layer(g, L, inverse ? EPI_IGDN : EPI_GDN, out, ld);
    seg_dense(g, in, ld, 0, L.K);
    g.square_a = 1;
    g.gx = in;
    g.ldx = ld;
    return gemm(g, s);
}

// context net (get_meanscale_fast, net:389-398) for the rows of `g`; the last layer's epilogue is
// plain (encode) or also emits the scale indexes (decode).  frame_pad: forward()'s full-frame semantics
// (get_meanscale as nn.Sequential, net:57-65): the layer-0 map is zero outside the frame.
// cells / ncells: the layer-0 cache cells of this wavefront step (cache mode, encoder and wavefront decoder); a
// raster step (g.raster) computes its own block's cell plus the border cell it owns (column -1 at h = 0, column Wb
// of the row above at h = Wb - 1).  Without either (forward(): every block at once) layer 0 runs at the five
// positions per block as before.
int run_ctx(lbc_model* m, Work& w, GemmArgs g, bool with_idx, hipStream_t s, bool frame_pad = false,
            const int4* cells = nullptr, int ncells = 0) {
    int rc;
    if (m->l0_on && (cells || g.raster)) {
        GemmArgs c = g;
        c.nseg = 0;
        c.square_a = 0;
        c.zero_oob = frame_pad;
        c.pos_dy[0] = c.pos_dx[0] = 0;
        if (cells) {
            c.blocks = cells;
            c.M = ncells;
            c.P = 1;
        } else {
            int P = 1;
            if (g.raster_h == 0) { c.pos_dy[P] = 0; c.pos_dx[P] = -1; ++P; }
            if (g.raster_h == g.geo.Wb - 1) { c.pos_dy[P] = -1; c.pos_dx[P] = 1; ++P; }
            c.P = P;
            c.M = g.M * P;
        }
        set_layer(c, m->net->ctx0, EPI_LEAKY_L0, m->l0.as<float>(), m->C1P);
        segs_ztaps(c, m->Cx);
        if ((rc = gemm(c, s))) return rc;
        GemmArgs d = g;
        d.nseg = 0;
        d.square_a = 0;
        set_layer(d, m->net->ctx1, EPI_LEAKY, w.ctx1.as<float>(), m->C2P);
        for (int t = 0; t < 5; ++t) {       // the 3x3 'B' taps of layer 1 = five cache cells, K order as packed
            Seg& sg = d.seg[d.nseg++];
            sg = Seg{m->l0.as<float>(), SEG_L0TAP, m->C1P, TAPS_B[t][0], TAPS_B[t][1], t * m->C1P, (t + 1) * m->C1P};
        }
        if ((rc = gemm(d, s))) return rc;
    } else {
    {
        GemmArgs c = g;
        c.nseg = 0;
        c.square_a = 0;
        c.zero_oob = frame_pad && m->P > 1;
        c.P = m->P;
        c.M = g.M * m->P;
        for (int p = 0; p < m->P; ++p) {
            c.pos_dy[p] = m->P == 1 ? 0 : TAPS_B[p][0];
            c.pos_dx[p] = m->P == 1 ? 0 : TAPS_B[p][1];
        }
        set_layer(c, m->net->ctx0, EPI_LEAKY, w.ctx0.as<float>(), m->C1P);
        segs_ztaps(c, m->Cx);
        if ((rc = gemm(c, s))) return rc;
    }
    if ((rc = run_dense(g, m->net->ctx1, w.ctx0.as<float>(), m->P * m->C1P, EPI_LEAKY, w.ctx1.as<float>(), m->C2P, s)))
        return rc;
    }
    if ((rc = run_dense(g, m->net->ctx2, w.ctx1.as<float>(), m->C2P, EPI_LEAKY, w.ctx2.as<float>(), m->C3P, s)))
        return rc;
    GemmArgs c = g;
    c.idx = w.idx.as<int32_t>();
    return run_dense(c, m->net->ctx3, w.ctx2.as<float>(), m->C3P, with_idx ? EPI_CTXIDX : EPI_BIAS, w.ksi.as<float>(),
                     m->C4, s);
}

// decoder transform (inverse_prtr_fast, net:384-387) + clamp + write-back into zpad (net:357); with
// xhat: the unclamped output scattered to xhat[img][v][h] instead (forward(), net:104)
int run_dec(lbc_model* m, Work& w, GemmArgs g, hipStream_t s, float* xhat = nullptr) {
    int rc;
    {
        GemmArgs c = g;
        c.nseg = 0;
        c.square_a = 0;
        set_layer(c, m->net->dec0, EPI_BIAS, w.d0.as<float>(), m->NP);
        segs_ztaps(c, m->Cx);
        seg_dense(c, w.yq.as<float>(), m->M, 4 * m->Cx, 4 * m->Cx + m->M);
        if ((rc = gemm(c, s))) return rc;
    }
    float *d0 = w.d0.as<float>(), *d1 = w.d1.as<float>();
    const int W = m->NP;
    if ((rc = run_gdn(g, m->net->ig0, d0, W, true, d1, s))) return rc;
    if ((rc = run_dense(g, m->net->d1, d1, W, EPI_BIAS, d0, W, s))) return rc;
    if ((rc = run_gdn(g, m->net->ig1, d0, W, true, d1, s))) return rc;
    if ((rc = run_dense(g, m->net->d2, d1, W, EPI_BIAS, d0, W, s))) return rc;
    if ((rc = run_gdn(g, m->net->ig2, d0, W, true, d1, s))) return rc;
    if (xhat) return run_dense(g, m->net->d3, d1, W, EPI_SCATTER, xhat, m->Cx, s);   // forward(): xhat, not clamped
    return run_dense(g, m->net->d3, d1, W, EPI_CLAMPZ, nullptr, 0, s);
}

// encoder transform (forward_prtr_fast, net:379-382) + quantize epilogue.  part: 0 all, 1 the layers before the
// quantising GEMM (they do not read the context net's output), 2 the quantising GEMM only
int run_enc(lbc_model* m, Work& w, GemmArgs g, int32_t* sym, int32_t* idx, float* bits, hipStream_t s, int part = 0) {
    int rc;
    float *e0 = w.e0.as<float>(), *e1 = w.e1.as<float>();
    const int W = m->NP;
    if (part != 2) {
    {
        GemmArgs c = g;
        c.nseg = 0;
        c.square_a = 0;
        set_layer(c, m->net->enc0, EPI_BIAS, e0, m->NP);
        segs_ztaps(c, m->Cx);
        Seg& sx = c.seg[c.nseg++];
        sx = Seg{c.geo.x, SEG_X, 0, 0, 0, 4 * m->Cx, 5 * m->Cx};
        if ((rc = gemm(c, s))) return rc;
    }
    if ((rc = run_gdn(g, m->net->g0, e0, W, false, e1, s))) return rc;
    if ((rc = run_dense(g, m->net->e1, e1, W, EPI_BIAS, e0, W, s))) return rc;
    if ((rc = run_gdn(g, m->net->g1, e0, W, false, e1, s))) return rc;
    if ((rc = run_dense(g, m->net->e2, e1, W, EPI_BIAS, e0, W, s))) return rc;
    if ((rc = run_gdn(g, m->net->g2, e0, W, false, e1, s))) return rc;
    if (part == 1) return LBC_OK;
    }
    GemmArgs c = g;
    c.ksi = w.ksi.as<float>();
    c.ldk = m->C4;
    c.sym = sym;
    c.idx = idx;
    c.bits = bits;
    return run_dense(c, m->net->e3, e1, W, EPI_QUANT, w.yq.as<float>(), m->M, s);
}

}  // namespace

extern "C" {

int lbc_create(const lbc_config* cfg, lbc_model** out) {
    if (!cfg || !out) return set_error(LBC_E_ARG, "null argument");
    if (cfg->block_size <= 0 || cfg->n <= 0 || cfg->m <= 0 || cfg->ks[0] != 3 || (cfg->ks[1] != 1 && cfg->ks[1] != 3))
        return set_error(LBC_E_ARG, "unsupported geometry (KS[0] must be 3, KS[1] 1 or 3)");
    if (cfg->ks[2] != 1 && cfg->ks[2] != 3) return set_error(LBC_E_ARG, "bad KS");
    auto* m = new lbc_model();   // no HIP call here: host-only entry points work without a GPU
    m->cfg = *cfg;
    m->B = cfg->block_size;
    m->Cx = 3 * m->B * m->B;
    m->N = cfg->n;
    m->M = cfg->m;
    m->N7 = m->N / 8 * 7;
    m->N6 = m->N / 8 * 6;
    m->C1 = m->N / 8 * 12;
    m->C2 = m->N / 8 * 10;
    m->C3 = m->N / 8 * 8;
    m->C4 = 2 * m->M;
    m->NP = pad16(m->N);
    m->C1P = pad16(m->C1);
    m->C2P = pad16(m->C2);
    m->C3P = pad16(m->C3);
    if (m->Cx % 16 || m->M % 16) {
        delete m;
        return set_error(LBC_E_ARG, "3*B^2 and M must be multiples of 16");
    }
    m->P = cfg->ks[1] == 3 ? 5 : 1;
    const char* lc = getenv("LBIC_L0CACHE");       // 0: layer 0 at five positions per block (A/B runs)
    m->l0_on = m->P == 5 && !(lc && atoi(lc) == 0);
    *out = m;
    return LBC_OK;
}

int lbc_create_sibling(const lbc_model* src, lbc_model** out) {
    if (!src || !out) return set_error(LBC_E_ARG, "null argument");
    if (!src->finalized) return set_error(LBC_E_STATE, "lbc_finalize() not called on the source handle");
    auto* m = new lbc_model();
    m->cfg = src->cfg;
    m->B = src->B; m->Cx = src->Cx; m->N = src->N; m->M = src->M; m->N7 = src->N7; m->N6 = src->N6;
    m->C1 = src->C1; m->C2 = src->C2; m->C3 = src->C3; m->C4 = src->C4; m->P = src->P;
    m->NP = src->NP; m->C1P = src->C1P; m->C2P = src->C2P; m->C3P = src->C3P;
    m->l0_on = src->l0_on;
    m->enc_lds_floor = src->enc_lds_floor;
    m->enc_fork = src->enc_fork;
    m->net = src->net;                    // shared, read-only
    m->finalized = true;
    if (src->tabs_set) {                  // host copies; this handle uploads its own device tables on first use
        m->tabs = src->tabs;
        m->total16 = src->total16;
        m->c16_host = src->c16_host;
        m->meta_host = src->meta_host;
        m->tabs_set = true;
        m->tabs_dirty = true;
    }
    *out = m;
    return LBC_OK;
}

int lbc_set_option(lbc_model* m, int option, long long value) {
    if (!m) return set_error(LBC_E_ARG, "null argument");
    switch (option) {
        case LBC_OPT_ENC_LDS_FLOOR:
            if (value < 0 || value > 160 * 1024) return set_error(LBC_E_ARG, "LDS floor out of range [0, 160 KB]");
            m->enc_lds_floor = (int)value;
            return LBC_OK;
        case LBC_OPT_TEAM_WG_PER_CU:
            if (value < 1 || value > 2) return set_error(LBC_E_ARG, "team workgroups per CU must be 1 or 2");
            m->team_wpc = (int)value;
            return LBC_OK;
        case LBC_OPT_TEAM_SIZE:
            if (value < 0 || value > 32) return set_error(LBC_E_ARG, "team size must be 0 (CUs / 8) .. 32");
            m->team_size = (int)value;
            return LBC_OK;
        case LBC_OPT_ENC_FORK:
            if (value < -1 || value > 1) return set_error(LBC_E_ARG, "encoder fork must be -1 (auto), 0 or 1");
            m->enc_fork = (int)value;
            return LBC_OK;
    }
    return set_error(LBC_E_ARG, "unknown option");
}

void lbc_destroy(lbc_model* m) {
    if (!m) return;
    for (auto& e : m->ev)
        if (e) (void)hipEventDestroy(e);
    for (auto& e : m->lev)
        if (e) (void)hipEventDestroy(e);
    for (auto& st : m->lstream)
        if (st) (void)hipStreamDestroy(st);
    if (m->prof.slots) (void)hipFree(m->prof.slots);
    if (m->prof.snap) (void)hipHostFree(m->prof.snap);
    if (m->enc_exec) (void)hipGraphExecDestroy(m->enc_exec);
    if (m->wf_exec) (void)hipGraphExecDestroy(m->wf_exec);
    for (auto e : m->dec_exec) (void)hipGraphExecDestroy(e);
    for (auto& kv : m->band_exec) (void)hipGraphExecDestroy(kv.second);
    if (m->cap) (void)hipStreamDestroy(m->cap);
    if (m->cap2) (void)hipStreamDestroy(m->cap2);
    for (auto e : m->fev)
        if (e) (void)hipEventDestroy(e);
    if (m->aux) (void)hipStreamDestroy(m->aux);
    if (m->aux_ev) (void)hipEventDestroy(m->aux_ev);
    delete m;
}

int lbc_set_tensor(lbc_model* m, const char* name, const float* host, const int64_t* shape, int ndim) {
    if (!m || !name || !host || (ndim > 0 && !shape)) return set_error(LBC_E_ARG, "null argument");
    std::string n(name);
    auto ends = [&](const char* suf) {
        const size_t l = strlen(suf);
        return n.size() >= l && n.compare(n.size() - l, l, suf) == 0;
    };
    if (ends(".mask") || ends(".pedestal") || ends(".bound") || n.rfind("conditional_gaussian_model.", 0) == 0)
        return LBC_OK;   // derived constants / entropy buffers (set through lbc_set_entropy_tables)
    HostT t;
    size_t cnt = 1;
    for (int i = 0; i < ndim; ++i) {
        t.shape.push_back(shape[i]);
        cnt *= (size_t)shape[i];
    }
    t.v.assign(host, host + cnt);
    m->host[n] = std::move(t);
    m->finalized = false;
    return LBC_OK;
}

int lbc_finalize(lbc_model* m) {
    if (!m) return set_error(LBC_E_ARG, "null model");
    HIPCHK(hipSetDevice(m->cfg.device));
    // pack into a new set and install it only when every layer packed: a failing call (or one on a sibling, which
    // holds no host tensors) leaves the handle's working weights, graphs and finalized state untouched
    auto net = std::make_shared<Net>();   // a new packed set: siblings made earlier keep theirs
    const int Cx = m->Cx, N = m->N, M = m->M;
    static const int one[1][2] = {{0, 0}};
    int rc;
    // context net: layer 0 = 4 masked taps; layer 1 = 1x1, or 3x3 'B' over the 5 layer-0 positions
    if ((rc = pack_conv(m, net->ctx0, "get_meanscale.0", Cx, m->C1, 4, TAPS_A))) return rc;
    if (m->P == 5) rc = pack_conv(m, net->ctx1, "get_meanscale.2", m->C1, m->C2, 5, TAPS_B);
    else rc = pack_conv(m, net->ctx1, "get_meanscale.2", m->C1, m->C2, 1, one);
    if (rc) return rc;
    if ((rc = pack_conv(m, net->ctx2, "get_meanscale.4", m->C2, m->C3, 1, one))) return rc;
    if ((rc = pack_conv(m, net->ctx3, "get_meanscale.6", m->C3, m->C4, 1, one))) return rc;
    if ((rc = pack_first(m, net->enc0, "prtr_forward2", "prtr_forward1", Cx))) return rc;
    if ((rc = pack_gdn(m, net->g0, "prtr_forward3.0", N))) return rc;
    if ((rc = pack_conv(m, net->e1, "prtr_forward3.1", N, m->N7, 1, one))) return rc;
    if ((rc = pack_gdn(m, net->g1, "prtr_forward3.2", m->N7))) return rc;
    if ((rc = pack_conv(m, net->e2, "prtr_forward3.3", m->N7, m->N6, 1, one))) return rc;
    if ((rc = pack_gdn(m, net->g2, "prtr_forward3.4", m->N6))) return rc;
    if ((rc = pack_conv(m, net->e3, "prtr_forward3.5", m->N6, M, 1, one))) return rc;
    if ((rc = pack_first(m, net->dec0, "prtr_inverse2", "prtr_inverse1", M))) return rc;
    if ((rc = pack_gdn(m, net->ig0, "prtr_inverse3.0", N))) return rc;
    if ((rc = pack_conv(m, net->d1, "prtr_inverse3.1", N, m->N7, 1, one))) return rc;
    if ((rc = pack_gdn(m, net->ig1, "prtr_inverse3.2", m->N7))) return rc;
    if ((rc = pack_conv(m, net->d2, "prtr_inverse3.3", m->N7, m->N6, 1, one))) return rc;
    if ((rc = pack_gdn(m, net->ig2, "prtr_inverse3.4", m->N6))) return rc;
    if ((rc = pack_conv(m, net->d3, "prtr_inverse3.5", m->N6, Cx, 1, one))) return rc;
    // the captured graphs and the recorded team program hold the old weight pointers
    if (m->enc_exec) { (void)hipGraphExecDestroy(m->enc_exec); m->enc_exec = nullptr; }
    if (m->wf_exec) { (void)hipGraphExecDestroy(m->wf_exec); m->wf_exec = nullptr; }
    for (auto e : m->dec_exec) (void)hipGraphExecDestroy(e);
    m->dec_exec.clear();
    for (auto& kv : m->band_exec) (void)hipGraphExecDestroy(kv.second);
    m->band_exec.clear();
    m->band_key.clear();
    m->team_key.clear();
    m->net = std::move(net);
    m->finalized = true;
    return LBC_OK;
}

int lbc_pmf_to_quantized_cdf(const float* pmf, int n, int precision, uint32_t* cdf_out) {
    if (!pmf || !cdf_out) return set_error(LBC_E_ARG, "null argument");
    return pmf_to_quantized_cdf(pmf, n, precision, cdf_out);
}

int lbc_set_entropy_tables(lbc_model* m, const float* scale_table, int n_tables, const int32_t* cdf, int cdf_stride,
                           const int32_t* cdf_length, const int32_t* offset) {
    if (!m || !scale_table || !cdf || !cdf_length || !offset) return set_error(LBC_E_ARG, "null argument");
    if (n_tables != 64) return set_error(LBC_E_ARG, "expected the 64-entry scale table (net:13-18)");
    EntropyTables& t = m->tabs;
    t.n_tables = n_tables;
    t.stride = cdf_stride;
    t.table.assign(scale_table, scale_table + n_tables);
    t.cdf.assign(cdf, cdf + (size_t)n_tables * cdf_stride);
    t.length.assign(cdf_length, cdf_length + n_tables);
    t.offset.assign(offset, offset + n_tables);
    // device copies: scale table, and the GPU rANS decoder's LDS image of the CDF rows
    std::vector<uint16_t> c16;
    std::vector<int> meta;
    if (int rc = build_rans_gpu_tables(t, c16, meta)) return rc;
    m->total16 = (int)c16.size();
    m->c16_host = std::move(c16);
    m->meta_host = std::move(meta);
    m->tabs_set = true;
    m->tabs_dirty = true;
    return LBC_OK;
}

int lbc_encode(lbc_model* m, const float* x_dev, int n_img, int Hb, int Wb, float* zhat_dev, int32_t* sym_dev,
               int32_t* idx_dev, float* bits_dev, void* stream) {
    return lbc_encode_ex(m, x_dev, n_img, Hb, Wb, zhat_dev, sym_dev, idx_dev, bits_dev, 0, stream);
}

int lbc_encode_ex(lbc_model* m, const float* x_dev, int n_img, int Hb, int Wb, float* zhat_dev, int32_t* sym_dev,
                  int32_t* idx_dev, float* bits_dev, int flags, void* stream) {
    if (flags & ~LBC_ENC_FRAME_PAD) return set_error(LBC_E_ARG, "unknown encode flags");
    const bool frame_pad = (flags & LBC_ENC_FRAME_PAD) != 0;
    if (!m || !x_dev || !zhat_dev || !sym_dev || !idx_dev) return set_error(LBC_E_ARG, "null argument");
    if (!m->finalized) return set_error(LBC_E_STATE, "lbc_finalize() not called");
    // the validation loop (frame_pad) uses forward()'s likelihood, not the CDFs: it runs before update()
    // too (scale indexes are then not produced)
    if (!m->tabs_set && !frame_pad) return set_error(LBC_E_NOT_UPDATED, "Uninitialized CDFs. Run update() first");
    if (n_img <= 0 || Hb <= 0 || Wb <= 0) return set_error(LBC_E_ARG, "empty frame");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    int rc;
    if ((rc = prepare_device(m))) return rc;
    if ((rc = ensure_workspace(m, n_img, Hb, Wb, s))) return rc;
    const size_t nx = (size_t)n_img * Hb * Wb * m->Cx, nsym = (size_t)n_img * Hb * Wb * m->M;
    if ((rc = m->x_in.alloc(nx * 4)) || (rc = m->sym_buf.alloc(nsym * 4)) || (rc = m->idx_buf.alloc(nsym * 4)) ||
        (rc = m->bits_buf.alloc(nsym * 4)))
        return rc;
    // the graph works on library-owned buffers only, so it survives new caller tensors
    const std::vector<long long> key = {n_img, Hb, Wb, (long long)m->x_in.p, (long long)m->zpad.p,
                                        (long long)m->sym_buf.p, (long long)m->lane[0].ctx0.p,
                                        (long long)m->table_dev.p, m->prof.sample_every, flags,
                                        m->enc_lds_floor, m->enc_fork};
    if (!m->enc_exec || key != m->enc_key) {
        std::lock_guard<std::mutex> lk(g_capture_mu);
        if (m->enc_exec) { (void)hipGraphExecDestroy(m->enc_exec); m->enc_exec = nullptr; }
        HIPCHK(hipStreamBeginCapture(m->cap, hipStreamCaptureModeThreadLocal));
        int crc = prof_range_begin(&m->prof, 0, m->cap);
        drop_recs(m->prof, 0);
        const int4* blocks = m->blocks_enc.as<int4>();
        const bool fork = enc_fork_on(m->Mmax, m->enc_fork);   // (sampled: launch spans only, no launch-to-launch period)
        g_prof = &m->prof;
        m->prof.nochain = fork;
        for (size_t t = 0; t < m->step_off.size(); ++t)
            if (m->step_cnt[t] > m->lane[0].rows) crc = set_error(LBC_E_STATE, "encoder workspace too small");
        for (size_t t = 0; t < m->step_off.size() && !crc; ++t) {
            m->prof.step(m->prof.sample_every > 0 && (t % m->prof.sample_every) == 0);
            GemmArgs g = base_args(m, blocks + m->step_off[t], m->step_cnt[t], m->x_in.as<float>(), n_img, Hb, Wb);
            const int4* cells = m->l0_on ? m->cells_enc.as<int4>() + m->cell_off[t] : nullptr;
            const int ncells = m->l0_on ? m->cell_cnt[t] : 0;
            if (fork) {
                // fork: the context net on cap2, the transform's first layers on cap; join before quantising
                if (!crc) crc = hip_rc(hipEventRecord(m->fev[0], m->cap));
                if (!crc) crc = hip_rc(hipStreamWaitEvent(m->cap2, m->fev[0], 0));
                if (!crc) crc = run_ctx(m, m->lane[0], g, false, m->cap2, frame_pad, cells, ncells);
                if (!crc) crc = hip_rc(hipEventRecord(m->fev[1], m->cap2));
                if (!crc) crc = run_enc(m, m->lane[0], g, nullptr, nullptr, nullptr, m->cap, 1);
                if (!crc) crc = hip_rc(hipStreamWaitEvent(m->cap, m->fev[1], 0));
                if (!crc) crc = run_enc(m, m->lane[0], g, m->sym_buf.as<int32_t>(), m->idx_buf.as<int32_t>(),
                                        m->bits_buf.as<float>(), m->cap, 2);
            } else {
                if (!crc) crc = run_ctx(m, m->lane[0], g, false, m->cap, frame_pad, cells, ncells);
                if (!crc) crc = run_enc(m, m->lane[0], g, m->sym_buf.as<int32_t>(), m->idx_buf.as<int32_t>(),
                                        m->bits_buf.as<float>(), m->cap);
            }
            if (!crc) crc = run_dec(m, m->lane[0], g, m->cap);
        }
        m->prof.active = false;
        m->prof.nochain = false;
        m->prof.used0 = m->prof.next;
        g_prof = nullptr;
        hipGraph_t graph = nullptr;
        const hipError_t e = hipStreamEndCapture(m->cap, &graph);
        if (crc) { if (graph) (void)hipGraphDestroy(graph); return crc; }
        if (e != hipSuccess) return set_error(LBC_E_HIP, std::string("encoder capture: ") + hipGetErrorString(e));
        const hipError_t ei = hipGraphInstantiate(&m->enc_exec, graph, nullptr, nullptr, 0);
        (void)hipGraphDestroy(graph);
        if (ei != hipSuccess) return set_error(LBC_E_HIP, std::string("encoder instantiate: ") + hipGetErrorString(ei));
        m->enc_key = key;
    }
    HIPCHK(hipEventRecord(m->ev[0], s));
    HIPCHK(hipMemcpyAsync(m->x_in.p, x_dev, nx * 4, hipMemcpyDeviceToDevice, s));
    HIPCHK(hipMemsetAsync(m->zpad.p, 0, (size_t)n_img * (Hb + 2) * (Wb + 4) * m->Cx * sizeof(float), s));
    if (m->l0_on &&
        (rc = launch_l0_border(m->l0.as<float>(), n_img, Hb, Wb, m->C1P, frame_pad ? nullptr : m->net->ctx0.bias.as<float>(), s)))
        return rc;
    HIPCHK(hipGraphLaunch(m->enc_exec, s));
    m->prof.replays[0] += 1;
    if (m->prof.sample_every && m->prof.slots && m->prof.snap && m->prof.used0 > 0 && m->prof.nsnap < Prof::kSnaps) {
        // this replay's stamps, before the next replay zeroes them (stream order)
        HIPCHK(hipMemcpyAsync(m->prof.snap + (size_t)m->prof.nsnap * kSlotsPerRange * kSlotU64, m->prof.slots,
                              (size_t)m->prof.used0 * kSlotU64 * 8, hipMemcpyDeviceToHost, s));
        m->prof.nsnap += 1;
    }
    if ((rc = launch_copy_interior(m->zpad.as<float>(), zhat_dev, n_img, Hb, Wb, m->Cx, s))) return rc;
    HIPCHK(hipMemcpyAsync(sym_dev, m->sym_buf.p, nsym * 4, hipMemcpyDeviceToDevice, s));
    HIPCHK(hipMemcpyAsync(idx_dev, m->idx_buf.p, nsym * 4, hipMemcpyDeviceToDevice, s));
    if (bits_dev) HIPCHK(hipMemcpyAsync(bits_dev, m->bits_buf.p, nsym * 4, hipMemcpyDeviceToDevice, s));
    HIPCHK(hipEventRecord(m->ev[1], s));
    m->enc_timed = true;
    return LBC_OK;
}

// ---------------------------------------------------------------- band pipeline for frames split over GPUs
// Block rows [v0, v0 + Hb_band) of n_img frames.  The workspace is the band's: zpad rows 0..1 (the zero border of a
// whole frame) hold the two block rows above the band, which the caller hands over before every step range.
int lbc_band_begin(lbc_model* m, const float* x_dev, int n_img, int Hb_band, int Wb, int v0, void* stream) {
    if (!m || !x_dev) return set_error(LBC_E_ARG, "null argument");
    if (!m->finalized) return set_error(LBC_E_STATE, "lbc_finalize() not called");
    if (!m->tabs_set) return set_error(LBC_E_NOT_UPDATED, "Uninitialized CDFs. Run update() first");
    if (n_img <= 0 || Hb_band <= 0 || Wb <= 0 || v0 < 0) return set_error(LBC_E_ARG, "empty band");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    int rc;
    if ((rc = prepare_device(m))) return rc;
    if ((rc = ensure_workspace(m, n_img, Hb_band, Wb, s))) return rc;
    const size_t nx = (size_t)n_img * Hb_band * Wb * m->Cx, nsym = (size_t)n_img * Hb_band * Wb * m->M;
    if ((rc = m->x_in.alloc(nx * 4)) || (rc = m->sym_buf.alloc(nsym * 4)) || (rc = m->idx_buf.alloc(nsym * 4)) ||
        (rc = m->bits_buf.alloc(nsym * 4)))
        return rc;
    // the step-range graphs hold workspace pointers: rebuilt when any of them (or the band) changed
    const std::vector<long long> key = {n_img, Hb_band, Wb, v0, (long long)m->x_in.p, (long long)m->zpad.p,
                                        (long long)m->sym_buf.p, (long long)m->lane[0].ctx0.p,
                                        (long long)m->table_dev.p, (long long)m->net.get()};
    if (key != m->band_key) {
        m->band_key = key;
        for (auto& kv : m->band_exec) (void)hipGraphExecDestroy(kv.second);
        m->band_exec.clear();
    }
    m->band_v0 = v0;
    HIPCHK(hipMemcpyAsync(m->x_in.p, x_dev, nx * 4, hipMemcpyDeviceToDevice, s));
    HIPCHK(hipMemsetAsync(m->zpad.p, 0, (size_t)n_img * (Hb_band + 2) * (Wb + 4) * m->Cx * sizeof(float), s));
    return LBC_OK;
}

// two block rows [n_img][2][Wb][Cx] <-> zpad rows r0, r0 + 1 (interior columns)
static int band_rows_copy(lbc_model* m, float* rows, int r0, bool to_zpad, hipStream_t s) {
    const size_t w = (size_t)m->ws_Wb * m->Cx * sizeof(float), pitch = (size_t)(m->ws_Wb + 4) * m->Cx * sizeof(float);
    for (int i = 0; i < m->ws_n; ++i) {
        float* z = m->zpad.as<float>() + (((size_t)i * (m->ws_Hb + 2) + r0) * (m->ws_Wb + 4) + 2) * m->Cx;
        float* h = rows + (size_t)i * 2 * m->ws_Wb * m->Cx;
        HIPCHK(to_zpad ? hipMemcpy2DAsync(z, pitch, h, w, w, 2, hipMemcpyDeviceToDevice, s)
                       : hipMemcpy2DAsync(h, w, z, pitch, w, 2, hipMemcpyDeviceToDevice, s));
    }
    return LBC_OK;
}

int lbc_band_run(lbc_model* m, int t0, int t1, const float* halo_dev, float* edge_dev, void* stream) {
    if (!m || m->band_v0 < 0) return set_error(LBC_E_STATE, "lbc_band_begin() not called");
    if (t1 < t0) return set_error(LBC_E_ARG, "bad step range");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    int rc;
    if (halo_dev && (rc = band_rows_copy(m, const_cast<float*>(halo_dev), 0, true, s))) return rc;
    // global step t codes block (v, h) with h + 2 v = t: the band's local step t - 2 v0
    const int T = (int)m->step_off.size();
    const int a = std::max(0, t0 - 2 * m->band_v0), b = std::min(T, t1 - 2 * m->band_v0);
    if (a < b) {
        auto it = m->band_exec.find({a, b});
        if (it == m->band_exec.end()) {
            std::lock_guard<std::mutex> lk(g_capture_mu);
            HIPCHK(hipStreamBeginCapture(m->cap, hipStreamCaptureModeThreadLocal));
            int crc = LBC_OK;
            const int4* blocks = m->blocks_enc.as<int4>();
            for (int t = a; t < b && !crc; ++t) {
                GemmArgs g = base_args(m, blocks + m->step_off[t], m->step_cnt[t], m->x_in.as<float>(), m->ws_n,
                                       m->ws_Hb, m->ws_Wb);
                // layer 0 at five positions (no layer-0 cache): the band's row -1 is real data, not the frame border
                crc = run_ctx(m, m->lane[0], g, false, m->cap);
                if (!crc) crc = run_enc(m, m->lane[0], g, m->sym_buf.as<int32_t>(), m->idx_buf.as<int32_t>(),
                                        m->bits_buf.as<float>(), m->cap);
                if (!crc) crc = run_dec(m, m->lane[0], g, m->cap);
            }
            hipGraph_t graph = nullptr;
            const hipError_t e = hipStreamEndCapture(m->cap, &graph);
            if (crc) { if (graph) (void)hipGraphDestroy(graph); return crc; }
            if (e != hipSuccess) return set_error(LBC_E_HIP, std::string("band capture: ") + hipGetErrorString(e));
            hipGraphExec_t ex = nullptr;
            const hipError_t ei = hipGraphInstantiate(&ex, graph, nullptr, nullptr, 0);
            (void)hipGraphDestroy(graph);
            if (ei != hipSuccess) return set_error(LBC_E_HIP, std::string("band instantiate: ") + hipGetErrorString(ei));
            it = m->band_exec.emplace(std::make_pair(a, b), ex).first;
        }
        HIPCHK(hipGraphLaunch(it->second, s));
    }
    if (edge_dev && (rc = band_rows_copy(m, edge_dev, m->ws_Hb, false, s))) return rc;
    return LBC_OK;
}

int lbc_band_end(lbc_model* m, float* zhat_dev, int32_t* sym_dev, int32_t* idx_dev, float* bits_dev, void* stream) {
    if (!m || m->band_v0 < 0) return set_error(LBC_E_STATE, "lbc_band_begin() not called");
    if (!zhat_dev || !sym_dev || !idx_dev) return set_error(LBC_E_ARG, "null argument");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    int rc;
    if ((rc = launch_copy_interior(m->zpad.as<float>(), zhat_dev, m->ws_n, m->ws_Hb, m->ws_Wb, m->Cx, s))) return rc;
    const size_t nsym = (size_t)m->ws_n * m->ws_Hb * m->ws_Wb * m->M;
    HIPCHK(hipMemcpyAsync(sym_dev, m->sym_buf.p, nsym * 4, hipMemcpyDeviceToDevice, s));
    HIPCHK(hipMemcpyAsync(idx_dev, m->idx_buf.p, nsym * 4, hipMemcpyDeviceToDevice, s));
    if (bits_dev) HIPCHK(hipMemcpyAsync(bits_dev, m->bits_buf.p, nsym * 4, hipMemcpyDeviceToDevice, s));
    m->band_v0 = -1;
    return LBC_OK;
}

int lbc_forward(lbc_model* m, const float* x_dev, const float* zhat_dev, int n_img, int Hb, int Wb, float* xhat_dev,
                float* info_dev, void* stream) {
    if (!m || !x_dev || !zhat_dev || !xhat_dev || !info_dev) return set_error(LBC_E_ARG, "null argument");
    if (!m->finalized) return set_error(LBC_E_STATE, "lbc_finalize() not called");   // (no CDFs needed)
    if (n_img <= 0 || Hb <= 0 || Wb <= 0) return set_error(LBC_E_ARG, "empty frame");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    int rc;
    if ((rc = prepare_device(m))) return rc;
    if ((rc = ensure_workspace(m, n_img, Hb, Wb, s))) return rc;
    const size_t nsym = (size_t)n_img * Hb * Wb * m->M;
    if ((rc = m->sym_buf.alloc(nsym * 4)) || (rc = m->idx_buf.alloc(nsym * 4))) return rc;
    // teacher forcing: the given zhat is the reconstruction every block sees (zero border as before)
    HIPCHK(hipMemsetAsync(m->zpad.p, 0, (size_t)n_img * (Hb + 2) * (Wb + 4) * m->Cx * sizeof(float), s));
    if ((rc = launch_fill_interior(zhat_dev, m->zpad.as<float>(), n_img, Hb, Wb, m->Cx, s))) return rc;
    // every block is independent here: chunks of the encoder workspace's row capacity, eager launches
    Work& w = m->lane[0];
    const int total = n_img * Hb * Wb;
    const int4* blocks = m->blocks_enc.as<int4>();    // all blocks (wavefront order; outputs go by block)
    for (int off = 0; off < total && !rc; off += w.rows) {
        const int cnt = std::min(w.rows, total - off);
        GemmArgs g = base_args(m, blocks + off, cnt, x_dev, n_img, Hb, Wb);
        if (!rc) rc = run_ctx(m, w, g, false, s, true);
        if (!rc) rc = run_enc(m, w, g, m->sym_buf.as<int32_t>(), m->idx_buf.as<int32_t>(), info_dev, s);
        if (!rc) rc = run_dec(m, w, g, s, xhat_dev);
    }
    return rc;
}

int lbc_rans_encode(const lbc_model* m, const int32_t* sym, const int32_t* idx, size_t n, uint8_t** out, size_t* len) {
    if (!m || !sym || !idx || !out || !len) return set_error(LBC_E_ARG, "null argument");
    if (!m->tabs_set) return set_error(LBC_E_NOT_UPDATED, "Uninitialized CDFs. Run update() first");
    std::vector<uint8_t> bytes;
    int rc = rans_encode(m->tabs, sym, idx, n, bytes);
    if (rc) return rc;
    *out = static_cast<uint8_t*>(malloc(std::max<size_t>(bytes.size(), 1)));
    std::memcpy(*out, bytes.data(), bytes.size());
    *len = bytes.size();
    return LBC_OK;
}

int lbc_rans_decode_host(const lbc_model* m, const uint8_t* data, size_t len, const int32_t* idx, size_t n,
                         int32_t* sym_out) {
    if (!m || !data || !idx || !sym_out) return set_error(LBC_E_ARG, "null argument");
    if (!m->tabs_set) return set_error(LBC_E_NOT_UPDATED, "Uninitialized CDFs. Run update() first");
    return rans_decode_host(m->tabs, data, len, idx, n, sym_out);
}

int lbc_rans_decode_gpu(lbc_model* m, const uint8_t* const* streams, const size_t* lens, int n_streams,
                        const int32_t* idx_dev, int n_chunks, int32_t* sym_dev, void* stream) {
    if (!m || !streams || !lens || !idx_dev || !sym_dev) return set_error(LBC_E_ARG, "null argument");
    if (!m->tabs_set) return set_error(LBC_E_NOT_UPDATED, "Uninitialized CDFs. Run update() first");
    if (n_streams <= 0 || n_chunks < 0) return set_error(LBC_E_ARG, "bad stream / chunk count");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    int rc;
    if ((rc = prepare_device(m))) return rc;
    std::vector<std::pair<const uint8_t*, size_t>> subs;
    for (int i = 0; i < n_streams; ++i) subs.emplace_back(streams[i], lens[i]);
    if ((rc = upload_streams(m, subs, s))) return rc;
    RansArgs r = rans_args(m);
    r.rows = n_streams;
    double nsym = (double)n_streams * n_chunks * m->M;
    r.sparse = rans_sparse_choice(lens, n_streams, nsym);
    for (int c = 0; c < n_chunks && !rc; ++c) {
        r.idx = idx_dev + (size_t)c * n_streams * m->M;
        r.sym_out = sym_dev + (size_t)c * n_streams * m->M;
        rc = launch_rans_decode(r, s);
    }
    if (rc) return rc;
    return check_status(m, (size_t)n_streams, s, false);
}

// ---------------------------------------------------------------------------------------------- single image
// k_dec_one's program for this handle (one.hip): the raster step's 12 operations (context net x 4, rANS, decoder x 7,
// exactly the layers, segments and epilogues run_ctx / run_dec give the graph decoder) and the placement of every weight
// column tile in the LDS of one workgroup (greedy: each tile to the workgroup holding the fewest tiles of its GEMM, then
// the least bytes).  KS[1] = 3 runs the context net under the layer-0 cache as the graph decoder does (run_ctx, raster):
// layer 0 computes its block's cell (and at a row end the border cell it owns) into the cache, layer 1 reads its five
// 'B' taps as four cache cells and layer 0's granules; a column tile whose K x 16 weights exceed one workgroup's LDS
// (B4_highrate's layer 1, K = 3,840) is held as two halves (OneOp::half).  Applies to Mlat <= 256, K slices of <= 11
// k-blocks (<= 32 for a half-tile op), weights that fit the grid's LDS; returns with m->one_ok = 0 otherwise.
static int one_prepare(lbc_model* m, int Hb, int Wb, int cus) {
    const std::vector<long long> key = {Hb, Wb, cus, m->net->gen, (long long)m->zpad.p, (long long)m->words.p,
                                        (long long)m->table_dev.p, (long long)m->st_x.p, (long long)m->cdf16_dev.p,
                                        (long long)m->tmeta_dev.p, (long long)m->word_base.p, (long long)m->st_status.p,
                                        (long long)m->st_ptr.p, (long long)m->word_count.p, (long long)m->l0.p};
    if (key == m->one_key) return LBC_OK;
    m->one_ok = 0;
    m->one_key = key;
    if ((m->P != 1 && !m->l0_on) || m->M > 256 || cus < 16) return LBC_OK;
    const bool l0 = m->l0_on;
    const Net& n = *m->net;
    std::vector<OneOp> ops(ONE_MAXOPS);
    auto gemm_op = [&](int o, const Layer& L, int epi, int sq) {
        OneOp& q = ops[o];
        q = OneOp{};
        q.W = L.W.as<float>();
        q.bias = L.bias.as<float>();
        q.K = L.K;
        q.N = L.N;
        q.NB16 = L.NB16;
        q.epi = epi;
        q.sq = sq;
        q.gx_src = -1;
        q.gw = (L.N + 15) / 16 * 16;
    };
    auto gran_seg = [&](int o, int src, int k0, int k1) {
        ops[o].seg[ops[o].nseg++] = OneSeg{ONE_GRAN, src, 0, 0, 0, k0, k1};
    };
    auto ztaps = [&](int o) {
        for (int t = 0; t < 4; ++t)
            ops[o].seg[ops[o].nseg++] = OneSeg{ONE_ZTAP, -1, 0, TAPS_A[t][0], TAPS_A[t][1], t * m->Cx, (t + 1) * m->Cx};
    };
    gemm_op(0, n.ctx0, EPI_LEAKY, 0);  ztaps(0);                       // get_meanscale.0 ('A' 3x3 on the window)
    gemm_op(1, n.ctx1, EPI_LEAKY, 0);
    if (l0) {       // layer 0 into the cache; layer 1 = the 3x3 'B' taps: four cache cells, then layer 0's own output
        ops[0].l0out = 1;
        for (int t = 0; t < 4; ++t)
            ops[1].seg[ops[1].nseg++] = OneSeg{ONE_L0TAP, 0, 0, TAPS_B[t][0], TAPS_B[t][1], t * m->C1P, (t + 1) * m->C1P};
        gran_seg(1, 0, 4 * m->C1P, 5 * m->C1P);
        ops[1].l0seg = 1;
        if (n.ctx1.K != 5 * m->C1P || n.ctx0.N != m->C1 || !m->l0.p) return LBC_OK;
    } else {
        gran_seg(1, 0, 0, n.ctx1.K);
    }
    gemm_op(2, n.ctx2, EPI_LEAKY, 0);  gran_seg(2, 1, 0, n.ctx2.K);
    gemm_op(3, n.ctx3, EPI_CTXIDX, 0); gran_seg(3, 2, 0, n.ctx3.K);
    ops[4] = OneOp{};                                                 // the rANS decode: y_qnt granules
    ops[4].N = m->M;
    ops[4].gw = (m->M + 15) / 16 * 16;
    ops[4].gx_src = -1;
    gemm_op(5, n.dec0, EPI_BIAS, 0);   ztaps(5); gran_seg(5, 4, 4 * m->Cx, 4 * m->Cx + m->M);
    gemm_op(6, n.ig0, EPI_IGDN, 1);    gran_seg(6, 5, 0, n.ig0.K);  ops[6].gx_src = 5;
    gemm_op(7, n.d1, EPI_BIAS, 0);     gran_seg(7, 6, 0, n.d1.K);
    gemm_op(8, n.ig1, EPI_IGDN, 1);    gran_seg(8, 7, 0, n.ig1.K);  ops[8].gx_src = 7;
    gemm_op(9, n.d2, EPI_BIAS, 0);     gran_seg(9, 8, 0, n.d2.K);
    gemm_op(10, n.ig2, EPI_IGDN, 1);   gran_seg(10, 9, 0, n.ig2.K); ops[10].gx_src = 9;
    gemm_op(11, n.d3, EPI_CLAMPZ, 0);  gran_seg(11, 10, 0, n.d3.K);
    if (n.d3.N != m->Cx || n.dec0.K != 4 * m->Cx + m->M || n.ctx0.K != 4 * m->Cx || n.ctx3.N != 2 * m->M) return LBC_OK;
    // weight capacity of one workgroup's LDS; a column tile larger than that, or with K slices past ONE_LL_MAX - 1
    // k-blocks, is held as two halves (only layer-0 cache taps and granules as inputs there)
    const int red_rows = l0 ? 3 : 1;
    const size_t cap_f4 = (160 * 1024 - one_lds_bytes(0, red_rows)) / 16;
    for (int o = 0; o < ONE_MAXOPS; ++o) {
        if (o == 4) continue;
        const int nkb = ops[o].K / 16;
        if ((size_t)nkb * 64 > cap_f4 || nkb / KSPLIT > ONE_LL_MAX - 1) {
            bool ok = l0 && (nkb + KSPLIT - 1) / KSPLIT <= ONE_LLH_MAX && ops[o].epi == EPI_LEAKY && !ops[o].sq;
            // (one_gemm_half: cache taps, then granules -- every cache segment before the first granule segment)
            bool gran_seen = false;
            for (int i = 0; i < ops[o].nseg; ++i) {
                ok &= ops[o].seg[i].kind != ONE_ZTAP && !(gran_seen && ops[o].seg[i].kind == ONE_L0TAP);
                gran_seen |= ops[o].seg[i].kind == ONE_GRAN;
            }
            if (!ok) return LBC_OK;
            ops[o].half = 1;
        }
    }
    // shape checks: K slices of 0..12 k-blocks (half-tile ops: 0..32), granule sources wide enough, segments contiguous
    for (int o = 0; o < ONE_MAXOPS; ++o) {
        const OneOp& q = ops[o];
        if (o == 4) continue;
        const int nkb = q.K / 16;
        if (q.K % 16 || nkb < 1 || !q.W || !q.bias) return LBC_OK;
        if (!q.half && nkb / KSPLIT > ONE_LL_MAX - 1) return LBC_OK;
        for (int i = 0; i < q.nseg; ++i) {
            const OneSeg& sg = q.seg[i];
            if ((sg.k0 & 15) || (i == 0 ? sg.k0 != 0 : sg.k0 != q.seg[i - 1].k1)) return LBC_OK;
            if (sg.kind == ONE_GRAN && sg.c0 + sg.k1 - sg.k0 > ops[sg.src].gw) return LBC_OK;
        }
        if (q.seg[q.nseg - 1].k1 != q.K) return LBC_OK;
    }
    // granule buffers (+ the half-tile ops' partials: two step parities x column tiles x 4 slices x 16)
    size_t ng = 0;
    for (const OneOp& q : ops) ng += (size_t)q.gw + (q.half ? (size_t)2 * q.gw * 4 : 0);
    int rc;
    if ((rc = m->one_gran.alloc(ng * 8))) return rc;
    size_t at = 0;
    for (OneOp& q : ops) {
        q.gran = m->one_gran.as<unsigned long long>() + at;
        at += (size_t)q.gw;
        if (q.half) {
            q.pgran = m->one_gran.as<unsigned long long>() + at;
            at += (size_t)2 * q.gw * 4;
        }
    }
    // weight placement: workgroups 0 .. G - 2 hold tiles, G - 1 decodes the stream.  The half-tile pieces first (the
    // largest), each to a workgroup that holds no other piece of a half-tile op (half 1 waits for half 0's partials
    // inside the same operation: the two must run on different workgroups)
    const int G = cus;
    std::vector<size_t> load(G, 0);
    std::vector<int> held(G, 0), has_half(G, 0);
    std::vector<int4> tiles((size_t)G * ONE_NT_MAX, make_int4(-1, 0, 0, 0));
    std::vector<int> order;
    for (int o = 0; o < ONE_MAXOPS; ++o)
        if (o != 4 && ops[o].half) order.push_back(o);
    for (int o = 0; o < ONE_MAXOPS; ++o)
        if (o != 4 && !ops[o].half) order.push_back(o);
    for (int o : order) {
        const int nt_n = (ops[o].N + 15) / 16;
        const int nkb = ops[o].K / 16;
        std::vector<int> of_op(G, 0);
        for (int nt = 0; nt < nt_n; ++nt) {
            for (int pc = ops[o].half ? 1 : 0; pc <= (ops[o].half ? 2 : 0); ++pc) {
                const int kb_lo = pc == 2 ? 4 * nkb / KSPLIT : 0, kb_hi = pc == 1 ? 4 * nkb / KSPLIT : nkb;
                const size_t sz = (size_t)(kb_hi - kb_lo) * 64;
                int best = -1;
                for (int g = 0; g < G - 1; ++g) {
                    if (held[g] >= ONE_NT_MAX || load[g] + sz > cap_f4 || (pc && has_half[g])) continue;
                    if (best < 0 || of_op[g] < of_op[best] || (of_op[g] == of_op[best] && load[g] < load[best])) best = g;
                }
                if (best < 0) return LBC_OK;       // does not fit: the graph decoder keeps single images
                tiles[(size_t)best * ONE_NT_MAX + held[best]] = make_int4(o, nt, (int)load[best], pc);
                load[best] += sz;
                held[best] += 1;
                of_op[best] += 1;
                has_half[best] |= pc ? 1 : 0;
            }
        }
    }
    size_t wmax = 0;
    for (size_t l : load) wmax = std::max(wmax, l);
    if ((rc = dev_upload(m->one_ops, ops.data(), ops.size() * sizeof(OneOp)))) return rc;
    if ((rc = dev_upload(m->one_tiles, tiles.data(), tiles.size() * sizeof(int4)))) return rc;
    RansArgs r = rans_args(m);
    r.rows = 1;
    r.sparse = 1;
    if ((rc = dev_upload(m->one_rans, &r, sizeof(r)))) return rc;
    if ((rc = m->one_fail.alloc(64))) return rc;
    OneArgs& a = m->one_args;
    a = OneArgs{};
    a.ops = m->one_ops.as<OneOp>();
    a.nops = ONE_MAXOPS;
    a.rans_op = 4;
    a.rans_wg = G - 1;
    a.tiles = m->one_tiles.as<int4>();
    a.wlds_f4 = (int)wmax;
    a.zpad = m->zpad.as<float>();
    a.Hp = Hb + 2;
    a.Wp = Wb + 4;
    a.Cx = m->Cx;
    a.Hb = Hb;
    a.Wb = Wb;
    a.l0 = l0 ? m->l0.as<float>() : nullptr;
    a.C1P = m->C1P;
    a.red_rows = red_rows;
    a.rans = m->one_rans.as<RansArgs>();
    a.Mlat = m->M;
    a.table = m->table_dev.as<float>();
    a.fail = m->one_fail.as<unsigned>();
    a.tmo = 100000000ull;     // 1 s per wait (100 MHz)
    a.lazy_z = Wb >= 3 ? 1 : 0;
    a.rans_lds_tab = (size_t)m->total16 * 2 <= wmax * 16 && m->total16 % 8 == 0 ? 1 : 0;
    a.ts_step = (Hb / 2) * Wb + Wb / 2;
    if ((rc = m->one_ts.alloc(ONE_TS_WORDS * sizeof(unsigned long long)))) return rc;
    if (one_blocks_per_cu(one_lds_bytes(a.wlds_f4, a.red_rows), l0) < 1) return LBC_OK;
    m->one_grid = G;
    m->one_ok = 1;
    return LBC_OK;
}

// One image through k_dec_one when it applies (LBIC_ONE=0 keeps the row graphs: A/B runs).  *used = 1: decoded (zpad
// holds the reconstruction); 0: not applicable; -1: the launch timed out (counted; the caller decodes with the graphs
// after re-uploading the stream).
static int decode_one(lbc_model* m, const size_t* lens, int Hb, int Wb, hipStream_t s, int* used) {
    *used = 0;
    const char* e = getenv("LBIC_ONE");
    // (no_one: a team fallback after a residency timeout -- the chip's CUs are held elsewhere, and k_dec_one needs
    // every one of them co-resident, so it would likely time out again: go to the row graphs directly)
    // k_dec_one decodes with the sparse rANS variant at any rate (its misses search the table image, copied into the
    // rANS workgroup's LDS; bit-identical to the dense coder); LBIC_RANS_SPARSE=0 (the dense coder forced) keeps the
    // row graphs
    const char* rs = getenv("LBIC_RANS_SPARSE");
    (void)lens;
    if ((e && atoi(e) == 0) || m->no_one || (rs && atoi(rs) == 0)) return LBC_OK;
    int cus = 0, rc;
    HIPCHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, m->cfg.device));
    if ((rc = one_prepare(m, Hb, Wb, cus))) return rc;
    if (!m->one_ok) return LBC_OK;
    OneArgs a = m->one_args;
    if (const char* t = getenv("LBIC_ONE_TMO")) a.tmo = std::max(1ull, strtoull(t, nullptr, 10));   // test hook
    const char* st = getenv("LBIC_ONE_STAMPS");
    std::vector<unsigned long long> ts0(ONE_TS_WORDS, 0ull);
    if (st && atoi(st)) {
        for (int o = 0; o < ONE_MAXOPS; ++o) ts0[o * 4] = ~0ull;
        HIPCHK(hipMemcpyAsync(m->one_ts.p, ts0.data(), ts0.size() * 8, hipMemcpyHostToDevice, s));
        a.ts = m->one_ts.as<unsigned long long>();
    }
    HIPCHK(hipMemsetAsync(m->one_gran.p, 0, m->one_gran.bytes, s));
    HIPCHK(hipMemsetAsync(m->one_fail.p, 0, 64, s));
    // (KS[1] = 3) the layer-0 cache's row -1, as the graph decoder sets it: constant LeakyReLU(bias)
    if (a.l0 && (rc = launch_l0_border(m->l0.as<float>(), 1, Hb, Wb, m->C1P, m->net->ctx0.bias.as<float>(), s))) return rc;
    if ((rc = launch_dec_one(a, m->one_grid, s))) return rc;
    if (a.ts) {
        m->one_ts_host.assign(ONE_TS_WORDS, 0ull);
        HIPCHK(hipMemcpyAsync(m->one_ts_host.data(), a.ts, ONE_TS_WORDS * 8, hipMemcpyDeviceToHost, s));
    }
    unsigned fail = 0;
    HIPCHK(hipMemcpyAsync(&fail, m->one_fail.p, sizeof(unsigned), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (fail > 1)   // k_dec_one writes 1 (a wait timed out) and nothing else: any other word is a protocol error
        return set_error(LBC_E_STATE, "single-image decode: unexpected failure word " + std::to_string(fail));
    if (fail == 1) {
        m->one_timeouts += 1;
        static std::atomic<bool> noted{false};
        if (!noted.exchange(true))
            fprintf(stderr, "[lbic] single-image decode: wait timeout, decoding through the row graphs (counted)\n");
        *used = -1;
        return LBC_OK;
    }
    *used = 1;
    return LBC_OK;
}

int lbc_decode(lbc_model* m, const uint8_t* const* streams, const size_t* lens, int n_img, int Hb, int Wb,
               float* zhat_dev, void* stream) {
    if (!m || !streams || !lens || !zhat_dev) return set_error(LBC_E_ARG, "null argument");
    if (!m->finalized) return set_error(LBC_E_STATE, "lbc_finalize() not called");
    if (!m->tabs_set) return set_error(LBC_E_NOT_UPDATED, "Uninitialized CDFs. Run update() first");
    if (n_img <= 0 || Hb <= 0 || Wb <= 0) return set_error(LBC_E_ARG, "empty frame");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    int rc;
    if ((rc = prepare_device(m))) return rc;
    if ((rc = ensure_workspace(m, n_img, Hb, Wb, s))) return rc;
    std::vector<std::pair<const uint8_t*, size_t>> subs;
    for (int i = 0; i < n_img; ++i) subs.emplace_back(streams[i], lens[i]);
    if ((rc = upload_streams(m, subs, s))) return rc;
    HIPCHK(hipEventRecord(m->ev[2], s));
    HIPCHK(hipMemsetAsync(m->zpad.p, 0, (size_t)n_img * (Hb + 2) * (Wb + 4) * m->Cx * sizeof(float), s));
    m->dec_path_last = 0;
    if (n_img == 1) {     // one image: the persistent single-image decoder (one.hip) where it applies
        int used = 0;
        if ((rc = decode_one(m, lens, Hb, Wb, s, &used))) return rc;
        if (used == 1) {
            m->dec_path_last = 1;
            if ((rc = launch_copy_interior(m->zpad.as<float>(), zhat_dev, n_img, Hb, Wb, m->Cx, s))) return rc;
            HIPCHK(hipEventRecord(m->ev[3], s));
            m->dec_timed = true;
            return check_status(m, (size_t)n_img, s, true);
        }
        if (used == -1) {   // a timed-out launch advanced the coder state: start again
            if ((rc = upload_streams(m, subs, s))) return rc;
            HIPCHK(hipEventRecord(m->ev[2], s));
            HIPCHK(hipMemsetAsync(m->zpad.p, 0, (size_t)n_img * (Hb + 2) * (Wb + 4) * m->Cx * sizeof(float), s));
        }
    }
    // image groups -> lanes: every lane runs its own raster chain on its own stream, so the small
    // per-step kernels of different groups fill the GPU side by side.  Each lane's block row (Wb raster
    // steps, 13 launches each) is one captured HIP graph replayed Hb times: its kernels read the row
    // from the lane's device counter, which the graph's last node advances.
    // one lane by default: on ROCm 7.2 several streams' graphs did not overlap usefully
    int G = 1;
    if (const char* e = getenv("LBIC_DEC_LANES")) G = std::max(1, std::min(std::min(kLanes, n_img), atoi(e)));
    int g0[kLanes + 1];
    for (int l = 0; l <= G; ++l) g0[l] = l * n_img / G;
    if ((rc = m->ctr.alloc(kLanes * sizeof(int)))) return rc;
    // rANS decoder variant: the sparse one (centre-interval fast path, no LDS table image) when the streams
    // average under LBIC_RANS_SPARSE_BPS bits per symbol (default 1.0; LBIC_RANS_SPARSE=0/1 forces it)
    int sparse = rans_sparse_choice(lens, n_img, (double)n_img * Hb * Wb * m->M);
    const std::vector<long long> key = {n_img, Hb, Wb, G, (long long)m->words.p, (long long)m->zpad.p,
                                        (long long)m->lane[0].ctx0.p, (long long)m->table_dev.p,
                                        (long long)m->st_x.p, m->prof.sample_every, sparse};
    if ((int)m->dec_exec.size() != G || key != m->dec_key) {
        std::lock_guard<std::mutex> lk(g_capture_mu);
        for (auto e : m->dec_exec) (void)hipGraphExecDestroy(e);
        m->dec_exec.clear();
        g_prof = &m->prof;
        for (int l = 0; l < G; ++l) {
            Work& w = m->lane[l];
            const int rows = g0[l + 1] - g0[l];
            if (rows > w.rows) { g_prof = nullptr; return set_error(LBC_E_STATE, "decoder lane workspace too small"); }
            RansArgs r = rans_args(m);
            r.cdf16 = m->cdf16_dev.as<uint16_t>();
            r.tmeta = m->tmeta_dev.as<int>();
            r.total16 = m->total16;
                    r.words = m->words.as<uint32_t>();
            r.word_base = m->word_base.as<long long>();
            r.word_count = m->word_count.as<int>();
            r.state_x = m->st_x.as<unsigned long long>();
            r.state_ptr = m->st_ptr.as<int>();
            r.status = m->st_status.as<int>();
            r.idx = w.idx.as<int32_t>();
            r.ksi = w.ksi.as<float>();
            r.ldk = m->C4;
            r.Mlat = m->M;
            r.yq = w.yq.as<float>();
            r.ldy = m->M;
            r.rows = rows;
            r.ctr = m->ctr.as<int>() + l;
            r.ctr_stride = Wb * n_img;
            r.sparse = sparse;
            HIPCHK(hipStreamBeginCapture(m->cap, hipStreamCaptureModeThreadLocal));
            int crc = prof_range_begin(&m->prof, 1 + l, m->cap);
            drop_recs(m->prof, 1 + l);
            for (int h = 0; h < Wb && !crc; ++h) {
                m->prof.step(m->prof.sample_every > 0 && (h % m->prof.sample_every) == 0);
                const int4* blocks = m->blocks_dec.as<int4>() + (size_t)h * n_img + g0[l];
                GemmArgs g = base_args(m, blocks, rows, nullptr, n_img, Hb, Wb);
                g.ctr = r.ctr;
                g.ctr_stride = r.ctr_stride;
                g.raster = 1;            // block of row r = (g0 + r, row counter, h): computed, not loaded
                g.raster_img0 = g0[l];
                g.raster_h = h;
                if (!crc) crc = run_ctx(m, w, g, true, m->cap);
                r.blocks = blocks;
                r.ts = m->prof.active ? m->prof.take() : nullptr;
                m->prof.per_replay[1 + l][2] += 1;
                if (!crc) crc = launch_rans_decode(r, m->cap);
                if (!crc && r.ts) {
                    // algorithmic bytes: the CDF tables staged into LDS + idx/mean in + y_qnt out
                    const double b = (double)m->total16 * 2 * ((rows + 7) / 8) + 12.0 * rows * m->M;
                    m->prof.add(2, r.ts, 0.0, b);
                }
                if (!crc) crc = run_dec(m, w, g, m->cap);
            }
            if (!crc) crc = launch_ctr_add(m->ctr.as<int>() + l, 1, m->cap);
            hipGraph_t graph = nullptr;
            const hipError_t e = hipStreamEndCapture(m->cap, &graph);
            if (crc) { if (graph) (void)hipGraphDestroy(graph); g_prof = nullptr; return crc; }
            if (e != hipSuccess) return set_error(LBC_E_HIP, std::string("decoder capture: ") + hipGetErrorString(e));
            hipGraphExec_t ex = nullptr;
            const hipError_t ei = hipGraphInstantiate(&ex, graph, nullptr, nullptr, 0);
            (void)hipGraphDestroy(graph);
            if (ei != hipSuccess) return set_error(LBC_E_HIP, std::string("decoder instantiate: ") + hipGetErrorString(ei));
            m->dec_exec.push_back(ex);
        }
        m->prof.active = false;
        g_prof = nullptr;
        m->dec_key = key;
    }
    HIPCHK(hipMemsetAsync(m->ctr.p, 0, kLanes * sizeof(int), s));
    if (m->l0_on && (rc = launch_l0_border(m->l0.as<float>(), n_img, Hb, Wb, m->C1P, m->net->ctx0.bias.as<float>(), s))) return rc;
    if (G == 1) {      // one lane: the row graphs run on the caller's stream
        for (int v = 0; v < Hb; ++v) HIPCHK(hipGraphLaunch(m->dec_exec[0], s));
        m->prof.replays[1] += Hb;
    } else {
        for (int l = 0; l < G; ++l)
            if (!m->lstream[l]) HIPCHK(hipStreamCreateWithFlags(&m->lstream[l], hipStreamNonBlocking));
        HIPCHK(hipEventRecord(m->lev[kLanes], s));
        for (int l = 0; l < G; ++l) HIPCHK(hipStreamWaitEvent(m->lstream[l], m->lev[kLanes], 0));
        for (int v = 0; v < Hb; ++v)
            for (int l = 0; l < G; ++l) HIPCHK(hipGraphLaunch(m->dec_exec[l], m->lstream[l]));
        for (int l = 0; l < G; ++l) m->prof.replays[1 + l] += Hb;
        for (int l = 0; l < G; ++l) {
            HIPCHK(hipEventRecord(m->lev[l], m->lstream[l]));
            HIPCHK(hipStreamWaitEvent(s, m->lev[l], 0));
        }
    }
    m->prof.active = false;
    g_prof = nullptr;
    if ((rc = launch_copy_interior(m->zpad.as<float>(), zhat_dev, n_img, Hb, Wb, m->Cx, s))) return rc;
    HIPCHK(hipEventRecord(m->ev[3], s));
    m->dec_timed = true;
    return check_status(m, (size_t)n_img, s, true);
}

// ---------------------------------------------------------------------------------------------- team decode
// lbc_decode_team: T batches (one per handle) decoded by ONE persistent k_dec_team launch, S workgroups per batch.
// The raster step each team replays is recorded from the same run_ctx / run_dec calls that build the graph decoder
// (three column classes: the KS3311 layer-0 cache computes border cells at h = 0 and h = Wb - 1), so the team
// decoder computes exactly what lbc_decode computes.  Falls back to lbc_decode per batch where the team kernel does
// not apply (M > 256, buffers past the 4 GB reach of its buffer loads, LBIC_TEAM=0, an LDS image past 160 KB).
static std::mutex g_team_mu;   // one team launch at a time per process: its grid must be resident as a whole

static int team_fallback(lbc_model* const* ms, int T, const uint8_t* const* streams, const size_t* lens, int n_img,
                         int Hb, int Wb, float* const* zhat, void* stream, bool after_timeout = false) {
    ms[0]->team_mode_last = 0;
    for (int t = 0; t < T; ++t) {
        ms[t]->no_one = after_timeout;
        const int rc = lbc_decode(ms[t], streams + (size_t)t * n_img, lens + (size_t)t * n_img, n_img, Hb, Wb, zhat[t],
                                  stream);
        ms[t]->no_one = false;
        if (rc) return rc;
    }
    return LBC_OK;
}

// The team program (held by ms[0]): every team's raster step recorded from the same run_ctx / run_dec calls that build
// the graph decoder, for the geometry (S, spread); rebuilt when the geometry, any team's buffers or any team's
// weight set (Net::gen) changed.  Sets ms[0]->team_args (without the per-launch fields) and the step's algorithmic work.
static int team_record(lbc_model* const* ms, int T, int n_img, int Hb, int Wb, int S, int spread, int sparse,
                       hipStream_t us) {
    lbc_model* m0 = ms[0];
    int rc;
    std::vector<long long> key = {T, S, spread, n_img, Hb, Wb, sparse};
    for (int t = 0; t < T; ++t) {
        lbc_model* m = ms[t];
        for (long long x : {(long long)m->words.p, (long long)m->zpad.p, (long long)m->lane[0].ctx0.p,
                            (long long)m->lane[0].d0.p, (long long)m->table_dev.p, (long long)m->tmeta_dev.p,
                            (long long)m->st_x.p, (long long)m->l0.p, m->net->gen})
            key.push_back(x);
    }
    if (key == m0->team_key) return LBC_OK;
    std::vector<GemmArgs> gem;
    std::vector<RansArgs> rans;
    std::vector<int> ops;
    int NG = -1;
    for (int t = 0; t < T; ++t) {
        lbc_model* m = ms[t];
        Work& w = m->lane[0];
        for (int c = 0; c < 3; ++c) {
            const int hc = c == 0 ? 0 : c == 1 ? std::min(1, Wb - 1) : Wb - 1;
            Recorder rec;
            GemmArgs g = base_args(m, m->blocks_dec.as<int4>(), n_img, nullptr, n_img, Hb, Wb);
            g.ctr = m->ctr.as<int>();
            g.ctr_stride = Wb * n_img;
            g.raster = 1;
            g.raster_img0 = 0;
            g.raster_h = hc;
            g_rec = &rec;
            int crc = run_ctx(m, w, g, true, nullptr);
            rec.ops.push_back(-1);
            if (!crc) crc = run_dec(m, w, g, nullptr);
            g_rec = nullptr;
            if (crc) return crc;
            if (NG < 0) {
                NG = (int)rec.gemms.size();
                ops = rec.ops;
            }
            if ((int)rec.gemms.size() != NG || rec.ops != ops || (int)ops.size() > TEAM_MAXOPS)
                return set_error(LBC_E_STATE, "team decoder: raster steps differ in shape");
            gem.insert(gem.end(), rec.gemms.begin(), rec.gemms.end());
        }
        RansArgs r = rans_args(m);
        r.idx = w.idx.as<int32_t>();
        r.ksi = w.ksi.as<float>();
        r.yq = w.yq.as<float>();
        r.rows = n_img;
        r.sparse = sparse;
        rans.push_back(r);
    }
    const size_t gb = gem.size() * sizeof(GemmArgs), rb = rans.size() * sizeof(RansArgs);
    if ((rc = m0->team_prog.alloc(gb + rb))) return rc;
    // (on the launch's stream: a legacy-stream copy fails while another thread captures a graph)
    HIPCHK(hipMemcpyAsync(m0->team_prog.p, gem.data(), gb, hipMemcpyHostToDevice, us));
    HIPCHK(hipMemcpyAsync(static_cast<char*>(m0->team_prog.p) + gb, rans.data(), rb, hipMemcpyHostToDevice, us));
    HIPCHK(hipStreamSynchronize(us));
    if ((rc = m0->team_sync.alloc((size_t)(TEAM_MAX + 2) * 32 * sizeof(unsigned)))) return rc;
    if ((rc = m0->team_ts.alloc((size_t)TEAM_MAX * TEAM_TS_WORDS * sizeof(unsigned long long)))) return rc;
    TeamArgs& a = m0->team_args;
    a = TeamArgs{};
    a.gemm = m0->team_prog.as<GemmArgs>();
    a.rans = reinterpret_cast<const RansArgs*>(static_cast<char*>(m0->team_prog.p) + gb);
    for (size_t i = 0; i < ops.size(); ++i) a.opk[i] = ops[i];
    a.nops = (int)ops.size();
    a.NG = NG;
    a.T = T;
    a.S = S;
    a.spread = spread;
    a.sub = T > TEAM_SLOTS ? 2 : 1;
    a.Hb = Hb;
    a.Wb = Wb;
    a.sync = m0->team_sync.as<unsigned>();
    // most tiles per workgroup over the step's GEMMs (the partials' LDS; the slower path needs 2)
    a.ni_max = 2;
    a.tab16 = rans[0].total16;
    for (const GemmArgs& d : gem) {
        const int items = ((d.M + 15) >> 4) * ((d.N + 15) >> 4);
        if (!team_fast_path(d, S)) continue;
        a.ni_max = std::max(a.ni_max, (items + S - 1) / S);
    }
    // rANS waves per workgroup: two once the team has more images than workgroups (each wave then keeps one image's
    // coder state in LDS up to 2 S images; beyond that each wave decodes its rows one after another)
    a.nrw = n_img > S ? 2 : 1;
    a.rows0 = n_img;
    // the GEMM after the rANS decode (the decoder's first layer): its last K segment is y_qnt; the K slices that end
    // before it run beside the rANS decode (on the waves the rANS decode leaves free) when every workgroup takes the
    // fast path for it
    a.split_op = -1;
    a.split_wy = 0;
    for (int i = 0; i + 1 < (int)ops.size(); ++i) {
        if (ops[i] != -1 || ops[i + 1] < 0) continue;
        bool fast = true;
        for (int t = 0; t < T; ++t)
            for (int c = 0; c < 3; ++c) {
                fast = fast && team_fast_path(gem[((size_t)t * 3 + c) * NG + ops[i + 1]], S);
            }
        const GemmArgs& d = gem[ops[i + 1]];
        const Seg& last = d.seg[d.nseg - 1];
        if (last.kind != SEG_DENSE || last.base != ms[0]->lane[0].yq.as<float>() || !fast) continue;
        const int nkb = d.K >> 4, kby = last.k0 >> 4;
        int wy = 0;
        while (wy < KSPLIT && (wy + 1) * nkb / KSPLIT <= kby) ++wy;
        wy = std::min(wy, KSPLIT - a.nrw);
        if (wy >= 1) {
            a.split_op = i + 1;
            a.split_wy = wy;
        }
    }
    // algorithmic work of one raster step (the graph decoder's accounting, gemm(): weights + A rows + outputs [+ the
    // GDN input] once per GEMM; rANS: indexes and means in, y_qnt out, the step's stream words)
    double sb = 0, sf = 0;
    for (int gi = 0; gi < NG; ++gi) {
        const GemmArgs& d = gem[(size_t)1 * NG + gi];     // team 0, inner column class
        sb += 4.0 * ((double)d.K * d.N + (double)d.M * d.K + (double)d.M * d.N * (d.square_a ? 2 : 1));
        sf += 2.0 * d.M * d.K * d.N;
    }
    sb += 12.0 * n_img * m0->M;
    m0->team_step_bytes = sb;
    m0->team_step_flops = sf;
    m0->team_key = key;
    return LBC_OK;
}

int lbc_decode_team(lbc_model* const* ms, int n_teams, const uint8_t* const* streams, const size_t* lens, int n_img,
                    int Hb, int Wb, float* const* zhat_devs, void* stream) {
    if (!ms || !streams || !lens || !zhat_devs) return set_error(LBC_E_ARG, "null argument");
    if (n_teams < 1 || n_teams > TEAM_MAX) return set_error(LBC_E_ARG, "1 to 16 image sets per team decode");
    if (n_img <= 0 || Hb <= 0 || Wb <= 0) return set_error(LBC_E_ARG, "empty frame");
    const int T = n_teams;
    for (int t = 0; t < T; ++t) {
        lbc_model* m = ms[t];
        if (!m || !zhat_devs[t]) return set_error(LBC_E_ARG, "null handle or output");
        if (!m->finalized) return set_error(LBC_E_STATE, "lbc_finalize() not called");
        if (!m->tabs_set) return set_error(LBC_E_NOT_UPDATED, "Uninitialized CDFs. Run update() first");
        for (int u = 0; u < t; ++u)
            if (ms[u] == m) return set_error(LBC_E_ARG, "every batch needs its own handle (lbc_create_sibling)");
        if (m->B != ms[0]->B || m->N != ms[0]->N || m->M != ms[0]->M || m->P != ms[0]->P || m->l0_on != ms[0]->l0_on ||
            m->cfg.device != ms[0]->cfg.device)
            return set_error(LBC_E_ARG, "team decode handles must share one geometry and device");
    }
    const char* te = getenv("LBIC_TEAM");
    if (T == 1 && n_img == 1 && !(te && atoi(te) == 0)) {
        // one image: the whole chip is its team -- lbc_decode runs the single-image decoder (k_dec_one) where it
        // applies, else the row graphs (faster than a team of 32 or 64 workgroups for one image: 0.59 vs 0.75 s per
        // 768x768 frame, profiles/r04/r04_c5_b1_s*.log)
        const int rc1 = lbc_decode(ms[0], streams, lens, 1, Hb, Wb, zhat_devs[0], stream);
        if (rc1) return rc1;
        ms[0]->team_mode_last = ms[0]->dec_path_last == 1 ? 3 : 4;
        ms[0]->team_launch_bytes = ms[0]->team_launch_flops = 0;
        ms[0]->team_plain_last = -1;    // no team launch: lbc_team_stats reports the decode's own events (ev[2..3])
        return LBC_OK;
    }
    int sparse = rans_sparse_choice(lens, T * n_img, (double)T * n_img * Hb * Wb * ms[0]->M);
    const double zbytes = (double)n_img * (Hb + 2) * (Wb + 4) * ms[0]->Cx * 4;
    const double lbytes = ms[0]->l0_on ? (double)n_img * (Hb + 2) * (Wb + 4) * ms[0]->C1P * 4 : 0.0;
    if ((te && atoi(te) == 0) || ms[0]->M > 256 || zbytes >= 4294967296.0 || lbytes >= 4294967296.0)
        return team_fallback(ms, T, streams, lens, n_img, Hb, Wb, zhat_devs, stream);
    std::lock_guard<std::mutex> team_lock(g_team_mu);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    lbc_model* m0 = ms[0];
    int rc;
    int dev = m0->cfg.device, cus = 0;
    HIPCHK(hipSetDevice(dev));
    HIPCHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    for (int t = 0; t < T; ++t) {
        lbc_model* m = ms[t];
        if ((rc = prepare_device(m))) return rc;
        if ((rc = ensure_workspace(m, n_img, Hb, Wb, s))) return rc;
        if ((rc = m->ctr.alloc(kLanes * sizeof(int)))) return rc;
        std::vector<std::pair<const uint8_t*, size_t>> subs;
        for (int i = 0; i < n_img; ++i) subs.emplace_back(streams[(size_t)t * n_img + i], lens[(size_t)t * n_img + i]);
        if ((rc = upload_streams(m, subs, s))) return rc;
    }
    // team geometry: grid 8 x S, one XCD slot per team, S = one (or, LBC_OPT_TEAM_WG_PER_CU, two) workgroups per CU
    // of an XCD.  The whole grid must be resident (team barriers): the occupancy query below uses the kernel instance
    // and the dynamic LDS of the launch, and a geometry that does not fit is shrunk (two workgroups per CU -> one) or
    // decoded by lbc_decode per batch.
    int wpc = std::max(1, m0->team_wpc);
    int S = 0, spread = 1, sub = 1;
    TeamArgs a{};
    for (;;) {
        // more than 8 teams: two per XCD slot, each half the slot's CUs
        sub = T > TEAM_SLOTS ? 2 : 1;
        S = std::min(32, cus / TEAM_SLOTS) / sub * wpc;
        if (m0->team_size > 0) S = std::min(S, m0->team_size * wpc);
        // at most four batches: each team takes two XCDs (twice the workgroups, write-through hand-offs; 4 batches
        // alone: 0.917 vs 0.969 s per launch, profiles/r02_exp/team_spread.txt); LBIC_TEAM_SPREAD=P (1, 2, 4, 8 with
        // T <= 8 / P) sets the XCD slots per team (A/B runs)
        const char* spe = getenv("LBIC_TEAM_SPREAD");
        spread = T <= TEAM_SLOTS / 2 ? 2 : 1;
        if (spe) {
            const int p = atoi(spe);
            if ((p == 1 || p == 2 || p == 4 || p == 8) && T <= TEAM_SLOTS / p) spread = p;
        }
        S *= spread;
        if (S < 1) return team_fallback(ms, T, streams, lens, n_img, Hb, Wb, zhat_devs, stream);
        if ((rc = team_record(ms, T, n_img, Hb, Wb, S, spread, sparse, s))) return rc;
        a = m0->team_args;
        // high rates: the tables staged in every workgroup's LDS (rans_row<true>); low rates: rans_row_sparse, its rare
        // far symbols searched in the table image in global memory
        a.dense = sparse ? 0 : 1;
        size_t lds = team_lds_bytes(a);
        if (lds > 160 * 1024 && a.dense) {
            // the dense tables do not fit beside this geometry's partials (high rates with many tiles per workgroup):
            // the sparse coder -- tables read from global memory, any rate, bit-identical -- instead of the row graphs
            sparse = 1;
            if ((rc = team_record(ms, T, n_img, Hb, Wb, S, spread, sparse, s))) return rc;
            a = m0->team_args;
            a.dense = 0;
            lds = team_lds_bytes(a);
        }
        if (lds > 160 * 1024) return team_fallback(ms, T, streams, lens, n_img, Hb, Wb, zhat_devs, stream);
        const int nb = team_blocks_per_cu(a.dense, lds);
        if (nb >= wpc) break;
        if (nb < 1 || wpc == 1) return team_fallback(ms, T, streams, lens, n_img, Hb, Wb, zhat_devs, stream);
        wpc = nb;
    }
    const char* tmoe = getenv("LBIC_TEAM_TMO");   // test hook: s_memrealtime ticks one barrier waits (default 1 s)
    a.tmo = tmoe ? std::max(1ull, strtoull(tmoe, nullptr, 10)) : 100000000ull;
    const char* st = getenv("LBIC_TEAM_STAMPS");
    a.ts = st && atoi(st) ? m0->team_ts.as<unsigned long long>() : nullptr;
    a.sv = Hb / 2;
    a.sh = Wb / 2;
    auto reset = [&]() -> int {
        for (int t = 0; t < T; ++t) {
            lbc_model* m = ms[t];
            HIPCHK(hipMemsetAsync(m->zpad.p, 0, (size_t)n_img * (Hb + 2) * (Wb + 4) * m->Cx * sizeof(float), s));
            int rc_;
            if (m->l0_on &&
                (rc_ = launch_l0_border(m->l0.as<float>(), n_img, Hb, Wb, m->C1P, m->net->ctx0.bias.as<float>(), s)))
                return rc_;
        }
        return LBC_OK;
    };
    // plain hand-off stores unless LBIC_TEAM_SC1=1 (or a spread / column-split geometry); a launch that finds a team
    // spread over XCDs stops before its first operation (failure word 2, nothing decoded yet) and is rerun with
    // write-through hand-offs
    const char* sc1e = getenv("LBIC_TEAM_SC1");
    a.plain = (sc1e && atoi(sc1e)) || a.spread > 1 ? 0 : 1;
    unsigned fail = 0;
    for (int attempt = 0; attempt < 2; ++attempt) {
        if ((rc = reset())) return rc;
        HIPCHK(hipMemsetAsync(m0->team_sync.p, 0, (size_t)(TEAM_MAX + 2) * 32 * sizeof(unsigned), s));
        if (a.ts) HIPCHK(hipMemsetAsync(m0->team_ts.p, 0, (size_t)TEAM_MAX * TEAM_TS_WORDS * sizeof(unsigned long long), s));
        HIPCHK(hipEventRecord(m0->ev[2], s));
        if ((rc = launch_dec_team(a, s))) return rc;
        HIPCHK(hipEventRecord(m0->ev[3], s));
        HIPCHK(hipMemcpyAsync(&fail, m0->team_sync.as<unsigned>() + T * 32, sizeof(unsigned), hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        if (fail != 2 || !a.plain) break;
        a.plain = 0;
        m0->team_fallbacks += 1;
    }
    if (fail == 1) {
        // a workgroup gave up waiting at a team barrier (the grid was not co-resident in time: another process or
        // stream held CUs past the timeout).  Nothing is wrong with the streams: decode the batches again through
        // lbc_decode one after another (it re-uploads the streams and resets the workspaces), and count the event.
        m0->team_timeouts += 1;
        static std::atomic<bool> noted{false};
        const char* ev = getenv("LBIC_TEAM_VERBOSE");
        if (!noted.exchange(true) || (ev && atoi(ev)))
            fprintf(stderr, "[lbic] team decode: barrier timeout, decoding through lbc_decode (counted: lbc_team_events)\n");
        return team_fallback(ms, T, streams, lens, n_img, Hb, Wb, zhat_devs, stream, true);
    }
    if (fail)   // any other failure word is a protocol error, not a residency problem: report it
        return set_error(LBC_E_STATE, "team decode: unexpected failure word " + std::to_string(fail));
    m0->team_plain_last = a.plain;
    m0->team_mode_last = a.dense == 1 ? 2 : 1;
    m0->team_launch_bytes = m0->team_step_bytes * T * Hb * Wb;
    m0->team_launch_flops = m0->team_step_flops * T * Hb * Wb;
    m0->dec_timed = true;
    for (int t = 0; t < T; ++t)
        if ((rc = launch_copy_interior(ms[t]->zpad.as<float>(), zhat_devs[t], n_img, Hb, Wb, ms[t]->Cx, s))) return rc;
    if (a.ts) {
        m0->team_ts_host.assign((size_t)T * TEAM_TS_WORDS, 0ull);
        HIPCHK(hipMemcpyAsync(m0->team_ts_host.data(), m0->team_ts.p, (size_t)T * TEAM_TS_WORDS * sizeof(unsigned long long),
                              hipMemcpyDeviceToHost, s));
    }
    HIPCHK(hipStreamSynchronize(s));
    if (const char* e = getenv("LBIC_TEAM_VERBOSE"); e && atoi(e))
        fprintf(stderr, "[lbic] team decode: T=%d S=%d plain=%d reruns=%d lds=%zu\n", T, S, a.plain, m0->team_fallbacks,
                team_lds_bytes(a));
    for (int t = 0; t < T; ++t)
        if ((rc = check_status(ms[t], (size_t)n_img, s, true))) return rc;
    return LBC_OK;
}

int lbc_team_stats(const lbc_model* m, double* launch_ms, double* bytes, double* flops, int* plain) {
    if (!m || !launch_ms || !bytes || !flops || !plain) return set_error(LBC_E_ARG, "null argument");
    float ms = 0.f;
    if (m->dec_timed && m->ev[2]) HIPCHK(hipEventElapsedTime(&ms, m->ev[2], m->ev[3]));
    *launch_ms = ms;
    *bytes = m->team_launch_bytes;
    *flops = m->team_launch_flops;
    *plain = m->team_plain_last;
    return LBC_OK;
}

int lbc_one_stamps(const lbc_model* m, unsigned long long* out, int max_out, int* n_out) {
    if (!m || !out || !n_out) return set_error(LBC_E_ARG, "null argument");
    const int n = std::min(max_out, (int)m->one_ts_host.size());
    for (int i = 0; i < n; ++i) out[i] = m->one_ts_host[i];
    *n_out = n;
    return LBC_OK;
}

int lbc_decode_path(const lbc_model* m, int* path, int* timeouts) {
    if (!m || !path || !timeouts) return set_error(LBC_E_ARG, "null argument");
    *path = m->dec_path_last;
    *timeouts = m->one_timeouts;
    return LBC_OK;
}

int lbc_team_mode(const lbc_model* m, int* mode) {
    if (!m || !mode) return set_error(LBC_E_ARG, "null argument");
    *mode = m->team_mode_last;
    return LBC_OK;
}

int lbc_team_events(const lbc_model* m, int* sc1_reruns, int* timeouts) {
    if (!m || !sc1_reruns || !timeouts) return set_error(LBC_E_ARG, "null argument");
    *sc1_reruns = m->team_fallbacks;
    *timeouts = m->team_timeouts;
    return LBC_OK;
}

int lbc_team_stamps(const lbc_model* m, unsigned long long* out, int max_out, int* n_out) {
    if (!m || !n_out) return set_error(LBC_E_ARG, "null argument");
    const int n = (int)m->team_ts_host.size();
    *n_out = n;
    if (out)
        for (int i = 0; i < n && i < max_out; ++i) out[i] = m->team_ts_host[i];
    return LBC_OK;
}

static const uint32_t kRowsMagic = 0x3157424Cu;   // "LBW1"

int lbc_rans_encode_rows(const lbc_model* m, const int32_t* sym, const int32_t* idx, int Hb, int Wb, uint8_t** out,
                         size_t* len) {
    if (!m || !sym || !idx || !out || !len || Hb <= 0 || Wb <= 0) return set_error(LBC_E_ARG, "bad argument");
    if (!m->tabs_set) return set_error(LBC_E_NOT_UPDATED, "Uninitialized CDFs. Run update() first");
    const size_t per_row = (size_t)Wb * m->M;
    std::vector<std::vector<uint8_t>> rows(Hb);
    for (int v = 0; v < Hb; ++v) {
        int rc = rans_encode(m->tabs, sym + v * per_row, idx + v * per_row, per_row, rows[v]);
        if (rc) return rc;
    }
    size_t total = 8 + 4 * (size_t)Hb;
    for (auto& r : rows) total += r.size();
    uint8_t* buf = static_cast<uint8_t*>(malloc(total));
    uint32_t hdr[2] = {kRowsMagic, (uint32_t)Hb};
    std::memcpy(buf, hdr, 8);
    size_t off = 8 + 4 * (size_t)Hb;
    for (int v = 0; v < Hb; ++v) {
        const uint32_t n = (uint32_t)rows[v].size();
        std::memcpy(buf + 8 + 4 * (size_t)v, &n, 4);
        std::memcpy(buf + off, rows[v].data(), n);
        off += n;
    }
    *out = buf;
    *len = total;
    return LBC_OK;
}

int lbc_decode_rows(lbc_model* m, const uint8_t* const* streams, const size_t* lens, int n_img, int Hb, int Wb,
                    float* zhat_dev, void* stream) {
    if (!m || !streams || !lens || !zhat_dev) return set_error(LBC_E_ARG, "null argument");
    if (!m->finalized) return set_error(LBC_E_STATE, "lbc_finalize() not called");
    if (!m->tabs_set) return set_error(LBC_E_NOT_UPDATED, "Uninitialized CDFs. Run update() first");
    if (n_img <= 0 || Hb <= 0 || Wb <= 0) return set_error(LBC_E_ARG, "empty frame");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    int rc;
    if ((rc = prepare_device(m))) return rc;
    if ((rc = ensure_workspace(m, n_img, Hb, Wb, s))) return rc;
    std::vector<std::pair<const uint8_t*, size_t>> subs;       // stream (img, v) at img * Hb + v
    for (int i = 0; i < n_img; ++i) {
        uint32_t hdr[2];
        if (!streams[i] || lens[i] < 8 + 4 * (size_t)Hb) return set_error(LBC_E_STREAM, "invalid sub-stream container");
        std::memcpy(hdr, streams[i], 8);
        if (hdr[0] != kRowsMagic || (int)hdr[1] != Hb) return set_error(LBC_E_STREAM, "not a sub-stream container for this frame");
        size_t off = 8 + 4 * (size_t)Hb;
        for (int v = 0; v < Hb; ++v) {
            uint32_t n;
            std::memcpy(&n, streams[i] + 8 + 4 * (size_t)v, 4);
            if (off + n > lens[i]) return set_error(LBC_E_STREAM, "truncated sub-stream container");
            subs.emplace_back(streams[i] + off, (size_t)n);
            off += n;
        }
    }
    if ((rc = upload_streams(m, subs, s))) return rc;
    // the whole anti-diagonal wavefront (the encoder's schedule) as one graph: per step, context net of
    // every block on the diagonal -> one wave per (image, block row) decodes that row's next block ->
    // decoder transform of every block
    std::vector<size_t> sub_lens;
    for (const auto& sb : subs) sub_lens.push_back(sb.second);
    const int sparse = rans_sparse_choice(sub_lens.data(), (int)sub_lens.size(), (double)n_img * Hb * Wb * m->M);
    const std::vector<long long> key = {n_img, Hb, Wb, (long long)m->words.p, (long long)m->zpad.p,
                                        (long long)m->lane[0].ctx0.p, (long long)m->table_dev.p,
                                        (long long)m->st_x.p, m->prof.sample_every, sparse};
    if (!m->wf_exec || key != m->wf_key) {
        std::lock_guard<std::mutex> lk(g_capture_mu);
        if (m->wf_exec) { (void)hipGraphExecDestroy(m->wf_exec); m->wf_exec = nullptr; }
        Work& w = m->lane[0];
        HIPCHK(hipStreamBeginCapture(m->cap, hipStreamCaptureModeThreadLocal));
        int crc = prof_range_begin(&m->prof, kRanges - 1, m->cap);
        drop_recs(m->prof, kRanges - 1);
        const int4* blocks = m->blocks_enc.as<int4>();
        g_prof = &m->prof;
        for (size_t t = 0; t < m->step_off.size() && !crc; ++t) {
            m->prof.step(m->prof.sample_every > 0 && (t % m->prof.sample_every) == 0);
            const int rows = m->step_cnt[t];
            GemmArgs g = base_args(m, blocks + m->step_off[t], rows, nullptr, n_img, Hb, Wb);
            crc = run_ctx(m, w, g, true, m->cap, false, m->l0_on ? m->cells_enc.as<int4>() + m->cell_off[t] : nullptr,
                          m->l0_on ? m->cell_cnt[t] : 0);
            RansArgs r = rans_args(m);
            r.idx = w.idx.as<int32_t>();
            r.ksi = w.ksi.as<float>();
            r.yq = w.yq.as<float>();
            r.rows = rows;
            r.blocks = blocks + m->step_off[t];
            r.streams_per_img = Hb;
            r.sparse = sparse;
            r.ts = m->prof.active ? m->prof.take() : nullptr;
            m->prof.per_replay[kRanges - 1][2] += 1;
            if (!crc) crc = launch_rans_decode(r, m->cap);
            if (!crc && r.ts) {
                const double b = (double)m->total16 * 2 * ((rows + 7) / 8) + 12.0 * rows * m->M;
                m->prof.add(2, r.ts, 0.0, b);
            }
            if (!crc) crc = run_dec(m, w, g, m->cap);
        }
        m->prof.active = false;
        m->prof.nochain = false;
        // (used0 counts the ENCODER graph's range-0 slots: set by lbc_encode_ex's capture only -- ADVICE r4)
        g_prof = nullptr;
        hipGraph_t graph = nullptr;
        const hipError_t e = hipStreamEndCapture(m->cap, &graph);
        if (crc) { if (graph) (void)hipGraphDestroy(graph); return crc; }
        if (e != hipSuccess) return set_error(LBC_E_HIP, std::string("wavefront decoder capture: ") + hipGetErrorString(e));
        const hipError_t ei = hipGraphInstantiate(&m->wf_exec, graph, nullptr, nullptr, 0);
        (void)hipGraphDestroy(graph);
        if (ei != hipSuccess) return set_error(LBC_E_HIP, std::string("wavefront decoder instantiate: ") + hipGetErrorString(ei));
        m->wf_key = key;
    }
    HIPCHK(hipEventRecord(m->ev[2], s));
    HIPCHK(hipMemsetAsync(m->zpad.p, 0, (size_t)n_img * (Hb + 2) * (Wb + 4) * m->Cx * sizeof(float), s));
    if (m->l0_on && (rc = launch_l0_border(m->l0.as<float>(), n_img, Hb, Wb, m->C1P, m->net->ctx0.bias.as<float>(), s))) return rc;
    HIPCHK(hipGraphLaunch(m->wf_exec, s));
    m->prof.replays[kRanges - 1] += 1;
    if ((rc = launch_copy_interior(m->zpad.as<float>(), zhat_dev, n_img, Hb, Wb, m->Cx, s))) return rc;
    HIPCHK(hipEventRecord(m->ev[3], s));
    m->dec_timed = true;
    return check_status(m, subs.size(), s, true);
}

int lbc_profile_begin(lbc_model* m, int sample_every) {
    if (!m || sample_every < 0) return set_error(LBC_E_ARG, "bad argument");
    Prof& p = m->prof;
    if (sample_every && !p.slots) {
        HIPCHK(hipSetDevice(m->cfg.device));
        HIPCHK(hipMalloc(&p.slots, 8 * kSlotU64 * (size_t)kSlotsPerRange * kRanges));
        HIPCHK(hipMemset(p.slots, 0, 8 * kSlotU64 * (size_t)kSlotsPerRange * kRanges));
        if (getenv("LBIC_DEBUG_STAMPS"))
            fprintf(stderr, "handle %p slots %p..%p\n", (void*)m, (void*)p.slots,
                    (void*)(p.slots + kSlotU64 * (size_t)kSlotsPerRange * kRanges));
    }
    // sample_every is part of the graph keys: a change re-captures (and re-creates the sample records);
    // an unchanged value only restarts the launch counting.  Every stamp slot is zeroed here, so a graph
    // that is not replayed after this call (a warmup graph, another handle's idle pass) contributes no
    // sample: lbc_profile_end counts only launches executed since lbc_profile_begin.
    if (sample_every != p.sample_every) p.recs.clear();
    p.sample_every = sample_every;
    for (auto& r : p.replays) r = 0;
    if (sample_every && !p.snap)
        HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&p.snap), (size_t)Prof::kSnaps * kSlotsPerRange * kSlotU64 * 8));
    p.nsnap = 0;
    if (p.slots) {
        HIPCHK(hipSetDevice(m->cfg.device));
        HIPCHK(hipDeviceSynchronize());
        HIPCHK(hipMemset(p.slots, 0, 8 * kSlotU64 * (size_t)kSlotsPerRange * kRanges));
        HIPCHK(hipDeviceSynchronize());
    }
    return LBC_OK;
}

// Reads the stamps of the sampled launches as of the last replay of every graph (a decoder row graph
// is replayed Hb times: its stamps are those of the last block row).
int lbc_profile_end(lbc_model* m, lbc_kernel_stat* out, int max_out, int* n_out) {
    if (!m || !out || !n_out) return set_error(LBC_E_ARG, "null argument");
    Prof& p = m->prof;
    lbc_kernel_stat acc[kNClass];
    std::memset(acc, 0, sizeof(acc));
    for (int c = 0; c < kNClass; ++c)
        snprintf(acc[c].name, sizeof(acc[c].name), "%s", kKernelNames[c]);
    if (p.slots && !p.recs.empty()) {
        HIPCHK(hipDeviceSynchronize());
        std::vector<unsigned long long> h(kSlotU64 * (size_t)kSlotsPerRange * kRanges);
        HIPCHK(hipMemcpy(h.data(), p.slots, h.size() * 8, hipMemcpyDeviceToHost));
        // latest end stamp of a slot over the XCDs (0: not executed since the last reset)
        auto last_end = [&](int slot) -> unsigned long long {
            const unsigned long long* t = h.data() + kSlotU64 * (size_t)slot;
            unsigned long long e = 0;
            for (int x = 0; x < 8; ++x)
                if (t[2 * x] && t[2 * x + 1]) e = std::max(e, t[2 * x + 1]);
            return e;
        };
        // the launch's span: earliest workgroup start over the XCDs -> latest workgroup end over the XCDs (what a
        // dispatch trace measures; the XCDs do not start a launch at the same moment); -1: not executed
        auto span_of = [](const unsigned long long* t) -> long long {
            unsigned long long s0 = ~0ull, e1 = 0;
            for (int x = 0; x < 8; ++x) {
                if (!t[2 * x] || !t[2 * x + 1]) continue;
                s0 = std::min(s0, ~0ull - t[2 * x]);
                e1 = std::max(e1, t[2 * x + 1]);
            }
            return e1 && e1 >= s0 ? (long long)(e1 - s0) : -1;
        };
        for (const auto& r : p.recs) {
            const unsigned long long* t = h.data() + kSlotU64 * (size_t)r.slot;
            if (r.slot < kSlotsPerRange && p.nsnap > 0 && r.slot < p.used0) {
                // the encoder graph: every replay's copy (stream-ordered D2H after each replay)
                for (int q = 0; q < p.nsnap; ++q) {
                    const long long sp = span_of(p.snap + ((size_t)q * kSlotsPerRange + r.slot) * kSlotU64);
                    if (sp < 0) continue;
                    acc[r.cls].launches += 1;
                    acc[r.cls].total_ms += (double)sp * 1e-5;
                    acc[r.cls].flops += r.flops;
                    acc[r.cls].bytes += r.bytes;
                }
                continue;
            }
            const long long span = span_of(t);
            if (span >= 0 && r.prev >= 0) {    // launch-to-launch period in the stream chain
                const unsigned long long e0 = last_end(r.prev), e1 = last_end(r.slot);
                if (e0 && e1 > e0 && e1 - e0 < 100000000ull) {
                    acc[r.cls].launches_chain += 1;
                    acc[r.cls].total_ms_chain += (double)(e1 - e0) * 1e-5;
                }
            }
            if (getenv("LBIC_DEBUG_STAMPS") && span > 10000000) {
                fprintf(stderr, "handle %p bad slot %d cls %d:", (void*)m, r.slot, r.cls);
                for (int x = 0; x < 16; ++x) fprintf(stderr, " %llx", t[x]);
                fprintf(stderr, "\n");
            }
            if (span < 0) continue;   // not executed since the last reset
#ifdef LBIC_PHASE_DIAG
            if (r.cls == 0 && t[31]) {
                static double pmax[5], psum[5], nl;
                for (int i = 1; i <= 4; ++i) { pmax[i] += (double)t[16 + i]; psum[i] += (double)t[24 + i] / (double)t[31]; }
                nl += 1;
                if (&r == &p.recs.back() || true) {
                    static int printed = 0;
                    if (++printed % 50 == 0 || &r == &p.recs.back())
                        fprintf(stderr, "[diag k_gemm_s] launches %.0f  critical-WG cycles since start: prologue %.0f "
                                "loads+mfma %.0f reduce %.0f epilogue %.0f | mean WG: %.0f %.0f %.0f %.0f\n", nl,
                                pmax[1] / nl, pmax[2] / nl, pmax[3] / nl, pmax[4] / nl, psum[1] / nl, psum[2] / nl,
                                psum[3] / nl, psum[4] / nl);
                }
            }
#endif
            acc[r.cls].launches += 1;
            acc[r.cls].total_ms += (double)span * 1e-5;     // 100 MHz ticks -> ms
            acc[r.cls].flops += r.flops;
            acc[r.cls].bytes += r.bytes;
        }
    }
    // true launch counts since lbc_profile_begin (the stamps are a sample of them)
    for (int c = 0; c < kNClass; ++c) {
        long long tot = 0;
        for (int r = 0; r < 8; ++r) {
            tot += p.per_replay[r][c] * p.replays[r];
            acc[c].total_flops += p.work_replay[r][c][0] * p.replays[r];
            acc[c].total_bytes += p.work_replay[r][c][1] * p.replays[r];
        }
        acc[c].total_launches = tot;
    }
    int n = 0;
    for (int c = 0; c < kNClass && n < max_out; ++c)
        if (acc[c].launches || acc[c].total_launches) out[n++] = acc[c];
    *n_out = n;
    return LBC_OK;
}

void lbc_free(void* p) { free(p); }

const char* lbc_last_error(void) { return g_err.c_str(); }

int lbc_last_timing(const lbc_model* m, double* enc_ms, double* dec_ms) {
    if (!m) return set_error(LBC_E_ARG, "null model");
    float t = 0.f;
    if (enc_ms) {
        *enc_ms = -1.0;
        if (m->enc_timed && hipEventSynchronize(m->ev[1]) == hipSuccess &&
            hipEventElapsedTime(&t, m->ev[0], m->ev[1]) == hipSuccess)
            *enc_ms = t;
    }
    if (dec_ms) {
        *dec_ms = -1.0;
        if (m->dec_timed && hipEventSynchronize(m->ev[3]) == hipSuccess &&
            hipEventElapsedTime(&t, m->ev[2], m->ev[3]) == hipSuccess)
            *dec_ms = t;
    }
    return LBC_OK;
}

}  // extern "C"
