/* lbic.h -- C ABI of liblbic.so, the MI355X-native block-level masked-convolution codec.
 *
 * The reference's hot path is Python (graphs/models/BlockBasedImgCompLossy_net.py) over two native
 * layers: torch conv/elementwise kernels and CompressAI's C++ coder.  Each entry point below replaces
 * one reference interface (cited per function); the Python mirror in
 * learned-block-based-image-compression_amd/lbic/ binds them with ctypes.
 *
 * Conventions
 *   - All functions return 0 on success or a negative LBC_E* code; lbc_last_error() gives a
 *     thread-local message.  LBC_E_NOT_UPDATED mirrors the reference's
 *     ValueError("Uninitialized CDFs. Run update() first") (graphs/layers/entropy_layers_cai.py:185-204).
 *   - Image tensors are block-major fp32: [n_img][Hb][Wb][C] with C = 3*B*B and channel index
 *     (py*B + px)*3 + colour (arrange_block_pixels_to_channel_dim, agents/blkbsdimgcomp_agent.py:853-860).
 *   - *_dev pointers are HIP device pointers owned by the caller; `stream` is a hipStream_t (NULL =
 *     default stream).  The handle owns packed weights and workspaces; it is not thread-safe (the
 *     reference is single-threaded, agents/blkbsdimgcomp_agent.py:565-566).
 *   - Symbols / indexes are int32 in the reference's order: per image, raster block order, latent
 *     channel minor (graphs/models/BlockBasedImgCompLossy_net.py:353-354).
 */
#ifndef LBIC_H
#define LBIC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LBC_OK 0
#define LBC_E_ARG (-1)
#define LBC_E_HIP (-2)
#define LBC_E_STATE (-3)
#define LBC_E_NOT_UPDATED (-4)
#define LBC_E_STREAM (-5)

typedef struct lbc_model lbc_model;

typedef struct {
    int block_size;  /* config.block_size (configs/<name>.json) */
    int ks[4];       /* config.KS */
    int n;           /* config.N */
    int m;           /* config.M (latent channels) */
    int device;      /* HIP device ordinal */
} lbc_config;

/* BlockBasedImgCompLossyNetv9.__init__ (net:259-317): allocate a model of this geometry. */
int lbc_create(const lbc_config *cfg, lbc_model **out);
void lbc_destroy(lbc_model *m);

/* A second handle on the same finalized weights (no reference counterpart: the reference keeps one model per
 * process and codes one image at a time).  The packed device weights are shared read-only; the new handle has
 * its own workspaces, graphs and device entropy tables (copied from src's current ones), so it can code on
 * another stream from another thread while src is busy.  A later lbc_finalize on either handle gives that
 * handle a fresh weight set and leaves the other's untouched; destroy order is free. */
int lbc_create_sibling(const lbc_model *src, lbc_model **out);

/* Module.load_state_dict for one tensor under its reference state-dict name
 * (e.g. "prtr_forward3.0.gamma", "get_meanscale.6.bias").  Buffers (mask, pedestal, bound, the
 * entropy-model buffers) are accepted and ignored: masks and reparametrisation constants are
 * re-derived (masked_conv2d.py:9-17, utils/parametrizers.py:32-37). */
int lbc_set_tensor(lbc_model *m, const char *ref_name, const float *host, const int64_t *shape, int ndim);

/* Apply MaskedConv2d masks (masked_conv2d.py:19-21) and the GDN reparametrisation
 * (gdn_compressai.py:66-68), pack every layer for the fp32 MFMA kernels and upload. */
int lbc_finalize(lbc_model *m);

/* compressai._CXX.pmf_to_quantized_cdf (called at entropy_layers_cai.py:61-64): host C++.
 * cdf_out receives n+1 entries. */
int lbc_pmf_to_quantized_cdf(const float *pmf, int n, int precision, uint32_t *cdf_out);

/* GaussianConditional.update() results (entropy_layers_cai.py:590-613): the 64-entry scale table,
 * quantized CDF rows [n_tables][cdf_stride], cdf lengths and offsets.  Until this is called,
 * lbc_encode / lbc_decode return LBC_E_NOT_UPDATED. */
int lbc_set_entropy_tables(lbc_model *m, const float *scale_table, int n_tables, const int32_t *cdf,
                           int cdf_stride, const int32_t *cdf_length, const int32_t *offset);

/* compress() closed loop (net:319-361) for a batch of images, on the GPU: x_dev [n_img][Hb][Wb][C]
 * in [-1/2, 1/2] -> zhat_dev (same layout; the clamped reconstruction, net:357), sym_dev / idx_dev
 * [n_img][Hb*Wb*M] int32, bits_dev (nullable) [n_img][Hb*Wb*M] fp32 = -log2 of the Gaussian likelihood
 * (entropy_layers_cai.py:615-647, the per-latent self-information of net:103).  The raster
 * dependency is scheduled as an anti-diagonal wavefront t = h + 2v over all images at once. */
int lbc_encode(lbc_model *m, const float *x_dev, int n_img, int Hb, int Wb, float *zhat_dev,
               int32_t *sym_dev, int32_t *idx_dev, float *bits_dev, void *stream);

/* Options.  LBC_OPT_ENC_LDS_FLOOR (bytes, 0..160 KB): LDS reserved by each workgroup of the encoder's
 * large-M GEMM; above 80 KB one encoder workgroup per CU, which leaves room for a decoder running
 * concurrently on another stream (bench.py's two-stage pipeline).  Results are unchanged. */
#define LBC_OPT_ENC_LDS_FLOOR 1
/* LBC_OPT_TEAM_WG_PER_CU (1 or 2): workgroups per CU of the lbc_decode_team launches this handle leads (as the
 * first handle of the call).  1 (default): a team of CUs/8 workgroups per batch, one per CU, leaving registers and
 * LDS to an encoder running concurrently on another stream.  2: two per CU (teams of 2 * CUs/8), every register
 * of the CU -- for a decode with the GPU otherwise idle (e.g. the last launch of a pipeline).  Results unchanged. */
#define LBC_OPT_TEAM_WG_PER_CU 2
/* LBC_OPT_TEAM_SIZE (0..32): workgroups per team of the lbc_decode_team launches this handle leads, one per CU.  0
 * (default): CUs/8, every CU of an XCD.  Fewer: small teams (every workgroup then computes more output tiles and
 * decodes several rANS streams per step).  Results unchanged. */
#define LBC_OPT_TEAM_SIZE 3
/* LBC_OPT_ENC_FORK (-1, 0, 1): the encoder graph's wavefront steps as two branches (the context net beside the
 * transform's first six GEMMs, joined before the quantising GEMM) or as one chain.  -1 (default): forked when the
 * pass's largest wavefront step has at most 2,048 rows (a 32-frame 768^2 pass: 1,536), one chain for larger passes,
 * whose launches fill the chip for several rounds each.  The environment's LBIC_ENC_FORK=0/1, when set, overrides it
 * (experiments).  Results unchanged. */
#define LBC_OPT_ENC_FORK 4
int lbc_set_option(lbc_model *m, int option, long long value);

/* lbc_encode with flags.  LBC_ENC_FRAME_PAD: the context net's layer-0 map is zero outside the frame
 * (forward()'s 'same' padding) instead of being evaluated on the zero-padded zhat (compress()): the closed
 * loop of validate_recu_reco_fast (agents/blkbsdimgcomp_agent.py:491-520), which runs forward() on causal
 * crops.  Differs from compress() only for KS[1] = 3; bits_dev then holds its self-information. */
#define LBC_ENC_FRAME_PAD 1
int lbc_encode_ex(lbc_model *m, const float *x_dev, int n_img, int Hb, int Wb, float *zhat_dev,
                  int32_t *sym_dev, int32_t *idx_dev, float *bits_dev, int flags, void *stream);

/* Teacher-forced forward pass, BlockBasedImgCompLossyNetv4.forward(zhat, x) inherited by v9
 * (graphs/models/BlockBasedImgCompLossy_net.py:90-106), eval mode: every block sees the GIVEN zhat
 * (no closed loop), with the full-frame 'same' convolutions of the reference's nn.Sequential layers.
 * x_dev, zhat_dev: [n_img][Hb][Wb][3B^2] fp32 on the device.  Outputs: xhat_dev [n_img][Hb][Wb][3B^2]
 * (inverse transform of the dequantized latent, not clamped) and info_dev [n_img][Hb][Wb][M] =
 * -log2 of the Gaussian likelihood with the 1e-9 lower bound (entropy_layers_cai.py:615-647). */
int lbc_forward(lbc_model *m, const float *x_dev, const float *zhat_dev, int n_img, int Hb, int Wb, float *xhat_dev,
                float *info_dev, void *stream);

/* BufferedRansEncoder.encode_with_indexes + flush (net:328,359-360), host C++, one image.
 * *out is allocated by the library (release with lbc_free). */
int lbc_rans_encode(const lbc_model *m, const int32_t *sym, const int32_t *idx, size_t n, uint8_t **out,
                    size_t *len);

/* RansDecoder host-side reference decode of a whole stream (net:409-410,439 for every block),
 * given every symbol's table index: test/debug helper for the host coder. */
int lbc_rans_decode_host(const lbc_model *m, const uint8_t *data, size_t len, const int32_t *idx, size_t n,
                         int32_t *sym_out);

/* RansDecoder.decode_with_indexes (CompressAI C++; called once per block at net:439) on the GPU, for
 * n_streams independent streams at once: chunk c decodes the next M symbols (M = the model's latent
 * channels) of every stream with the table indexes idx_dev[c][stream][M] and writes the symbols to
 * sym_dev[c][stream][M] (both device int32).  The same k_rans_decode kernel lbc_decode runs per raster
 * step; streams are host bitstreams as lbc_rans_encode produced.  Returns LBC_E_STREAM for an overrun. */
int lbc_rans_decode_gpu(lbc_model *m, const uint8_t *const *streams, const size_t *lens, int n_streams,
                        const int32_t *idx_dev, int n_chunks, int32_t *sym_dev, void *stream);

/* decompress() (net:400-452) for a batch of images: streams[i] / lens[i] are the host bitstreams
 * lbc_rans_encode produced.  Strictly raster-serial within an image (the reference format has one
 * rANS stream per image); images are decoded together, rANS decode runs on the GPU.  The streams are
 * copied to the device in `stream` order (after that stream's earlier work).  The call is synchronous:
 * it returns after the whole decode has finished on `stream` (it reads back the per-stream status to
 * report a corrupt bitstream), so the caller may free or reuse its buffers on return.
 * Stream integrity (stricter than CompressAI's RansDecoder, which never checks): LBC_E_STREAM when a stream runs out
 * of words before its last block (truncated), or when its coder state after the last block is not the encoder's
 * initial state 2^31 (Rans64EncInit; the decoder retraces the encoder's states in reverse), which a corrupted stream
 * misses with near certainty.  Words after the last one the decode reads (trailing padding) are ignored, as the
 * reference's decoder ignores them.  Every decoder path (row graphs, k_dec_one, lbc_decode_team, lbc_decode_rows)
 * applies the same check. */
int lbc_decode(lbc_model *m, const uint8_t *const *streams, const size_t *lens, int n_img, int Hb, int Wb,
               float *zhat_dev, void *stream);
/* How the last lbc_decode of this handle ran (no reference counterpart: a query for tests and the bench).  *path: 0
 * the row graphs (k_gemm_s / k_rans_decode chains), 1 the single-image decoder k_dec_one (n_img = 1 wherever the raster
 * step's weights fit the grid's LDS -- B8_lowrate, B4_highrate with its KS[1] = 3 layer-0 cache -- at any rate: one
 * persistent launch over every CU, each weight tile resident in one or two workgroups' LDS, data-tagged hand-offs;
 * bit-identical to the row graphs; LBIC_ONE=0, or LBIC_RANS_SPARSE=0, disables it).  *timeouts: k_dec_one launches of this handle that timed out
 * waiting (CUs held elsewhere) and were decoded by the row graphs instead. */
int lbc_decode_path(const lbc_model *m, int *path, int *timeouts);
/* raw stamps of the last k_dec_one launch made with LBIC_ONE_STAMPS=1 (diagnostic): 4 per operation of the raster step
 * (Hb/2, Wb/2), s_memrealtime (100 MHz): [0] first workgroup entering the operation, [1] the last one's partials
 * reduced (inputs waited for, chains done), [2] the last one's outputs published, [3] the last one's inputs all there;
 * then [48] the rANS operation's decode started, [49] its symbols decoded, [50], [51] s_memtime (shader clock)
 * at those two points; then 32 per operation from the workgroup holding its column tile 0: [52 + 32 o] in, [+1 + w]
 * wave w's inputs there, [+9 + w] its A and weights in registers, [+17 + w] its chain done, [+25] partials reduced,
 * [+26] published, [+27] thread 0's granule store issued (436 words; written after the last step). */
int lbc_one_stamps(const lbc_model *m, unsigned long long *out, int max_out, int *n_out);

/* decompress() of n_teams batches at once (reference format; no reference counterpart for the batching: the
 * reference decodes one image at a time, agents/blkbsdimgcomp_agent.py:591-599 -> net:400-452).  Batch t is decoded by
 * handle ms[t] (distinct handles of one geometry, e.g. lbc_create_sibling) from streams[t * n_img + i] /
 * lens[t * n_img + i] into zhat_devs[t]; results are bit-identical to lbc_decode of each batch.  All batches run
 * in ONE persistent GPU launch (k_dec_team: one team of workgroups per batch, team barriers between the operations
 * of a raster step; n_teams 1..16: up to 8 teams one per XCD, 9-16 two per XCD).  The rANS operation picks its variant
 * by rate as lbc_decode does: below 1 bit per symbol the sparse one, otherwise the dense one on a copy of the tables
 * every workgroup stages in its LDS at launch start (the sparse one where those tables do not fit beside the
 * geometry's partials).
 * Batches the team kernel does not cover (M > 256, buffers past 4 GB) are decoded by lbc_decode one after another.  Synchronous like lbc_decode; one call at a time per process. */
int lbc_decode_team(lbc_model *const *ms, int n_teams, const uint8_t *const *streams, const size_t *lens, int n_img,
                    int Hb, int Wb, float *const *zhat_devs, void *stream);
/* raw stamps of the last lbc_decode_team launch made with LBIC_TEAM_STAMPS=1, 1024 per team (team rank 0), s_memrealtime
 * (100 MHz): [op] after each barrier of the sampled raster step (Hb/2, Wb/2), [32 + op] when rank 0's own share of the
 * operation was done, [60] end of the step before it, [61] end of the sampled step, [62] launch start, [63] launch
 * end; s_memtime (shader clock) [256 + 64 op + p] inside the operation's GEMM (p: entry, A loads issued, first chain, all
 * chains, outputs written, epilogue operands issued, first weights issued, offsets, partials reduced (8), first round
 * of outputs written (9), wave w's chains done (16 + w), its first chain done (24 + w), its A loads issued (32 + w), its first A fragment in (40 + w)).  m = the call's first handle. */
int lbc_team_stamps(const lbc_model *m, unsigned long long *out, int max_out, int *n_out);
/* the last lbc_decode_team launch led by m: its duration (HIP events around the launch), algorithmic bytes and FLOPs
 * (per raster step, the graph decoder's accounting: weights + A rows + outputs once per GEMM, rANS inputs and
 * outputs; times teams x Hb x Wb) and whether it ran with plain hand-off stores (1) or write-through ones (0). */
int lbc_team_stats(const lbc_model *m, double *launch_ms, double *bytes, double *flops, int *plain);
/* how the last lbc_decode_team call led by m decoded: 0 lbc_decode per batch (fallback), 1 one team launch with the
 * sparse rANS variant, 2 one team launch with the dense variant (tables in LDS); one batch of one image goes to
 * lbc_decode: 3 its single-image decoder (k_dec_one), 4 its row graphs (lbc_team_stats then reports that decode's
 * duration, no algorithmic work and plain = -1). */
int lbc_team_mode(const lbc_model *m, int *mode);
/* counters of the lbc_decode_team calls led by m: launches rerun with write-through hand-offs after the placement
 * census found a team spread over XCDs; and launches in which a workgroup timed out at a team barrier (the grid was
 * not co-resident in time, e.g. CUs held by another process) and whose batches were then decoded by lbc_decode one
 * after another (same results).  Any other launch failure is returned as LBC_E_STATE. */
int lbc_team_events(const lbc_model *m, int *sc1_reruns, int *timeouts);

/* OPT-IN sub-stream format (not the reference's bitstream): one rANS stream per block row,
 * container [u32 'LBW1'][u32 Hb][u32 bytes[Hb]][row streams...], each row stream in the same coder
 * format as lbc_rans_encode.  Costs 12 bytes per block row over the reference format and lets the
 * decoder run the encoder's anti-diagonal wavefront instead of a raster loop.  sym/idx: one image. */
int lbc_rans_encode_rows(const lbc_model *m, const int32_t *sym, const int32_t *idx, int Hb, int Wb, uint8_t **out,
                         size_t *len);
int lbc_decode_rows(lbc_model *m, const uint8_t *const *streams, const size_t *lens, int n_img, int Hb, int Wb,
                    float *zhat_dev, void *stream);

/* Band pipeline for frames split over GPUs by block rows (no reference counterpart: the reference
 * codes one image on one device).  compress() of block rows [v0, v0 + Hb_band) of n_img frames, x_dev
 * [n_img][Hb_band][Wb][3B^2].  The frames' anti-diagonal wavefront codes block (v, h) at global step t = h + 2v;
 * lbc_band_run runs this band's share of global steps [t0, t1).  halo_dev (nullable, [n_img][2][Wb][3B^2]) holds the
 * two block rows above the band (v0-2, v0-1) as the band above last returned them in its edge_dev; it must contain
 * every block that band coded before step t1 - 1 (so: the band above ran [t0, t1) first).  edge_dev (nullable,
 * same shape) receives this band's last two block rows after the range.  lbc_band_end writes zhat, symbols and
 * indexes of the band (layout as lbc_encode for Hb_band rows); the bands' symbols concatenated in row order are the
 * frame's.  Results are bit-identical to lbc_encode on the whole frame (compress() semantics). */
int lbc_band_begin(lbc_model *m, const float *x_dev, int n_img, int Hb_band, int Wb, int v0, void *stream);
int lbc_band_run(lbc_model *m, int t0, int t1, const float *halo_dev, float *edge_dev, void *stream);
int lbc_band_end(lbc_model *m, float *zhat_dev, int32_t *sym_dev, int32_t *idx_dev, float *bits_dev, void *stream);

void lbc_free(void *p);
const char *lbc_last_error(void);

/* Kernel-time instrumentation of the last lbc_encode / lbc_decode call (HIP events on `stream`):
 * total milliseconds of the encode and decode phases. */
int lbc_last_timing(const lbc_model *m, double *enc_ms, double *dec_ms);

/* Per-kernel instrumentation (bench.py's roofline).  HIP events cannot be recorded inside a captured
 * graph (ROCm 7.2), so while enabled every kernel of every `sample_every`-th wavefront / raster step is
 * captured with a timing slot: its workgroups stamp the earliest start and latest end on the GPU's
 * constant 100 MHz clock (s_memrealtime), per XCD.  The launch's algorithmic FLOPs and bytes are recorded
 * at capture.  lbc_profile_begin zeroes every slot; lbc_profile_end synchronises and returns one record
 * per kernel family from the launches executed since then (the last replay of each sampled graph). */
typedef struct {
    char name[40];
    long long launches;   /* sampled launches */
    long long total_launches; /* all launches of this kernel since lbc_profile_begin */
    double total_ms;      /* summed in-kernel spans (first workgroup start -> last workgroup end) */
    double flops;         /* summed algorithmic FLOPs (2 * rows * K_live * N for a GEMM) */
    double bytes;         /* summed algorithmic bytes (weights + A rows + outputs read/written once) */
    long long launches_chain; /* sampled launches whose predecessor in the stream chain was sampled too */
    double total_ms_chain;    /* summed launch-to-launch periods end(previous launch) -> end(this launch):
                                 the span plus the kernel boundary in front of it */
    double total_flops;       /* algorithmic FLOPs / bytes of ALL launches since lbc_profile_begin (GEMM families;
                                 sampled or not, also with sample_every = 0) */
    double total_bytes;
} lbc_kernel_stat;

int lbc_profile_begin(lbc_model *m, int sample_every);
int lbc_profile_end(lbc_model *m, lbc_kernel_stat *out, int max_out, int *n_out);

#ifdef __cplusplus
}
#endif
#endif /* LBIC_H */
