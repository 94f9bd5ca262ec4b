/*
 * rr.h — C-ABI of librr, the MI355X (gfx950) embed+search library.
 *
 * The reference (Mak-GIBA/research_image_retrieval, src/benchmark) is pure
 * Python/PyTorch and has no FFI of its own: its "operator API" is duck-typed
 * Python.  Every entry point below replaces one torch/numpy
 * call site on the reference's extract-and-rank hot path; the citation in
 * each comment names that site (paths relative to src/benchmark/).  The
 * Python mirror of the reference API (research_image_retrieval_amd/) binds
 * these with ctypes; INTEGRATION.md shows the binding.
 *
 * Conventions
 *   - All tensors are caller-owned DEVICE pointers (e.g. torch data_ptr()).
 *     Dense row-major, fp32 unless stated.  Images/activations are NHWC.
 *   - `stream` is a hipStream_t passed as void* (NULL = default stream).
 *     Every call is stream-ordered and asynchronous: no host sync inside,
 *     except the explicit *_collect / *_sync helpers.
 *   - Return value: 0 on success, a negative RR_E* code on error; the message
 *     is available from rr_last_error(h).  The library never aborts.
 *   - One handle per device; handles are independent across threads.  Every
 *     entry point runs on its handle's device: the calling thread's current
 *     HIP device is switched to it for the call and restored afterwards.
 */
#ifndef RR_H_
#define RR_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RR_OK 0
#define RR_EINVAL (-1)    /* bad argument / unsupported shape */
#define RR_EHIP (-2)      /* HIP runtime error */
#define RR_EWORKSPACE (-3) /* workspace too small */
#define RR_EOVERFLOW (-4) /* candidate buffer overflow (see rr_cosine_topk) */

/* Words of an activation's max-|x| record (rr_conv2d_h2, rr_amax_f32): the
 * float bit patterns of per-wave maxima, hashed over this many words so no
 * single address takes every atomic.  Zero them before the producing call. */
#define RR_AMAX_SLOTS 64

typedef struct rr_handle_s* rr_handle_t;

/* ABI revision of this header.  Bumped when an existing entry changes its
 * arguments under the same name (a caller built against an older header would
 * pass shifted arguments): 2 = rr_alpha_qe gained n_rows (round 2); 3 = the
 * f16x2 entries rr_conv2d_h2 / rr_bottleneck_out_h2 / rr_stem_pool_h2 /
 * rr_split2_f16 / rr_amax_f32 were added (no existing entry changed); 4 =
 * rr_linear_bf16_ln / rr_ln_partials_bf16 were added (round 4; the ViT
 * LayerNorm fold); 5 = rr_bottleneck_seam_h2 was added and the tuning keys
 * RR_TUNE_SWEEP_ORDER (6), RR_TUNE_SWEEP_PF (7) and RR_TUNE_LP_IL (12)
 * were retired (round 5: they lost their A/Bs; rr_set_tuning returns
 * RR_EINVAL for them, and their numbers are not reused); RR_TUNE_LP_CFG value
 * 6 (the gallery-in-VGPR sweep) was retired then too, and the number was
 * REDEFINED in the same revision as the tests' hook for the three-A-stage
 * persistent bf16 tile (a caller of the old value 6 now gets that tile on
 * stored-C GEMMs and the cost-based pick on sweeps); and rr_linear_bf16_ln /
 * rr_ln_partials_bf16 now centre the bf16 rows on their 256-column tile
 * means with colsum per k tile (same arguments, new layout); 6 = entries
 * REMOVED: rr_bottleneck_seam_h2 (round 5's block seam, measured slower
 * than the two launches it fused) and the split-bf16 core's rr_conv2d_s3 /
 * rr_linear_s3 / rr_split3_bf16 (superseded by the f16x2 core in round 3);
 * the tuning keys RR_TUNE_SWEEP_FORM (14) and RR_TUNE_HALO_2D (15) were
 * added (round 6).
 * Bindings compare rr_abi_version() with the RR_ABI_VERSION they were
 * written against.                                                          */
#define RR_ABI_VERSION 6
int rr_abi_version(void);

/* ---- handle ------------------------------------------------------------ */
const char* rr_version(void);
int rr_create(int device, rr_handle_t* out);
int rr_destroy(rr_handle_t h);
const char* rr_last_error(rr_handle_t h);

/* Per-kernel-class HIP-event timing (used by bench.py for the roofline).
 * When enabled, every launch of a timed class is bracketed by hipEvents on
 * the launch stream; rr_timing_collect synchronises those events and returns
 * the accumulated milliseconds and launch count for `cls`, then resets it.
 * Classes: 0 = cosine GEMM with the fused top-k filter epilogue,
 *          1 = conv/linear GEMM, 2 = top-k select/merge,
 *          3 = elementwise (preprocess/resize/pool/norm),
 *          4 = dense cosine GEMM (top-k threshold seed, rr_cosine_scores),
 *          5 = fused attention (ViT). */
int rr_timing_enable(rr_handle_t h, int enable);
int rr_timing_collect(rr_handle_t h, int cls, double* ms, long long* launches);

/* The device a handle was created for (rr_create's `device`). */
int rr_get_device(rr_handle_t h, int* device);

/* Kernel tile-config overrides for this handle (tests and tuning tools; the
 * default 0 = the library's own pick, which the product path always uses).
 *   RR_TUNE_GEMM_CFG: exact-fp32 core tile, 22 (128x128), 41 (256x64), 88 (256x256)
 *   RR_TUNE_GEMM_BK:  exact-fp32 core k-tile depth, 16 or 32
 *   RR_TUNE_LP_CFG:   bf16/fp8 core (0, the default: for the bf16 stored-C GEMMs with
 *                     the ViT epilogues, N % 256 == 0 and K <= 1024, the persistent
 *                     256x256 k-stream; its one-tile form is 3), 1 (128x128), 2 (256x64),
 *                     3 (256x256), 6 (the persistent form with three A stages for the
 *                     epilogues without the LayerNorm fold, at any K; tests; this
 *                     value's meaning changed in ABI 5, see above),
 *                     4 (256x320 for bf16 filter / score sweeps, 256x256 otherwise),
 *                     5 (bf16 sweeps with K % 128 == 0, fp8 sweeps with K % 256 == 0:
 *                     256x256 8-phase pipeline; otherwise as 3)
 *   RR_TUNE_S3_CFG:   f16x2 split core, 1..15 (gemm_s3.hip tile table; 13 = the halo-staged stride-1 3x3 tile on
 *                     v_mfma_f32_32x32x16_f16, 14 = the same on v_mfma_f32_16x16x32_f16
 *                     (the default picks 14's form for cout % 256 == 0, 13's for cout 64);
 *                     15 = the 256x256 tile (12) as a persistent k-stream (the default
 *                     for dense A with cout % 256 == 0, K >= 256, its 256x128 form
 *                     for dense cout 128, K >= 256, its 256x64 form for dense cout 64,
 *                     K >= 64; forced, every other
 *                     GEMM runs the library's pick; 12 forces the one-tile-per-block form);
 *                     7 also selects the implicit-GEMM fused stem over the halo stem)
 *   RR_TUNE_S3_STAGGER: split core first-round stagger, 0..200 sleeps of
 *                     ~1 us for every other resident block (-1 = the library's pick)
 *   RR_TUNE_SWEEP_MF16: the 256x320 bf16 filter sweep on v_mfma_f32_16x16x32_bf16 (1)
 *                     or v_mfma_f32_32x32x16_bf16 (0); -1 = the library's pick (0)
 *   RR_TUNE_SWEEP_IL: the bf16 / fp8 filter sweeps: 1 = the next k-tile's LDS-DMA
 *                     issued chunk by chunk among the k-tile's first MFMAs, 0 = one
 *                     burst at the top of the k-tile; -1 = the library's pick (1 for the
 *                     256x320 bf16 and the fp8 sweeps, 0 for the 256x256 bf16 one)
 *   RR_TUNE_CONV_IL:  the f16x2 256x256 conv tile (RR_TUNE_S3_CFG 12): 1 = the next
 *                     k-tiles' B DMA and A loads issued one group at a time among the
 *                     MFMAs, 0 = one burst at the top of the k-tile; 1 also selects the
 *                     halo-staged 3x3 tile's 16x16x32 form with its B DMA spread the
 *                     same way; -1 = the library's pick (0)
 *   RR_TUNE_HALO_MF:  the f16x2 halo-staged 3x3 tiles on v_mfma_f32_16x16x32_f16 (1) or
 *                     v_mfma_f32_32x32x16_f16 (0); for cout 64: 2 = the 512-row
 *                     single-buffer tile (the pick where its 640-row halo holds the map,
 *                     round 6), 3 = the persistent 256-row stream (round 5's pick); for
 *                     cout 128: 4 = the two-buffer one-tap tile (the pick is the
 *                     single-buffer three-tap one, round 6);
 *                     -1 = the library's pick (RR_TUNE_S3_CFG 13 / 14 override it)
 *   RR_TUNE_S3_CFG_RES: as RR_TUNE_S3_CFG, for the split-core GEMMs with a residual
 *                     epilogue only (0 = RR_TUNE_S3_CFG's choice)
 *   RR_TUNE_SWEEP_FORM: the bf16 filter sweeps (the prefilter's pass 2, bf16
 *                     rr_cosine_topk_lp): 0 = the gemm core's tiles (RR_TUNE_LP_CFG
 *                     applies), 1 = the hand-scheduled 16x16x32 sweep (csrc/sweep16.hip)
 *                     on 128-B LDS rows (K % 64 == 0; else as 2), 2 = the same on
 *                     64-B rows; -1 = the library's pick
 *   RR_TUNE_HALO_2D:  the f16x2 stride-1 3x3 convs on 2-D block halo tiles (16 x 16 or,
 *                     for cout 64, 16 x 32 outputs of one image; no residual epilogue):
 *                     -1 = where no raster halo tile holds the map (the library's pick),
 *                     1 = wherever one serves, 0 = never (ABI 6, round 6)
 * Any other key or value: RR_EINVAL. */
#define RR_TUNE_GEMM_CFG 1
#define RR_TUNE_GEMM_BK 2
#define RR_TUNE_LP_CFG 3
#define RR_TUNE_S3_CFG 4
#define RR_TUNE_S3_STAGGER 5
/* 6, 7: retired (ABI 5) */
#define RR_TUNE_SWEEP_MF16 8
#define RR_TUNE_SWEEP_IL 9
#define RR_TUNE_CONV_IL 10
#define RR_TUNE_HALO_MF 11
/* 12: retired (ABI 5) */
#define RR_TUNE_S3_CFG_RES 13
#define RR_TUNE_SWEEP_FORM 14
#define RR_TUNE_HALO_2D 15
int rr_set_tuning(rr_handle_t h, int key, int value);

/* ---- search (ranker) ----------------------------------------------------
 * Replaces iris_evaluate.py:383 `torch.mm(q, g.t())` + :386
 * `np.argsort(-similarity, axis=1)` (the only ranking driver), truncated to
 * the top k, with a STABLE order: score descending, then gallery index
 * ascending.  Scores are exact fp32 MFMA dot products (v_mfma_f32_32x32x2_f32,
 * a fixed k-ordered fmaf chain restated bit-for-bit by oracle/cosine_topk.c).
 *
 *   queries [nq][d], gallery [n][d]  (rows are expected L2-normalised by the
 *   caller, as iris_evaluate.py:379-380 does; the kernel does not renormalise)
 *   out_scores [nq][k] fp32, out_idx [nq][k] int64 = row + idx_offset.
 *   If n < k the tail is filled with (-inf, -1).
 *   1 <= k <= 16384, d % 4 == 0, 16-byte aligned rows.
 * Workspace: rr_cosine_topk_workspace_size(nq, n, d, k) bytes of device
 * memory, any alignment >= 256.  That size holds a worst-case candidate
 * buffer (every row of the gallery, per query: ~nq * n * 8 bytes), which can
 * never overflow.
 *
 * Bounded workspaces (all three rankers: rr_cosine_topk, rr_cosine_topk_lp,
 * rr_cosine_topk_prefilter with its _prefilter_ functions).  Any workspace of
 * at least rr_cosine_topk_workspace_size_cap(nq, n, d, k, k) bytes is
 * accepted; the ranker then keeps cap = rr_cosine_topk_cap_for(nq, n, d, k,
 * workspace_bytes) candidates per query (cap >= k; workspace_size_cap(...,
 * cap) gives the bytes for a chosen cap).  A query whose threshold filter
 * passes more than cap rows gets an incomplete candidate set: its output row
 * is NOT its exact top-k.  Every call zeroes and then sets the int32 at
 * rr_cosine_topk_overflow_offset (device, inside the workspace) to the number
 * of such queries; the int32 [nq] at rr_cosine_topk_counts_offset holds each
 * query's count (> cap = overflowed).  The caller re-runs those queries, e.g.
 * with a worst-case workspace for just them (ops.cosine_topk* with
 * max_workspace_bytes do this).  The status cannot be returned synchronously:
 * the counts exist only once the stream has run.  Offsets are valid for the
 * same (nq, n, d, k) until the workspace is reused.                         */
size_t rr_cosine_topk_workspace_size(int nq, long long n, int d, int k);
size_t rr_cosine_topk_workspace_size_cap(int nq, long long n, int d, int k, long long cap);
long long rr_cosine_topk_cap_for(int nq, long long n, int d, int k, size_t workspace_bytes);
size_t rr_cosine_topk_counts_offset(int nq, long long n, int d, int k);
size_t rr_cosine_topk_overflow_offset(int nq, long long n, int d, int k);
int rr_cosine_topk(rr_handle_t h, const float* queries, int nq,
                   const float* gallery, long long n, int d, int k,
                   long long idx_offset, float* out_scores, long long* out_idx,
                   void* workspace, size_t workspace_bytes, void* stream);

/* Dense cosine scores, gallery-major: scores[j][i] = <gallery_j, query_i>,
 * i.e. the transpose of iris_evaluate.py:383's similarity matrix. [n][nq]. */
int rr_cosine_scores(rr_handle_t h, const float* queries, int nq,
                     const float* gallery, long long n, int d, float* scores,
                     void* stream);

/* Merge nparts partial top-k lists (the per-shard results gathered over RCCL)
 * into one top-k_out list per query, same stable order.  Layout
 * part_scores/part_idx [nparts][nq][k_in]; entries with idx < 0 are padding.
 * Indices must be < 2^32 - 1 (ShardedGallery refuses larger galleries).
 * No reference counterpart (the reference never
 * shards); it is the k-way merge of SURVEY.md §8(e).        */
int rr_topk_merge(rr_handle_t h, const float* part_scores,
                  const long long* part_idx, int nparts, int nq, int k_in,
                  int k_out, float* out_scores, long long* out_idx,
                  void* stream);

/* ---- low-precision search (configs C4 bf16, C5 fp8) ---------------------
 * dtype: 1 = bf16 (RNE), 2 = fp8 OCP e4m3 with one fp32 scale per row.
 * rr_quantize_rows: x [rows][d] fp32 -> y [rows][d] (2 or 1 bytes/elem);
 * fp8 writes row_scale[r] = amax(row)/448 (x ~= q * scale).              */
int rr_quantize_rows(rr_handle_t h, const float* x, long long rows, int d,
                     int dtype, void* y, float* row_scale, void* stream);

/* rr_cosine_topk on bf16 / fp8 rows (fp32 accumulate, scores dequantised
 * by q_scale[i] * g_scale[j] when given; required for fp8).  Same workspace
 * and output contract as rr_cosine_topk; scores are the low-precision
 * ones, so parity vs fp32 is recall@k, not index equality.  d*size % 16 == 0. */
int rr_cosine_topk_lp(rr_handle_t h, const void* queries, const float* q_scale,
                      int nq, const void* gallery, const float* g_scale,
                      long long n, int d, int dtype, int k, long long idx_offset,
                      float* out_scores, long long* out_idx, void* workspace,
                      size_t workspace_bytes, void* stream);

/* alpha-weighted query expansion (config C5; absent from the reference,
 * SURVEY.md §8f row 3 — defined as in Radenovic et al., TPAMI 2018, the GeM
 * paper models/gem_pooling.py:3 cites):
 *   out[i] = normalize(q[i] + sum_{r<n} max(s[i][r],0)^alpha * g[idx[i][r]-idx_offset])
 * top_idx / top_scores [nq][k] as returned by rr_cosine_topk (idx < 0 =
 * padding, skipped); gallery [n_rows][d] = the local rows, holding global
 * indices [idx_offset, idx_offset + n_rows): an index outside that range is
 * skipped, never read.  Re-rank by calling rr_cosine_topk with `out` as the
 * queries.                                                                 */
int rr_alpha_qe(rr_handle_t h, const float* queries, int nq,
                const float* gallery, long long n_rows, int d, const long long* top_idx,
                const float* top_scores, int k, int n, float alpha,
                long long idx_offset, float* out, void* stream);

/* Exact cosine top-k through a bf16 prefilter: the SAME scores and indices,
 * bit for bit, as rr_cosine_topk (iris_evaluate.py:383-386 ranker), with the
 * full gallery sweep on the bf16 MFMA and only rows that can still reach the
 * exact top-k rescored with the fp32 core's fmaf chain (proof and bound in
 * csrc/prefilter.hip).  gallery_bf16 = rr_quantize_rows(gallery, bf16);
 * bound3 (device, 3 doubles) = rr_prefilter_gallery_bound of the same pair,
 * computed once per gallery.  d % 8 == 0.                                   */
int rr_prefilter_gallery_bound(rr_handle_t h, const float* gallery,
                               const void* gallery_bf16, long long n, int d,
                               double* bound3, void* stream);
size_t rr_cosine_topk_prefilter_workspace_size(int nq, long long n, int d, int k);
/* Byte offset, inside that workspace, of the int32 [nq] count of rows each
 * query kept through the bf16 filter pass (the rows then bounded and, where
 * they can still reach the top-k, rescored exactly); valid after a call with
 * the same (nq, n, d, k) until the workspace is reused. */
size_t rr_cosine_topk_prefilter_counts_offset(int nq, long long n, int d, int k);
/* Bounded workspaces, as for rr_cosine_topk (the count above > cap marks an
 * overflowed query). */
size_t rr_cosine_topk_prefilter_overflow_offset(int nq, long long n, int d, int k);
size_t rr_cosine_topk_prefilter_workspace_size_cap(int nq, long long n, int d, int k, long long cap);
long long rr_cosine_topk_prefilter_cap_for(int nq, long long n, int d, int k, size_t workspace_bytes);
int rr_cosine_topk_prefilter(rr_handle_t h, const float* queries, int nq,
                             const float* gallery, const void* gallery_bf16,
                             const double* bound3, long long n, int d, int k,
                             long long idx_offset, float* out_scores,
                             long long* out_idx, void* workspace,
                             size_t workspace_bytes, void* stream);

/* PCA-whitening learning, GPU half (replaces the
 * m = X.mean(0), Xc = X - m, np.dot(Xc.T, Xc) lines of
 * networks/backbone.py:46-49, called from networks/spca.py:215-217):
 *   mean_out [d]   fp64 column means of X [n][d] (fp32, row-major, device)
 *   gram_out [d*d] fp64 sum_i (x_i - m)(x_i - m)^T, symmetric (device)
 * fp32 MFMA partials over <= 8192-row slices, summed in fp64.  The caller
 * symmetrises / scales by 1/(2n) and runs the eigendecomposition on the host
 * (backbone.py:50-57).  Workspace is bounded (<= 131072-row chunks).          */
size_t rr_pcaw_gram_workspace_size(long long n, int d);
int rr_pcaw_gram(rr_handle_t h, const float* x, long long n, int d,
                 void* workspace, size_t workspace_bytes, double* mean_out,
                 double* gram_out, void* stream);

/* ---- embed (extractor) ---------------------------------------------------
 * uint8 HWC pixels -> fp32 NHWC, (x/255 - mean[c]) / std[c].
 * Replaces transforms.ToTensor + Normalize(mean=[.485,.456,.406],
 * std=[.229,.224,.225]) (dataset/configdataset.py:417, :430-436).          */
int rr_preprocess_u8(rr_handle_t h, const uint8_t* img_nhwc, int b, int hgt,
                     int wid, const float* mean3, const float* std3,
                     float* out_nhwc, void* stream);

/* Same with out_c in {3, 4}: out_c == 4 writes NHWC4 pixels with a zero
 * 4th channel, the stem conv's 16-byte tap layout (see rr_conv2d).          */
int rr_preprocess_u8_ex(rr_handle_t h, const uint8_t* img_nhwc, int b, int hgt,
                        int wid, const float* mean3, const float* std3,
                        int out_c, float* out_nhwc, void* stream);

/* fp32 NCHW -> NHWC relayout (the reference's forward_test input is NCHW). */
int rr_nchw_to_nhwc(rr_handle_t h, const float* in, int b, int c, int hgt,
                    int wid, float* out, void* stream);
/* Same, zero-padding the channel dim to out_c >= c.                       */
int rr_nchw_to_nhwc_ex(rr_handle_t h, const float* in, int b, int c, int hgt,
                       int wid, int out_c, float* out, void* stream);

/* 2-D convolution, NHWC, implicit GEMM on fp32 MFMA with a fused epilogue:
 * y = relu?( conv(x, w) + bias[co] + residual? ).  Weights [cout][kh][kw][cin]
 * with eval-mode BatchNorm already folded into w/bias by the host.
 * Replaces the torchvision ResNet conv/BN/ReLU/residual ops behind
 * networks/backbone.py:103-109 and models/gem_pooling.py:44,61.
 * residual may be NULL; output is [b][oh][ow][cout].
 * A-operand paths: 1x1/s1 = dense rows; cin % 32 == 0 = im2col with one
 * filter tap per 32-deep k-tile; cin == 4 = one tap per float4 (the stem on
 * NHWC4 input, zero 4th channel and zero 4th weight channel); other cin =
 * per-element gather.                                                      */
int rr_conv2d(rr_handle_t h, const float* x, int b, int hgt, int wid, int cin,
              const float* w, const float* bias, int cout, int kh, int kw,
              int stride, int pad, const float* residual, int relu, float* y,
              void* stream);

/* Bilinear resize, NHWC, align_corners=False, PyTorch source-index rule:
 * src = max(scale * (dst + 0.5) - 0.5, 0) with scale = 1/scale_factor when a
 * scale factor was given (inv_scale_h/w > 0) else in/out.  Replaces the
 * F.interpolate(..., mode='bilinear', align_corners=False) calls of
 * extract_vectors (utils/helpfunc.py:26, :38).                             */
int rr_resize_bilinear(rr_handle_t h, const float* x, int b, int hgt, int wid,
                       int c, int out_h, int out_w, float inv_scale_h,
                       float inv_scale_w, float* y, void* stream);

/* fp32-accurate convolution on the fp16 matrix cores (gemm_s3.hip, f16x2
 * split): the same operation, layouts and epilogue as rr_conv2d on the
 * 16-bit MFMA at three fp16 products per fp32 product.  Every fp32 operand is scaled by a power of two and split
 * into two fp16 pieces, x 2^e = x0 + x1 + r with |r| <= 2^-22 |x 2^e|; a.b
 * keeps a0b0 + (a0b1 + a1b0) (dropped terms <= 3 2^-22 |a||b|), three fp16
 * MFMAs with exact products and fp32 accumulation (a0b0 in its own
 * accumulator), and the accumulator is scaled back exactly.  Weights come
 * from rr_split2_f16: w2 = planes [2][cout][K] (fp16 bit patterns), w_iscale
 * [cout] the inverse row scales.  x_amax: the RR_AMAX_SLOTS-word max-|x|
 * record of x (from the producing call's y_amax, or rr_amax_f32); y_amax
 * (optional, zeroed by the caller): receives max |y| over the finite stored
 * values.  Needs cin % 32 == 0, or cin == 4 for the NHWC4 stem (w2 then holds
 * the flattened [kh][kw][4] filter zero-padded to K = kh*kw*4 rounded up to
 * 32).  y, bias and residual must be 16-byte aligned (RR_EINVAL otherwise).
 * The split scale of x is one per tensor: values more than 2^18 below its
 * max keep an absolute error <= 2^-40 max|x| instead of full relative
 * precision.  Replaces the same reference ops as rr_conv2d
 * (networks/backbone.py:103-109, :305-346; models/gem_pooling.py:44,61).    */
int rr_conv2d_h2(rr_handle_t h, const float* x, const unsigned* x_amax, int b,
                 int hgt, int wid, int cin, const void* w2,
                 const float* w_iscale, const float* bias, int cout, int kh,
                 int kw, int stride, int pad, const float* residual, int relu,
                 float* y, unsigned* y_amax, void* stream);

/* The output of a stage-entry bottleneck block on the f16x2 core, its 1x1
 * conv3 and its 1x1 strided downsample projection as ONE GEMM over
 * K = planes + cin:
 *   out = ReLU(y . W3^T + x[:, ::stride, ::stride] . Wd^T + bias)
 * (torchvision Bottleneck / the reference's ResBlock sum,
 * networks/backbone.py:327-346), so the projected identity is never written
 * or read back.  y: conv2's output [b][oh][ow][planes] with its max-|x|
 * record y_amax; x: the block input [b][hx][wx][cin] with x_amax;
 * (oh - 1) * stride < hx, (ow - 1) * stride < wx.  w2 / w_iscale:
 * rr_split2_f16 of the concatenated rows [W3 | Wd] [cout][planes + cin];
 * bias = the two folded biases' sum.  planes % 32 == 0, cin % 32 == 0,
 * cout % 256 == 0.  out_amax as rr_conv2d_h2's y_amax.                      */
int rr_bottleneck_out_h2(rr_handle_t h, const float* y, const unsigned* y_amax,
                         int b, int oh, int ow, int planes, const float* x,
                         const unsigned* x_amax, int hx, int wx, int cin,
                         int stride, const void* w2, const float* w_iscale,
                         const float* bias, int cout, float* out,
                         unsigned* out_amax, void* stream);

/* The ResNet stem on the f16x2 core with its max-pool fused: NHWC4 conv
 * (cin == 4, as rr_conv2d_h2) + bias + ReLU, then the 3x3 stride-2 padding-1
 * max-pool, written only pooled: y_pool [b][ph][pw][64] with
 * ph = (oh - 1) / 2 + 1, pw likewise (oh, ow the conv's output size).  Each
 * tile computes a 17 x 15 patch of conv outputs and pools its 8 x 7 windows
 * from LDS: the stem's 112 x 112 x 64 map never reaches HBM.  The max is taken
 * over the raw accumulators and scaled once (scale > 0, bias add and ReLU are
 * monotone): the same bits as rr_conv2d_h2 followed by the max-pool, for
 * finite inputs.  y_amax (optional, zeroed): max |y_pool|, which equals the
 * conv output's (every conv output lies in some window).  cout == 64.
 * Replaces networks/backbone.py:103-109's conv1 / bn1 / relu / maxpool.     */
int rr_stem_pool_h2(rr_handle_t h, const float* x, const unsigned* x_amax,
                    int b, int hgt, int wid, const void* w2,
                    const float* w_iscale, const float* bias, int cout, int kh,
                    int kw, int stride, int pad, float* y_pool,
                    unsigned* y_amax, void* stream);

/* fp16 2-way split of the rows of w [rows][k] (done once per weight tensor):
 * row n is scaled by 2^e_n, its max |w| then in [2^14, 2^15), and split into
 * planes [2][rows][kpad] (fp16 bit patterns, zero past k; kpad >= k, a
 * multiple of 32 for rr_conv2d_h2); iscale[n] = 2^-e_n.                    */
int rr_split2_f16(rr_handle_t h, const float* w, int rows, int k, int kpad,
                  void* planes, float* iscale, void* stream);

/* max |x| over the finite values of x[n] into the RR_AMAX_SLOTS words at
 * amax (atomic max; zero them first): the x_amax record rr_conv2d_h2 needs
 * for an input no earlier call produced.                                   */
int rr_amax_f32(rr_handle_t h, const float* x, long long n, unsigned* amax,
                void* stream);

/* Max pool (torchvision ResNet stem maxpool 3x3/2 pad 1), NHWC. */
int rr_maxpool2d(rr_handle_t h, const float* x, int b, int hgt, int wid, int c,
                 int k, int stride, int pad, float* y, void* stream);

/* GeM pooling over the spatial axis of an NHWC map [b][hw][c] -> [b][c]:
 * (mean_hw clamp(x, eps)^p)^(1/p).  Replaces networks/RetrievalNet.py:324-325
 * (gem, python-float p) and models/gem_pooling.py:20-23 (GeMPooling).      */
int rr_gem_pool(rr_handle_t h, const float* x, int b, int hw, int c, float p,
                float eps, float* out, void* stream);

/* y[m][n] = x[m][:] . w[n][:] + bias[n]   (bias may be NULL).
 * Replaces GeM.whiten 1x1 conv (networks/RetrievalNet.py:332,342),
 * GeMModel.feature_proj Linear (models/gem_pooling.py:50,68) and the
 * PCA-whitening ConvDimReduction apply (networks/spca.py:205-227).        */
int rr_linear(rr_handle_t h, const float* x, int m, int k, const float* w,
              const float* bias, int n, float* y, void* stream);

/* y = act(x . w^T + bias + residual); act 0 = none, 1 = ReLU, 2 = QuickGELU
 * (x * sigmoid(1.702 x)).  bias / residual ([m][n]) may be NULL.  Replaces the
 * ViT projections of networks/model.py:171-192 (MHA in/out_proj, c_fc +
 * QuickGELU, c_proj + residual) and `ln_post(x[:,0]) @ proj` (:239-241).   */
int rr_linear_ex(rr_handle_t h, const float* x, int m, int k, const float* w,
                 const float* bias, int n, const float* residual, int act,
                 float* y, void* stream);

/* bf16 x [m][k] . bf16 w [n][k]^T, fp32 accumulate, fp32 bias / residual,
 * act as rr_linear_ex; y fp32 or (out_bf16) bf16.  The C4 (ViT bf16) GEMMs. */
int rr_linear_bf16(rr_handle_t h, const void* x, int m, int k, const void* w,
                   const float* bias, int n, const float* residual, int act,
                   int out_bf16, void* y, void* stream);

/* rr_linear_bf16 with the ViT LayerNorms (networks/model.py:157-163, the ln_1
 * / ln_2 of :188-190) folded into the GEMMs, so no LayerNorm pass reads the
 * fp32 residual stream.  Exactly one of stats_in / stats_out is set:
 *  - stats_out (the out-proj / c_proj GEMMs: bias, residual, fp32 y, act 0,
 *    n % 256 == 0, k % 64 == 0): besides y, writes per row and 256-column tile
 *    t the LayerNorm partials of y, stats_out [m][n/256][2] = (mean_t, M2_t =
 *    sum (y - mean_t)^2 over the tile's 256 columns), and xb_out [m][n] =
 *    bf16(y - mean_t) (RNE), each tile centred on its own mean.
 *  - stats_in (the in-proj / c_fc GEMMs: bias, bf16 y, k % 64 == 0, k <= 768):
 *    x holds such centred bf16 rows (xb) with their partials
 *    [m][ceil(k/256)][2]; w = bf16(W o gamma) (columns scaled by the LayerNorm
 *    weight), colsum [ceil(k/256)][n] = sum over k-tile t of float(w[n][k]),
 *    bias = b + W beta:
 *      y = act(rstd_m (x.w^T + sum_t (mean_t - mean_m) colsum[t]) + bias),
 *    mean_m / rstd_m = 1 / sqrt(var + eps) from the partials (biased
 *    variance, combined as Chan et al.).  Equal to LayerNorm -> bf16 ->
 *    rr_linear_bf16 up to where bf16 rounding falls: the operand is
 *    bf16(y - mean_t) instead of bf16(LayerNorm(y)), an element rounding error
 *    of 2^-9 |y_k - mean_t| against the LayerNorm path's 2^-9 rstd |y_k -
 *    mean| -- the same scale, whatever the rows' |mean| / std (centring was
 *    added in ABI 5: with bf16(y) the error grew with |mean| / std;
 *    tests/test_gpu_vit.py::test_linear_bf16_ln_fold_large_mean).             */
int rr_linear_bf16_ln(rr_handle_t h, const void* x, int m, int k, const void* w,
                      const float* bias, int n, const float* residual, int act,
                      int out_bf16, void* y, const float* stats_in,
                      const float* colsum, float eps, float* stats_out,
                      void* xb_out, void* stream);

/* The producer side of rr_linear_bf16_ln for rows that no GEMM wrote (the
 * first block's ln_1 input): the partials stats [m][d/256][2] = (mean_t,
 * M2_t) of fp32 x [m][d] and xb [m][d] = bf16(x - mean_t); d % 256 == 0.   */
int rr_ln_partials_bf16(rr_handle_t h, const float* x, int m, int d, void* xb,
                        float* stats, void* stream);

/* ---- ViT-B/16 (networks/model.py:206-243) ------------------------------ */
/* LayerNorm over the last dim (fp32, biased variance), rows x + i*ldx ->
 * dense y [m][d].  Replaces LayerNorm (:157-163): ln_pre, ln_1, ln_2, and
 * ln_post on the CLS rows (ldx = seq*width).  d <= 4096.                   */
int rr_layernorm(rr_handle_t h, const float* x, long long ldx, int m, int d,
                 const float* gamma, const float* beta, float eps, float* y,
                 void* stream);

/* Same, output dtype 0 = fp32, 1 = bf16 (feeds rr_linear_bf16).           */
int rr_layernorm_ex(rr_handle_t h, const float* x, long long ldx, int m, int d,
                    const float* gamma, const float* beta, float eps,
                    int out_dtype, void* y, void* stream);

/* NHWC image -> non-overlapping patch rows [b*(H/p)*(W/p)][p*p*c], (kh,kw,c)
 * order: with weights [width][p][p][c] the patch conv (:223, stride = kernel
 * = p, no bias) becomes one dense GEMM (rr_linear).                        */
int rr_patchify(rr_handle_t h, const float* x, int b, int hgt, int wid, int c,
                int patch, float* y, void* stream);

/* Same, output dtype 0 = fp32, 1 = bf16 (RNE, the rows rr_linear_bf16 reads;
 * equal to rr_patchify followed by rr_quantize_rows bf16).                 */
int rr_patchify_ex(rr_handle_t h, const float* x, int b, int hgt, int wid,
                   int c, int patch, int out_dtype, void* y, void* stream);

/* tokens [b][1+np][width]: row 0 = cls + pos[0], row 1+i = patches[b][i] +
 * pos[1+i]  (class_embedding concat + positional_embedding, :226-227).     */
int rr_vit_tokens(rr_handle_t h, const float* patches, int b, int npatch,
                  int width, const float* cls, const float* pos, float* y,
                  void* stream);

/* Same with ln_pre (:229) fused when gamma and beta are given (both or
 * neither; width <= 4096): y = LayerNorm(tokens), bit-identical to
 * rr_vit_tokens followed by rr_layernorm, without the HBM round trip.      */
int rr_vit_tokens_ex(rr_handle_t h, const float* patches, int b, int npatch,
                     int width, const float* cls, const float* pos,
                     const float* gamma, const float* beta, float eps,
                     float* y, void* stream);

/* Multi-head self-attention core: qkv [b*seq][3*heads*64] (q | k | v, the
 * in_proj output) -> out [b*seq][heads*64] = softmax(q k^T / 8) v per head
 * (nn.MultiheadAttention, ResidualAttentionBlock.attention :184-186).
 * head_dim == 64, seq <= 256.  Fused on fp32 MFMA, scores never leave the
 * CU.                                                                      */
int rr_attention(rr_handle_t h, const float* qkv, int b, int seq, int heads,
                 int head_dim, float* out, void* stream);
/* Same, output dtype 0 = fp32, 1 = bf16.                                   */
/* (rr_attention_bf16 below: the C4 bf16 variant.)                          */
int rr_attention_ex(rr_handle_t h, const float* qkv, int b, int seq, int heads,
                    int head_dim, int out_dtype, void* out, void* stream);

/* The attention core on bf16 MFMA (config C4): q, k, v rounded to bf16 (RNE),
 * fp32 accumulation and fp32 softmax, P rounded to bf16 for P.V; output fp32
 * (out_dtype 0) or bf16 (1).  Same contract as rr_attention_ex.             */
int rr_attention_bf16(rr_handle_t h, const float* qkv, int b, int seq, int heads,
                      int head_dim, int out_dtype, void* out, void* stream);
/* Same, with the QKV rows already in bf16 (the QKV linear's bf16 output,
 * rr_linear_bf16 out_bf16 = 1: rounded RNE as rr_attention_bf16 rounds them,
 * so the result is bit-identical at half the bytes read).                  */
int rr_attention_bf16_qkv16(rr_handle_t h, const void* qkv_bf16, int b, int seq,
                            int heads, int head_dim, int out_dtype, void* out,
                            void* stream);

/* Row-wise L2 normalisation x / max(||x||_2, eps), in place allowed.
 * Replaces F.normalize (networks/RetrievalNet.py:343, models/gem_pooling.py:91,
 * utils/helpfunc.py:44, iris_evaluate.py:379-380).                        */
int rr_l2_normalize(rr_handle_t h, const float* x, int m, int d, float eps,
                    float* y, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* RR_H_ */
