// rr_internal.hpp — shared declarations for librr (gfx950 only).
#pragma once

#include <type_traits>

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>
#include <vector>

#include "../../include/rr.h"

struct rr_handle_s {
  int device = 0;
  std::string last_error;
  // kernel-config overrides (rr_set_tuning): tests and tools force each tile
  // config through these; the product path never sets them, and their
  // defaults (0 / -1) select the library's own picks
  struct Tuning {
    int gemm_cfg = 0;  // fp32 core: 22, 41 or 88
    int gemm_bk = 0;   // fp32 core k-tile depth: 16 or 32
    int lp_cfg = 0;    // bf16 / fp8 core: 1 = 128x128, 2 = 256x64, 3 = 256x256, 4 = 256x320 (filter sweeps), 5 = 8-phase 256x256 (bf16 / fp8 sweeps), 6 = the persistent bf16 tile with three A stages (tests); 0: the pick (the persistent 256x256 bf16 tile for the ViT epilogues, K <= 1024)
    int s3_cfg = 0;    // split cores: 1..15 (gemm_s3.hip tile table; 9-15 f16x2 only); 0: the pick
    int s3_stagger = -1;  // split-bf16 core round stagger in ~1 us sleeps (-1: the library's pick)
    int sweep_mf16 = -1;   // bf16 256x320 filter sweep on v_mfma_f32_16x16x32_bf16 (1) or 32x32x16 (0); -1: the pick (0)
    int sweep_il = -1;     // bf16 256x320 filter sweep: next k-tile's DMA spread among the MFMAs (1) or one burst (0); -1: the pick (1)
    int conv_il = -1;      // f16x2 256x256 conv tile (s3_cfg 12) and halo 16x16x32 tile: next k-tiles' loads spread among the MFMAs (1) or one burst (0); -1: the pick (0)
    int halo_mf = -1;      // f16x2 halo 3x3 tiles on v_mfma_f32_16x16x32_f16 (1) or 32x32x16 (0); -1: the pick (the 256x256 tile 1, the others 0)
    int halo_2d = -1;      // the 2-D block halo tiles: -1 where no raster halo holds the map, 1 wherever one serves, 0 never
    int s3_cfg_res = 0;    // split cores: forced tile config for the GEMMs with a residual epilogue only (0: s3_cfg's)
    int sweep_form = -1;   // bf16 filter sweeps: 0 = gemm_f32.hip's tiles, 1 / 2 = sweep16.hip on 128-B / 64-B LDS rows; -1: the pick
  } tune;
  int n_cu = 0;  // compute units of the handle's device (device_cu_count)
  // timing (see rr_timing_enable)
  bool timing = false;
  static constexpr int kClasses = 6;
  // event pairs per class, created on demand and reused across timing
  // windows; the pool grows with the launches of a window (no cap: a capped
  // pool silently dropped the launches past it)
  std::vector<hipEvent_t> ev_start[kClasses], ev_stop[kClasses];
  int n_ev[kClasses] = {};
  double acc_ms[kClasses] = {};
  long long acc_launches[kClasses] = {};
};

namespace rr {

// Every C-ABI entry runs on its handle's device (rr.h: one handle per
// device): the calling thread's current device is switched for the call and
// restored afterwards, so a NULL-stream launch, a memset or an event of a
// handle created for device d always lands on d.
struct DeviceGuard {
  int prev = -1;
  int rc = 0;
  explicit DeviceGuard(const rr_handle_s* h) {
    int cur = -1;
    if (hipGetDevice(&cur) != hipSuccess) {
      rc = RR_EHIP;
      return;
    }
    if (cur != h->device) {
      if (hipSetDevice(h->device) != hipSuccess) {
        rc = RR_EHIP;
        return;
      }
      prev = cur;
    }
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};
#define RR_ENTRY(h)                                                                 \
  if (!(h)) return RR_EINVAL;                                                       \
  rr::DeviceGuard rr_device_guard_(h);                                              \
  if (rr_device_guard_.rc) return rr::set_error(h, rr_device_guard_.rc, "cannot select the handle's device")

enum TimerClass { kTimeCosine = 0, kTimeGemm = 1, kTimeSelect = 2, kTimeElem = 3, kTimeCosineSeed = 4, kTimeAttn = 5 };

// RAII-style bracket: records start/stop events on `stream` when timing is on.
struct TimedLaunch {
  rr_handle_s* h;
  int cls;
  hipStream_t s;
  int slot = -1;
  TimedLaunch(rr_handle_s* h_, int cls_, hipStream_t s_);
  ~TimedLaunch();
};

int set_error(rr_handle_s* h, int code, const std::string& msg);
int check_hip(rr_handle_s* h, hipError_t e, const char* what);

// ---- ordered 64-bit keys: score descending, then index ascending --------
// key = (ord(score) << 32) | ~idx ; larger key = better rank.  Every NaN maps
// to ord 0, below -inf (0x007fffff): NaN scores rank last, among themselves by
// index, as np.argsort(-similarity) places them (iris_evaluate.py:386).  The
// all-zero key (ord 0, idx 0xffffffff) is reserved for "no entry"; gallery
// shards have < 2^32 rows, so a real key is never 0.
__host__ __device__ inline uint32_t ord_f32(float f) {
  uint32_t u;
  __builtin_memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return 0u;  // NaN
  if (u == 0x80000000u) u = 0u;  // -0.0 ranks as +0.0 (equal scores tie-break on index)
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__host__ __device__ inline float unord_f32(uint32_t o) {
  uint32_t u = (o & 0x80000000u) ? (o & 0x7fffffffu) : ~o;
  float f;
  __builtin_memcpy(&f, &u, 4);
  return f;
}
// next float toward -inf / +inf (finite inputs; -inf / +inf map to themselves)
__host__ __device__ inline float next_down(float f) {
  uint32_t u;
  __builtin_memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) == 0) u = 0x80000001u;                  // +-0 -> -min denormal
  else if (u == 0xff800000u || (u & 0x7fffffffu) > 0x7f800000u) {  // -inf, NaN
  } else if (u & 0x80000000u) ++u;
  else --u;
  __builtin_memcpy(&f, &u, 4);
  return f;
}
__host__ __device__ inline float next_up(float f) { return -next_down(-f); }
__host__ __device__ inline unsigned long long make_key(float s, uint32_t idx) {
  return ((unsigned long long)ord_f32(s) << 32) | (unsigned long long)(~idx);
}
__host__ __device__ inline uint32_t key_idx(unsigned long long k) {
  return ~(uint32_t)(k & 0xffffffffull);
}
__host__ __device__ inline float key_score(unsigned long long k) {
  return unord_f32((uint32_t)(k >> 32));
}

// ---- GEMM core launchers (gemm_f32.hip) ---------------------------------
// Rows of the threshold-seeding sample of the cosine top-k rankers (exact
// for any sample >= k rows).  About 2 % of the shard, capped at 32768 and
// floored at 4096: on a row-sharded gallery the seed GEMM + select cost per
// rank, nq x s with nq = all ranks' queries, then stays constant as the node
// grows (the later passes already scale as nq x n / ranks).
inline long long seed_sample_rows(long long n, int k) {
  long long s = n / 48;
  if (s > 32768) s = 32768;
  if (s < 4096) s = 4096;
  if (s < k) s = k;
  return n < s ? n : s;
}

// compute units of the handle's device (queried once)
inline int device_cu_count(rr_handle_s* h) {
  if (h->n_cu <= 0) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, h->device) != hipSuccess || v <= 0) v = 256;
    h->n_cu = v;
  }
  return h->n_cu;
}

// Candidate capacity per query that a workspace of `bytes` holds when the
// candidate buffer [nq][cap] of 8-byte keys starts at `off_cand` (256-aligned)
// and the layout's total is rounded up to 256 B; at most `worst`.
inline long long cap_that_fits(size_t off_cand, int nq, size_t bytes, long long worst) {
  const size_t usable = bytes & ~(size_t)255;
  if (nq <= 0 || usable <= off_cand) return 0;
  const long long cap = (long long)((usable - off_cand) / ((size_t)nq * 8));
  return cap < worst ? cap : worst;
}

enum AMode { A_DENSE = 0, A_CONV = 1, A_CONV_GENERIC = 2, A_CONV_C4 = 3 };
enum EMode { E_STORE = 0, E_SCORES_T = 1, E_FILTER = 2 };
enum DType { DT_F32 = 0, DT_BF16 = 1, DT_FP8 = 2 };

struct GemmArgs {
  // A operand (M rows x K): dense [M][lda] or implicit im2col of NHWC input
  const float* A = nullptr;
  long long lda = 0;
  int M = 0, K = 0;
  int H = 0, W = 0, Cin = 0, OH = 0, OW = 0, KH = 1, KW = 1, stride = 1, pad = 0;
  // B operand (N rows x K), dense [N][ldb], K contiguous
  const float* B = nullptr;
  long long ldb = 0;
  int N = 0;
  // epilogue
  float* C = nullptr;
  long long ldc = 0;
  const float* bias = nullptr;
  const float* residual = nullptr;
  int relu = 0;  // epilogue activation: 0 none, 1 ReLU, 2 QuickGELU
  // filter epilogue (cosine top-k candidates): per B-row (query) threshold
  const float* tau = nullptr;
  unsigned long long* cand = nullptr;
  int* cnt = nullptr;
  long long cap = 0;
  long long row_offset = 0;  // added to the A row index in candidate keys
  // per-row dequantisation scales (fp8 inputs), applied to the accumulator
  const float* scale_a = nullptr;  // [M]
  const float* scale_b = nullptr;  // [N]
  int out_bf16 = 0;                // E_STORE: write bf16 instead of fp32
  // split-K (dense A, E_STORE): blockIdx.y = split s covers k in
  // [s*k_split, (s+1)*k_split) and stores its partial C at C + s*c_split_stride
  int k_split = 0;
  long long c_split_stride = 0;
  int sym = 0;  // E_STORE of a symmetric product: skip tiles strictly below the diagonal
  // split GEMM (gemm_s3.hip): B = three bf16 planes (SP 3) or two fp16 planes
  // (SP 2), b_plane elements apart
  long long b_plane = 0;
  // f16x2 split (SP 2): B row n was split at scale 2^e_n, col_scale[n] = 2^-e_n;
  // A's max |x| is read from a_amax (RR_AMAX_SLOTS words); the epilogue
  // publishes max |C| to c_amax when it is set
  const float* col_scale = nullptr;
  const uint32_t* a_amax = nullptr;
  uint32_t* c_amax = nullptr;
  // round stagger: of the first stagger_blocks blocks (one full round of
  // resident blocks), every other XCD-slot one sleeps stagger_sleeps x ~2k
  // cycles before starting, so later rounds run half the CUs out of phase
  int stagger_blocks = 0, stagger_sleeps = 0;
  // two-segment dense A (gemm_s3p_kernel SEG2; the stage-entry bottleneck's
  // conv3 and downsample projection as one GEMM over K = K1 + K2): k < K1
  // reads row m of A (lda); k >= K1 reads channel k - K1 of A2 at the pixel
  // output pixel m (of the OH x OW map) samples at stride s2 from the H2 x W2
  // NHWC map A2 (lda2 channels); a2_amax: A2's max-|x| record
  const float* A2 = nullptr;
  long long lda2 = 0;
  int K1 = 0, H2 = 0, W2 = 0, s2 = 1;
  const uint32_t* a2_amax = nullptr;
  // stem conv + 3x3/2 pad-1 max-pool (gemm_s3_kernel POOL; rr_stem_pool_h2):
  // tile t = (image, pr, pc) covers the 17 x 15 conv outputs from
  // (16 pr - 1, 14 pc - 1), whose windows give pooled rows 8 pr .. +7 and
  // columns 7 pc .. +6 of the POH x POW pooled map pool_out (NHWC, N channels)
  float* pool_out = nullptr;
  int POH = 0, POW = 0, pool_tr = 0, pool_tc = 0;
  // ViT LayerNorm fold (bf16 stored-C GEMMs, 256-column tiles):
  //  stats_out: also write bf16(C) to c2 ([M][ldc]) and, per row and 256-column
  //   tile t, the LayerNorm partials (mean_t, M2_t) of C to stats_out[M][T][2];
  //  stats_in: A holds bf16 rows of a LayerNorm input with those partials
  //   (T = ceil(stats_k / 256)); C = rstd (A.B^T - mean colsum) + bias
  uint16_t* c2 = nullptr;
  float* stats_out = nullptr;
  const float* stats_in = nullptr;
  const float* colsum = nullptr;
  int stats_k = 0;
  float ln_eps = 0.f;
  // the 256x320 bf16 filter sweep's 16x16x32 MFMA form (gemm_kernel MF16 = 2)
  int mf16_sweep = 0;
  int issue_spread = 0;
  int halo_mf = -1;
  int halo_2d = -1;
};

// 64-lane sum, returned wave-uniform: DPP row_shr 1/2/4/8 sums each 16-lane
// row into its lane 15 (out-of-row sources read 0), then the four rows'
// lanes 15, 31, 47, 63 are added in that order.  VALU-only (no LDS
// crossbar), and the same order on every call.
__device__ __forceinline__ float wave_sum(float x) {
  auto shr = [](float v, auto ctrl) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), decltype(ctrl)::value, 0xf, 0xf, true));
  };
  x += shr(x, std::integral_constant<int, 0x111>{});  // row_shr:1
  x += shr(x, std::integral_constant<int, 0x112>{});  // row_shr:2
  x += shr(x, std::integral_constant<int, 0x114>{});  // row_shr:4
  x += shr(x, std::integral_constant<int, 0x118>{});  // row_shr:8
  const int xi = __float_as_int(x);
  return (__int_as_float(__builtin_amdgcn_readlane(xi, 15)) + __int_as_float(__builtin_amdgcn_readlane(xi, 31))) +
         (__int_as_float(__builtin_amdgcn_readlane(xi, 47)) + __int_as_float(__builtin_amdgcn_readlane(xi, 63)));
}

// Block -> (tm, tn) of a tiles_m x tiles_n grid, the bijective XCD remap:
// blocks b, b + 8, ... share an XCD (dispatch is round-robin over the 8 XCDs;
// used for speed only, never for correctness), and each XCD gets a contiguous
// range of tile ids, tn fastest (an XCD sweeps its rows against every panel).
// (Round 4 measured panel-grouped orders on the filter sweeps: +-1 %, not kept,
// profiles/r04b_sweep_order_ab.txt.)
__device__ __forceinline__ void tile_coords(int bid, int nwg, int tiles_n, int& tm, int& tn) {
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  tn = wgid % tiles_n;
  tm = wgid / tiles_n;
}

int launch_gemm(rr_handle_s* h, int amode, int emode, const GemmArgs& a, hipStream_t s, int timer_cls,
                int dt = DT_F32);

// fp32-accurate GEMM on the 16-bit matrix cores (gemm_s3.hip): A fp32
// (A_DENSE, A_CONV or A_CONV_C4), E_STORE epilogue; sp must be 2: B = fp16
// planes [2][N][ldb] + col_scale from launch_split2h, A scaled by its a_amax
int launch_gemm_s3(rr_handle_s* h, int amode, const GemmArgs& g, hipStream_t s, int timer_cls, int sp = 2);
// f16x2 two-segment GEMM (GemmArgs A2 / K1): the persistent tile, N % 256 == 0
int launch_gemm_h2_seg2(rr_handle_s* h, const GemmArgs& g, hipStream_t s, int timer_cls);
// f16x2 NHWC4 stem conv + ReLU + 3x3/2 pad-1 max-pool (GemmArgs pool_*), N == 64
int launch_stem_pool_h2(rr_handle_s* h, const GemmArgs& g, hipStream_t s, int timer_cls);
// fp16 2-way split of the rows of w [rows][k] into planes [2][rows][kpad]
// (zero-padded) at a per-row power-of-two scale, iscale[row] = its inverse
int launch_split2h(rr_handle_s* h, const float* w, int rows, int k, int kpad, uint16_t* planes, float* iscale,
                   hipStream_t s);
// max |x| over x[n] into the RR_AMAX_SLOTS words at slots (atomic max)
int launch_amax(rr_handle_s* h, const float* x, long long n, uint32_t* slots, hipStream_t s);

// 256x256 8-phase pipeline (gemm_8p.hip), bf16 or fp8 (16x16x128 block-scaled
// MFMA): dense A/B, K a multiple of two k-tiles
bool gemm_8p_eligible(const GemmArgs& g, int dt);
hipError_t launch_gemm_8p(const GemmArgs& g, int emode, hipStream_t s, int dt);

// ---- top-k kernels (topk.hip) -------------------------------------------
// Dense scores, query-major [nq][ld] (first `rows` valid) -> per query the
// top-min(k,rows) keys written to cand[q][0..), cnt[q], tau[q].
int launch_select_dense_seed(rr_handle_s* h, const float* scores_t, long long ld, int rows, int nq,
                             int k, long long row_offset, unsigned long long* cand, long long cap,
                             int* cnt, float* tau, hipStream_t s);
// candidates cand[q][0..cnt[q]) -> sorted top-k (scores, idx + idx_offset)
int launch_select_final(rr_handle_s* h, const unsigned long long* cand, long long cap,
                        const int* cnt, int nq, int k, long long idx_offset, float* out_scores,
                        long long* out_idx, int* overflow_flag, hipStream_t s);
// exact bf16-bound prefilter, pass 2: clear keys that cannot reach the exact
// top-k, rescore the others with the fp32 MFMA core's exact fmaf chain
int launch_prefilter_rescore(rr_handle_s* h, unsigned long long* cand, long long cap, const int* cnt, int nq, int k,
                             const float* eps2, float* t2, const float* q, const float* g, int d, hipStream_t s);
int launch_merge(rr_handle_s* h, const float* ps, const long long* pi, int nparts, int nq, int kin,
                 int kout, float* os, long long* oi, hipStream_t s);

// sweep16.hip: the bf16 filter sweep on 16x16x32 MFMA with a hand-placed
// k-loop (256 gallery rows x 320 queries per block, 8 waves); rows128: LDS
// rows of 128 B (K % 64 == 0; else 64-B rows)
bool sweep16_eligible(const GemmArgs& g);
hipError_t launch_sweep16(const GemmArgs& g, hipStream_t s, int rows128);

// gemm_lpp.hip: the bf16 stored-C GEMM as a persistent 256x256 k-stream
bool lpp_eligible(const GemmArgs& g);
hipError_t launch_lpp(const GemmArgs& g, hipStream_t s, int n_cu);
bool lpp3_eligible(const GemmArgs& g);
hipError_t launch_lpp3(const GemmArgs& g, hipStream_t s, int n_cu);

}  // namespace rr
