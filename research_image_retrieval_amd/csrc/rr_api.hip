// rr_api.hip — C-ABI entry points of librr (see include/rr.h).
#include <algorithm>
#include <cstring>
#include <initializer_list>

#include "gemm_epilogue.hpp"
#include "rr_internal.hpp"

namespace rr {

int set_error(rr_handle_s* h, int code, const std::string& msg) {
  if (h) h->last_error = msg;
  return code;
}

int check_hip(rr_handle_s* h, hipError_t e, const char* what) {
  if (e == hipSuccess) return RR_OK;
  return set_error(h, RR_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}

TimedLaunch::TimedLaunch(rr_handle_s* h_, int cls_, hipStream_t s_) : h(h_), cls(cls_), s(s_) {
  if (!h || !h->timing || cls < 0 || cls >= rr_handle_s::kClasses) return;
  const int i = h->n_ev[cls];
  if (i >= (int)h->ev_start[cls].size()) {
    hipEvent_t a = nullptr, b = nullptr;
    if (hipEventCreate(&a) != hipSuccess) return;
    if (hipEventCreate(&b) != hipSuccess) {
      (void)hipEventDestroy(a);
      return;
    }
    h->ev_start[cls].push_back(a);
    h->ev_stop[cls].push_back(b);
  }
  if (hipEventRecord(h->ev_start[cls][i], s) != hipSuccess) return;
  slot = i;
}

TimedLaunch::~TimedLaunch() {
  if (slot < 0) return;
  if (hipEventRecord(h->ev_stop[cls][slot], s) == hipSuccess) h->n_ev[cls] = slot + 1;
}

// Sample size of the threshold-seeding pass of rr_cosine_topk.
static long long seed_rows(long long n, int k) { return seed_sample_rows(n, k); }

static inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

struct TopkWs {
  long long s, ld, cap;
  size_t off_scores, off_tau, off_cnt, off_ovf, off_cand, total;
};

static TopkWs topk_layout(int nq, long long n, int k, long long cap = -1) {
  TopkWs w{};
  w.s = seed_rows(n, k);
  w.ld = (w.s + 3) & ~3LL;
  w.cap = k + (n - w.s);  // worst case: every non-seed row passes its threshold
  if (cap >= 0 && cap < w.cap) w.cap = cap;  // bounded candidate buffer (rr.h)
  size_t o = 0;
  w.off_scores = o;
  o = align256(o + (size_t)nq * w.ld * 4);
  w.off_tau = o;
  o = align256(o + (size_t)nq * 4);
  w.off_cnt = o;
  o = align256(o + (size_t)nq * 4);
  w.off_ovf = o;
  o = align256(o + 4);
  w.off_cand = o;
  o = align256(o + (size_t)nq * w.cap * 8);
  w.total = o;
  return w;
}

}  // namespace rr

using namespace rr;

extern "C" {

const char* rr_version(void) { return "librr 0.4.0 (gfx950: fp32 / f16x2 / bf16 / fp8 MFMA)"; }

int rr_abi_version(void) { return RR_ABI_VERSION; }

int rr_create(int device, rr_handle_t* out) {
  if (!out) return RR_EINVAL;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return RR_EHIP;
  rr_handle_s* h = new (std::nothrow) rr_handle_s();
  if (!h) return RR_EINVAL;
  h->device = device;
  *out = h;
  return RR_OK;
}

int rr_destroy(rr_handle_t h) {
  RR_ENTRY(h);
  for (int c = 0; c < rr_handle_s::kClasses; ++c)
    for (size_t i = 0; i < h->ev_start[c].size(); ++i) {
      (void)hipEventDestroy(h->ev_start[c][i]);
      (void)hipEventDestroy(h->ev_stop[c][i]);
    }
  delete h;
  return RR_OK;
}

const char* rr_last_error(rr_handle_t h) { return h ? h->last_error.c_str() : "null handle"; }

int rr_timing_enable(rr_handle_t h, int enable) {
  RR_ENTRY(h);
  h->timing = enable != 0;
  for (int c = 0; c < rr_handle_s::kClasses; ++c) {
    h->n_ev[c] = 0;
    h->acc_ms[c] = 0;
    h->acc_launches[c] = 0;
  }
  return RR_OK;
}

int rr_get_device(rr_handle_t h, int* device) {
  if (!h || !device) return RR_EINVAL;
  *device = h->device;
  return RR_OK;
}

int rr_set_tuning(rr_handle_t h, int key, int value) {
  if (!h) return RR_EINVAL;
  auto in = [&](std::initializer_list<int> ok) {
    for (int v : ok)
      if (v == value) return true;
    return false;
  };
  switch (key) {
    case RR_TUNE_GEMM_CFG:
      if (!in({0, 22, 41, 88})) break;
      h->tune.gemm_cfg = value;
      return RR_OK;
    case RR_TUNE_GEMM_BK:
      if (!in({0, 16, 32})) break;
      h->tune.gemm_bk = value;
      return RR_OK;
    case RR_TUNE_LP_CFG:
      if (value < 0 || value > 6) break;
      h->tune.lp_cfg = value;
      return RR_OK;
    case RR_TUNE_S3_CFG:
      if (value < 0 || value > 15) break;
      h->tune.s3_cfg = value;
      return RR_OK;
    case RR_TUNE_S3_STAGGER:
      if (value < -1 || value > 200) break;
      h->tune.s3_stagger = value;
      return RR_OK;
    case RR_TUNE_SWEEP_MF16:
      if (!in({-1, 0, 1})) break;
      h->tune.sweep_mf16 = value;
      return RR_OK;
    case RR_TUNE_SWEEP_IL:
      if (!in({-1, 0, 1})) break;
      h->tune.sweep_il = value;
      return RR_OK;
    case RR_TUNE_CONV_IL:
      if (!in({-1, 0, 1})) break;
      h->tune.conv_il = value;
      return RR_OK;
    case RR_TUNE_HALO_MF:
      if (!in({-1, 0, 1, 2, 3, 4})) break;
      h->tune.halo_mf = value;
      return RR_OK;
    case RR_TUNE_S3_CFG_RES:
      if (value < 0 || value > 15) break;
      h->tune.s3_cfg_res = value;
      return RR_OK;
    case RR_TUNE_SWEEP_FORM:
      if (!in({-1, 0, 1, 2})) break;
      h->tune.sweep_form = value;
      return RR_OK;
    case RR_TUNE_HALO_2D:
      if (!in({-1, 0, 1})) break;
      h->tune.halo_2d = value;
      return RR_OK;
    default:
      return set_error(h, RR_EINVAL, "rr_set_tuning: unknown key");
  }
  return set_error(h, RR_EINVAL, "rr_set_tuning: value out of range for this key");
}

int rr_timing_collect(rr_handle_t h, int cls, double* ms, long long* launches) {
  if (!h || cls < 0 || cls >= rr_handle_s::kClasses) return RR_EINVAL;
  DeviceGuard dg(h);
  for (int i = 0; i < h->n_ev[cls]; ++i) {
    if (int rc = check_hip(h, hipEventSynchronize(h->ev_stop[cls][i]), "timing sync")) return rc;
    float t = 0.f;
    if (int rc = check_hip(h, hipEventElapsedTime(&t, h->ev_start[cls][i], h->ev_stop[cls][i]), "timing elapsed"))
      return rc;
    h->acc_ms[cls] += t;
    h->acc_launches[cls] += 1;
  }
  h->n_ev[cls] = 0;
  if (ms) *ms = h->acc_ms[cls];
  if (launches) *launches = h->acc_launches[cls];
  h->acc_ms[cls] = 0;
  h->acc_launches[cls] = 0;
  return RR_OK;
}

size_t rr_cosine_topk_workspace_size(int nq, long long n, int d, int k) {
  (void)d;
  if (nq <= 0 || k <= 0) return 256;
  return topk_layout(nq, n > 0 ? n : 1, k).total;
}

size_t rr_cosine_topk_workspace_size_cap(int nq, long long n, int d, int k, long long cap) {
  (void)d;
  if (nq <= 0 || k <= 0 || cap < k) return 0;
  return topk_layout(nq, n > 0 ? n : 1, k, cap).total;
}

long long rr_cosine_topk_cap_for(int nq, long long n, int d, int k, size_t workspace_bytes) {
  (void)d;
  if (nq <= 0 || k <= 0) return 0;
  const TopkWs L = topk_layout(nq, n > 0 ? n : 1, k);
  return workspace_bytes >= L.total ? L.cap : cap_that_fits(L.off_cand, nq, workspace_bytes, L.cap);
}

size_t rr_cosine_topk_counts_offset(int nq, long long n, int d, int k) {
  (void)d;
  if (nq <= 0 || k <= 0) return 0;
  return topk_layout(nq, n > 0 ? n : 1, k).off_cnt;
}

size_t rr_cosine_topk_overflow_offset(int nq, long long n, int d, int k) {
  (void)d;
  if (nq <= 0 || k <= 0) return 0;
  return topk_layout(nq, n > 0 ? n : 1, k).off_ovf;
}

}  // extern "C"

namespace rr {
// Fused top-k over a gallery of any GEMM input dtype (fp32 / bf16 / fp8 with
// per-row scales); see rr_cosine_topk for the algorithm.
static int cosine_topk_impl(rr_handle_t h, const void* queries, const float* q_scale, int nq, const void* gallery,
                            const float* g_scale, long long n, int d, int k, long long idx_offset, float* out_scores,
                            long long* out_idx, void* workspace, size_t workspace_bytes, hipStream_t s, int dt) {
  if (nq < 0 || n < 0 || d <= 0 || (d & 3) || k < 1 || k > 16384)
    return set_error(h, RR_EINVAL, "rr_cosine_topk: need nq,n >= 0, d % 4 == 0, 1 <= k <= 16384");
  if (n >= 0xffffffffLL) return set_error(h, RR_EINVAL, "rr_cosine_topk: gallery shard must have < 2^32 rows");
  if (nq == 0) return RR_OK;
  if (!queries || !out_scores || !out_idx || (n > 0 && !gallery))
    return set_error(h, RR_EINVAL, "rr_cosine_topk: null pointer");
  if (((uintptr_t)queries & 15) || ((uintptr_t)gallery & 15))
    return set_error(h, RR_EINVAL, "rr_cosine_topk: queries/gallery must be 16-byte aligned");
  const int es = dt == DT_F32 ? 4 : (dt == DT_BF16 ? 2 : 1);
  TopkWs L = topk_layout(nq, n > 0 ? n : 1, k);
  if (workspace && workspace_bytes < L.total) {  // bounded candidate buffer
    const long long cap = cap_that_fits(L.off_cand, nq, workspace_bytes, L.cap);
    if (cap >= k) L = topk_layout(nq, n > 0 ? n : 1, k, cap);
  }
  if (!workspace || workspace_bytes < L.total)
    return set_error(h, RR_EWORKSPACE,
                     "rr_cosine_topk: workspace too small (at least rr_cosine_topk_workspace_size_cap(..., k))");
  char* ws = (char*)workspace;
  float* scores_t = (float*)(ws + L.off_scores);
  float* tau = (float*)(ws + L.off_tau);
  int* cnt = (int*)(ws + L.off_cnt);
  int* ovf = (int*)(ws + L.off_ovf);
  unsigned long long* cand = (unsigned long long*)(ws + L.off_cand);
  // the overflow count is zeroed on every call (rr.h), the empty gallery included
  if (int rc = check_hip(h, hipMemsetAsync(ovf, 0, 4, s), "memset")) return rc;
  if (n == 0) {  // nothing to rank: all padding
    if (int rc = check_hip(h, hipMemsetAsync(cnt, 0, (size_t)nq * 4, s), "memset")) return rc;
    return launch_select_final(h, cand, L.cap, cnt, nq, k, idx_offset, out_scores, out_idx, ovf, s);
  }
  // 1. exact scores of the first s gallery rows (query-major)
  GemmArgs g;
  g.A = (const float*)gallery;
  g.lda = d;
  g.M = (int)L.s;
  g.K = d;
  g.B = (const float*)queries;
  g.ldb = d;
  g.N = nq;
  g.C = scores_t;
  g.ldc = L.ld;
  g.scale_a = g_scale;
  g.scale_b = q_scale;
  if (int rc = launch_gemm(h, A_DENSE, E_SCORES_T, g, s, kTimeCosineSeed, dt)) return rc;
  // 2. seed candidates with their exact top-k; tau = k-th best score
  if (int rc = launch_select_dense_seed(h, scores_t, L.ld, (int)L.s, nq, k, 0, cand, L.cap, cnt, tau, s)) return rc;
  // 3. remaining rows: fused GEMM + threshold filter (scores never hit HBM)
  long long done = L.s;
  while (done < n) {
    const long long rows = std::min<long long>(n - done, 0x7fffff00LL);
    GemmArgs f;
    f.A = (const float*)((const char*)gallery + done * d * es);
    f.lda = d;
    f.M = (int)rows;
    f.K = d;
    f.B = (const float*)queries;
    f.ldb = d;
    f.N = nq;
    f.tau = tau;
    f.cand = cand;
    f.cnt = cnt;
    f.cap = L.cap;
    f.row_offset = done;
    f.scale_a = g_scale ? g_scale + done : nullptr;
    f.scale_b = q_scale;
    if (int rc = launch_gemm(h, A_DENSE, E_FILTER, f, s, kTimeCosine, dt)) return rc;
    done += rows;
  }
  // 4. exact top-k of the survivors, stable order
  return launch_select_final(h, cand, L.cap, cnt, nq, k, idx_offset, out_scores, out_idx, ovf, s);
}
}  // namespace rr

extern "C" {

int rr_cosine_topk(rr_handle_t h, const float* queries, int nq, const float* gallery, long long n, int d, int k,
                   long long idx_offset, float* out_scores, long long* out_idx, void* workspace,
                   size_t workspace_bytes, void* stream) {
  RR_ENTRY(h);
  return cosine_topk_impl(h, queries, nullptr, nq, gallery, nullptr, n, d, k, idx_offset, out_scores, out_idx,
                          workspace, workspace_bytes, (hipStream_t)stream, DT_F32);
}

int rr_cosine_topk_lp(rr_handle_t h, const void* queries, const float* q_scale, int nq, const void* gallery,
                      const float* g_scale, long long n, int d, int dtype, int k, long long idx_offset,
                      float* out_scores, long long* out_idx, void* workspace, size_t workspace_bytes,
                      void* stream) {
  RR_ENTRY(h);
  if (dtype != DT_BF16 && dtype != DT_FP8) return set_error(h, RR_EINVAL, "rr_cosine_topk_lp: dtype must be 1 or 2");
  if (dtype == DT_FP8 && (!q_scale || !g_scale))
    return set_error(h, RR_EINVAL, "rr_cosine_topk_lp: fp8 needs per-row scales");
  if ((d % (dtype == DT_BF16 ? 8 : 16)) != 0)
    return set_error(h, RR_EINVAL, "rr_cosine_topk_lp: rows must be multiples of 16 bytes");
  return cosine_topk_impl(h, queries, q_scale, nq, gallery, g_scale, n, d, k, idx_offset, out_scores, out_idx,
                          workspace, workspace_bytes, (hipStream_t)stream, dtype);
}

int rr_linear_bf16(rr_handle_t h, const void* x, int m, int k, const void* w, const float* bias, int n,
                   const float* residual, int act, int out_bf16, void* y, void* stream) {
  RR_ENTRY(h);
  if (!x || !w || !y || m < 0 || k <= 0 || n <= 0 || (k & 7) || act < 0 || act > 2)
    return set_error(h, RR_EINVAL, "rr_linear_bf16: bad argument (k % 8 == 0)");
  if (((uintptr_t)x & 15) || ((uintptr_t)w & 15)) return set_error(h, RR_EINVAL, "rr_linear_bf16: 16-B alignment");
  GemmArgs g;
  g.A = (const float*)x;
  g.lda = k;
  g.M = m;
  g.K = k;
  g.B = (const float*)w;
  g.ldb = k;
  g.N = n;
  g.C = (float*)y;
  g.ldc = n;
  g.bias = bias;
  g.residual = residual;
  g.relu = act;
  g.out_bf16 = out_bf16 ? 1 : 0;
  return launch_gemm(h, A_DENSE, E_STORE, g, (hipStream_t)stream, kTimeGemm, DT_BF16);
}

int rr_linear_bf16_ln(rr_handle_t h, const void* x, int m, int k, const void* w, const float* bias, int n,
                      const float* residual, int act, int out_bf16, void* y, const float* stats_in,
                      const float* colsum, float eps, float* stats_out, void* xb_out, void* stream) {
  RR_ENTRY(h);
  if (!x || !w || !y || m < 0 || k <= 0 || n <= 0 || (k & 7) || act < 0 || act > 2)
    return set_error(h, RR_EINVAL, "rr_linear_bf16_ln: bad argument (k % 8 == 0)");
  if (((uintptr_t)x & 15) || ((uintptr_t)w & 15) || ((uintptr_t)y & 15) || (bias && ((uintptr_t)bias & 15)) ||
      (residual && ((uintptr_t)residual & 15)))
    return set_error(h, RR_EINVAL, "rr_linear_bf16_ln: 16-B alignment");
  if ((stats_in == nullptr) == (stats_out == nullptr))
    return set_error(h, RR_EINVAL, "rr_linear_bf16_ln: exactly one of stats_in (fold) and stats_out (produce)");
  if (stats_out) {
    // the producer: the residual GEMM (fp32 output) writing the bf16 copy and the partials
    // (k % 64: the 256x256 tile with the partials epilogue stages whole 64-deep k-tiles)
    if (!xb_out || !residual || !bias || act != 0 || out_bf16 || (n % 256) || (k % 64) || ((uintptr_t)xb_out & 15) ||
        ((uintptr_t)stats_out & 7))
      return set_error(h, RR_EINVAL,
                       "rr_linear_bf16_ln: stats_out needs bias, residual, fp32 output, n % 256 == 0, k % 64 == 0");
  } else {
    // the consumer: bias, bf16 output, K in whole 64-deep k-tiles, at most
    // three 256-column LayerNorm tiles (LN_TMAX)
    if (!colsum || !bias || residual || !out_bf16 || (k % 64) || k > 256 * LN_TMAX || (n & 3) ||
        ((uintptr_t)colsum & 15) || !(eps >= 0.f))
      return set_error(h, RR_EINVAL,
                       "rr_linear_bf16_ln: stats_in needs colsum, bias, bf16 output, k % 64 == 0, k <= 768");
  }
  if (m == 0) return RR_OK;
  GemmArgs g;
  g.A = (const float*)x;
  g.lda = k;
  g.M = m;
  g.K = k;
  g.B = (const float*)w;
  g.ldb = k;
  g.N = n;
  g.C = (float*)y;
  g.ldc = n;
  g.bias = bias;
  g.residual = residual;
  g.relu = act;
  g.out_bf16 = out_bf16 ? 1 : 0;
  g.stats_out = stats_out;
  g.c2 = (uint16_t*)xb_out;
  g.stats_in = stats_in;
  g.colsum = colsum;
  g.stats_k = k;
  g.ln_eps = eps;
  return launch_gemm(h, A_DENSE, E_STORE, g, (hipStream_t)stream, kTimeGemm, DT_BF16);
}

int rr_cosine_scores(rr_handle_t h, const float* queries, int nq, const float* gallery, long long n, int d,
                     float* scores, void* stream) {
  RR_ENTRY(h);
  if (nq < 0 || n < 0 || n > 0x7fffffffLL || d <= 0 || (d & 3))
    return set_error(h, RR_EINVAL, "rr_cosine_scores: bad shape");
  if (nq == 0 || n == 0) return RR_OK;
  if (!queries || !gallery || !scores) return set_error(h, RR_EINVAL, "rr_cosine_scores: null pointer");
  GemmArgs g;
  g.A = gallery;
  g.lda = d;
  g.M = (int)n;
  g.K = d;
  g.B = queries;
  g.ldb = d;
  g.N = nq;
  g.C = scores;
  g.ldc = nq;
  return launch_gemm(h, A_DENSE, E_STORE, g, (hipStream_t)stream, kTimeCosineSeed);
}

int rr_topk_merge(rr_handle_t h, const float* ps, const long long* pi, int nparts, int nq, int k_in, int k_out,
                  float* os, long long* oi, void* stream) {
  RR_ENTRY(h);
  if (!ps || !pi || !os || !oi) return set_error(h, RR_EINVAL, "rr_topk_merge: null pointer");
  return launch_merge(h, ps, pi, nparts, nq, k_in, k_out, os, oi, (hipStream_t)stream);
}

int rr_conv2d(rr_handle_t h, const float* x, int b, int hgt, int wid, int cin, const float* w, const float* bias,
              int cout, int kh, int kw, int stride, int pad, const float* residual, int relu, float* y,
              void* stream) {
  RR_ENTRY(h);
  if (!x || !w || !y || b < 0 || hgt <= 0 || wid <= 0 || cin <= 0 || cout <= 0 || kh <= 0 || kw <= 0 ||
      stride <= 0 || pad < 0)
    return set_error(h, RR_EINVAL, "rr_conv2d: bad argument");
  const int oh = (hgt + 2 * pad - kh) / stride + 1, ow = (wid + 2 * pad - kw) / stride + 1;
  if (oh <= 0 || ow <= 0) return set_error(h, RR_EINVAL, "rr_conv2d: empty output");
  const long long M = (long long)b * oh * ow;
  if (M > 0x7fffffffLL) return set_error(h, RR_EINVAL, "rr_conv2d: too many output pixels");
  GemmArgs g;
  g.A = x;
  g.M = (int)M;
  g.K = kh * kw * cin;
  g.H = hgt;
  g.W = wid;
  g.Cin = cin;
  g.OH = oh;
  g.OW = ow;
  g.KH = kh;
  g.KW = kw;
  g.stride = stride;
  g.pad = pad;
  g.B = w;
  g.ldb = g.K;
  g.N = cout;
  g.C = y;
  g.ldc = cout;
  g.bias = bias;
  g.residual = residual;
  g.relu = relu;
  int amode;
  if (kh == 1 && kw == 1 && stride == 1 && pad == 0 && (cin & 3) == 0) {
    amode = A_DENSE;
    g.lda = cin;
  } else if (cin % 32 == 0) {
    amode = A_CONV;
  } else if (cin == 4) {
    amode = A_CONV_C4;
  } else {
    amode = A_CONV_GENERIC;
  }
  if (amode != A_CONV_GENERIC && (((uintptr_t)x & 15) || ((uintptr_t)w & 15)))
    return set_error(h, RR_EINVAL, "rr_conv2d: x/w must be 16-byte aligned");
  // cout % 4 == 0: the epilogue's vector path (f32x4 bias, 16-byte C / residual rows)
  if ((cout & 3) == 0 && (((uintptr_t)y & 15) || (bias && ((uintptr_t)bias & 15)) || (residual && ((uintptr_t)residual & 15))))
    return set_error(h, RR_EINVAL, "rr_conv2d: bias/residual/y must be 16-byte aligned");
  return launch_gemm(h, amode, E_STORE, g, (hipStream_t)stream, kTimeGemm);
}

int rr_conv2d_h2(rr_handle_t h, const float* x, const unsigned* x_amax, int b, int hgt, int wid, int cin,
                 const void* w2, const float* w_iscale, const float* bias, int cout, int kh, int kw, int stride,
                 int pad, const float* residual, int relu, float* y, unsigned* y_amax, void* stream) {
  RR_ENTRY(h);
  if (!x || !x_amax || !w2 || !w_iscale || !y || b < 0 || hgt <= 0 || wid <= 0 || cin <= 0 || cout <= 0 ||
      kh <= 0 || kw <= 0 || stride <= 0 || pad < 0 || relu < 0 || relu > 1)
    return set_error(h, RR_EINVAL, "rr_conv2d_h2: bad argument");
  if (cin % 32 && cin != 4) return set_error(h, RR_EINVAL, "rr_conv2d_h2: cin must be a multiple of 32, or 4 (NHWC4 stem)");
  if (cout % 4) return set_error(h, RR_EINVAL, "rr_conv2d_h2: cout must be a multiple of 4");
  const int oh = (hgt + 2 * pad - kh) / stride + 1, ow = (wid + 2 * pad - kw) / stride + 1;
  if (oh <= 0 || ow <= 0) return set_error(h, RR_EINVAL, "rr_conv2d_h2: empty output");
  const long long M = (long long)b * oh * ow;
  if (M > 0x7fffffffLL) return set_error(h, RR_EINVAL, "rr_conv2d_h2: too many output pixels");
  // the epilogues load bias / col_scale as f32x4 and store C / read the
  // residual in 16-byte pieces
  if (((uintptr_t)x & 15) || ((uintptr_t)w2 & 15) || ((uintptr_t)w_iscale & 15) || ((uintptr_t)y & 15) ||
      (bias && ((uintptr_t)bias & 15)) || (residual && ((uintptr_t)residual & 15)))
    return set_error(h, RR_EINVAL, "rr_conv2d_h2: x/w2/w_iscale/bias/residual/y must be 16-byte aligned");
  GemmArgs g;
  g.A = x;
  g.M = (int)M;
  g.K = kh * kw * cin;
  g.H = hgt;
  g.W = wid;
  g.Cin = cin;
  g.OH = oh;
  g.OW = ow;
  g.KH = kh;
  g.KW = kw;
  g.stride = stride;
  g.pad = pad;
  if (cin == 4) g.K = (g.K + 31) / 32 * 32;  // NHWC4 stem: planes zero-padded to a multiple of 32
  g.B = reinterpret_cast<const float*>(w2);
  g.ldb = g.K;
  g.b_plane = (long long)cout * g.K;
  g.N = cout;
  g.C = y;
  g.ldc = cout;
  g.bias = bias;
  g.residual = residual;
  g.relu = relu;
  g.col_scale = w_iscale;
  g.a_amax = x_amax;
  g.c_amax = y_amax;
  const bool dense = kh == 1 && kw == 1 && stride == 1 && pad == 0 && cin != 4;
  if (dense) g.lda = cin;
  return launch_gemm_s3(h, dense ? A_DENSE : (cin == 4 ? A_CONV_C4 : A_CONV), g, (hipStream_t)stream, kTimeGemm, 2);
}

int rr_stem_pool_h2(rr_handle_t h, const float* x, const unsigned* x_amax, int b, int hgt, int wid, const void* w2,
                    const float* w_iscale, const float* bias, int cout, int kh, int kw, int stride, int pad,
                    float* y_pool, unsigned* y_amax, void* stream) {
  RR_ENTRY(h);
  if (!x || !x_amax || !w2 || !w_iscale || !y_pool || b < 0 || hgt <= 0 || wid <= 0 || kh <= 0 || kw <= 0 ||
      stride <= 0 || pad < 0)
    return set_error(h, RR_EINVAL, "rr_stem_pool_h2: bad argument");
  if (cout != 64) return set_error(h, RR_EINVAL, "rr_stem_pool_h2: cout must be 64");
  const int oh = (hgt + 2 * pad - kh) / stride + 1, ow = (wid + 2 * pad - kw) / stride + 1;
  if (oh <= 0 || ow <= 0) return set_error(h, RR_EINVAL, "rr_stem_pool_h2: empty output");
  const int ph = (oh - 1) / 2 + 1, pw = (ow - 1) / 2 + 1;  // 3x3 / 2, padding 1
  if ((long long)b * oh * ow > 0x7fffffffLL || (long long)b * ph * pw * cout > (1LL << 40))
    return set_error(h, RR_EINVAL, "rr_stem_pool_h2: too many output pixels");
  if (((uintptr_t)x & 15) || ((uintptr_t)w2 & 15) || ((uintptr_t)w_iscale & 15) || ((uintptr_t)y_pool & 15) ||
      (bias && ((uintptr_t)bias & 15)))
    return set_error(h, RR_EINVAL, "rr_stem_pool_h2: x/w2/w_iscale/bias/y_pool must be 16-byte aligned");
  GemmArgs g;
  g.A = x;
  g.M = (int)((long long)b * oh * ow);
  g.K = (kh * kw * 4 + 31) / 32 * 32;  // NHWC4 planes zero-padded to a multiple of 32
  g.H = hgt;
  g.W = wid;
  g.Cin = 4;
  g.OH = oh;
  g.OW = ow;
  g.KH = kh;
  g.KW = kw;
  g.stride = stride;
  g.pad = pad;
  g.B = reinterpret_cast<const float*>(w2);
  g.ldb = g.K;
  g.b_plane = (long long)cout * g.K;
  g.N = cout;
  g.ldc = cout;
  g.bias = bias;
  g.relu = 1;
  g.col_scale = w_iscale;
  g.a_amax = x_amax;
  g.c_amax = y_amax;
  g.pool_out = y_pool;
  g.POH = ph;
  g.POW = pw;
  g.pool_tr = (ph + 7) / 8;
  g.pool_tc = (pw + 6) / 7;
  return launch_stem_pool_h2(h, g, (hipStream_t)stream, kTimeGemm);
}

int rr_bottleneck_out_h2(rr_handle_t h, const float* y, const unsigned* y_amax, int b, int oh, int ow, int planes,
                         const float* x, const unsigned* x_amax, int hx, int wx, int cin, int stride, const void* w2,
                         const float* w_iscale, const float* bias, int cout, float* out, unsigned* out_amax,
                         void* stream) {
  RR_ENTRY(h);
  if (!y || !y_amax || !x || !x_amax || !w2 || !w_iscale || !out || b < 0 || oh <= 0 || ow <= 0 || planes <= 0 ||
      hx <= 0 || wx <= 0 || cin <= 0 || stride <= 0 || cout <= 0)
    return set_error(h, RR_EINVAL, "rr_bottleneck_out_h2: bad argument");
  if ((planes % 32) || (cin % 32) || (cout % 256))
    return set_error(h, RR_EINVAL, "rr_bottleneck_out_h2: planes % 32, cin % 32 and cout % 256 must be 0");
  if ((long long)(oh - 1) * stride >= hx || (long long)(ow - 1) * stride >= wx)
    return set_error(h, RR_EINVAL, "rr_bottleneck_out_h2: the strided samples leave x");
  const long long M = (long long)b * oh * ow;
  if (M > 0x7fffffffLL || (long long)b * hx * wx > 0x7fffffffLL)
    return set_error(h, RR_EINVAL, "rr_bottleneck_out_h2: too many pixels");
  if (((uintptr_t)y & 15) || ((uintptr_t)x & 15) || ((uintptr_t)w2 & 15) || ((uintptr_t)w_iscale & 15) ||
      ((uintptr_t)out & 15) || (bias && ((uintptr_t)bias & 15)))
    return set_error(h, RR_EINVAL, "rr_bottleneck_out_h2: y/x/w2/w_iscale/bias/out must be 16-byte aligned");
  GemmArgs g;
  g.A = y;
  g.lda = planes;
  g.M = (int)M;
  g.K = planes + cin;
  g.K1 = planes;
  g.A2 = x;
  g.lda2 = cin;
  g.H2 = hx;
  g.W2 = wx;
  g.s2 = stride;
  g.OH = oh;
  g.OW = ow;
  g.B = reinterpret_cast<const float*>(w2);
  g.ldb = g.K;
  g.b_plane = (long long)cout * g.K;
  g.N = cout;
  g.C = out;
  g.ldc = cout;
  g.bias = bias;
  g.relu = 1;
  g.col_scale = w_iscale;
  g.a_amax = y_amax;
  g.a2_amax = x_amax;
  g.c_amax = out_amax;
  return launch_gemm_h2_seg2(h, g, (hipStream_t)stream, kTimeGemm);
}

int rr_split2_f16(rr_handle_t h, const float* w, int rows, int k, int kpad, void* planes, float* iscale,
                  void* stream) {
  RR_ENTRY(h);
  if (!w || !planes || !iscale || rows < 0 || k <= 0 || kpad < k) return set_error(h, RR_EINVAL, "rr_split2_f16: bad argument");
  TimedLaunch tl(h, kTimeElem, (hipStream_t)stream);
  return launch_split2h(h, w, rows, k, kpad, reinterpret_cast<uint16_t*>(planes), iscale, (hipStream_t)stream);
}

int rr_amax_f32(rr_handle_t h, const float* x, long long n, unsigned* amax, void* stream) {
  RR_ENTRY(h);
  if (!x || !amax || n < 0) return set_error(h, RR_EINVAL, "rr_amax_f32: bad argument");
  TimedLaunch tl(h, kTimeElem, (hipStream_t)stream);
  return launch_amax(h, x, n, amax, (hipStream_t)stream);
}


int rr_linear(rr_handle_t h, const float* x, int m, int k, const float* w, const float* bias, int n, float* y,
              void* stream) {
  return rr_linear_ex(h, x, m, k, w, bias, n, nullptr, 0, y, stream);
}

int rr_linear_ex(rr_handle_t h, const float* x, int m, int k, const float* w, const float* bias, int n,
                 const float* residual, int act, float* y, void* stream) {
  RR_ENTRY(h);
  if (!x || !w || !y || m < 0 || k <= 0 || n <= 0 || (k & 3)) return set_error(h, RR_EINVAL, "rr_linear: bad argument");
  if (((uintptr_t)x & 15) || ((uintptr_t)w & 15)) return set_error(h, RR_EINVAL, "rr_linear: x/w must be 16-byte aligned");
  GemmArgs g;
  g.A = x;
  g.lda = k;
  g.M = m;
  g.K = k;
  g.B = w;
  g.ldb = k;
  g.N = n;
  g.C = y;
  g.ldc = n;
  g.bias = bias;
  g.residual = residual;
  if (act < 0 || act > 2) return set_error(h, RR_EINVAL, "rr_linear_ex: act must be 0, 1 or 2");
  g.relu = act;
  return launch_gemm(h, A_DENSE, E_STORE, g, (hipStream_t)stream, kTimeGemm);
}

}  // extern "C"
