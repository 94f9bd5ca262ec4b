// prefilter.hip — exact cosine top-k through a bf16 prefilter (gfx950).
//
// rr_cosine_topk_prefilter returns the SAME scores and indices, bit for bit,
// as rr_cosine_topk (the exhaustive fp32 ranker of iris_evaluate.py:383-386),
// while the full gallery sweep runs on the bf16 MFMA (16x the fp32 rate, half
// the bytes).  Only rows that can still be in the exact top-k are rescored in
// fp32, with the fp32 core's own fmaf chain.
//
// Bound.  For a query q and gallery row g (fp32), q^ = bf16(q), g^ = bf16(g),
// s = the fp32 chain score and s' = the bf16 MFMA score:
//   |s - s'| <= |s - q.g| + |q.g - q^.g^| + |q^.g^ - s'|
//            <= g_d |q||g| + |q - q^||g| + |q^||g - g^| + g'_d |q^||g^|
// (Cauchy-Schwarz for the middle term; g_d = d u / (1 - d u), u = 2^-24, for
// the fp32 chain; g'_d with u = 2^-23 for the bf16 MFMA accumulation, which
// covers any rounding mode of its fp32 adds; bf16 x bf16 products are exact
// in fp32).  With the gallery maxima G = max|g|, E = max|g - g^|,
// H = max|g^| (rr_prefilter_gallery_bound, once per gallery) this gives one
// eps(q) for all rows, computed in fp64 and rounded up.
//
// Passes (one query = one column of the GEMMs):
//   1. bf16 scores of the first s rows (seed_sample_rows: <= 32768); their k-th best s'_seed;
//      T1 = s'_seed - 2 eps.  At least k rows have s >= s'_seed - eps, so the
//      exact k-th best S_k >= s'_seed - eps and any row of the exact top-k
//      has s' >= S_k - eps >= T1.
//   2. bf16 GEMM over ALL rows with the filter epilogue keeping s' >= T1.
//   3. (topk.hip) s'_k = k-th best s' among the survivors (= over all rows),
//      T2 = s'_k - 2 eps >= T1 by the same argument; survivors with s' >= T2
//      are rescored exactly in place, the rest cleared.
//   4. select_final: stable exact top-k of the rescored keys.
// The rescored set contains the exact top-k, so the result equals the
// exhaustive one, ties included (a tie at S_k has s' >= S_k - eps).
#include <algorithm>

#include "rr_internal.hpp"

namespace rr {

__device__ inline float round_up_f(double x) {
  float f = (float)x;
  if ((double)f < x) f = next_up(f);
  return f;
}
__device__ inline float round_down_f(double x) {
  float f = (float)x;
  if ((double)f > x) f = next_down(f);
  return f;
}

__device__ inline double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// grid-stride, one wave per row: |g|, |g - g^|, |g^| in fp64; per-wave
// maxima, one atomic per wave (the bit order of non-negative doubles is their
// numeric order)
__global__ __launch_bounds__(256) void gallery_bound_kernel(const float* __restrict__ g,
                                                            const uint16_t* __restrict__ gb, long long n, int d,
                                                            unsigned long long* __restrict__ out3) {
  const int lane = threadIdx.x & 63;
  const long long waves = (long long)gridDim.x * (blockDim.x >> 6);
  double ma = 0.0, me = 0.0, mb = 0.0;
  for (long long row = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6; row < n; row += waves) {
    double a = 0.0, e = 0.0, b = 0.0;
    for (int i = lane; i < d; i += 64) {
      const double x = (double)g[row * d + i];
      const double y = (double)__builtin_bit_cast(float, (uint32_t)gb[row * d + i] << 16);
      a += x * x;
      e += (x - y) * (x - y);
      b += y * y;
    }
    ma = fmax(ma, wave_sum(a));
    me = fmax(me, wave_sum(e));
    mb = fmax(mb, wave_sum(b));
  }
  if (lane == 0) {
    atomicMax(out3 + 0, __builtin_bit_cast(unsigned long long, sqrt(ma)));
    atomicMax(out3 + 1, __builtin_bit_cast(unsigned long long, sqrt(me)));
    atomicMax(out3 + 2, __builtin_bit_cast(unsigned long long, sqrt(mb)));
  }
}

// one wave per query: eps2 = 2 * eps(q), rounded up
__global__ __launch_bounds__(256) void query_eps_kernel(const float* __restrict__ q, const uint16_t* __restrict__ qb,
                                                        int nq, int d, const double* __restrict__ bound3,
                                                        float* __restrict__ eps2) {
  const int row = (int)(((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= nq) return;
  double a = 0.0, e = 0.0, b = 0.0;
  for (int i = lane; i < d; i += 64) {
    const double x = (double)q[(long long)row * d + i];
    const double y = (double)__builtin_bit_cast(float, (uint32_t)qb[(long long)row * d + i] << 16);
    a += x * x;
    e += (x - y) * (x - y);
    b += y * y;
  }
  a = wave_sum(a);
  e = wave_sum(e);
  b = wave_sum(b);
  if (lane == 0) {
    const double G = bound3[0], E = bound3[1], H = bound3[2];
    const double u32 = 0x1p-24, u23 = 0x1p-23;
    const double gd = d * u32 / (1.0 - d * u32), gbd = d * u23 / (1.0 - d * u23);
    const double eps = sqrt(e) * G + sqrt(b) * E + gd * sqrt(a) * G + gbd * sqrt(b) * H;
    eps2[row] = round_up_f(2.0 * eps * (1.0 + 1e-6) + 1e-12);
  }
}

// pass-1 threshold: keep s' >= tau - eps2 (the filter epilogue is strict `>`)
__global__ void pass1_tau_kernel(float* __restrict__ tau, const float* __restrict__ eps2, int* __restrict__ cnt,
                                 int nq) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nq) return;
  const float t = tau[i];
  if (t == -__builtin_inff()) {
    tau[i] = t;
  } else {
    tau[i] = next_down(round_down_f((double)t - (double)eps2[i]));
  }
  cnt[i] = 0;
}

struct PrefilterWs {
  long long s, ld, cap;
  size_t off_scores, off_tau, off_cnt, off_ovf, off_eps, off_qb, off_cand, total;
};

static inline size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

static PrefilterWs prefilter_layout(int nq, long long n, int d, int k, long long cap = -1) {
  PrefilterWs w{};
  w.s = seed_sample_rows(n, k);
  w.ld = (w.s + 3) & ~3LL;
  w.cap = std::max<long long>(n, k);  // worst case: every row passes pass 1
  if (cap >= 0 && cap < w.cap) w.cap = cap;  // bounded candidate buffer (rr.h)
  size_t o = 0;
  w.off_scores = o;
  o = al256(o + (size_t)nq * w.ld * 4);
  w.off_tau = o;
  o = al256(o + (size_t)nq * 4);
  w.off_cnt = o;
  o = al256(o + (size_t)nq * 4);
  w.off_ovf = o;
  o = al256(o + 4);
  w.off_eps = o;
  o = al256(o + (size_t)nq * 4);
  w.off_qb = o;
  o = al256(o + (size_t)nq * d * 2);
  w.off_cand = o;
  o = al256(o + (size_t)nq * w.cap * 8);
  w.total = o;
  return w;
}

}  // namespace rr

using namespace rr;

extern "C" {

int rr_prefilter_gallery_bound(rr_handle_t h, const float* gallery, const void* gallery_bf16, long long n, int d,
                               double* bound3, void* stream) {
  RR_ENTRY(h);
  if (n < 0 || d <= 0 || !bound3 || (n > 0 && (!gallery || !gallery_bf16)))
    return set_error(h, RR_EINVAL, "rr_prefilter_gallery_bound: bad argument");
  hipStream_t s = (hipStream_t)stream;
  if (int rc = check_hip(h, hipMemsetAsync(bound3, 0, 3 * sizeof(double), s), "memset")) return rc;
  if (n == 0) return RR_OK;
  TimedLaunch tl(h, kTimeElem, s);
  const long long blocks = std::min<long long>((n + 3) / 4, 4096);
  hipLaunchKernelGGL(gallery_bound_kernel, dim3((unsigned)blocks), dim3(256), 0, s, gallery,
                     (const uint16_t*)gallery_bf16, n, d, (unsigned long long*)bound3);
  return check_hip(h, hipGetLastError(), "gallery bound launch");
}

size_t rr_cosine_topk_prefilter_workspace_size(int nq, long long n, int d, int k) {
  if (nq < 0 || n < 0 || d <= 0 || k < 1) return 0;
  return prefilter_layout(nq, n > 0 ? n : 1, d, k).total;
}

size_t rr_cosine_topk_prefilter_counts_offset(int nq, long long n, int d, int k) {
  if (nq < 0 || n < 0 || d <= 0 || k < 1) return 0;
  return prefilter_layout(nq, n > 0 ? n : 1, d, k).off_cnt;
}

size_t rr_cosine_topk_prefilter_overflow_offset(int nq, long long n, int d, int k) {
  if (nq < 0 || n < 0 || d <= 0 || k < 1) return 0;
  return prefilter_layout(nq, n > 0 ? n : 1, d, k).off_ovf;
}

size_t rr_cosine_topk_prefilter_workspace_size_cap(int nq, long long n, int d, int k, long long cap) {
  if (nq < 0 || n < 0 || d <= 0 || k < 1 || cap < k) return 0;
  return prefilter_layout(nq, n > 0 ? n : 1, d, k, cap).total;
}

long long rr_cosine_topk_prefilter_cap_for(int nq, long long n, int d, int k, size_t workspace_bytes) {
  if (nq <= 0 || n < 0 || d <= 0 || k < 1) return 0;
  const PrefilterWs L = prefilter_layout(nq, n > 0 ? n : 1, d, k);
  return workspace_bytes >= L.total ? L.cap : cap_that_fits(L.off_cand, nq, workspace_bytes, L.cap);
}

int rr_cosine_topk_prefilter(rr_handle_t h, const float* queries, int nq, const float* gallery,
                             const void* gallery_bf16, const double* bound3, long long n, int d, int k,
                             long long idx_offset, float* out_scores, long long* out_idx, void* workspace,
                             size_t workspace_bytes, void* stream) {
  RR_ENTRY(h);
  if (nq < 0 || n < 0 || d <= 0 || (d & 7) || k < 1 || k > 16384)
    return set_error(h, RR_EINVAL, "rr_cosine_topk_prefilter: need nq,n >= 0, d % 8 == 0, 1 <= k <= 16384");
  if (n >= 0xffffffffLL) return set_error(h, RR_EINVAL, "rr_cosine_topk_prefilter: shard must have < 2^32 rows");
  if (nq == 0) return RR_OK;
  if (!queries || !out_scores || !out_idx || (n > 0 && (!gallery || !gallery_bf16 || !bound3)))
    return set_error(h, RR_EINVAL, "rr_cosine_topk_prefilter: null pointer");
  if (((uintptr_t)queries & 15) || ((uintptr_t)gallery & 15) || ((uintptr_t)gallery_bf16 & 15))
    return set_error(h, RR_EINVAL, "rr_cosine_topk_prefilter: buffers must be 16-byte aligned");
  PrefilterWs L = prefilter_layout(nq, n > 0 ? n : 1, d, k);
  if (workspace && workspace_bytes < L.total) {  // bounded candidate buffer
    const long long cap = cap_that_fits(L.off_cand, nq, workspace_bytes, L.cap);
    if (cap >= k) L = prefilter_layout(nq, n > 0 ? n : 1, d, k, cap);
  }
  if (!workspace || workspace_bytes < L.total)
    return set_error(h, RR_EWORKSPACE, "rr_cosine_topk_prefilter: workspace too small (at least "
                                       "rr_cosine_topk_prefilter_workspace_size_cap(..., k))");
  hipStream_t s = (hipStream_t)stream;
  char* ws = (char*)workspace;
  float* scores_t = (float*)(ws + L.off_scores);
  float* tau = (float*)(ws + L.off_tau);
  int* cnt = (int*)(ws + L.off_cnt);
  int* ovf = (int*)(ws + L.off_ovf);
  float* eps2 = (float*)(ws + L.off_eps);
  uint16_t* qb = (uint16_t*)(ws + L.off_qb);
  unsigned long long* cand = (unsigned long long*)(ws + L.off_cand);
  // the overflow count is zeroed on every call (rr.h), the empty gallery included
  if (int rc = check_hip(h, hipMemsetAsync(ovf, 0, 4, s), "memset")) return rc;
  if (n == 0) {
    if (int rc = check_hip(h, hipMemsetAsync(cnt, 0, (size_t)nq * 4, s), "memset")) return rc;
    return launch_select_final(h, cand, L.cap, cnt, nq, k, idx_offset, out_scores, out_idx, ovf, s);
  }
  if (int rc = rr_quantize_rows(h, queries, nq, d, DT_BF16, qb, nullptr, s)) return rc;
  {
    TimedLaunch tl(h, kTimeElem, s);
    hipLaunchKernelGGL(query_eps_kernel, dim3((unsigned)(((long long)nq * 64 + 255) / 256)), dim3(256), 0, s, queries,
                       qb, nq, d, bound3, eps2);
  }
  if (int rc = check_hip(h, hipGetLastError(), "eps launch")) return rc;
  // 1. bf16 seed scores -> k-th best s'_seed -> T1
  GemmArgs g;
  g.A = (const float*)gallery_bf16;
  g.lda = d;
  g.M = (int)L.s;
  g.K = d;
  g.B = (const float*)qb;
  g.ldb = d;
  g.N = nq;
  g.C = scores_t;
  g.ldc = L.ld;
  if (int rc = launch_gemm(h, A_DENSE, E_SCORES_T, g, s, kTimeCosineSeed, DT_BF16)) return rc;
  if (int rc = launch_select_dense_seed(h, scores_t, L.ld, (int)L.s, nq, k, 0, cand, L.cap, cnt, tau, s)) return rc;
  {
    TimedLaunch tl(h, kTimeElem, s);
    hipLaunchKernelGGL(pass1_tau_kernel, dim3((nq + 255) / 256), dim3(256), 0, s, tau, eps2, cnt, nq);
  }
  if (int rc = check_hip(h, hipGetLastError(), "tau launch")) return rc;
  // 2. bf16 GEMM + filter over every row
  long long done = 0;
  while (done < n) {
    const long long rows = std::min<long long>(n - done, 0x7fffff00LL);
    GemmArgs f;
    f.A = (const float*)((const char*)gallery_bf16 + done * d * 2);
    f.lda = d;
    f.M = (int)rows;
    f.K = d;
    f.B = (const float*)qb;
    f.ldb = d;
    f.N = nq;
    f.tau = tau;
    f.cand = cand;
    f.cnt = cnt;
    f.cap = L.cap;
    f.row_offset = done;
    if (int rc = launch_gemm(h, A_DENSE, E_FILTER, f, s, kTimeCosine, DT_BF16)) return rc;
    done += rows;
  }
  // 3. tighten to s'_k - 2 eps, rescore the survivors exactly
  if (int rc = launch_prefilter_rescore(h, cand, L.cap, cnt, nq, k, eps2, tau, queries, gallery, d, s)) return rc;
  // 4. stable exact top-k
  return launch_select_final(h, cand, L.cap, cnt, nq, k, idx_offset, out_scores, out_idx, ovf, s);
}

}  // extern "C"
