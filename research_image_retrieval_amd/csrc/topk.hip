// topk.hip — per-query top-k selection for the cosine ranker (gfx950).
//
// Replaces the full `np.argsort(-similarity, axis=1)` of iris_evaluate.py:386
// with an exact top-k under a STABLE order (score desc, gallery index asc).
// Every candidate is a 64-bit key  (ord(score) << 32) | ~index  whose unsigned
// order is exactly that ranking order, so selection is an integer problem:
//   1. MSB-first radix select (8 passes x 8 bits, 256-bin LDS histogram,
//      parallel suffix scan) finds the k-th largest key; a pass stops early as
//      soon as the bucket holding the k-th key is entirely selected;
//   2. the <= k winning keys are gathered into LDS and bitonic-sorted
//      descending (power-of-two padded with key 0 = "no entry").
// One 256-thread workgroup per query.
#include "rr_internal.hpp"

namespace rr {

constexpr int SEL_NT = 256;
constexpr int SEL_MAX_K = 16384;

struct SelShared {
  unsigned int scan[SEL_NT];
  int digit, above, dcnt, gcount, all;
};

// MSB-first radix select of the k largest keys: on return, the winners are
// exactly the keys with (key >> fshift) >= (prefix >> fshift), or every
// non-zero key when `all` (<= k of them).
// Src: callable int64 index -> key (0 = empty / padding, never selected)
template <class Src>
__device__ void block_radix_select(Src src, long long count, int k, SelShared& sh, unsigned long long& prefix_out,
                                   int& fshift_out, bool& all_out, int max_passes = 8) {
  const int tid = threadIdx.x;
  unsigned long long prefix = 0, mask = 0;
  int remaining = k;
  int fshift = 0;
  bool all = false;
  for (int pass = 0; pass < max_passes; ++pass) {
    const int shift = 56 - 8 * pass;
    sh.scan[tid] = 0;
    __syncthreads();
    for (long long i = tid; i < count; i += SEL_NT) {
      const unsigned long long key = src(i);
      if (key != 0ull && (key & mask) == prefix) atomicAdd(&sh.scan[(key >> shift) & 255u], 1u);
    }
    __syncthreads();
    // inclusive suffix sum over digits: scan[t] = sum_{e >= t} hist[e]
    const unsigned int mine = sh.scan[tid];
    for (int off = 1; off < SEL_NT; off <<= 1) {
      const unsigned int add = (tid + off < SEL_NT) ? sh.scan[tid + off] : 0u;
      __syncthreads();
      sh.scan[tid] += add;
      __syncthreads();
    }
    if (pass == 0 && tid == 0) sh.all = (sh.scan[0] <= (unsigned)k) ? 1 : 0;
    {
      const unsigned int incl = sh.scan[tid];
      const unsigned int excl = incl - mine;
      if (mine > 0 && incl >= (unsigned)remaining && excl < (unsigned)remaining) {
        sh.digit = tid;
        sh.above = (int)excl;
        sh.dcnt = (int)mine;
      }
    }
    __syncthreads();
    if (sh.all) {
      all = true;
      break;
    }
    remaining -= sh.above;
    prefix |= (unsigned long long)sh.digit << shift;
    mask |= 0xffull << shift;
    const bool done = (sh.dcnt == remaining);
    fshift = shift;
    __syncthreads();
    if (done) break;
  }
  prefix_out = prefix;
  fshift_out = fshift;
  all_out = all;
}

template <class Src>
__device__ int block_select_sort(Src src, long long count, int k, int P, unsigned long long* skeys,
                                 SelShared& sh) {
  const int tid = threadIdx.x;
  unsigned long long prefix;
  int fshift;
  bool all;
  block_radix_select(src, count, k, sh, prefix, fshift, all);

  // gather winners
  if (tid == 0) sh.gcount = 0;
  __syncthreads();
  const unsigned long long ptop = prefix >> fshift;
  for (long long i = tid; i < count; i += SEL_NT) {
    const unsigned long long key = src(i);
    if (key != 0ull && (all || (key >> fshift) >= ptop)) {
      const int pos = atomicAdd(&sh.gcount, 1);
      if (pos < P) skeys[pos] = key;
    }
  }
  __syncthreads();
  const int nsel = sh.gcount < P ? sh.gcount : P;
  for (int i = nsel + tid; i < P; i += SEL_NT) skeys[i] = 0ull;
  __syncthreads();

  // bitonic sort, descending
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = tid; i < (P >> 1); i += SEL_NT) {
        const int pos = 2 * i - (i & (stride - 1));
        const int par = pos + stride;
        const bool desc = (pos & size) == 0;
        const unsigned long long a = skeys[pos], b = skeys[par];
        if ((a < b) == desc && a != b) {
          skeys[pos] = b;
          skeys[par] = a;
        }
      }
      __syncthreads();
    }
  }
  return nsel < k ? nsel : k;
}

__device__ inline void write_out(const unsigned long long* skeys, int nsel, int k, long long offset,
                                 float* os, long long* oi) {
  for (int r = threadIdx.x; r < k; r += SEL_NT) {
    const unsigned long long key = r < nsel ? skeys[r] : 0ull;
    if (key != 0ull) {
      os[r] = key_score(key);
      oi[r] = (long long)key_idx(key) + offset;
    } else {
      os[r] = -__builtin_inff();
      oi[r] = -1;
    }
  }
}

// Dense query-major scores -> seed the candidate buffer with the exact top-k
// of the first `rows` gallery rows, and the threshold tau = k-th best score.
__global__ __launch_bounds__(SEL_NT) void select_dense_seed_kernel(const float* __restrict__ st, long long ld,
                                                                   int rows, int k, int P, long long row_offset,
                                                                   unsigned long long* cand, long long cap,
                                                                   int* cnt, float* tau) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long skeys[];
  __shared__ SelShared sh;
  const int q = blockIdx.x;
  const float* col = st + (long long)q * ld;
  auto src = [&](long long i) -> unsigned long long { return make_key(col[i], (uint32_t)(row_offset + i)); };
  const int nsel = block_select_sort(src, rows, k, P, skeys, sh);
  unsigned long long* cq = cand + (long long)q * cap;
  for (int r = threadIdx.x; r < nsel; r += SEL_NT) cq[r] = skeys[r];
  if (threadIdx.x == 0) {
    cnt[q] = nsel;
    tau[q] = (nsel >= k) ? key_score(skeys[k - 1]) : -__builtin_inff();
  }
}

__global__ __launch_bounds__(SEL_NT) void select_final_kernel(const unsigned long long* __restrict__ cand,
                                                              long long cap, const int* __restrict__ cnt, int k,
                                                              int P, long long offset, float* os, long long* oi,
                                                              int* overflow) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long skeys[];
  __shared__ SelShared sh;
  const int q = blockIdx.x;
  const long long c = cnt[q];
  if (c > cap && threadIdx.x == 0) atomicAdd(overflow, 1);
  const long long count = c < cap ? c : cap;
  const unsigned long long* cq = cand + (long long)q * cap;
  auto src = [&](long long i) -> unsigned long long { return cq[i]; };
  const int nsel = block_select_sort(src, count, k, P, skeys, sh);
  write_out(skeys, nsel, k, offset, os + (long long)q * k, oi + (long long)q * k);
}

__global__ __launch_bounds__(SEL_NT) void merge_kernel(const float* __restrict__ ps, const long long* __restrict__ pi,
                                                       int nparts, int nq, int kin, int kout, int P, float* os,
                                                       long long* oi) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long skeys[];
  __shared__ SelShared sh;
  const int q = blockIdx.x;
  auto src = [&](long long i) -> unsigned long long {
    const long long p = i / kin, r = i - p * kin;
    const long long o = (p * nq + q) * (long long)kin + r;
    const long long idx = pi[o];
    return idx < 0 ? 0ull : make_key(ps[o], (uint32_t)idx);
  };
  const int nsel = block_select_sort(src, (long long)nparts * kin, kout, P, skeys, sh);
  write_out(skeys, nsel, kout, 0, os + (long long)q * kout, oi + (long long)q * kout);
}

// Pass 2 of the exact bf16-bound prefilter (rr_cosine_topk_prefilter).
// cand[q][0..cnt) holds (bf16 score, row) keys of every row whose bf16 score
// passed pass 1.  With s'_k the k-th largest of them and eps2 = 2 * (bound on
// |exact - bf16| for this query), a row can be in the exact top-k only if
// s' >= s'_k - eps2: those keys are rescored exactly in place, all others are
// cleared to 0 (empty); select_final then ranks them.  Any lower bound of s'_k
// is as valid: three 8-bit radix passes give the k-th key's top 24 bits, and
// the key with those bits and zeros below bounds it from beneath.
//
// Two launches: prefilter_threshold (one block per query) writes T2 into
// tau[q]; prefilter_rescore runs on a (query, part) grid, each part owning
// 1/RS_PARTS of the candidate positions, so 4x more blocks stream rows (the
// threshold must be final before any part rewrites keys).
// Rescoring is wave-cooperative: survivors are compacted into an LDS list;
// a wave takes 64 of them (lane j <-> survivor j) and walks the feature
// dimension in 32-wide segments: each segment of the 64 rows is loaded
// coalesced (8 lanes x 16 B per 128-B row piece, two segments in flight in
// registers) into a padded LDS tile; each lane then runs its row's exact fmaf
// chain in the order the fp32 MFMA core accumulates (gemm_f32.hip: within
// each 16-deep chunk k = 16c + e from lane half 0, then 16c + 8 + e from lane
// half 1, e = 0..7; zero terms up to the 16-padded k extent), so the scores
// are bit-identical to rr_cosine_topk's.
constexpr int RS_PARTS = 4;
constexpr int RS_CAP = 512;
constexpr int RS_SEG = 32;
constexpr int RS_LD = 36;  // tile row stride (floats): conflict-free ds_read_b128

__global__ __launch_bounds__(SEL_NT) void prefilter_threshold_kernel(const unsigned long long* __restrict__ cand,
                                                                     long long cap, const int* __restrict__ cnt, int k,
                                                                     const float* __restrict__ eps2,
                                                                     float* __restrict__ t2_out) {
  __shared__ SelShared sh;
  const int qi = blockIdx.x;
  const long long c0 = cnt[qi];
  const long long c = c0 < cap ? c0 : cap;
  const unsigned long long* cq = cand + (long long)qi * cap;
  float t2 = -__builtin_inff();
  if (c > k) {
    auto src = [&](long long i) -> unsigned long long { return cq[i]; };
    unsigned long long prefix;
    int fshift;
    bool all;
    block_radix_select(src, c, k, sh, prefix, fshift, all, 3);
    if (!all) {
      const double t = (double)key_score((prefix >> fshift) << fshift) - (double)eps2[qi];
      t2 = (float)t;
      if ((double)t2 > t) t2 = next_down(t2);
    }
  }
  if (threadIdx.x == 0) t2_out[qi] = t2;
}

__global__ __launch_bounds__(SEL_NT) void prefilter_rescore_kernel(unsigned long long* __restrict__ cand, long long cap,
                                                                   const int* __restrict__ cnt,
                                                                   const float* __restrict__ t2v,
                                                                   const float* __restrict__ q,
                                                                   const float* __restrict__ g, int d, int dpad) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* qs = smem;          // [dpad] (zero beyond d)
  float* tiles = smem + dpad;  // [4 waves][64][RS_LD]
  __shared__ uint32_t lpos[RS_CAP];
  __shared__ uint32_t lrow[RS_CAP];
  __shared__ int lcount;
  const int qi = blockIdx.x, part = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < dpad; i += SEL_NT) qs[i] = i < d ? q[(long long)qi * d + i] : 0.f;
  const long long c0 = cnt[qi];
  const long long c = c0 < cap ? c0 : cap;
  unsigned long long* cq = cand + (long long)qi * cap;
  const float t2 = t2v[qi];
  __syncthreads();
  const long long lo = c * part / RS_PARTS, hi = c * (part + 1) / RS_PARTS;
  const int dk = (d + 15) & ~15;  // the MFMA core's k extent (zero-padded 16-deep chunks)
  float* tile = tiles + wave * 64 * RS_LD;
  long long base = lo;
  while (base < hi) {
    // ---- compact the next survivors of this part into the LDS list ----
    if (tid == 0) lcount = 0;
    __syncthreads();
    int filled = 0;
    while (base < hi && filled <= RS_CAP - SEL_NT) {
      const long long i = base + tid;
      if (i < hi) {
        const unsigned long long key = cq[i];
        if (key != 0ull) {
          if (!(key_score(key) < t2)) {  // NaN score or NaN T2: rescore (NaN ranks last)
            const int p = atomicAdd(&lcount, 1);
            lpos[p] = (uint32_t)i;
            lrow[p] = key_idx(key);
          } else {
            cq[i] = 0ull;
          }
        }
      }
      base += SEL_NT;
      __syncthreads();
      filled = lcount;
      __syncthreads();
    }
    const int m = filled;
    // ---- rescore them, 64 per wave ----
    for (int g0 = 0; g0 < m; g0 += SEL_NT) {
      const int mine0 = g0 + wave * 64;
      const int my = mine0 + lane;
      // this lane's 8 pieces of a segment: row r = 8t + (lane >> 3), float4 (lane & 7)
      const float* rp[8];
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const int sidx = mine0 + 8 * t + (lane >> 3);
        rp[t] = sidx < m ? g + (long long)lrow[sidx] * d + 4 * (lane & 7) : nullptr;
      }
      auto load_seg = [&](int seg, float4* v) {
        const int col = seg + 4 * (lane & 7);
#pragma unroll
        for (int t = 0; t < 8; ++t)
          v[t] = (rp[t] != nullptr && col < d) ? *reinterpret_cast<const float4*>(rp[t] + seg)
                                               : float4{0.f, 0.f, 0.f, 0.f};
      };
      float4 cur[8], nxt[8];
      load_seg(0, cur);
      float acc = 0.f;
      for (int seg = 0; seg < dk; seg += RS_SEG) {
        if (seg + RS_SEG < dk) load_seg(seg + RS_SEG, nxt);
#pragma unroll
        for (int t = 0; t < 8; ++t)
          *reinterpret_cast<float4*>(tile + (8 * t + (lane >> 3)) * RS_LD + 4 * (lane & 7)) = cur[t];
        __syncthreads();
        if (my < m) {
          const int nch = (dk - seg) < RS_SEG ? (dk - seg) >> 4 : RS_SEG / 16;
          for (int ch = 0; ch < nch; ++ch) {
            float gv[16], qv[16];
#pragma unroll
            for (int v = 0; v < 4; ++v) {
              const float4 x = *reinterpret_cast<const float4*>(tile + lane * RS_LD + 16 * ch + 4 * v);
              const float4 y = *reinterpret_cast<const float4*>(qs + seg + 16 * ch + 4 * v);
              gv[4 * v] = x.x, gv[4 * v + 1] = x.y, gv[4 * v + 2] = x.z, gv[4 * v + 3] = x.w;
              qv[4 * v] = y.x, qv[4 * v + 1] = y.y, qv[4 * v + 2] = y.z, qv[4 * v + 3] = y.w;
            }
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              acc = __builtin_fmaf(gv[e], qv[e], acc);
              acc = __builtin_fmaf(gv[8 + e], qv[8 + e], acc);
            }
          }
        }
        __syncthreads();
#pragma unroll
        for (int t = 0; t < 8; ++t) cur[t] = nxt[t];
      }
      if (my < m) cq[lpos[my]] = make_key(acc, lrow[my]);
    }
    __syncthreads();
  }
}

static int pow2_at_least(int k) {
  int p = 1;
  while (p < k) p <<= 1;
  return p;
}

static int check_k(rr_handle_s* h, int k) {
  if (k < 1 || k > SEL_MAX_K) return set_error(h, RR_EINVAL, "top-k: k must be in [1, 16384]");
  return RR_OK;
}

static hipError_t set_lds(const void* fn, size_t bytes) {
  if (bytes <= 64 * 1024) return hipSuccess;
  return hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

int launch_select_dense_seed(rr_handle_s* h, const float* st, long long ld, int rows, int nq, int k,
                             long long row_offset, unsigned long long* cand, long long cap, int* cnt, float* tau,
                             hipStream_t s) {
  if (int rc = check_k(h, k)) return rc;
  if (nq <= 0) return RR_OK;
  const int P = pow2_at_least(k);
  const size_t lds = (size_t)P * 8;
  hipError_t e = set_lds((const void*)select_dense_seed_kernel, lds);
  if (e != hipSuccess) return check_hip(h, e, "select_dense_seed attr");
  TimedLaunch tl(h, kTimeSelect, s);
  hipLaunchKernelGGL(select_dense_seed_kernel, dim3(nq), dim3(SEL_NT), lds, s, st, ld, rows, k, P, row_offset,
                     cand, cap, cnt, tau);
  return check_hip(h, hipGetLastError(), "select_dense_seed launch");
}

int launch_select_final(rr_handle_s* h, const unsigned long long* cand, long long cap, const int* cnt, int nq, int k,
                        long long offset, float* os, long long* oi, int* overflow, hipStream_t s) {
  if (int rc = check_k(h, k)) return rc;
  if (nq <= 0) return RR_OK;
  const int P = pow2_at_least(k);
  const size_t lds = (size_t)P * 8;
  hipError_t e = set_lds((const void*)select_final_kernel, lds);
  if (e != hipSuccess) return check_hip(h, e, "select_final attr");
  TimedLaunch tl(h, kTimeSelect, s);
  hipLaunchKernelGGL(select_final_kernel, dim3(nq), dim3(SEL_NT), lds, s, cand, cap, cnt, k, P, offset, os, oi,
                     overflow);
  return check_hip(h, hipGetLastError(), "select_final launch");
}

int launch_merge(rr_handle_s* h, const float* ps, const long long* pi, int nparts, int nq, int kin, int kout,
                 float* os, long long* oi, hipStream_t s) {
  if (int rc = check_k(h, kout)) return rc;
  if (nparts <= 0 || kin <= 0) return set_error(h, RR_EINVAL, "merge: nparts and k_in must be positive");
  if (nq <= 0) return RR_OK;
  const int P = pow2_at_least(kout);
  const size_t lds = (size_t)P * 8;
  hipError_t e = set_lds((const void*)merge_kernel, lds);
  if (e != hipSuccess) return check_hip(h, e, "merge attr");
  TimedLaunch tl(h, kTimeSelect, s);
  hipLaunchKernelGGL(merge_kernel, dim3(nq), dim3(SEL_NT), lds, s, ps, pi, nparts, nq, kin, kout, P, os, oi);
  return check_hip(h, hipGetLastError(), "merge launch");
}

int launch_prefilter_rescore(rr_handle_s* h, unsigned long long* cand, long long cap, const int* cnt, int nq, int k,
                             const float* eps2, float* t2, const float* q, const float* g, int d, hipStream_t s) {
  if (int rc = check_k(h, k)) return rc;
  if (nq <= 0) return RR_OK;
  {
    TimedLaunch tl(h, kTimeSelect, s);
    hipLaunchKernelGGL(prefilter_threshold_kernel, dim3(nq), dim3(SEL_NT), 0, s, cand, cap, cnt, k, eps2, t2);
  }
  if (int rc = check_hip(h, hipGetLastError(), "prefilter_threshold launch")) return rc;
  const int dpad = (d + RS_SEG - 1) / RS_SEG * RS_SEG;
  const size_t lds = (size_t)dpad * 4 + (size_t)4 * 64 * RS_LD * 4;
  hipError_t e = set_lds((const void*)prefilter_rescore_kernel, lds);
  if (e != hipSuccess) return check_hip(h, e, "prefilter_rescore attr");
  TimedLaunch tl(h, kTimeSelect, s);
  hipLaunchKernelGGL(prefilter_rescore_kernel, dim3(nq, RS_PARTS), dim3(SEL_NT), lds, s, cand, cap, cnt, t2, q, g, d,
                     dpad);
  return check_hip(h, hipGetLastError(), "prefilter_rescore launch");
}

}  // namespace rr
