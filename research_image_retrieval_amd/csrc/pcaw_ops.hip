// pcaw_ops.hip — the GPU half of PCA-whitening learning:
// the column mean and the centred Gram matrix Xc^T Xc of a descriptor set
// X [n, d] (networks/backbone.py:46-50: m = X.mean(0); Xc = X - m;
// Xcov = Xc^T Xc).  The eigendecomposition stays on the host (np.linalg.eig,
// backbone.py:51), as does the 1/(2n) symmetrisation (cheap, d x d).
//
// Pipeline per chunk of R rows (R <= 131072, bounded workspace at any n):
//   1. center_transpose: Xt[j][i] = X[r0+i][j] - m[j] (fp32, 64x64 LDS tiles,
//      both sides coalesced; rows past n are written as 0 so they add nothing)
//   2. gram GEMM on the MFMA core: G_s = Xt[:, ks] . Xt[:, ks]^T, split-K over
//      S slices of the chunk (fp32 MFMA partials), upper-triangle tiles only
//   3. reduce: gram64[i][j] += sum_s G_s[i][j] in fp64 (i <= j)
// then a final mirror makes gram64 symmetric.  Column sums for the mean are
// accumulated in fp64 (two passes: per-row-group partials, then a sum).
//
// Algorithmic cost: 2 n d^2 FLOP (half of it skipped by symmetry) and n d 4 B
// read twice (mean, transpose) + n d 4 B written and read once (Xt).
#include "rr_internal.hpp"

namespace rr {

constexpr int kMeanGroups = 256;
constexpr long long kChunkRows = 131072;
constexpr int kSplitK = 8192;

__global__ __launch_bounds__(256) void column_sum_kernel(const float* __restrict__ x, long long n, int d,
                                                         double* __restrict__ part) {
  const int col = blockIdx.x * 256 + threadIdx.x;
  if (col >= d) return;
  const long long per = (n + gridDim.y - 1) / gridDim.y;
  const long long r0 = (long long)blockIdx.y * per;
  const long long r1 = r0 + per < n ? r0 + per : n;
  double acc = 0.0;
  for (long long r = r0; r < r1; ++r) acc += (double)x[r * d + col];
  part[(long long)blockIdx.y * d + col] = acc;
}

__global__ __launch_bounds__(256) void column_mean_kernel(const double* __restrict__ part, int groups, long long n,
                                                          int d, double* __restrict__ mean64,
                                                          float* __restrict__ mean32) {
  const int col = blockIdx.x * 256 + threadIdx.x;
  if (col >= d) return;
  double acc = 0.0;
  for (int gi = 0; gi < groups; ++gi) acc += part[(long long)gi * d + col];
  const double m = n > 0 ? acc / (double)n : 0.0;
  mean64[col] = m;
  mean32[col] = (float)m;
}

// Xt[j][i] = x[r0 + i][j] - mean[j] for i < rows, 0 for rows <= i < rpad
__global__ __launch_bounds__(256) void center_transpose_kernel(const float* __restrict__ x, long long r0,
                                                               long long rows, int rpad, int d,
                                                               const float* __restrict__ mean,
                                                               float* __restrict__ xt) {
  __shared__ float tile[64][65];
  const int i0 = blockIdx.x * 64, j0 = blockIdx.y * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;  // 64 x 4
  for (int r = ty; r < 64; r += 4) {
    const int i = i0 + r, j = j0 + tx;
    float v = 0.f;
    if (i < rows && j < d) v = x[(r0 + i) * d + j] - mean[j];
    tile[r][tx] = v;
  }
  __syncthreads();
  for (int c = ty; c < 64; c += 4) {
    const int j = j0 + c, i = i0 + tx;
    if (j < d && i < rpad) xt[(long long)j * rpad + i] = tile[tx][c];
  }
}

__global__ __launch_bounds__(256) void gram_reduce_kernel(const float* __restrict__ part, int splits, int d,
                                                          double* __restrict__ gram) {
  const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long dd = (long long)d * d;
  if (e >= dd) return;
  const int i = (int)(e / d), j = (int)(e - (long long)i * d);
  if (i > j) return;
  double acc = gram[e];
  for (int s = 0; s < splits; ++s) acc += (double)part[(long long)s * dd + e];
  gram[e] = acc;
}

__global__ __launch_bounds__(256) void gram_mirror_kernel(int d, double* __restrict__ gram) {
  const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
  if (e >= (long long)d * d) return;
  const int i = (int)(e / d), j = (int)(e - (long long)i * d);
  if (i > j) gram[e] = gram[(long long)j * d + i];
}

struct GramLayout {
  long long rpad, splits;
  size_t off_mean_part, off_mean32, off_xt, off_part, total;
};

static GramLayout gram_layout(long long n, int d) {
  GramLayout L{};
  long long r = n < kChunkRows ? n : kChunkRows;
  L.rpad = ((r > 0 ? r : 1) + 31) / 32 * 32;
  L.splits = (L.rpad + kSplitK - 1) / kSplitK;
  auto al = [](size_t v) { return (v + 255) & ~(size_t)255; };
  size_t o = 0;
  L.off_mean_part = o;
  o = al(o + sizeof(double) * kMeanGroups * (size_t)d);
  L.off_mean32 = o;
  o = al(o + sizeof(float) * (size_t)d);
  L.off_xt = o;
  o = al(o + sizeof(float) * (size_t)d * L.rpad);
  L.off_part = o;
  o = al(o + sizeof(float) * (size_t)L.splits * d * d);
  L.total = o;
  return L;
}

}  // namespace rr

using namespace rr;

extern "C" size_t rr_pcaw_gram_workspace_size(long long n, int d) {
  if (n < 0 || d <= 0) return 0;
  return gram_layout(n, d).total;
}

extern "C" int rr_pcaw_gram(rr_handle_t h, const float* x, long long n, int d, void* workspace,
                            size_t workspace_bytes, double* mean_out, double* gram_out, void* stream) {
  RR_ENTRY(h);
  if (!x || n <= 0 || d <= 0 || !mean_out || !gram_out || !workspace)
    return set_error(h, RR_EINVAL, "rr_pcaw_gram: bad argument (n > 0, d > 0, non-null buffers)");
  if (d > 65535 * 64) return set_error(h, RR_EINVAL, "rr_pcaw_gram: d too large");
  const GramLayout L = gram_layout(n, d);
  if (workspace_bytes < L.total) return set_error(h, RR_EWORKSPACE, "rr_pcaw_gram: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  char* ws = static_cast<char*>(workspace);
  double* mean_part = reinterpret_cast<double*>(ws + L.off_mean_part);
  float* mean32 = reinterpret_cast<float*>(ws + L.off_mean32);
  float* xt = reinterpret_cast<float*>(ws + L.off_xt);
  float* part = reinterpret_cast<float*>(ws + L.off_part);
  const int cb = (d + 255) / 256;
  const long long dd = (long long)d * d;
  {
    TimedLaunch tl(h, kTimeElem, s);
    const int groups = (int)(n < kMeanGroups ? n : kMeanGroups);
    hipLaunchKernelGGL(column_sum_kernel, dim3(cb, groups), dim3(256), 0, s, x, n, d, mean_part);
    hipLaunchKernelGGL(column_mean_kernel, dim3(cb), dim3(256), 0, s, mean_part, groups, n, d, mean_out, mean32);
    if (hipError_t e = hipMemsetAsync(gram_out, 0, sizeof(double) * dd, s)) return check_hip(h, e, "gram memset");
  }
  if (int rc = check_hip(h, hipGetLastError(), "mean launch")) return rc;
  for (long long r0 = 0; r0 < n; r0 += L.rpad) {
    const long long rows = n - r0 < L.rpad ? n - r0 : L.rpad;
    // the last chunk is shortened to its own 32-row padding
    const int rpad = (int)((rows + 31) / 32 * 32);
    {
      TimedLaunch tl(h, kTimeElem, s);
      hipLaunchKernelGGL(center_transpose_kernel, dim3((rpad + 63) / 64, (d + 63) / 64), dim3(256), 0, s, x, r0,
                         rows, rpad, d, mean32, xt);
    }
    if (int rc = check_hip(h, hipGetLastError(), "center/transpose launch")) return rc;
    GemmArgs g;
    g.A = xt;
    g.lda = rpad;
    g.M = d;
    g.K = rpad;
    g.B = xt;
    g.ldb = rpad;
    g.N = d;
    g.C = part;
    g.ldc = d;
    g.k_split = kSplitK;
    g.c_split_stride = dd;
    g.sym = 1;
    if (int rc = launch_gemm(h, A_DENSE, E_STORE, g, s, kTimeGemm)) return rc;
    const int splits = (rpad + kSplitK - 1) / kSplitK;
    {
      TimedLaunch tl(h, kTimeElem, s);
      hipLaunchKernelGGL(gram_reduce_kernel, dim3((unsigned)((dd + 255) / 256)), dim3(256), 0, s, part, splits, d,
                         gram_out);
    }
    if (int rc = check_hip(h, hipGetLastError(), "gram reduce launch")) return rc;
  }
  {
    TimedLaunch tl(h, kTimeElem, s);
    hipLaunchKernelGGL(gram_mirror_kernel, dim3((unsigned)((dd + 255) / 256)), dim3(256), 0, s, d, gram_out);
  }
  return check_hip(h, hipGetLastError(), "gram mirror launch");
}
