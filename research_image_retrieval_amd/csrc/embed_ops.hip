// embed_ops.hip — HBM-bound embed-path kernels (gfx950): input normalisation,
// NCHW->NHWC relayout, stem max-pool, GeM pooling, row L2 normalisation.
// All are single-pass streaming kernels with coalesced 4-/16-byte accesses
// along the innermost (channel) axis; reductions use wavefront shuffles.
#include "rr_internal.hpp"

namespace rr {

// (x/255 - mean[c]) / std[c]; same op order and IEEE division as
// torchvision ToTensor().div(255) + Normalize().sub_(mean).div_(std)
// (dataset/configdataset.py:417,430-436).
// out_c == 4 appends a zero channel (16-B pixels for the stem conv's tap loads).
__global__ void preprocess_u8_kernel(const uint8_t* __restrict__ in, long long n_px, float m0, float m1, float m2,
                                     float s0, float s1, float s2, int out_c, float* __restrict__ out) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x; p < n_px; p += stride) {
    const uint8_t* px = in + p * 3;
    const float r = ((float)px[0] / 255.0f - m0) / s0;
    const float g = ((float)px[1] / 255.0f - m1) / s1;
    const float b = ((float)px[2] / 255.0f - m2) / s2;
    if (out_c == 4) {
      *reinterpret_cast<float4*>(out + p * 4) = make_float4(r, g, b, 0.f);
    } else {
      float* o = out + p * 3;
      o[0] = r;
      o[1] = g;
      o[2] = b;
    }
  }
}

// out[b][hw][c'] = in[b][c'][hw] for c' < C, 0 for C <= c' < CO (channel pad)
__global__ void nchw_to_nhwc_kernel(const float* __restrict__ in, int C, int CO, long long HW, long long total,
                                    float* __restrict__ out) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long o = (long long)blockIdx.x * blockDim.x + threadIdx.x; o < total; o += stride) {
    const int c = (int)(o % CO);
    const long long t = o / CO;
    const long long hw = t % HW;
    const long long b = t / HW;
    out[o] = c < C ? in[(b * C + c) * HW + hw] : 0.f;
  }
}

// bilinear, align_corners=False (ATen upsample_bilinear2d source-index rule)
__global__ void resize_bilinear_kernel(const float* __restrict__ x, int B, int H, int W, int C, int OH, int OW,
                                       float sh, float sw, float* __restrict__ y) {
  const long long total = (long long)B * OH * OW * C;
  const long long gstride = (long long)gridDim.x * blockDim.x;
  for (long long o = (long long)blockIdx.x * blockDim.x + threadIdx.x; o < total; o += gstride) {
    const int c = (int)(o % C);
    long long t = o / C;
    const int ow = (int)(t % OW);
    t /= OW;
    const int oh = (int)(t % OH);
    const int b = (int)(t / OH);
    float rh = sh * ((float)oh + 0.5f) - 0.5f;
    float rw = sw * ((float)ow + 0.5f) - 0.5f;
    rh = rh < 0.f ? 0.f : rh;
    rw = rw < 0.f ? 0.f : rw;
    const int h0 = (int)rh, w0 = (int)rw;
    const int h1 = h0 + (h0 < H - 1 ? 1 : 0), w1 = w0 + (w0 < W - 1 ? 1 : 0);
    const float lh1 = fminf(fmaxf(rh - (float)h0, 0.f), 1.f), lw1 = fminf(fmaxf(rw - (float)w0, 0.f), 1.f);
    const float lh0 = 1.f - lh1, lw0 = 1.f - lw1;
    const float* xb = x + (long long)b * H * W * C + c;
    const float v00 = xb[((long long)h0 * W + w0) * C], v01 = xb[((long long)h0 * W + w1) * C];
    const float v10 = xb[((long long)h1 * W + w0) * C], v11 = xb[((long long)h1 * W + w1) * C];
    y[o] = (v00 * lw0 + v01 * lw1) * lh0 + (v10 * lw0 + v11 * lw1) * lh1;
  }
}

// max pool, NHWC, one block per output row (b, oh), 4 channels per thread
// (C % 4 == 0); padding taps are -inf.  A block's outputs share their input
// columns and consecutive blocks share an input row, so the overlapping 3x3
// windows are re-read from L2 instead of HBM (the flat grid-stride form below
// read 6.4 GB per 4.1 GB stem output at 1280 images); 32-bit index math.
__global__ __launch_bounds__(256) void maxpool4_row_kernel(const float* __restrict__ x, int H, int W, int C, int k,
                                                           int stride, int pad, int OH, int OW, float* __restrict__ y) {
  const int C4 = C >> 2;
  const int row = blockIdx.x;  // b * OH + oh
  const int b = row / OH, oh = row - b * OH;
  const float* xb = x + (long long)b * H * W * C;
  float* yr = y + (long long)row * OW * C;
  const int n = OW * C4;
  for (int o = threadIdx.x; o < n; o += blockDim.x) {
    const int ow = o / C4, c4 = o - ow * C4;
    float4 m = make_float4(-__builtin_inff(), -__builtin_inff(), -__builtin_inff(), -__builtin_inff());
    for (int dh = 0; dh < k; ++dh) {
      const int ih = oh * stride - pad + dh;
      if ((unsigned)ih >= (unsigned)H) continue;
      const float* xr = xb + (long long)ih * W * C + c4 * 4;
      for (int dw = 0; dw < k; ++dw) {
        const int iw = ow * stride - pad + dw;
        if ((unsigned)iw >= (unsigned)W) continue;
        const float4 v = *reinterpret_cast<const float4*>(xr + iw * C);
        m.x = fmaxf(m.x, v.x);
        m.y = fmaxf(m.y, v.y);
        m.z = fmaxf(m.z, v.z);
        m.w = fmaxf(m.w, v.w);
      }
    }
    *reinterpret_cast<float4*>(yr + o * 4) = m;
  }
}

// The ResNet stem's 3x3 / stride 2 / pad 1 max pool, NHWC, C % 4 == 0: one
// block per pair of output rows, each thread a 2x2 block of outputs x 4
// channels from the 5x5 input window they share (25 loads for 4 outputs
// instead of 36), row by row: per input row the max of columns 0-2 and of
// columns 2-4.  Padding taps are -inf.
typedef float mp_f32x4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void maxpool3s2_kernel(const float* __restrict__ x, int H, int W, int C, int OH,
                                                         int OW, float* __restrict__ y) {
  const int C4 = C >> 2;
  const int OH2 = (OH + 1) >> 1, OW2 = (OW + 1) >> 1;
  const int b = blockIdx.x / OH2, oh0 = 2 * (blockIdx.x - b * OH2);
  const float* xb = x + (long long)b * H * W * C;
  float* yb = y + (long long)b * OH * OW * C;
  const float ninf = -__builtin_inff();
  const int n = OW2 * C4;
  for (int o = threadIdx.x; o < n; o += blockDim.x) {
    const int owp = o / C4, c4 = o - owp * C4;
    const int ow0 = 2 * owp;
    mp_f32x4 m[2][2];  // [output row][output col]
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int q = 0; q < 2; ++q) m[r][q] = mp_f32x4{ninf, ninf, ninf, ninf};
#pragma unroll
    for (int dr = 0; dr < 5; ++dr) {
      const int ih = 2 * oh0 - 1 + dr;
      if ((unsigned)ih >= (unsigned)H) continue;
      const float* xr = xb + (long long)ih * W * C + c4 * 4;
      mp_f32x4 col[5];
#pragma unroll
      for (int dc = 0; dc < 5; ++dc) {
        const int iw = 2 * ow0 - 1 + dc;
        col[dc] = (unsigned)iw < (unsigned)W ? *reinterpret_cast<const mp_f32x4*>(xr + iw * C) : mp_f32x4{ninf, ninf, ninf, ninf};
      }
      mp_f32x4 p0, p1;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        p0[e] = fmaxf(fmaxf(col[0][e], col[1][e]), col[2][e]);
        p1[e] = fmaxf(fmaxf(col[2][e], col[3][e]), col[4][e]);
      }
      // input row dr feeds output row 0 (dr 0-2) and output row 1 (dr 2-4)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (dr <= 2) {
          m[0][0][e] = fmaxf(m[0][0][e], p0[e]);
          m[0][1][e] = fmaxf(m[0][1][e], p1[e]);
        }
        if (dr >= 2) {
          m[1][0][e] = fmaxf(m[1][0][e], p0[e]);
          m[1][1][e] = fmaxf(m[1][1][e], p1[e]);
        }
      }
    }
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      if (oh0 + r >= OH) continue;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        if (ow0 + q >= OW) continue;
        *reinterpret_cast<mp_f32x4*>(yb + ((long long)(oh0 + r) * OW + ow0 + q) * C + c4 * 4) = m[r][q];
      }
    }
  }
}

// max pool, NHWC, 4 channels per thread (C % 4 == 0); padding taps are -inf.
__global__ void maxpool4_kernel(const float* __restrict__ x, int B, int H, int W, int C, int k, int stride, int pad,
                                int OH, int OW, float* __restrict__ y) {
  const int C4 = C >> 2;
  const long long total = (long long)B * OH * OW * C4;
  const long long gstride = (long long)gridDim.x * blockDim.x;
  for (long long o = (long long)blockIdx.x * blockDim.x + threadIdx.x; o < total; o += gstride) {
    const int c4 = (int)(o % C4);
    long long t = o / C4;
    const int ow = (int)(t % OW);
    t /= OW;
    const int oh = (int)(t % OH);
    const int b = (int)(t / OH);
    float4 m = make_float4(-__builtin_inff(), -__builtin_inff(), -__builtin_inff(), -__builtin_inff());
    for (int dh = 0; dh < k; ++dh) {
      const int ih = oh * stride - pad + dh;
      if ((unsigned)ih >= (unsigned)H) continue;
      for (int dw = 0; dw < k; ++dw) {
        const int iw = ow * stride - pad + dw;
        if ((unsigned)iw >= (unsigned)W) continue;
        const float4 v = *reinterpret_cast<const float4*>(x + (((long long)b * H + ih) * W + iw) * C + c4 * 4);
        m.x = fmaxf(m.x, v.x);
        m.y = fmaxf(m.y, v.y);
        m.z = fmaxf(m.z, v.z);
        m.w = fmaxf(m.w, v.w);
      }
    }
    *reinterpret_cast<float4*>(y + o * 4) = m;
  }
}

// max pool, NHWC; out-of-bounds taps are -inf (PyTorch max_pool2d padding).
__global__ void maxpool_kernel(const float* __restrict__ x, int B, int H, int W, int C, int k, int stride, int pad,
                               int OH, int OW, float* __restrict__ y) {
  const long long total = (long long)B * OH * OW * C;
  const long long gstride = (long long)gridDim.x * blockDim.x;
  for (long long o = (long long)blockIdx.x * blockDim.x + threadIdx.x; o < total; o += gstride) {
    const int c = (int)(o % C);
    long long t = o / C;
    const int ow = (int)(t % OW);
    t /= OW;
    const int oh = (int)(t % OH);
    const int b = (int)(t / OH);
    float m = -__builtin_inff();
    for (int dh = 0; dh < k; ++dh) {
      const int ih = oh * stride - pad + dh;
      if ((unsigned)ih >= (unsigned)H) continue;
      for (int dw = 0; dw < k; ++dw) {
        const int iw = ow * stride - pad + dw;
        if ((unsigned)iw >= (unsigned)W) continue;
        m = fmaxf(m, x[(((long long)b * H + ih) * W + iw) * C + c]);
      }
    }
    y[o] = m;
  }
}

// GeM over the spatial axis of [B][HW][C]: (sum_hw clamp(x,eps)^p / HW)^(1/p).
// p == 3 uses (x*x)*x, the op torch's pow(tensor, 3.0) kernel emits
// (networks/RetrievalNet.py:325); other p use powf.
__global__ void gem_kernel(const float* __restrict__ x, int B, int HW, int C, float p, float eps, int p_is_3,
                           float* __restrict__ out) {
  const long long total = (long long)B * C;
  const long long gstride = (long long)gridDim.x * blockDim.x;
  const float inv_p = 1.0f / p;
  for (long long o = (long long)blockIdx.x * blockDim.x + threadIdx.x; o < total; o += gstride) {
    const int c = (int)(o % C);
    const long long b = o / C;
    const float* xp = x + b * (long long)HW * C + c;
    float acc = 0.f;
    for (int i = 0; i < HW; ++i) {
      const float v = fmaxf(xp[(long long)i * C], eps);
      acc += p_is_3 ? (v * v) * v : powf(v, p);
    }
    out[o] = powf(acc / (float)HW, inv_p);
  }
}

// One wave per row: x / max(||x||_2, eps)  (F.normalize semantics).
__global__ __launch_bounds__(256) void l2norm_kernel(const float* __restrict__ x, int M, int D, float eps,
                                                     float* __restrict__ y) {
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (wave >= M) return;
  const float* xr = x + (long long)wave * D;
  float* yr = y + (long long)wave * D;
  float ss = 0.f;
  for (int i = lane; i < D; i += 64) ss = fmaf(xr[i], xr[i], ss);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) ss += __shfl_xor(ss, off, 64);
  const float nrm = fmaxf(sqrtf(ss), eps);
  for (int i = lane; i < D; i += 64) yr[i] = xr[i] / nrm;
}

static dim3 grid_for(long long n, int block) {
  long long g = (n + block - 1) / block;
  if (g > 256 * 16) g = 256 * 16;
  if (g < 1) g = 1;
  return dim3((unsigned)g);
}

}  // namespace rr

using namespace rr;

extern "C" int rr_preprocess_u8(rr_handle_t h, const uint8_t* img, int b, int hgt, int wid, const float* mean3,
                                const float* std3, float* out, void* stream) {
  return rr_preprocess_u8_ex(h, img, b, hgt, wid, mean3, std3, 3, out, stream);
}

extern "C" int rr_preprocess_u8_ex(rr_handle_t h, const uint8_t* img, int b, int hgt, int wid, const float* mean3,
                                   const float* std3, int out_c, float* out, void* stream) {
  RR_ENTRY(h);
  if (!img || !out || !mean3 || !std3 || b < 0 || hgt < 0 || wid < 0 || (out_c != 3 && out_c != 4) ||
      (out_c == 4 && ((uintptr_t)out & 15)))
    return set_error(h, RR_EINVAL, "rr_preprocess_u8: bad argument (out_c 3 or 4, 16-B aligned out)");
  const long long npx = (long long)b * hgt * wid;
  if (npx == 0) return RR_OK;
  hipStream_t s = (hipStream_t)stream;
  TimedLaunch tl(h, kTimeElem, s);
  hipLaunchKernelGGL(preprocess_u8_kernel, grid_for(npx, 256), dim3(256), 0, s, img, npx, mean3[0], mean3[1],
                     mean3[2], std3[0], std3[1], std3[2], out_c, out);
  return check_hip(h, hipGetLastError(), "preprocess launch");
}

extern "C" int rr_nchw_to_nhwc(rr_handle_t h, const float* in, int b, int c, int hgt, int wid, float* out,
                               void* stream) {
  return rr_nchw_to_nhwc_ex(h, in, b, c, hgt, wid, c, out, stream);
}

extern "C" int rr_nchw_to_nhwc_ex(rr_handle_t h, const float* in, int b, int c, int hgt, int wid, int out_c,
                                  float* out, void* stream) {
  RR_ENTRY(h);
  if (!in || !out || b < 0 || c <= 0 || hgt < 0 || wid < 0 || out_c < c)
    return set_error(h, RR_EINVAL, "rr_nchw_to_nhwc: bad argument");
  const long long total = (long long)b * out_c * hgt * wid;
  if (total == 0) return RR_OK;
  hipStream_t s = (hipStream_t)stream;
  TimedLaunch tl(h, kTimeElem, s);
  hipLaunchKernelGGL(nchw_to_nhwc_kernel, grid_for(total, 256), dim3(256), 0, s, in, c, out_c, (long long)hgt * wid,
                     total, out);
  return check_hip(h, hipGetLastError(), "nchw_to_nhwc launch");
}

extern "C" int rr_maxpool2d(rr_handle_t h, const float* x, int b, int hgt, int wid, int c, int k, int stride, int pad,
                            float* y, void* stream) {
  RR_ENTRY(h);
  if (!x || !y || b < 0 || c <= 0 || k <= 0 || stride <= 0 || pad < 0 || 2 * pad > k)
    return set_error(h, RR_EINVAL, "rr_maxpool2d: bad argument");
  const int oh = (hgt + 2 * pad - k) / stride + 1, ow = (wid + 2 * pad - k) / stride + 1;
  if (oh <= 0 || ow <= 0) return set_error(h, RR_EINVAL, "rr_maxpool2d: empty output");
  const long long total = (long long)b * oh * ow * c;
  if (total == 0) return RR_OK;
  hipStream_t s = (hipStream_t)stream;
  TimedLaunch tl(h, kTimeElem, s);
  const bool vec = (c & 3) == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 15) == 0;
  if (vec && k == 3 && stride == 2 && pad == 1 && (long long)b * ((oh + 1) / 2) <= 0x7fffffffLL &&
      (long long)wid * c < 0x7fffffffLL)
    hipLaunchKernelGGL(maxpool3s2_kernel, dim3((unsigned)((long long)b * ((oh + 1) / 2))), dim3(256), 0, s, x, hgt,
                       wid, c, oh, ow, y);
  else if (vec && (long long)b * oh <= 0x7fffffffLL && (long long)wid * c < 0x7fffffffLL)
    hipLaunchKernelGGL(maxpool4_row_kernel, dim3((unsigned)((long long)b * oh)), dim3(256), 0, s, x, hgt, wid, c, k,
                       stride, pad, oh, ow, y);
  else if (vec)
    hipLaunchKernelGGL(maxpool4_kernel, grid_for(total / 4, 256), dim3(256), 0, s, x, b, hgt, wid, c, k, stride, pad,
                       oh, ow, y);
  else
    hipLaunchKernelGGL(maxpool_kernel, grid_for(total, 256), dim3(256), 0, s, x, b, hgt, wid, c, k, stride, pad, oh,
                       ow, y);
  return check_hip(h, hipGetLastError(), "maxpool launch");
}

extern "C" int rr_gem_pool(rr_handle_t h, const float* x, int b, int hw, int c, float p, float eps, float* out,
                           void* stream) {
  RR_ENTRY(h);
  if (!x || !out || b < 0 || hw <= 0 || c <= 0 || !(p > 0.f)) return set_error(h, RR_EINVAL, "rr_gem_pool: bad argument");
  const long long total = (long long)b * c;
  if (total == 0) return RR_OK;
  hipStream_t s = (hipStream_t)stream;
  TimedLaunch tl(h, kTimeElem, s);
  hipLaunchKernelGGL(gem_kernel, grid_for(total, 256), dim3(256), 0, s, x, b, hw, c, p, eps, p == 3.0f ? 1 : 0, out);
  return check_hip(h, hipGetLastError(), "gem launch");
}

extern "C" int rr_l2_normalize(rr_handle_t h, const float* x, int m, int d, float eps, float* y, void* stream) {
  RR_ENTRY(h);
  if (!x || !y || m < 0 || d <= 0) return set_error(h, RR_EINVAL, "rr_l2_normalize: bad argument");
  if (m == 0) return RR_OK;
  hipStream_t s = (hipStream_t)stream;
  TimedLaunch tl(h, kTimeElem, s);
  const long long threads = (long long)m * 64;
  hipLaunchKernelGGL(l2norm_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s, x, m, d, eps, y);
  return check_hip(h, hipGetLastError(), "l2norm launch");
}

extern "C" int rr_resize_bilinear(rr_handle_t h, const float* x, int b, int hgt, int wid, int c, int out_h, int out_w,
                                  float inv_scale_h, float inv_scale_w, float* y, void* stream) {
  RR_ENTRY(h);
  if (!x || !y || b < 0 || hgt <= 0 || wid <= 0 || c <= 0 || out_h <= 0 || out_w <= 0)
    return set_error(h, RR_EINVAL, "rr_resize_bilinear: bad argument");
  const float sh = inv_scale_h > 0.f ? inv_scale_h : (float)hgt / (float)out_h;
  const float sw = inv_scale_w > 0.f ? inv_scale_w : (float)wid / (float)out_w;
  const long long total = (long long)b * out_h * out_w * c;
  if (total == 0) return RR_OK;
  hipStream_t s = (hipStream_t)stream;
  TimedLaunch tl(h, kTimeElem, s);
  hipLaunchKernelGGL(resize_bilinear_kernel, grid_for(total, 256), dim3(256), 0, s, x, b, hgt, wid, c, out_h, out_w, sh,
                     sw, y);
  return check_hip(h, hipGetLastError(), "resize launch");
}

// ---- alpha-weighted query expansion (config C5) --------------------------
// q'[i] = normalize(q[i] + sum_{r < n} max(s[i][r], 0)^alpha * g[idx[i][r]])
// One workgroup per query; the n neighbour rows are gathered with coalesced
// float4 loads and accumulated in registers, then the row is L2-normalised
// with a block reduction.  Padding entries (idx < 0) and indices outside the
// local rows [idx_offset, idx_offset + n_rows) are skipped (never read).
namespace rr {
__global__ __launch_bounds__(256) void alpha_qe_kernel(const float* __restrict__ q, const float* __restrict__ g,
                                                       const long long* __restrict__ idx,
                                                       const float* __restrict__ sc, int k, int n, int d,
                                                       float alpha, long long idx_offset, long long n_rows,
                                                       float* __restrict__ out) {
  __shared__ float red[256 / 64];
  const int qi = blockIdx.x;
  const int d4 = d >> 2;
  float ss = 0.f;
  for (int c = threadIdx.x; c < d4; c += 256) {
    float4 acc = reinterpret_cast<const float4*>(q + (long long)qi * d)[c];
    for (int r = 0; r < n; ++r) {
      const long long j = idx[(long long)qi * k + r] - idx_offset;
      if (j < 0 || j >= n_rows) continue;
      const float s = sc[(long long)qi * k + r];
      const float w = s > 0.f ? powf(s, alpha) : 0.f;
      const float4 v = reinterpret_cast<const float4*>(g + j * d)[c];
      acc.x = fmaf(w, v.x, acc.x);
      acc.y = fmaf(w, v.y, acc.y);
      acc.z = fmaf(w, v.z, acc.z);
      acc.w = fmaf(w, v.w, acc.w);
    }
    reinterpret_cast<float4*>(out + (long long)qi * d)[c] = acc;
    ss = fmaf(acc.x, acc.x, fmaf(acc.y, acc.y, fmaf(acc.z, acc.z, fmaf(acc.w, acc.w, ss))));
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) ss += __shfl_xor(ss, off, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
  __syncthreads();
  const float tot = red[0] + red[1] + red[2] + red[3];
  const float inv = 1.0f / fmaxf(sqrtf(tot), 1e-12f);
  for (int c = threadIdx.x; c < d4; c += 256) {
    float4 v = reinterpret_cast<float4*>(out + (long long)qi * d)[c];
    v.x *= inv;
    v.y *= inv;
    v.z *= inv;
    v.w *= inv;
    reinterpret_cast<float4*>(out + (long long)qi * d)[c] = v;
  }
}
}  // namespace rr

extern "C" int rr_alpha_qe(rr_handle_t h, const float* queries, int nq, const float* gallery, long long n_rows,
                           int d, const long long* top_idx, const float* top_scores, int k, int n, float alpha,
                           long long idx_offset, float* out, void* stream) {
  RR_ENTRY(h);
  if (!queries || !top_idx || !top_scores || !out || nq < 0 || n_rows < 0 || (n_rows > 0 && !gallery) || d <= 0 ||
      (d & 3) || k <= 0 || n < 0 ||
      n > k || ((uintptr_t)queries & 15) || ((uintptr_t)gallery & 15) || ((uintptr_t)out & 15))
    return set_error(h, RR_EINVAL, "rr_alpha_qe: bad argument (d % 4 == 0, 0 <= n <= k, 16-B aligned rows)");
  if (nq == 0) return RR_OK;
  hipStream_t s = (hipStream_t)stream;
  TimedLaunch tl(h, kTimeElem, s);
  hipLaunchKernelGGL(alpha_qe_kernel, dim3((unsigned)nq), dim3(256), 0, s, queries, gallery, top_idx, top_scores, k,
                     n, d, alpha, idx_offset, n_rows, out);
  return check_hip(h, hipGetLastError(), "alpha_qe launch");
}
