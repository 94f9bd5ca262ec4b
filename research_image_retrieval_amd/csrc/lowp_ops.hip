// lowp_ops.hip — fp32 -> bf16 / fp8 row quantisation for the low-precision
// (C4 bf16, C5 fp8) search and ViT paths (gfx950).
//   bf16: round-to-nearest-even (v_cvt_pk_bf16_f32 via the __bf16 cast).
//   fp8 : OCP e4m3 (gfx950 native, v_cvt_pk_fp8_f32) with one fp32 scale per
//         row: q = x * 448 / amax(row), scale = amax / 448, so x ~= q * scale
//         ("fp8-e4m3 with per-row scale").
#include "rr_internal.hpp"

namespace rr {

constexpr float kFp8Max = 448.0f;

// one wave per row, 4 consecutive elements per lane-step (d % 4 == 0)
__global__ __launch_bounds__(256) void quantize_rows_kernel(const float* __restrict__ x, long long rows, int d,
                                                            int dtype, void* __restrict__ y,
                                                            float* __restrict__ row_scale) {
  const long long row = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float4* xr = reinterpret_cast<const float4*>(x + row * d);
  const int d4 = d >> 2;
  if (dtype == DT_BF16) {
    typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
    bf16x4* yr = reinterpret_cast<bf16x4*>(reinterpret_cast<uint16_t*>(y) + row * d);
    for (int i = lane; i < d4; i += 64) {
      const float4 v = xr[i];
      yr[i] = bf16x4{(__bf16)v.x, (__bf16)v.y, (__bf16)v.z, (__bf16)v.w};
    }
    if (row_scale != nullptr && lane == 0) row_scale[row] = 1.0f;
    return;
  }
  float amax = 0.f;
  for (int i = lane; i < d4; i += 64) {
    const float4 v = xr[i];
    amax = fmaxf(amax, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) amax = fmaxf(amax, __shfl_xor(amax, off, 64));
  const float scale = amax > 0.f ? amax / kFp8Max : 1.0f;
  const float inv = amax > 0.f ? kFp8Max / amax : 0.0f;
  int* yr = reinterpret_cast<int*>(reinterpret_cast<uint8_t*>(y) + row * d);
  for (int i = lane; i < d4; i += 64) {
    const float4 v = xr[i];
    int p = 0;
    p = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(v.x * inv, -kFp8Max), kFp8Max),
                                        fminf(fmaxf(v.y * inv, -kFp8Max), kFp8Max), p, false);
    p = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(v.z * inv, -kFp8Max), kFp8Max),
                                        fminf(fmaxf(v.w * inv, -kFp8Max), kFp8Max), p, true);
    yr[i] = p;
  }
  if (row_scale != nullptr && lane == 0) row_scale[row] = scale;
}

}  // namespace rr

using namespace rr;

extern "C" int rr_quantize_rows(rr_handle_t h, const float* x, long long rows, int d, int dtype, void* y,
                                float* row_scale, void* stream) {
  RR_ENTRY(h);
  if (!x || !y || rows < 0 || d <= 0 || (d & 3) || (dtype != DT_BF16 && dtype != DT_FP8) ||
      ((uintptr_t)x & 15) || (dtype == DT_FP8 && !row_scale))
    return set_error(h, RR_EINVAL, "rr_quantize_rows: bad argument (d % 4 == 0, dtype 1|2, fp8 needs row_scale)");
  if (rows == 0) return RR_OK;
  hipStream_t s = (hipStream_t)stream;
  TimedLaunch tl(h, kTimeElem, s);
  const long long threads = rows * 64;
  hipLaunchKernelGGL(quantize_rows_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s, x, rows, d, dtype,
                     y, row_scale);
  return check_hip(h, hipGetLastError(), "quantize launch");
}
