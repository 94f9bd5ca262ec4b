// hbm_pattern.hip — HBM read rate of the trunk convs' access patterns, apart
// from any MFMA work: does reading a 1 GB NHWC activation 128 B per row per
// k-tile (the implicit-GEMM A loads: 256 rows of a tile, 32 channels at a
// time, rows 1-4 KB apart) or 1 KB per row per N-tile (the residual reads of
// a 256-column tile) cost bandwidth against a plain stream, and does a
// channel-blocked layout ([C/32][pixels][32]: a k-tile of 256 rows is one
// contiguous 32 KB) get it back?  One 512-thread block per CU-slot, four
// k-tiles of loads in flight per thread, loads summed (kept live).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/hbm_pattern.hip -o tools/hbm_pattern
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

constexpr int NT = 512;

// plain stream: block b reads bytes [b * chunk, (b + 1) * chunk), 1 KB per wave instruction
__global__ __launch_bounds__(NT, 1) void stream_read(const f32x4* __restrict__ x, long long n4, float* out) {
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  const long long per = (n4 + gridDim.x - 1) / gridDim.x;
  const long long b0 = blockIdx.x * per, b1 = min(n4, b0 + per);
  for (long long i = b0 + threadIdx.x; i < b1; i += 4 * NT) {
    f32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = (i + u * NT < b1) ? x[i + u * NT] : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < 4; ++u) s += v[u];
  }
  if (s[0] + s[1] + s[2] + s[3] == 1.2345f) out[0] = s[0];
}

// conv A pattern: rows of K fp32 (4 K bytes apart), 256-row tiles; k-tile kt
// reads columns 32 kt .. +31 of the tile's 256 rows: lane l -> row 16 w + l / 4
// (+ 128 for the second chunk), 32 B at column slot l % 4 (two 16-B loads)
__global__ __launch_bounds__(NT, 1) void conv_a_read(const float* __restrict__ x, int M, int K, int tiles,
                                                     float* out) {
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  const int tid = threadIdx.x, slot = tid % 4, row = tid / 4;
  const int nk = K / 32;
  for (int t = blockIdx.x; t < tiles; t += gridDim.x) {
    const long long r0 = (long long)t * 256 + row, r1 = r0 + 128;
    const float* p0 = x + (r0 < M ? r0 : 0) * K + slot * 8;
    const float* p1 = x + (r1 < M ? r1 : 0) * K + slot * 8;
    for (int kt = 0; kt < nk; kt += 4) {
      f32x4 v[16];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int k = (kt + u < nk ? kt + u : kt) * 32;
        v[4 * u + 0] = *reinterpret_cast<const f32x4*>(p0 + k);
        v[4 * u + 1] = *reinterpret_cast<const f32x4*>(p0 + k + 4);
        v[4 * u + 2] = *reinterpret_cast<const f32x4*>(p1 + k);
        v[4 * u + 3] = *reinterpret_cast<const f32x4*>(p1 + k + 4);
      }
#pragma unroll
      for (int u = 0; u < 16; ++u) s += v[u];
    }
  }
  if (s[0] + s[1] + s[2] + s[3] == 1.2345f) out[0] = s[0];
}

// channel-blocked layout [K/32][M][32]: k-tile kt of tile t is the contiguous
// 256 x 128 B = 32 KB at ((kt M) + 256 t) * 32 floats; the same lane -> (row,
// slot) map as conv_a_read
__global__ __launch_bounds__(NT, 1) void blocked_a_read(const float* __restrict__ x, int M, int K, int tiles,
                                                        float* out) {
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  const int tid = threadIdx.x, slot = tid % 4, row = tid / 4;
  const int nk = K / 32;
  for (int t = blockIdx.x; t < tiles; t += gridDim.x) {
    const long long r0 = (long long)t * 256 + row, r1 = r0 + 128;
    for (int kt = 0; kt < nk; kt += 4) {
      f32x4 v[16];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const long long base = (long long)(kt + u < nk ? kt + u : kt) * M * 32;
        const float* p0 = x + base + (r0 < M ? r0 : 0) * 32 + slot * 8;
        const float* p1 = x + base + (r1 < M ? r1 : 0) * 32 + slot * 8;
        v[4 * u + 0] = *reinterpret_cast<const f32x4*>(p0);
        v[4 * u + 1] = *reinterpret_cast<const f32x4*>(p0 + 4);
        v[4 * u + 2] = *reinterpret_cast<const f32x4*>(p1);
        v[4 * u + 3] = *reinterpret_cast<const f32x4*>(p1 + 4);
      }
#pragma unroll
      for (int u = 0; u < 16; ++u) s += v[u];
    }
  }
  if (s[0] + s[1] + s[2] + s[3] == 1.2345f) out[0] = s[0];
}

// epilogue pattern: [M][N] fp32, tile (tm, tn) of 256 rows x 256 columns
// (1 KB per row): 64 lanes per row segment, 8 rows per pass; tn fastest over
// consecutive tiles (the XCD remap's order); write = 1 stores the segment
template <int WRITE>
__global__ __launch_bounds__(NT, 1) void epi_seg(float* __restrict__ x, int M, int N, int tiles, float* out) {
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  const int tid = threadIdx.x, c4 = tid % 64, r = tid / 64;
  const int tn_n = N / 256;
  for (int t = blockIdx.x; t < tiles; t += gridDim.x) {
    const int tm = t / tn_n, tn = t - tm * tn_n;
    for (int rr = 0; rr < 256; rr += 32) {
      f32x4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const long long m = (long long)tm * 256 + rr + u * 8 + r;
        f32x4* p = reinterpret_cast<f32x4*>(x + (m < M ? m : 0) * N + tn * 256 + c4 * 4);
        if (WRITE) *p = f32x4{1.f, 2.f, 3.f, (float)u};
        else v[u] = *p;
      }
      if (!WRITE) {
#pragma unroll
        for (int u = 0; u < 4; ++u) s += v[u];
      }
    }
  }
  if (s[0] + s[1] + s[2] + s[3] == 1.2345f) out[0] = s[0];
}

__global__ void stream_write(f32x4* __restrict__ x, long long n4) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x)
    x[i] = f32x4{1.f, 2.f, 3.f, 4.f};
}

template <typename F>
static void timeit(const char* name, double bytes, F launch) {
  launch();
  CK(hipDeviceSynchronize());
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventRecord(a));
  for (int r = 0; r < 10; ++r) launch();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  ms /= 10;
  printf("%-60s %8.3f ms  %7.0f GB/s\n", name, ms, bytes / ms / 1e6);
  fflush(stdout);
}

int main() {
  const int M = 1280 * 196;  // the 14x14 stage at 1280 images
  const long long n = (long long)M * 1024;
  float *x, *out;
  CK(hipMalloc(&x, n * 4));
  CK(hipMalloc(&out, 64));
  hipLaunchKernelGGL(stream_write, dim3(4096), dim3(256), 0, 0, (f32x4*)x, n / 4);
  CK(hipDeviceSynchronize());
  const int tiles = (M + 255) / 256;
  const dim3 g(256), b(NT);
  timeit("stream read 1.03 GB", n * 4.0, [&] { hipLaunchKernelGGL(stream_read, g, b, 0, 0, (const f32x4*)x, n / 4, out); });
  timeit("stream write 1.03 GB", n * 4.0, [&] { hipLaunchKernelGGL(stream_write, dim3(4096), dim3(256), 0, 0, (f32x4*)x, n / 4); });
  timeit("conv A: K=1024 rows (4 KB), 128 B per row per k-tile", n * 4.0,
         [&] { hipLaunchKernelGGL(conv_a_read, g, b, 0, 0, x, M, 1024, tiles, out); });
  timeit("conv A: K=256 rows (1 KB), 128 B per row per k-tile (x4 M)", n * 4.0,
         [&] { hipLaunchKernelGGL(conv_a_read, g, b, 0, 0, x, M * 4, 256, tiles * 4, out); });
  timeit("blocked [K/32][M][32], K=1024: 32 KB contiguous per k-tile", n * 4.0,
         [&] { hipLaunchKernelGGL(blocked_a_read, g, b, 0, 0, x, M, 1024, tiles, out); });
  timeit("epilogue read: 1 KB row segments of 256-col tiles, N=1024", n * 4.0,
         [&] { hipLaunchKernelGGL(epi_seg<0>, g, b, 0, 0, x, M, 1024, tiles * 4, out); });
  timeit("epilogue write: 1 KB row segments of 256-col tiles, N=1024", n * 4.0,
         [&] { hipLaunchKernelGGL(epi_seg<1>, g, b, 0, 0, x, M, 1024, tiles * 4, out); });
  CK(hipFree(x));
  CK(hipFree(out));
  return 0;
}
