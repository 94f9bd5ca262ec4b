// fetch_ceiling.hip — how fast can every CU fill its LDS with the operands of
// the C3 cosine sweep, and what does the sweep's MFMA work leave of that?
//
// The bf16 filter sweep (gemm_f32.hip, lp_cfg 4: 256 gallery rows x 320
// queries per block, 8 waves, 1 block per CU, two 73.7 KB LDS stages, one
// 64-deep k-tile = 576 rows x 128 B per stage) is re-created here without its
// filter epilogue, with each part switchable:
//   G  stream the block's 256 gallery rows (HBM: every row is fetched by the
//      blocks of the 4 query panels)
//   Q  stream the block's 320-row query panel (1.3 MB, read by every block:
//      L2 / Infinity-Cache resident)
//   MF the sweep's MFMAs (per wave 2x5 v_mfma_f32_32x32x16_bf16 per 16-deep
//      k-step, fragments read from LDS exactly as the real tile does)
//   VG register staging (global_load_dwordx4 -> ds_write_b128) instead of
//      LDS-DMA (global_load_lds_dwordx4)
//   PF   prefetch the gallery k-slice two k-tiles ahead into L2 (4-byte
//        LDS-DMA per 128-B line into a dummy LDS word, left in flight across
//        the barrier: counted vmcnt + raw s_barrier instead of vmcnt(0))
//   ORD block -> (gallery tile, query panel) order: 0 = the library's (each
//      XCD a contiguous range of gallery tiles x all 4 panels); 2 / 4 = the 8
//      XCDs split into 2 / 4 panel groups x 4 / 2 gallery ranges, so an XCD
//      keeps 2 / 1 panels L2-resident and XCDs of one range stream the same
//      gallery rows at about the same time
// Gallery 1.6 M x 2048 bf16 (6.55 GB), 1280 queries: the C3 bench shape.
// Output per variant: ms, LDS fill rate (B/s per CU and chip), TFLOP/s.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/fetch_ceiling.hip -o tools/fetch_ceiling
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

constexpr int BM = 256, BN = 320, ROWS = BM + BN, K = 2048, EPR = 64, NK = K / EPR;
constexpr int NT = 512, SLOTS = 8, PASS = NT / SLOTS;  // 64 rows per staging pass
constexpr int BUFB = ROWS * 128;                      // bytes per stage

__device__ __forceinline__ int swz(int row, int slot) { return slot ^ ((row >> 1) & 7); }

// block -> (tm, tn); false: a padding block of the ORD grids
template <int ORD>
__device__ __forceinline__ bool tile_of(int bid, int nwg, int Mt, int T, int& tm, int& tn) {
  if constexpr (ORD == 0) {
    const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    tn = wgid % T;
    tm = wgid / T;
    return true;
  } else {
    constexpr int NP = ORD, NR = 8 / ORD;  // panel groups x gallery ranges = the 8 XCDs
    const int x = bid & 7, j = bid >> 3;
    const int tpg = T / NP;                 // panels per group
    const int R = (Mt + NR - 1) / NR;       // gallery tiles per range
    tm = (x / NP) * R + j / tpg;
    tn = (x % NP) * tpg + j % tpg;
    return tm < Mt && j < R * tpg;
  }
}

// IL > 0 (LDS-DMA only): instead of one burst of the next k-tile's 9 DMA
// instructions per wave at the top of the k-tile, chunk c goes out just
// before MFMA number (c * IL) / 9 of the k-tile's sequence (40 MFMAs of
// 32x32x16, 80 of 16x16x32), pinned there by sched_barriers: does spreading
// the issue over the MFMAs relieve the vector-memory issue queue?
template <int G, int Q, int MF, int VG, int ORD, int PF = 0, int M16 = 0, int IL = 0>
__global__ __launch_bounds__(NT, 1) void sweep_fill(const uint16_t* __restrict__ gal, const uint16_t* __restrict__ qry,
                                                    int Mt, int T, float* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) unsigned char lds[2 * BUFB + 256];
  int tm, tn;
  if (!tile_of<ORD>(blockIdx.x, gridDim.x, Mt, T, tm, tn)) return;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int slot = tid % SLOTS, crow = tid / SLOTS;
  // chunk i: LDS row crow + 64 i = gallery row crow + 64 i (i < 4) or query row crow + 64 (i - 4)
  const uint16_t* gsrc = gal + ((long long)tm * BM + crow) * K;
  const uint16_t* qsrc = qry + ((long long)tn * BN + crow) * K;
  auto src_of = [&](int i) { return i < 4 ? gsrc + (long long)i * PASS * K : qsrc + (long long)(i - 4) * PASS * K; };
  auto on = [&](int i) { return i < 4 ? G != 0 : Q != 0; };
  f32x4 rv[9];
  static_assert(!IL || (!VG && MF), "IL: LDS-DMA with MFMAs");
  auto issue_one = [&](int kt, int buf, int i) {
    if (!on(i)) return;
    const int row = crow + i * PASS;
    __builtin_amdgcn_global_load_lds((const void*)(src_of(i) + kt * EPR + swz(row, slot) * 8),
                                     (__attribute__((address_space(3))) void*)(lds + buf * BUFB +
                                                                               (i * PASS + wv * 8) * 128),
                                     16, 0, 0);
  };
  // the chunks due before MFMA number idx of the k-tile (IL > 0)
  auto issue_at = [&](int kt, int buf, int idx) {
    if constexpr (IL > 0) {
      if (kt >= NK) return;
#pragma unroll
      for (int c = 0; c < 9; ++c)
        if ((c * IL) / 9 == idx) {
          __builtin_amdgcn_sched_barrier(0);
          issue_one(kt, buf, c);
          __builtin_amdgcn_sched_barrier(0);
        }
    }
  };
  auto issue = [&](int kt, int buf) {
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      if (!on(i)) continue;
      const int row = crow + i * PASS;
      const uint16_t* s = src_of(i) + kt * EPR + swz(row, slot) * 8;
      if constexpr (VG) {
        rv[i] = *reinterpret_cast<const f32x4*>(s);
      } else {
        __builtin_amdgcn_global_load_lds((const void*)s,
                                         (__attribute__((address_space(3))) void*)(lds + buf * BUFB +
                                                                                   (i * PASS + wv * 8) * 128),
                                         16, 0, 0);
      }
    }
  };
  auto vstore = [&](int buf) {  // VG: chunk of (row, slot) at its swizzled LDS position
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      if (!on(i)) continue;
      const int row = crow + i * PASS;
      *reinterpret_cast<f32x4*>(lds + buf * BUFB + row * 128 + slot * 16) = rv[i];
    }
  };
  // PF: waves 0-3 each touch 64 of the block's 256 gallery rows' 128-B line
  // of k-tile kt (one 4-byte LDS-DMA per lane into a dummy word)
  const uint16_t* pf_src = gal + ((long long)tm * BM + (wv & 3) * 64 + lane) * K;
  auto prefetch = [&](int kt) {
    if (PF && wv < 4 && kt < NK)
      __builtin_amdgcn_global_load_lds((const void*)(pf_src + kt * EPR),
                                       (__attribute__((address_space(3))) void*)(lds + 2 * BUFB), 4, 0, 0);
  };
  f32x16 acc[M16 ? 1 : 2][M16 ? 1 : 5];
  f32x4 acc16[M16 ? 4 : 1][M16 ? 10 : 1];
#pragma unroll
  for (int i = 0; i < (M16 ? 1 : 2); ++i)
#pragma unroll
    for (int j = 0; j < (M16 ? 1 : 5); ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
#pragma unroll
  for (int i = 0; i < (M16 ? 4 : 1); ++i)
#pragma unroll
    for (int j = 0; j < (M16 ? 10 : 1); ++j) acc16[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int wm = wv % 4, wn = wv / 4, lr = lane & 31, lh = lane >> 5;
  issue(0, 0);
  if constexpr (VG) vstore(0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  prefetch(1);
  for (int kt = 0; kt < NK; ++kt) {
    const int cur = kt & 1;
    if (!IL && kt + 1 < NK) issue(kt + 1, cur ^ 1);
    prefetch(kt + 2);
    if constexpr (MF && M16) {
      // v_mfma_f32_16x16x32_bf16: per 32-deep k-step 4 A and 10 B fragments
      // (16 rows each; lane group l >> 4 holds k 8 (l >> 4) .. +7 = slot
      // 4 st + (l >> 4)), 40 MFMAs into acc16[4][10]
      const unsigned char* la = lds + cur * BUFB;
      const unsigned char* lb = la + BM * 128;
      const int l16 = lane & 15, lg = lane >> 4;
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        bf16x8 af[4], bfr[10];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = wm * 64 + i * 16 + l16;
          af[i] = *reinterpret_cast<const bf16x8*>(la + row * 128 + swz(row, 4 * st + lg) * 16);
        }
#pragma unroll
        for (int j = 0; j < 10; ++j) {
          const int row = wn * 160 + j * 16 + l16;
          bfr[j] = *reinterpret_cast<const bf16x8*>(lb + row * 128 + swz(row, 4 * st + lg) * 16);
        }
#pragma unroll
        for (int j = 0; j < 10; ++j)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            issue_at(kt + 1, cur ^ 1, st * 40 + j * 4 + i);
            acc16[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc16[i][j], 0, 0, 0);
          }
      }
    } else if constexpr (MF) {
      const unsigned char* la = lds + cur * BUFB;
      const unsigned char* lb = la + BM * 128;
#pragma unroll
      for (int st = 0; st < 4; ++st) {
        bf16x8 af[2], bfr[5];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int row = wm * 64 + i * 32 + lr;
          af[i] = *reinterpret_cast<const bf16x8*>(la + row * 128 + swz(row, 2 * st + lh) * 16);
        }
#pragma unroll
        for (int j = 0; j < 5; ++j) {
          const int row = wn * 160 + j * 32 + lr;
          bfr[j] = *reinterpret_cast<const bf16x8*>(lb + row * 128 + swz(row, 2 * st + lh) * 16);
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 5; ++j) {
            issue_at(kt + 1, cur ^ 1, st * 10 + i * 5 + j);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
          }
      }
    }
    if constexpr (VG) {
      if (kt + 1 < NK) vstore(cur ^ 1);
    }
    if constexpr (PF) {
      // everything but this iteration's prefetch (the youngest VMEM op of
      // waves 0-3) has landed; it stays in flight across the raw barrier
      if (wv < 4 && kt + 2 < NK) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < (M16 ? 1 : 2); ++i)
#pragma unroll
    for (int j = 0; j < (M16 ? 1 : 5); ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) s += acc[i][j][r];
#pragma unroll
  for (int i = 0; i < (M16 ? 4 : 1); ++i)
#pragma unroll
    for (int j = 0; j < (M16 ? 10 : 1); ++j) s += acc16[i][j][0] + acc16[i][j][1] + acc16[i][j][2] + acc16[i][j][3];
  if (!MF) s = (float)lds[(tid * 16) % (2 * BUFB)];
  if (lane == 0) out[blockIdx.x * 8 + wv] = s;
}

// The chip's sustained bf16 MFMA rate on random operands held in registers
// (no memory traffic at all): WPS waves per SIMD, each with independent
// accumulators (16 of 16x16, 4 of 32x32), for the two MFMA shapes the sweeps use.  This is the ceiling
// any bf16 sweep can reach at the clock the chip holds under that load.
template <int MF16, int WPS>
__global__ __launch_bounds__(256 * WPS, 1) void mfma_only(const uint16_t* __restrict__ seed, int iters,
                                                          float* __restrict__ out) {
  const int tid = threadIdx.x, lane = tid & 63;
  bf16x8 a, b;
  for (int e = 0; e < 8; ++e) {
    uint16_t u = seed[(blockIdx.x * 97 + tid * 8 + e) & 65535];
    uint16_t v = seed[(blockIdx.x * 31 + tid * 8 + e + 4096) & 65535];
    a[e] = __builtin_bit_cast(__bf16, u);
    b[e] = __builtin_bit_cast(__bf16, v);
  }
  float s = 0.f;
  if constexpr (MF16) {
    f32x4 acc[16];
    for (int i = 0; i < 16; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[i], 0, 0, 0);
    }
    for (int i = 0; i < 16; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  } else {
    f32x16 acc[4];
    for (int i = 0; i < 4; ++i)
      for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[i], 0, 0, 0);
    }
    for (int i = 0; i < 4; ++i)
      for (int r = 0; r < 16; ++r) s += acc[i][r];
  }
  if (lane == 0) out[blockIdx.x * 16 + (tid >> 6)] = s;
}

template <int MF16, int WPS>
static void run_mfma(const char* name, const uint16_t* seed, float* out) {
  // per wave and iteration: 16 x (16x16x32) = 262144 FLOP, 4 x (32x32x16) = 131072 FLOP
  const int iters = 20000;
  auto k = mfma_only<MF16, WPS>;
  hipLaunchKernelGGL(k, dim3(256), dim3(256 * WPS), 0, 0, seed, iters, out);
  CK(hipDeviceSynchronize());
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventRecord(a));
  for (int r = 0; r < 20; ++r) hipLaunchKernelGGL(k, dim3(256), dim3(256 * WPS), 0, 0, seed, iters, out);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  ms /= 20;
  const double flop = 256.0 * 4 * WPS * iters * (MF16 ? 262144.0 : 131072.0);
  printf("%-44s %8.3f ms  %7.1f TF/s (%.3f of 2500)\n", name, ms, flop / ms / 1e9, flop / ms / 1e9 / 2500.0);
  fflush(stdout);
}

__global__ void fill_rand(uint16_t* p, long long n, unsigned seed) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    unsigned h = (unsigned)i * 2654435761u ^ seed;
    h ^= h >> 13;
    h *= 0x5bd1e995u;
    h ^= h >> 15;
    // bf16 in +-[2^-8, 2^-6): unit-norm-like 2048-d rows
    p[i] = (uint16_t)(((h & 1) << 15) | ((119 + ((h >> 1) & 1)) << 7) | ((h >> 2) & 0x7f));
  }
}

template <int G, int Q, int MF, int VG, int ORD, int PF = 0, int M16 = 0, int IL = 0>
static void run(const char* name, const uint16_t* gal, const uint16_t* qry, int Mt, int T, float* out, int reps) {
  int nblk = Mt * T;
  if (ORD) {
    const int NR = 8 / ORD, R = (Mt + NR - 1) / NR;
    nblk = 8 * R * (T / ORD);
  }
  auto k = sweep_fill<G, Q, MF, VG, ORD, PF, M16, IL>;
  hipLaunchKernelGGL(k, dim3(nblk), dim3(NT), 0, 0, gal, qry, Mt, T, out);
  CK(hipDeviceSynchronize());
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k, dim3(nblk), dim3(NT), 0, 0, gal, qry, Mt, T, out);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  ms /= reps;
  const double tiles = (double)Mt * T;
  const double bytes = tiles * NK * ((G ? BM : 0) + (Q ? BN : 0)) * 128.0;  // LDS fill bytes
  const double flop = MF ? tiles * 2.0 * BM * BN * K : 0.0;
  printf("%-44s %8.3f ms  fill %6.2f TB/s (%5.1f GB/s per CU)  %7.1f TF/s (%.3f of 2500)\n", name, ms,
         bytes / ms / 1e9, bytes / ms / 1e6 / 256.0, flop / ms / 1e9, flop / ms / 1e9 / 2500.0);
  fflush(stdout);
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 5;
  const long long N = 1600000 - 32768, NQ = 1280;  // the C3 filter sweep's rows (seed rows excluded)
  const int Mt = (int)(N / BM), T = (int)(NQ / BN);
  uint16_t *gal, *qry;
  float* out;
  CK(hipMalloc(&gal, (size_t)Mt * BM * K * 2));
  CK(hipMalloc(&qry, (size_t)NQ * K * 2));
  CK(hipMalloc(&out, (size_t)8 * 8 * ((Mt + 7) / 8 + 8) * T * sizeof(float)));
  hipLaunchKernelGGL(fill_rand, dim3(4096), dim3(256), 0, 0, gal, (long long)Mt * BM * K, 1u);
  hipLaunchKernelGGL(fill_rand, dim3(1024), dim3(256), 0, 0, qry, NQ * K, 7u);
  CK(hipDeviceSynchronize());
  printf("C3 sweep shape: %d gallery tiles x %d query panels (256 x 320 x 2048 bf16), %d reps\n", Mt, T, reps);
  run_mfma<0, 1>("register-only MFMA 32x32x16, 1 wave/SIMD", qry, out);
  run_mfma<0, 2>("register-only MFMA 32x32x16, 2 waves/SIMD", qry, out);
  run_mfma<1, 1>("register-only MFMA 16x16x32, 1 wave/SIMD", qry, out);
  run_mfma<1, 2>("register-only MFMA 16x16x32, 2 waves/SIMD", qry, out);
  run<1, 1, 0, 0, 0>("DMA  gallery+query, no MFMA, order 0", gal, qry, Mt, T, out, reps);
  run<0, 1, 0, 0, 0>("DMA  query panel only (L2), no MFMA", gal, qry, Mt, T, out, reps);
  run<1, 0, 0, 0, 0>("DMA  gallery only (HBM), no MFMA", gal, qry, Mt, T, out, reps);
  run<1, 1, 0, 1, 0>("VGPR gallery+query, no MFMA, order 0", gal, qry, Mt, T, out, reps);
  run<0, 1, 0, 1, 0>("VGPR query panel only (L2), no MFMA", gal, qry, Mt, T, out, reps);
  run<0, 0, 1, 0, 0>("MFMA only (stale LDS operands)", gal, qry, Mt, T, out, reps);
  run<1, 1, 1, 0, 0>("DMA  + MFMA, order 0 (the sweep, no epilogue)", gal, qry, Mt, T, out, reps);
  run<1, 1, 1, 0, 2>("DMA  + MFMA, order 2 (2 panel groups)", gal, qry, Mt, T, out, reps);
  run<1, 1, 1, 0, 4>("DMA  + MFMA, order 4 (4 panel groups)", gal, qry, Mt, T, out, reps);
  run<1, 1, 0, 0, 2>("DMA  gallery+query, no MFMA, order 2", gal, qry, Mt, T, out, reps);
  run<1, 1, 0, 0, 4>("DMA  gallery+query, no MFMA, order 4", gal, qry, Mt, T, out, reps);
  run<1, 1, 1, 1, 0>("VGPR + MFMA, order 0", gal, qry, Mt, T, out, reps);
  run<0, 1, 1, 0, 0>("DMA  query only + MFMA (gallery stale)", gal, qry, Mt, T, out, reps);
  run<1, 0, 1, 0, 0>("DMA  gallery only + MFMA (queries stale)", gal, qry, Mt, T, out, reps);
  run<1, 1, 1, 0, 0, 1>("DMA  + MFMA + L2 prefetch 2 ahead, order 0", gal, qry, Mt, T, out, reps);
  run<1, 1, 1, 0, 2, 1>("DMA  + MFMA + L2 prefetch 2 ahead, order 2", gal, qry, Mt, T, out, reps);
  run<1, 1, 1, 0, 4, 1>("DMA  + MFMA + L2 prefetch 2 ahead, order 4", gal, qry, Mt, T, out, reps);
  run<1, 1, 0, 0, 0, 1>("DMA  gallery+query + L2 prefetch, no MFMA", gal, qry, Mt, T, out, reps);
  run<0, 0, 1, 0, 0, 0, 1>("16x16x32: MFMA only (stale LDS operands)", gal, qry, Mt, T, out, reps);
  run<1, 1, 1, 0, 0, 0, 1>("16x16x32: DMA + MFMA, order 0", gal, qry, Mt, T, out, reps);
  run<1, 1, 1, 0, 2, 0, 1>("16x16x32: DMA + MFMA, order 2", gal, qry, Mt, T, out, reps);
  if (argc > 2) {  // issue spread only (the r04e A/B)
    run<1, 1, 1, 0, 0>("DMA  + MFMA, burst issue (as above)", gal, qry, Mt, T, out, reps);
    run<1, 1, 1, 0, 0, 0, 0, 9>("DMA  + MFMA, issue over MFMAs 0-8", gal, qry, Mt, T, out, reps);
    run<1, 1, 1, 0, 0, 0, 0, 18>("DMA  + MFMA, issue over MFMAs 0-17", gal, qry, Mt, T, out, reps);
    run<1, 1, 1, 0, 0, 0, 0, 36>("DMA  + MFMA, issue over MFMAs 0-35", gal, qry, Mt, T, out, reps);
    run<1, 1, 1, 0, 0, 0, 1>("16x16x32: DMA + MFMA, burst issue", gal, qry, Mt, T, out, reps);
    run<1, 1, 1, 0, 0, 0, 1, 18>("16x16x32: DMA + MFMA, issue over MFMAs 0-17", gal, qry, Mt, T, out, reps);
    run<1, 1, 1, 0, 0, 0, 1, 36>("16x16x32: DMA + MFMA, issue over MFMAs 0-35", gal, qry, Mt, T, out, reps);
    run<1, 1, 1, 0, 0, 0, 1, 72>("16x16x32: DMA + MFMA, issue over MFMAs 0-71", gal, qry, Mt, T, out, reps);
  }
  CK(hipFree(gal));
  CK(hipFree(qry));
  CK(hipFree(out));
  return 0;
}
