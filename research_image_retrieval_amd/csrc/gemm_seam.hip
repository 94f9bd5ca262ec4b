// gemm_seam.hip — the seam between two bottleneck blocks as one f16x2 launch.
//
// Inside a ResNet stage the blocks chain (torchvision Bottleneck behind
// networks/backbone.py:60-109; the reference's own ResBlock /
// BottleneckTransform, networks/backbone.py:305-346):
//   y_i      = ReLU(conv3_i(h2_i) + b3 + y_{i-1})   (1x1, K = P,  N = 4P)
//   h1_{i+1} = ReLU(conv1_{i+1}(y_i) + b1)          (1x1, K = 4P, N = P)
// As two launches y_i is written by conv3 and read straight back by conv1
// (1 GB each way at 14 x 14 x 1024 and 1280 images), and each launch runs its
// own k-loop / epilogue phases.  Here one workgroup of 8 waves owns 128
// output rows and walks conv3's 4P output columns in chunks of 128:
//   - conv3 of the chunk (P deep) into a 128 x 128 accumulator, while the
//     chunk's residual rows stream by LDS-DMA into a 64 KB LDS region;
//   - the chunk epilogue: scale, bias, residual, ReLU in the accumulator
//     layout, y_i stored, and the chunk split into the f16x2 planes of
//     conv1's A operand in that same region (its own power-of-two scale: the
//     running max of the block's y rows so far, block-reduced in LDS);
//   - conv1's 128-deep slice of the chunk into the block's 128 x P conv1
//     accumulator (exactly rescaled, by a power of two, when the running max
//     grows).
// After the last chunk the conv1 epilogue (scale, bias, ReLU, max-|h1|
// record) stores h1_{i+1}.  Per 128 rows the launch moves the conv3 input
// (128 x P), the residual and y_i (128 x 4P each) and h1 (128 x P), fp32:
// y_i is never read back.
//
// Arithmetic: conv3 at P = 256 is config 12's (one accumulator,
// v_mfma_f32_32x32x16_f16, per 16-deep k-step a0b0 then a0b1 + a1b0, the
// conv3 input split at its tensor's scale; at P < 256 a0b0 and the two small
// products in separate accumulators, as configs 4 / 8) and its epilogue
// store_slab's (acc * scale + bias + residual, ReLU), so y_i is bit-identical
// to rr_conv2d_h2's conv3 on config 12 at K = 256.  conv1 runs the same k order and MFMA
// order as config 12 over K = 4P; its A pieces are split at the chunk's
// running-max scale instead of one scale per tensor.  A power-of-two scale
// moves no rounding (products of fp16 pieces are exact, fp32 sums scale
// exactly) except where a low piece falls below fp16's normal range, which a
// smaller scale makes rarer: the split never loses precision against the
// per-tensor record (tests/test_gpu_seam.py checks both outputs against
// float64 and against the two-launch path).
#include <utility>

#include "gemm_epilogue.hpp"
#include "h2_common.hpp"
#include "rr_internal.hpp"

namespace rr {

struct SeamArgs {
  const float* A3 = nullptr;         // h2_i [M][P], conv3's input
  const uint32_t* a3_amax = nullptr;  // its max-|x| record
  const float* R = nullptr;          // y_{i-1} [M][4P], the residual
  const uint16_t* W3 = nullptr;      // conv3 planes [2][4P][P] (rr_split2_f16)
  const float* w3_iscale = nullptr;  // [4P]
  const float* b3 = nullptr;         // [4P] or NULL
  const uint16_t* W1 = nullptr;      // conv1 planes [2][P][4P]
  const float* w1_iscale = nullptr;  // [P]
  const float* b1 = nullptr;         // [P] or NULL
  float* Y = nullptr;                // y_i [M][4P]
  uint32_t* y_amax = nullptr;        // optional
  float* H1 = nullptr;               // h1_{i+1} [M][P]
  uint32_t* h1_amax = nullptr;       // optional
  int M = 0;
};

template <int N>
__device__ __forceinline__ void seam_vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void seam_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
template <class F, int... Is>
__device__ __forceinline__ void seam_static_for(F&& f, std::integer_sequence<int, Is...>) {
  (f(std::integral_constant<int, Is>{}), ...);
}

// Diagnostic build only (-DRR_SEAM_PHASES=1, tools/phase_build.sh): per-wave
// s_memtime deltas of the seam kernel's phases, summed per wave role
// (0 = residual waves, 1 = loader waves) into seam_phase_sum (read by
// rr_debug_seam_phases).  Phases: 0 conv3 MFMAs, 1 DMA issue, 2 k-tile end
// wait, 3 k-tile barrier, 4 residual wait + barrier, 5 chunk epilogue,
// 6 conv1 MFMAs, 7 prologue + conv1 epilogue.
#ifndef RR_SEAM_PHASES
#define RR_SEAM_PHASES 0
#endif
#if RR_SEAM_PHASES
__device__ unsigned long long seam_phase_sum[2][8];
#define SP_DECL unsigned long long sp_t = __builtin_amdgcn_s_memtime(), sp_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#define SP(i)                                                   \
  do {                                                          \
    const unsigned long long sp_n = __builtin_amdgcn_s_memtime(); \
    sp_acc[i] += sp_n - sp_t;                                   \
    sp_t = sp_n;                                                \
  } while (0)
#define SP_FLUSH(role)                                                              \
  do {                                                                              \
    if ((threadIdx.x & 63) == 0)                                                    \
      for (int i = 0; i < 8; ++i) atomicAdd(&seam_phase_sum[role][i], sp_acc[i]);   \
  } while (0)
#else
#define SP_DECL
#define SP(i) ((void)0)
#define SP_FLUSH(role) ((void)0)
#endif

// the fp32 chunk's granule swizzle (gemm_seam.hip dma_res)
__device__ __forceinline__ int rsw(int row) { return ((row >> 2) & 3) << 2; }

template <int P>
__global__ __launch_bounds__(512, 1) void seam_h2_kernel(SeamArgs a) {
  static_assert(P == 64 || P == 128 || P == 256, "planes");
  typedef f16x8 frag_t;
  constexpr int BM = 128, CW = 128;      // rows per workgroup, conv3 columns per chunk
  constexpr int N3 = 4 * P;              // conv3 output channels = conv1 input channels
  constexpr int NC = N3 / CW;            // chunks
  constexpr int NK3 = P / 32;            // conv3 k-tiles per chunk
  constexpr int NK1 = CW / 32;           // conv1 k-tiles per chunk
  // conv1's 128 x P output: 2 x 4 waves of 64 x P/4 (P = 64: 4 x 2 waves of 32 x 32)
  constexpr int WM1 = P == 64 ? 4 : 2;
  constexpr int FM1 = BM / (32 * WM1);
  constexpr int FN1 = P / (32 * (8 / WM1));
  static_assert(FN1 >= 1 && 32 * FN1 * (8 / WM1) == P, "conv1 wave columns");
  constexpr int NB3 = 4;                 // conv3 B DMA per loader wave: 2 planes x 128 rows x 64 B = 16 KB / 4 waves
  constexpr int NB1 = P / 32;            // conv1 B DMA per loader wave: 2 planes x P rows x 64 B / 4 waves
  constexpr int NR = 16;                 // residual DMA per residual wave per chunk: 64 KB / 4 waves
  // conv3 at K = P < 256: a0b0 and a0b1 + a1b0 in two accumulators, as configs
  // 4 / 8 keep them (one measured up to 1.27x the exact-fp32 core's error at
  // K = 64, profiles/r03j_acc1_ab.txt)
  constexpr bool ACC2 = P < 256;
  // LDS (16-bit units): [0, 32768) the chunk region (fp32 residual -> y ->
  // conv1's A planes [NK1][2][128][32]); NS 32 KB stages (conv3's B planes
  // [2][128][32] or conv1's [2][P][32]); the epilogue's 8 block-max words go
  // in the stage its chunk's last conv3 k-tile has released
  // NS stages: three (the weight DMA two k-tiles ahead) when a chunk's
  // k-tiles divide by three, so every chunk starts on stage 0; else two
  constexpr int NS = (NK3 + NK1) % 3 == 0 ? 3 : 2;
  constexpr int A1 = 0, STG = 32768, STG_SZ = 16384;
  static_assert(2 * P * 32 <= STG_SZ, "conv1 B tile must fit a stage");
  __shared__ __attribute__((aligned(16))) uint16_t lds[STG + NS * STG_SZ];
  float* const lds_f = reinterpret_cast<float*>(lds);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // roles: waves 4-7 issue every weight DMA (their counter holds nothing
  // else, so each k-tile waits only for its own short L2 fetch); waves 0-3
  // issue the chunk's residual rows (HBM) at the chunk's start and wait for
  // them only before its epilogue.  A workgroup's waves 0-3 land on four
  // different SIMDs, and so do 4-7: every SIMD pairs one of each.
  const bool ldw = wave >= 4;
  const int lw = wave & 3;
  const int l16 = lane & 15, lg = lane >> 4;     // 16x16x32 lane roles
  const int lr = lane & 31, lh = lane >> 5;      // 32x32x16 lane roles
  const int wm1 = wave % WM1, wn1 = wave / WM1;  // conv1 wave grid
  const int M = a.M, m0 = blockIdx.x * BM;
  SP_DECL

  // ---- conv3's A: wave w's 16 rows x P, split once into 16x16x32 fragments
  // held in registers for every chunk (lane: row 16 w + l16, k 32 q + 8 lg ..
  // +7); rows past M clamped to row M - 1 (never stored: they duplicate row
  // M - 1 and leave every max unchanged) ----
  frag_t a3f[NK3][2];
  float a_isc;
  {
    const uint32_t a3_w = amax_load_slot(a.a3_amax);
    const float* ap = a.A3 + (long long)min(m0 + 16 * wave + l16, M - 1) * P + 8 * lg;
    const int e = __builtin_amdgcn_readfirstlane(h2_exp(amax_reduce(a3_w)));
    const float sc = __int_as_float((127 + e) << 23);
    a_isc = __int_as_float((127 - e) << 23);
#pragma unroll
    for (int q = 0; q < NK3; ++q) {
      f32x4 ra[2];
      ra[0] = *reinterpret_cast<const f32x4*>(ap + 32 * q);
      ra[1] = *reinterpret_cast<const f32x4*>(ap + 32 * q + 4);
      u32x4 p0, p1;
      split2h8(ra, sc, p0, p1);
      a3f[q][0] = __builtin_bit_cast(frag_t, p0);
      a3f[q][1] = __builtin_bit_cast(frag_t, p1);
    }
  }

  // ---- weight DMA (loader waves): conv3 B (chunk c, k-tile q) = plane-rows
  // 16 (4 i + lw) + lane / 4 of [2][128] (plane = row / 128); conv1 B (chunk
  // c, k-tile t) = plane-rows of [2][P] ----
  auto dma_b3 = [&](int c, int q, int st) __attribute__((always_inline)) {
    const int ln = s3_opaque(lane);
#pragma unroll
    for (int i = 0; i < NB3; ++i) {
      const int pr = (4 * i + lw) * 16 + (ln >> 2);
      const int p = pr >> 7, r = pr & 127;
      const uint16_t* src =
          a.W3 + (long long)p * N3 * P + (long long)(CW * c + r) * P + 32 * q + pswz<32, 2>(r, ln & 3) * 8;
      __builtin_amdgcn_global_load_lds((const void*)src,
                                       (__attribute__((address_space(3))) void*)(lds + STG + st * STG_SZ + (4 * i + lw) * 512),
                                       16, 0, 0);
    }
  };
  auto dma_b1 = [&](int c, int t, int st) __attribute__((always_inline)) {
    const int ln = s3_opaque(lane);
#pragma unroll
    for (int i = 0; i < NB1; ++i) {
      const int pr = (4 * i + lw) * 16 + (ln >> 2);
      const int p = pr / P, r = pr - p * P;
      const uint16_t* src =
          a.W1 + (long long)p * P * N3 + (long long)r * N3 + CW * c + 32 * t + pswz<32, 2>(r, ln & 3) * 8;
      __builtin_amdgcn_global_load_lds((const void*)src,
                                       (__attribute__((address_space(3))) void*)(lds + STG + st * STG_SZ + (4 * i + lw) * 512),
                                       16, 0, 0);
    }
  };
  // ---- the chunk's residual rows (residual waves): fp32 [128][128] in the
  // chunk region, instruction i of wave lw = rows 2 (4 i + lw) + {0, 1} ----
  // (addresses from an opaque base, recomputed per chunk: hoisted out of
  // the chunk loop, the 16 per-lane pointers were spilled)
  // Granule swizzle of the fp32 chunk: 16-B granule g of row r sits at
  // g ^ rsw(r) (rows 4 apart in different 16-bank windows: the epilogue's
  // accumulator-layout reads are conflict-free); the DMA moves it on the
  // source side (its LDS destination is lane-linear).
  auto dma_res = [&](int c) __attribute__((always_inline)) {
    const int rb = s3_opaque(m0 + 2 * lw + lh);
    const float* base = a.R + CW * c;
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      const int row = 2 * (4 * i + lw) + lh;  // local row
      const float* src = base + (long long)min(rb + 8 * i, M - 1) * N3 + 4 * (lr ^ rsw(row));
      __builtin_amdgcn_global_load_lds((const void*)src,
                                       (__attribute__((address_space(3))) void*)(lds + A1 + 2 * (4 * i + lw) * 256), 16,
                                       0, 0);
    }
  };

  // ---- accumulators ----
  f32x4 acc3[8], acc3lo[ACC2 ? 8 : 1];
  f32x16 acc1[FM1][FN1];
#pragma unroll
  for (int i = 0; i < FM1; ++i)
#pragma unroll
    for (int j = 0; j < FN1; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc1[i][j][r] = 0.f;

  // conv3 k-tile q from stage st: wave w = rows 16 w + [0, 16) x the chunk's
  // 128 columns (eight 16x16 tiles), A from registers, B from LDS
  auto mma3 = [&](int q, int st) __attribute__((always_inline)) {
    const uint16_t* lb = lds + STG + st * STG_SZ;
#pragma unroll
    for (int n = 0; n < 8; ++n) {
      const int row = 16 * n + l16;
      const frag_t b0 = *reinterpret_cast<const frag_t*>(lb + row * 32 + pswz<32, 2>(row, lg) * 8);
      const frag_t b1 = *reinterpret_cast<const frag_t*>(lb + (128 + row) * 32 + pswz<32, 2>(row, lg) * 8);
      acc3[n] = s3_mf16<2>(a3f[q][0], b0, acc3[n]);
      f32x4& L = ACC2 ? acc3lo[ACC2 ? n : 0] : acc3[n];
      L = s3_mf16<2>(a3f[q][0], b1, L);
      L = s3_mf16<2>(a3f[q][1], b0, L);
    }
    // the reads one column tile ahead of its MFMAs (two tiles' fragments live)
    __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);  // DS read: tiles 0, 1
#pragma unroll
    for (int n = 0; n < 6; ++n) {
      __builtin_amdgcn_sched_group_barrier(0x008, 3, 0);  // tile n's MFMAs
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);  // tile n + 2's reads
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 6, 0);
  };
  // conv1 k-tile t: A from the chunk region's planes, B from stage st
  auto mma1 = [&](int t, int st) __attribute__((always_inline)) {
    const uint16_t* la = lds + A1 + t * (2 * 128 * 32);
    const uint16_t* lb = lds + STG + st * STG_SZ;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      frag_t fa[2][FM1], fb[2][FN1];
#pragma unroll
      for (int p = 0; p < 2; ++p) {
#pragma unroll
        for (int i = 0; i < FM1; ++i) {
          const int row = wm1 * 32 * FM1 + i * 32 + lr;
          fa[p][i] = *reinterpret_cast<const frag_t*>(la + (p * 128 + row) * 32 + pswz<32, 2>(row, 2 * s + lh) * 8);
        }
#pragma unroll
        for (int j = 0; j < FN1; ++j) {
          const int row = wn1 * 32 * FN1 + j * 32 + lr;
          fb[p][j] = *reinterpret_cast<const frag_t*>(lb + (p * P + row) * 32 + pswz<32, 2>(row, 2 * s + lh) * 8);
        }
      }
#pragma unroll
      for (int i = 0; i < FM1; ++i)
#pragma unroll
        for (int j = 0; j < FN1; ++j) acc1[i][j] = s3_mf32<2>(fa[0][i], fb[0][j], acc1[i][j]);
#pragma unroll
      for (int i = 0; i < FM1; ++i)
#pragma unroll
        for (int j = 0; j < FN1; ++j) {
          acc1[i][j] = s3_mf32<2>(fa[0][i], fb[1][j], acc1[i][j]);
          acc1[i][j] = s3_mf32<2>(fa[1][i], fb[0][j], acc1[i][j]);
        }
    }
  };

  float run_max = 0.f;  // max |y| of the block's rows so far (finite values)
  int e_prev = 0;       // conv1's A scale exponent the accumulator holds
  float y_am = 0.f;     // y's max for its record

  // ---- chunk epilogue: y = ReLU(acc3 scale + b3 + residual), stored, split
  // into conv1's A planes.  Entered after the barrier that ends the chunk's
  // last conv3 k-tile, behind the residual waves' wait for their DMA ----
  // the stage the chunk's last conv3 k-tile released: the block-max words
  constexpr int AMX_F = (STG + ((NK3 - 1) % NS) * STG_SZ) / 2;
  auto epi3 = [&](int c) __attribute__((always_inline)) {
    float am = 0.f;
#pragma unroll
    for (int n = 0; n < 8; ++n) {
      const int col = 16 * n + l16;
      const float sc = a.w3_iscale[CW * c + col] * a_isc;
      const float bb = a.b3 != nullptr ? a.b3[CW * c + col] : 0.f;
      f32x4 v = acc3[n];
      if constexpr (ACC2) v += acc3lo[n];
      float rv[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * wave + 4 * lg + r;
        rv[r] = lds_f[row * CW + 4 * ((col >> 2) ^ rsw(row)) + (col & 3)];
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * wave + 4 * lg + r;
        float x = v[r] * sc;
        x += bb;
        x += rv[r];
        x = fmaxf(x, 0.f);
        am = amax_acc(am, x);
        lds_f[row * CW + 4 * ((col >> 2) ^ rsw(row)) + (col & 3)] = x;
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) am = __builtin_fmaxf(am, __shfl_xor(am, o));
    if (lane == 0) lds_f[AMX_F + wave] = am;
    seam_barrier();
    // row-contiguous: thread = (row r0 + 16 it, columns 4 c4 .. + 3)
    // (s3_opaque: recomputed here, not hoisted and held through the k-loop)
    const int te = s3_opaque(tid);
    const int c4 = te & 31, r0 = te >> 5;
    f32x4 yv[8];
#pragma unroll
    for (int it = 0; it < 8; ++it) {
      const int row = r0 + 16 * it;
      yv[it] = *reinterpret_cast<const f32x4*>(lds_f + row * CW + 4 * (c4 ^ rsw(row)));
    }
    float bm = lds_f[AMX_F];
#pragma unroll
    for (int w = 1; w < 8; ++w) bm = __builtin_fmaxf(bm, lds_f[AMX_F + w]);
    y_am = __builtin_fmaxf(y_am, bm);
    run_max = __builtin_fmaxf(run_max, bm);
    // y stored by the residual waves only (their counter holds nothing the
    // k-loop waits on): rows r0 + 16 it of their own and r0 + 8 + 16 it
    if (!ldw) {
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        const int m = m0 + r0 + 16 * it;
        if (m < M) *reinterpret_cast<f32x4*>(a.Y + (long long)m * N3 + CW * c + c4 * 4) = yv[it];
      }
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        const int row = r0 + 8 + 16 * it, m = m0 + row;
        const f32x4 v2 = *reinterpret_cast<const f32x4*>(lds_f + row * CW + 4 * (c4 ^ rsw(row)));
        if (m < M) *reinterpret_cast<f32x4*>(a.Y + (long long)m * N3 + CW * c + c4 * 4) = v2;
      }
    }
    const int e = __builtin_amdgcn_readfirstlane(h2_exp(run_max));
    const float ysc = __int_as_float((127 + e) << 23);
    seam_barrier();  // every read of the fp32 chunk done
    // the chunk as conv1's A planes: k-tile c4 / 8, 8-B half (c4 & 1) of slot (c4 & 7) / 2
    {
      const int t = c4 >> 3, slot = (c4 & 7) >> 1, half = c4 & 1;
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        const int row = r0 + 16 * it;
        uint32_t h[2], l[2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const f32x2 v = f32x2{yv[it][2 * q], yv[it][2 * q + 1]} * ysc;
          const f16x2 hh = __builtin_convertvector(v, f16x2);
          const f16x2 ll = __builtin_convertvector(v - __builtin_convertvector(hh, f32x2), f16x2);
          h[q] = __builtin_bit_cast(uint32_t, hh);
          l[q] = __builtin_bit_cast(uint32_t, ll);
        }
        uint16_t* dst = lds + A1 + t * (2 * 128 * 32) + row * 32 + pswz<32, 2>(row, slot) * 8 + half * 4;
        *reinterpret_cast<uint2*>(dst) = uint2{h[0], h[1]};
        *reinterpret_cast<uint2*>(dst + 128 * 32) = uint2{l[0], l[1]};
      }
    }
    // conv1's accumulator moves to the new scale exactly (e <= e_prev: the max only grows)
    if (c > 0 && e != e_prev) {
#pragma unroll
      for (int i = 0; i < FM1; ++i)
#pragma unroll
        for (int j = 0; j < FN1; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc1[i][j][r] = __builtin_amdgcn_ldexpf(acc1[i][j][r], e - e_prev);
    }
    e_prev = e;
    seam_barrier();
  };

  // ---- conv1 epilogue (after the last chunk; nothing in flight but the
  // last y stores): ReLU(acc1 scale + b1) staged [128][P] fp32, stored
  // row-contiguous ----
  auto epi1 = [&]() __attribute__((always_inline)) {
    const float isc = __int_as_float((127 - e_prev) << 23);
    float am = 0.f;
#pragma unroll
    for (int j = 0; j < FN1; ++j) {
      const int col = wn1 * 32 * FN1 + j * 32 + lr;
      const float sc = a.w1_iscale[col] * isc;
      const float bb = a.b1 != nullptr ? a.b1[col] : 0.f;
#pragma unroll
      for (int i = 0; i < FM1; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = wm1 * 32 * FM1 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
          float v = acc1[i][j][r] * sc;
          v += bb;
          v = fmaxf(v, 0.f);
          am = amax_acc(am, v);
          lds_f[row * P + col] = v;
        }
    }
    if (a.h1_amax != nullptr) amax_publish(a.h1_amax, am, blockIdx.x * 8 + wave);
    seam_barrier();
    constexpr int C4 = P / 4, RP = 512 / C4;  // float4 per row, rows per pass
    const int te = s3_opaque(tid);
    const int c4 = te % C4, r0 = te / C4;
#pragma unroll
    for (int it = 0; it < BM / RP; ++it) {
      const int row = r0 + RP * it, m = m0 + row;
      if (m < M)
        *reinterpret_cast<f32x4*>(a.H1 + (long long)m * P + c4 * 4) =
            *reinterpret_cast<const f32x4*>(lds_f + row * P + c4 * 4);
    }
  };

  // ---- the k-stream: per chunk NK3 conv3 k-tiles, the chunk epilogue, NK1
  // conv1 k-tiles; stage = position & 1 (a chunk starts on stage 0).  A
  // loader wave issues the next k-tile's weight DMA at the top of each
  // k-tile and waits for it (vmcnt 0: nothing else is in its counter) before
  // the k-tile's closing barrier ----
  // position k of chunk c (0 .. NK3 + NK1 - 1; the next chunk's 0, 1 past
  // the end): its weight DMA into stage (k % NS)
  auto dma_pos = [&](int c, int k) __attribute__((always_inline)) {
    if (k < NK3) dma_b3(c, k, k % NS);
    else if (k < NK3 + NK1) dma_b1(c, k - NK3, k % NS);
    else if (c + 1 < NC) dma_b3(c + 1, k - NK3 - NK1, k % NS);
  };
  // ---- the k-stream: per chunk NK3 conv3 k-tiles, the chunk epilogue, NK1
  // conv1 k-tiles on a ring of NS stages (a chunk starts on stage 0).  A
  // loader wave issues position k + NS - 1's weight DMA at the top of k-tile
  // k and waits for k + 1's (counted vmcnt: only its own DMA are in its
  // counter) before the k-tile's closing barrier ----
  auto chunk = [&](int c) __attribute__((always_inline)) {
    const bool last = c + 1 == NC;
#pragma unroll
    for (int n = 0; n < 8; ++n) {
      acc3[n] = f32x4{0.f, 0.f, 0.f, 0.f};
      if constexpr (ACC2) acc3lo[n] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    // the chunk region is free (the previous chunk's conv1 ended on a barrier)
    if (!ldw) dma_res(c);
    SP(1);
    auto kstep = [&](auto kc) __attribute__((always_inline)) {
      constexpr int k = decltype(kc)::value;
      constexpr int ahead = k + NS - 1;  // the position whose DMA goes out now
      constexpr bool crosses = ahead >= NK3 + NK1;
      if (ldw) dma_pos(c, ahead);
      SP(1);
      if constexpr (k < NK3) {
        mma3(k, k % NS);
        SP(0);
      } else {
        mma1(k - NK3, k % NS);
        SP(6);
      }
      if (ldw) {
        // every DMA but the one just issued has landed (position k + 1's)
        if constexpr (NS == 3) {
          if (crosses && last) seam_vm_wait<0>();
          else seam_vm_wait<(ahead < NK3 ? NB3 : ahead < NK3 + NK1 ? NB1 : NB3)>();
        } else {
          seam_vm_wait<0>();
        }
      }
      SP(2);
      seam_barrier();
      SP(3);
      if constexpr (k == NK3 - 1) {
        if (!ldw) seam_vm_wait<0>();  // the residual rows (and this wave's older y stores)
        seam_barrier();
        SP(4);
        epi3(c);
        SP(5);
      }
    };
    seam_static_for(kstep, std::make_integer_sequence<int, NK3 + NK1>{});
  };

  // ---- prologue: the first NS - 1 positions' weight DMA (the A fragments are loaded above) ----
  if (ldw) {
    dma_pos(0, 0);
    if constexpr (NS == 3) {
      dma_pos(0, 1);
      seam_vm_wait<NB3>();
    } else {
      seam_vm_wait<0>();
    }
  }
  seam_barrier();
  SP(7);
#pragma unroll 1
  for (int c = 0; c < NC; ++c) chunk(c);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  epi1();
  if (a.y_amax != nullptr) amax_publish(a.y_amax, y_am, blockIdx.x * 8 + wave);
  SP(7);
  SP_FLUSH(ldw ? 1 : 0);
}

static int launch_seam_h2(rr_handle_s* h, const SeamArgs& a, int planes, hipStream_t s, int timer_cls) {
  if (a.M == 0) return RR_OK;
  const unsigned grid = (unsigned)((a.M + 127) / 128);
  hipError_t e;
  {
    TimedLaunch tl(h, timer_cls, s);
    switch (planes) {
      case 64: hipLaunchKernelGGL(seam_h2_kernel<64>, dim3(grid), dim3(512), 0, s, a); break;
      case 128: hipLaunchKernelGGL(seam_h2_kernel<128>, dim3(grid), dim3(512), 0, s, a); break;
      default: hipLaunchKernelGGL(seam_h2_kernel<256>, dim3(grid), dim3(512), 0, s, a); break;
    }
    e = hipGetLastError();
  }
  return check_hip(h, e, "seam_h2 launch");
}

}  // namespace rr

using namespace rr;

extern "C" int rr_bottleneck_seam_h2(rr_handle_t h, const float* y2, const unsigned* y2_amax, int m, int planes,
                                     const float* res, const void* w3, const float* w3_iscale, const float* b3,
                                     const void* w1, const float* w1_iscale, const float* b1, float* out,
                                     unsigned* out_amax, float* h1, unsigned* h1_amax, void* stream) {
  RR_ENTRY(h);
  if (m < 0 || (planes != 64 && planes != 128 && planes != 256))
    return set_error(h, RR_EINVAL, "rr_bottleneck_seam_h2: m >= 0 and planes 64, 128 or 256");
  if (m == 0) return RR_OK;  // (empty tensors may carry NULL pointers)
  if (!y2 || !y2_amax || !res || !w3 || !w3_iscale || !w1 || !w1_iscale || !out || !h1)
    return set_error(h, RR_EINVAL, "rr_bottleneck_seam_h2: bad argument");
  const void* ptrs[] = {y2, res, w3, w3_iscale, w1, w1_iscale, out, h1, b3, b1};
  for (const void* p : ptrs)
    if ((uintptr_t)p & 15) return set_error(h, RR_EINVAL, "rr_bottleneck_seam_h2: pointers must be 16-byte aligned");
  if (((uintptr_t)y2_amax & 3) || ((uintptr_t)out_amax & 3) || ((uintptr_t)h1_amax & 3))
    return set_error(h, RR_EINVAL, "rr_bottleneck_seam_h2: max-|x| records must be 4-byte aligned");
  SeamArgs a;
  a.A3 = y2;
  a.a3_amax = y2_amax;
  a.R = res;
  a.W3 = reinterpret_cast<const uint16_t*>(w3);
  a.w3_iscale = w3_iscale;
  a.b3 = b3;
  a.W1 = reinterpret_cast<const uint16_t*>(w1);
  a.w1_iscale = w1_iscale;
  a.b1 = b1;
  a.Y = out;
  a.y_amax = out_amax;
  a.H1 = h1;
  a.h1_amax = h1_amax;
  a.M = m;
  return launch_seam_h2(h, a, planes, (hipStream_t)stream, kTimeGemm);
}

#if RR_SEAM_PHASES
extern "C" int rr_debug_seam_phases(unsigned long long* out) {
  // out[16] <- seam_phase_sum (residual waves 0-7, loader waves 8-15), then cleared
  unsigned long long h[16] = {};
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(rr::seam_phase_sum), sizeof(h)) != hipSuccess) return RR_EHIP;
  for (int i = 0; i < 16; ++i) out[i] = h[i];
  const unsigned long long z[16] = {};
  return hipMemcpyToSymbol(HIP_SYMBOL(rr::seam_phase_sum), z, sizeof(z)) == hipSuccess ? RR_OK : RR_EHIP;
}
#endif
