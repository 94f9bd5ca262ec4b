// gemm_8p.hip — bf16 GEMM on a 256x256 tile with an 8-phase LDS-DMA pipeline
// (cdna_hip_programming.md §5 'The 256² 8-phase template') for the long-K
// cosine sweeps (iris_evaluate.py:383): the filter epilogue (survivors above
// each query's threshold) and the transposed score store of the seed pass.
// Measured (tools/sweep_ab.py, profiles/r02c_sweep_ab.txt): 1.22-1.25x the
// 256x320 sweep tile at 256 / 512 / 768 queries x 1.6 M x 2048, 1.03x at 1280;
// on the ViT linears (K = 768, stored C) it was 2-4 % slower than gemm_f32.hip's
// 256x256 tile, so stored-C GEMMs do not come here.
//
// C[M,N] = A[M,K] . B[N,K]^T, bf16 in, fp32 accumulate, K % 128 == 0.
// LDS: two k-tile buffers, each four 16 KB half-tiles (A rows 0-127, A rows
// 128-255, B rows 0-127, B rows 128-255) of 128-B rows (64 bf16 = one k-tile),
// 16-B slots XOR-swizzled by (row >> 1) & 7.  A k-tile is computed in four
// phases, one 128x128 block quadrant each, in the order (A0,B0), (A0,B1),
// (A1,B1), (A1,B0): every phase reads one A half and/or one B half from LDS
// into registers, so each half-tile's last read is at a known phase and it can
// be restaged two phases later.  8 waves (2 x 4) each own a 64x32 piece of
// every quadrant (16 MFMAs of 16x16x32 per phase).
//
// Two k-tiles per iteration (phases P1..P8; even buffer in P1-P4, odd in
// P5-P8).  Each phase issues exactly one half-tile (two global_load_lds per
// thread):  P1: A1 of tile 2j+1, P2: B0 of 2j+1, P3: A0 of 2j+2, P4: B1 of
// 2j+2, P5: A1 of 2j+2, P6: B0 of 2j+2, P7: A0 of 2j+3, P8: B1 of 2j+3 (tile
// indices clamped to nk-1; a clamped copy lands in a half nobody reads again).
// Every restage is >= 2 phases after that half's last ds_read (WAR).  RAW:
// P4 waits vmcnt(4) (everything up to P2's loads landed: tile 2j+1 complete),
// read from P5 on; P8 waits vmcnt(4) (up to P6: tile 2j+2 complete), read from
// the next P1.  The counted waits never drain to 0 inside the loop, so the
// DMA stays in flight across the raw barriers.
//
// fp8 (OCP e4m3, DT_FP8; the C5 sweep): the same 128-B rows hold 128 k.  A
// wave's 64x32 piece of a quadrant is two 32x32 tiles on the block-scaled
// v_mfma_scale_f32_32x32x64_f8f6f4 with unit E8M0 scales (the rows' fp32
// scales are applied to the accumulator in the epilogue, as gemm_f32.hip's
// fp8 tiles do), two 64-deep k-steps per k-tile: 4 MFMAs per phase, each
// twice the cycles of the bf16 32x32x16 at 4x the k, so the phase is as long
// as the bf16 phase over the same LDS bytes.  Lane half h holds the 32 bytes
// of 16-B slots 4 step + 2h, +1 (gemm_f32.hip's fp8 reads); A and B use the
// same lane -> k map, so each dot product covers every k once.  (The
// 16x16x128 form of this tile left the compiler copying its accumulators and
// spilling, 68-128 B per lane, which broke the counted waits.)
#include "gemm_epilogue.hpp"
#include "rr_internal.hpp"

namespace rr {

namespace {

constexpr int P8_HALF = 128 * 128;  // bytes per half-tile (128 rows x 128 B)

__device__ __forceinline__ int swz8(int row, int slot) { return slot ^ ((row >> 1) & 7); }

template <int EM, int DT>
__global__ __launch_bounds__(512, 1) void gemm_8p_kernel(GemmArgs g, int tiles_n) {
  constexpr bool F8 = DT == DT_FP8;
  constexpr int EPR = F8 ? 128 : 64;  // elements per 128-B row (k per k-tile)
  __shared__ __attribute__((aligned(16))) unsigned char lds[8 * P8_HALF];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave & 1, wc = wave >> 1;  // 2 x 4 waves: 64 rows x 32 cols per quadrant
  const int l16 = lane & 15, lg = lane >> 4;

  // XCD-aware block -> tile order (rr_internal.hpp tile_coords)
  int tm, tn;
  tile_coords(blockIdx.x, gridDim.x, tiles_n, tm, tn);
  const int m0 = tm * 256, n0 = tn * 256;
  const int nk = g.K / EPR;  // even (K % (2 EPR) == 0, checked on the host)

  // LDS-DMA sources: instruction i of wave w fills rows (i*8 + w)*8 .. +7 of a
  // half, lane l -> row + l/8, physical slot l%8 (logical slot swz8 of it)
  const unsigned char* src[4][2];
#pragma unroll
  for (int h = 0; h < 4; ++h)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = (i * 8 + wave) * 8 + (lane >> 3);
      const bool isa = h < 2;
      const int row = (isa ? m0 : n0) + (h & 1) * 128 + r;
      const int lim = (isa ? g.M : g.N) - 1;
      const unsigned char* base = reinterpret_cast<const unsigned char*>(isa ? g.A : g.B);
      src[h][i] = base + ((long long)min(row, lim) * (isa ? g.lda : g.ldb)) * (F8 ? 1 : 2) + swz8(r, lane & 7) * 16;
    }
  auto stage = [&](int h, int kt, int buf) {
    const int t = min(kt, nk - 1);
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_global_load_lds(
          (const void*)(src[h][i] + (long long)t * 128),
          (__attribute__((address_space(3))) void*)(lds + (buf * 4 + h) * P8_HALF + (i * 8 + wave) * 8 * 128), 16, 0, 0);
  };

  f32x4 acc[F8 ? 1 : 4][4][2];  // bf16: [quadrant][16-row group][16-col group]
  f32x16 acc8[F8 ? 4 : 1][2];    // fp8: [quadrant][32-row tile]
#pragma unroll
  for (int q = 0; q < (F8 ? 1 : 4); ++q)
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) acc[q][a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int q = 0; q < (F8 ? 4 : 1); ++q)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc8[q][i][r] = 0.f;
  const int l32 = lane & 31, lh = lane >> 5;
  // fragments, 8 registers each.  bf16: fa[mg] / fb[ng] = 16-B slots lg (k-step
  // 0) and 4 + lg (k-step 1) of row l16 of a 16-row group; fp8: fa[2 i + st] /
  // fb[st] = the 32 bytes of k-step st of row l32 of 32-row tile i
  i32x8 fa[4], fb[2];
  auto rd32 = [&](const unsigned char* base, int row, int s0, int s1) {
    const i32x4 x = *reinterpret_cast<const i32x4*>(base + row * 128 + swz8(row, s0) * 16);
    const i32x4 y = *reinterpret_cast<const i32x4*>(base + row * 128 + swz8(row, s1) * 16);
    return __builtin_shufflevector(x, y, 0, 1, 2, 3, 4, 5, 6, 7);
  };

  auto read_a = [&](int buf, int ha) {
    const unsigned char* base = lds + (buf * 4 + ha) * P8_HALF;
    if constexpr (F8) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int st = 0; st < 2; ++st) fa[2 * i + st] = rd32(base, wr * 64 + i * 32 + l32, 4 * st + 2 * lh, 4 * st + 2 * lh + 1);
    } else {
#pragma unroll
      for (int mg = 0; mg < 4; ++mg) fa[mg] = rd32(base, wr * 64 + mg * 16 + l16, lg, 4 + lg);
    }
  };
  auto read_b = [&](int buf, int hb) {
    const unsigned char* base = lds + (buf * 4 + 2 + hb) * P8_HALF;
    if constexpr (F8) {
#pragma unroll
      for (int st = 0; st < 2; ++st) fb[st] = rd32(base, wc * 32 + l32, 4 * st + 2 * lh, 4 * st + 2 * lh + 1);
    } else {
#pragma unroll
      for (int ng = 0; ng < 2; ++ng) fb[ng] = rd32(base, wc * 32 + ng * 16 + l16, lg, 4 + lg);
    }
  };
  auto half_bf = [](const i32x8& v, int s) {
    const i32x4 h = s ? __builtin_shufflevector(v, v, 4, 5, 6, 7) : __builtin_shufflevector(v, v, 0, 1, 2, 3);
    return __builtin_bit_cast(bf16x8, h);
  };
  auto mfma_q = [&](int q) {
    __builtin_amdgcn_s_setprio(1);
    if constexpr (F8) {
#pragma unroll
      for (int st = 0; st < 2; ++st)
#pragma unroll
        for (int i = 0; i < 2; ++i)
          acc8[q][i] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(fa[2 * i + st], fb[st], acc8[q][i], 0, 0, 0, 127,
                                                                       0, 127);
    } else {
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int mg = 0; mg < 4; ++mg)
#pragma unroll
          for (int ng = 0; ng < 2; ++ng)
            acc[q][mg][ng] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(half_bf(fa[mg], s), half_bf(fb[ng], s),
                                                                     acc[q][mg][ng], 0, 0, 0);
    }
    __builtin_amdgcn_s_setprio(0);
  };
  auto sync_mid = [&]() {
    __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  };
  auto sync_end = [&]() {
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  // prologue: tile 0 (even) whole, then A0 and B1 of tile 1 (as P7/P8 would)
  stage(0, 0, 0);
  stage(1, 0, 0);
  stage(2, 0, 0);
  stage(3, 0, 0);
  stage(0, 1, 1);
  stage(3, 1, 1);
  asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // tile 0 landed
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  for (int kt = 0; kt < nk; kt += 2) {
    // P1: (A0,B0) of the even tile
    read_a(0, 0);
    read_b(0, 0);
    stage(1, kt + 1, 1);
    sync_mid();
    mfma_q(0);
    sync_end();
    // P2: (A0,B1)
    read_b(0, 1);
    stage(2, kt + 1, 1);
    sync_mid();
    mfma_q(1);
    sync_end();
    // P3: (A1,B1)
    read_a(0, 1);
    stage(0, kt + 2, 0);
    sync_mid();
    mfma_q(2);
    sync_end();
    // P4: (A1,B0); the odd tile kt+1 has landed once P2's loads have
    read_b(0, 0);
    stage(3, kt + 2, 0);
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    sync_mid();
    mfma_q(3);
    sync_end();
    // P5-P8: the odd tile
    read_a(1, 0);
    read_b(1, 0);
    stage(1, kt + 2, 0);
    sync_mid();
    mfma_q(0);
    sync_end();
    read_b(1, 1);
    stage(2, kt + 2, 0);
    sync_mid();
    mfma_q(1);
    sync_end();
    read_a(1, 1);
    stage(0, kt + 3, 1);
    sync_mid();
    mfma_q(2);
    sync_end();
    read_b(1, 0);
    stage(3, kt + 3, 1);
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // tile kt+2 landed (P6's loads)
    sync_mid();
    mfma_q(3);
    sync_end();
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // the epilogue reuses the LDS

  // acc[q][mg][ng][e]: row = qa*128 + wr*64 + mg*16 + 4*lg + e, col = qb*128 + wc*32 + ng*16 + l16
  constexpr int QA[4] = {0, 0, 1, 1}, QB[4] = {0, 1, 1, 0};
  if constexpr (F8) {
    // acc8[q][i][r]: row = qa*128 + wr*64 + 32 i + (r & 3) + 8 (r >> 2) + 4 lh,
    // col = qb*128 + wc*32 + l32; the rows' fp32 scales first (gemm_f32.hip's
    // fp8 order: acc * s_a * s_b), one quadrant at a time (all at once spilled)
    const bool scaled = g.scale_a != nullptr || g.scale_b != nullptr;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int n = n0 + QB[q] * 128 + wc * 32 + l32;
      const bool nok = n < g.N;
      if (scaled) {
        const float sb = (g.scale_b != nullptr && nok) ? g.scale_b[n] : 1.f;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int m = m0 + QA[q] * 128 + wr * 64 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lh;
            const float sa = (g.scale_a != nullptr && m < g.M) ? g.scale_a[m] : 1.f;
            acc8[q][i][r] = acc8[q][i][r] * sa * sb;
          }
      }
      if constexpr (EM == E_FILTER) {
        const float t = nok ? g.tau[n] : __builtin_inff();
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int m = m0 + QA[q] * 128 + wr * 64 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lh;
            const float v = acc8[q][i][r];
            if (nok && m < g.M && !(v <= t)) {
              const int pos = atomicAdd(g.cnt + n, 1);
              if (pos < g.cap) g.cand[(long long)n * g.cap + pos] = make_key(v, (uint32_t)(g.row_offset + m));
            }
          }
      } else if constexpr (EM == E_SCORES_T) {
        if (nok) {
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int b = 0; b < 4; ++b) {
              const int mb = m0 + QA[q] * 128 + wr * 64 + 32 * i + 8 * b + 4 * lh;
              float* dst = g.C + (long long)n * g.ldc + mb;
              if (mb + 3 < g.M) {
                *reinterpret_cast<f32x4*>(dst) =
                    f32x4{acc8[q][i][4 * b], acc8[q][i][4 * b + 1], acc8[q][i][4 * b + 2], acc8[q][i][4 * b + 3]};
              } else {
#pragma unroll
                for (int e = 0; e < 4; ++e)
                  if (mb + e < g.M) dst[e] = acc8[q][i][4 * b + e];
              }
            }
        }
      }
      asm volatile("" ::: "memory");
    }
    return;
  }
  if constexpr (EM == E_FILTER) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int ng = 0; ng < 2; ++ng) {
        const int n = n0 + QB[q] * 128 + wc * 32 + ng * 16 + l16;
        const bool nok = n < g.N;
        const float t = nok ? g.tau[n] : __builtin_inff();
#pragma unroll
        for (int mg = 0; mg < 4; ++mg)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int m = m0 + QA[q] * 128 + wr * 64 + mg * 16 + 4 * lg + e;
            const float v = acc[q][mg][ng][e];
            if (nok && m < g.M && !(v <= t)) {
              const int pos = atomicAdd(g.cnt + n, 1);
              if (pos < g.cap) g.cand[(long long)n * g.cap + pos] = make_key(v, (uint32_t)(g.row_offset + m));
            }
          }
      }
  } else if constexpr (EM == E_SCORES_T) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int ng = 0; ng < 2; ++ng) {
        const int n = n0 + QB[q] * 128 + wc * 32 + ng * 16 + l16;
        if (n >= g.N) continue;
#pragma unroll
        for (int mg = 0; mg < 4; ++mg) {
          const int mb = m0 + QA[q] * 128 + wr * 64 + mg * 16 + 4 * lg;
          float* dst = g.C + (long long)n * g.ldc + mb;
          if (mb + 3 < g.M) {
            *reinterpret_cast<f32x4*>(dst) = acc[q][mg][ng];
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
              if (mb + e < g.M) dst[e] = acc[q][mg][ng][e];
          }
        }
      }
  }
}

}  // namespace

// Host side: dense A and B, K a multiple of two k-tiles (bf16 128, fp8 256),
// 16-B aligned rows (checked by launch_gemm), no split-K / symmetric; row
// scales only for fp8.
bool gemm_8p_eligible(const GemmArgs& g, int dt) {
  const int ktp = dt == DT_FP8 ? 256 : 128;
  return (dt == DT_BF16 || dt == DT_FP8) && (g.K % ktp) == 0 && g.k_split == 0 && !g.sym &&
         (dt == DT_FP8 || (g.scale_a == nullptr && g.scale_b == nullptr)) &&
         (((uintptr_t)g.A | (uintptr_t)g.B) & 15) == 0;
}

hipError_t launch_gemm_8p(const GemmArgs& g, int emode, hipStream_t s, int dt) {
  const long long tiles_m = (g.M + 255) / 256, tiles_n = (g.N + 255) / 256;
  const long long nblk = tiles_m * tiles_n;
  if (nblk <= 0) return hipSuccess;
  if (nblk > 0x7fffffffLL) return hipErrorInvalidValue;
  if (emode == E_FILTER && dt == DT_FP8)
    hipLaunchKernelGGL((gemm_8p_kernel<E_FILTER, DT_FP8>), dim3((unsigned)nblk), dim3(512), 0, s, g, (int)tiles_n);
  else if (emode == E_SCORES_T && dt == DT_FP8)
    hipLaunchKernelGGL((gemm_8p_kernel<E_SCORES_T, DT_FP8>), dim3((unsigned)nblk), dim3(512), 0, s, g, (int)tiles_n);
  else if (emode == E_FILTER)
    hipLaunchKernelGGL((gemm_8p_kernel<E_FILTER, DT_BF16>), dim3((unsigned)nblk), dim3(512), 0, s, g, (int)tiles_n);
  else if (emode == E_SCORES_T)
    hipLaunchKernelGGL((gemm_8p_kernel<E_SCORES_T, DT_BF16>), dim3((unsigned)nblk), dim3(512), 0, s, g, (int)tiles_n);
  else
    return hipErrorInvalidValue;  // stored C: the 256x256 tile of gemm_f32.hip (config 3)
  return hipGetLastError();
}

}  // namespace rr
