// gemm_epilogue.hpp — the stored-C epilogue shared by the GEMM kernels
// (gemm_f32.hip, gemm_s3.hip): bias, residual, ReLU / QuickGELU, fp32 or
// bf16 output, written as whole rows through an LDS-staged tile.
#pragma once

#include "rr_internal.hpp"

namespace rr {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x8 __attribute__((ext_vector_type(8)));

// Accumulator register r of MFMA tile (i, j), lane `lane` -> (row, col) in
// the wave's block.  32x32x16 C/D map: col = lane & 31, row = (r&3) + 8(r>>2)
// + 4(lane>>5).  MF16 (four 16x16x32 tiles, sub-tile t = r >> 2 = 2a + b):
// row = 16a + 4(lane>>4) + (r&3), col = 16b + (lane&15).
template <bool MF16>
__device__ __forceinline__ int acc_row(int i, int r, int lane) {
  if constexpr (MF16) return 32 * i + 16 * (r >> 3) + 4 * ((lane >> 4) & 3) + (r & 3);
  else return 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
}
template <bool MF16>
__device__ __forceinline__ int acc_col(int j, int r, int lane) {
  if constexpr (MF16) return 32 * j + 16 * ((r >> 2) & 1) + (lane & 15);
  else return 32 * j + (lane & 31);
}

// QuickGELU, x * sigmoid(1.702 x) (networks/model.py:166-168), on the
// hardware exp2 and reciprocal (v_exp_f32, v_rcp_f32: ~1 ulp each; expf and a
// division cost ~20 VALU per element, 0.3 ms per ViT-B/16 fc1 at 1280 images);
// x -> -inf: exp2 -> inf, rcp -> 0, result -0 as x * sigmoid gives
__device__ __forceinline__ float quick_gelu(float x) {
  const float e = __builtin_amdgcn_exp2f(x * (-1.702f * 1.4426950408889634f));
  return x * __builtin_amdgcn_rcpf(1.0f + e);
}

// Flags of a stored-C launch (GemmArgs bias / residual / relu / out_bf16).
// The launchers compile the flag sets the networks use into their own kernel
// instances (template EPI = the flags, checked against ep_flags(g) on the
// host); EPI = -1 reads them from g per element.  One set per kernel, not a
// switch inside it: several inlined variants held extra values live through
// the k-loop and spilled it.
// EP_SCALE / EP_AMAX (the f16x2 split core only, always compiled-in flag
// sets): the accumulator times a per-column power-of-two scale before the
// bias, and the max |C| of the stored values published to c_amax.
// EP_STATS / EP_LNFOLD (the bf16 ViT linears, 256-column tiles): the
// LayerNorm partials + bf16 copy of C, and the LayerNorm folded into a
// consumer's epilogue (GemmArgs stats_out / stats_in).
// EP_SC1: fp32 C stored with sc1 (the line leaves the XCD's L2 instead of
// staying in it, MI355X_MICROARCH.md: a streamed output then does not evict
// the operand tiles other blocks of the XCD still re-read)
enum { EP_BIAS = 1, EP_RES = 2, EP_RELU = 4, EP_GELU = 8, EP_BF16 = 16, EP_SCALE = 32, EP_AMAX = 64, EP_STATS = 128,
       EP_LNFOLD = 256, EP_SC1 = 512 };
inline int ep_flags(const GemmArgs& g) {
  return (g.bias != nullptr ? EP_BIAS : 0) | (g.residual != nullptr ? EP_RES : 0) |
         (g.relu == 1 ? EP_RELU : g.relu == 2 ? EP_GELU : 0) | (g.out_bf16 ? EP_BF16 : 0) |
         (g.stats_out != nullptr ? EP_STATS : 0) | (g.stats_in != nullptr ? EP_LNFOLD : 0);
}

// The LayerNorm fold's consumer handles rows of up to LN_TMAX 256-column
// tiles (d <= 768: the ViT-B/16 in-proj / c_fc inputs); per row it stages
// LN_ROW floats: rstd and the tile-mean offsets d_t = mean_t - mean.
constexpr int LN_TMAX = 3, LN_ROW = 4;
// Row m's LayerNorm rstd = 1/sqrt(var + eps) and tile-mean offsets from the
// producer's per-tile partials (mean_t, M2_t over n_t = min(256, d - 256 t)
// columns), combined as Chan et al.: mean = sum n_t mean_t / d, M2 = sum M2_t
// + n_t (mean_t - mean)^2 (biased variance M2 / d, as nn.LayerNorm).  The
// consumer GEMM computes its tile's rows once, before its k-loop, into LDS.
__device__ __forceinline__ f32x4 ln_row_stats(const float* st, long long m, int d, float eps) {
  const int T = (d + 255) >> 8;
  const float* p = st + m * T * 2;
  float s = 0.f;
  for (int t = 0; t < T; ++t) s += (float)min(256, d - 256 * t) * p[2 * t];
  const float mean = s / (float)d;
  float m2 = 0.f;
  for (int t = 0; t < T; ++t) {
    const float dm = p[2 * t] - mean;
    m2 += p[2 * t + 1] + (float)min(256, d - 256 * t) * dm * dm;
  }
  f32x4 r = {1.0f / sqrtf(m2 / (float)d + eps), 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < LN_TMAX; ++t)
    if (t < T) r[1 + t] = p[2 * t] - mean;
  return r;
}

// ---- f16x2 split scales (gemm_s3.hip, SP 2) ----
// A tensor's max |x| lives in RR_AMAX_SLOTS words (float bit patterns of
// non-negative values, so unsigned order = float order), each the max over
// the waves that hashed to it: no single hot address.  Non-finite values are
// left out (an inf / NaN input still turns its own outputs into NaN).
__device__ __forceinline__ float amax_acc(float am, float x) {
  const float a = __builtin_fabsf(x);
  return a < __builtin_inff() ? __builtin_fmaxf(am, a) : am;
}
// (the wave max by DPP row shifts as wave_sum: out-of-row sources read 0,
// below every value; no lane-address registers, which a __shfl_xor tree
// holds from the kernel's start in the register-bound persistent kernels)
__device__ __forceinline__ void amax_publish(uint32_t* slots, float am, int slot) {
  auto shr = [](float v, auto ctrl) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), decltype(ctrl)::value, 0xf, 0xf, true));
  };
  am = __builtin_fmaxf(am, shr(am, std::integral_constant<int, 0x111>{}));  // row_shr:1
  am = __builtin_fmaxf(am, shr(am, std::integral_constant<int, 0x112>{}));  // row_shr:2
  am = __builtin_fmaxf(am, shr(am, std::integral_constant<int, 0x114>{}));  // row_shr:4
  am = __builtin_fmaxf(am, shr(am, std::integral_constant<int, 0x118>{}));  // row_shr:8
  const int xi = __float_as_int(am);
  const float w = __builtin_fmaxf(
      __builtin_fmaxf(__int_as_float(__builtin_amdgcn_readlane(xi, 15)), __int_as_float(__builtin_amdgcn_readlane(xi, 31))),
      __builtin_fmaxf(__int_as_float(__builtin_amdgcn_readlane(xi, 47)), __int_as_float(__builtin_amdgcn_readlane(xi, 63))));
  // (lane 0 by mbcnt: nothing held from the kernel's start for it)
  if (__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)) == 0)
    __hip_atomic_fetch_max(slots + (slot & (RR_AMAX_SLOTS - 1)), __float_as_uint(w), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}
// the max over the slots (every lane of the wave gets it)
__device__ __forceinline__ uint32_t amax_load_slot(const uint32_t* slots) {
  return __hip_atomic_load(slots + (threadIdx.x & (RR_AMAX_SLOTS - 1)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float amax_reduce(uint32_t u) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t v = (uint32_t)__shfl_xor((int)u, o);
    u = v > u ? v : u;
  }
  return __uint_as_float(u);
}
// Power-of-two split exponent: amax * 2^e in [2^14, 2^15), so the fp16 high
// piece of every scaled value is finite (< 65504) and values down to 2^-18 of
// the max keep both pieces normal (22 significant bits); 0 for a zero or
// non-finite max.  e >= -113 for every finite max; capped at 126 (a max
// below 2^-111) so 2^e and 2^-e stay normal floats.
__device__ __forceinline__ int h2_exp(float amax) {
  if (!(amax > 0.f && amax < __builtin_inff())) return 0;
  const int e = 15 - __builtin_amdgcn_frexp_expf(amax);
  return e > 126 ? 126 : e;
}

// a fresh, opaque copy of v (loads addressed by it are not hoisted)
__device__ __forceinline__ int ep_opaque(int v) {
  asm volatile("" : "+v"(v));
  return v;
}

// Row maps of epilogue_store / store_slab: (slab base mb, slab row) -> output
// row, >= g.M for a row that is not stored.  RowsLinear: the raster tiles
// (rows mb + row).  Rows2D<TW>: gemm_h2_halo_kernel's 2-D block tiles, tile
// row r = mb + row is output pixel (y0 + r / TW, x0 + r % TW) of the image
// whose first output row is img (H x W map), stored only inside the map.
struct RowsLinear {
  __device__ __forceinline__ int operator()(int mb, int row) const { return mb + row; }
};
template <int TW>
struct Rows2D {
  static constexpr int kTW = TW;
  int img, y0, x0, H, W;
  __device__ __forceinline__ int operator()(int mb, int row) const {
    const int r = mb + row, y = y0 + r / TW, x = x0 + r % TW;
    return (y < H && x < W) ? img + y * W + x : 0x7fffffff;
  }
};

// Write one staged slab (rows mb.. of the tile, row-major in ct): the LDS
// reads of a group of row chunks first (counted lgkmcnt waits instead of an
// LDS round trip between consecutive stores; the whole slab at once when no
// other slab's accumulators are still live), then bias / residual /
// activation and the 16-B (fp32) or 8-B (bf16) store.  FL >= 0: the flags
// fixed at compile time and (BI == 1) one column per thread, so the loop is
// the arithmetic, a row bound and an address step; FL = -1: the flags read
// from g per element.
// CSW: the staged rows are unpadded with their 16-B chunks XOR-swizzled,
// chunk c of row r at c ^ (((r >> 2) & 1) << 2) (csw_chunk; gemm_lpp.hip)
__device__ __forceinline__ int csw_chunk(int row, int c4) { return c4 ^ (((row >> 2) & 1) << 2); }
template <int FL, int P, int ITERS, int NT, int C4, int CS, int BI, int CSW = 0, class RM = RowsLinear>
__device__ __forceinline__ void store_slab(const GemmArgs& g, float* Cb, const float* ct, const f32x4 (&bias_v)[BI],
                                           const f32x4 (&res)[ITERS], int tid, int mb, int n0, const f32x4 (&sc_v)[BI],
                                           float& am, const float* ln_l = nullptr, const float* ln_cs = nullptr,
                                           RM rm = RM{}) {
  constexpr bool LIN = __is_same(RM, RowsLinear);
  typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
  constexpr bool FIXED = FL >= 0;
  // (the LayerNorm fold's epilogue holds two more values per row: fewer LDS reads ahead)
  constexpr int GR = (FIXED && (FL & EP_LNFOLD) != 0) ? 1 : ITERS < 4 ? ITERS : (P == 1 ? 8 : 4);
  // EP_STATS: one row of the 256-column tile per wave and iteration
  static_assert(!(FIXED && (FL & (EP_STATS | EP_LNFOLD))) || (BI == 1 && C4 == 64), "LayerNorm fold: 256-column tiles");
  const bool has_bias = FIXED ? (FL & EP_BIAS) != 0 : g.bias != nullptr;
  const bool has_res = FIXED ? (FL & EP_RES) != 0 : g.residual != nullptr;
  const int act = FIXED ? ((FL & EP_RELU) ? 1 : (FL & EP_GELU) ? 2 : 0) : g.relu;
  const bool obf = FIXED ? (FL & EP_BF16) != 0 : g.out_bf16 != 0;
  // BI == 1: every iteration of a thread is the same column, NT / C4 rows on
  const int c40 = tid % C4, r0 = tid / C4;
  constexpr int RSTEP = NT / C4;

  const int n_fix = n0 + c40 * 4;
  const long long o0 = (long long)(mb + r0) * g.ldc + n_fix;
  // (Rows2D: the thread's first row's pixel and output row)
  int r2y = 0, r2x = 0, r2m = 0;
  if constexpr (!LIN) {
    const int rb = mb + r0;
    r2y = rm.y0 + rb / RM::kTW;
    r2x = rm.x0 + rb % RM::kTW;
    r2m = rm.img + r2y * rm.W + r2x;
  }
  const long long ostep = (long long)RSTEP * g.ldc;
  f32x4 cv[ITERS];
#pragma unroll
  for (int it = 0; it < ITERS; ++it) {
    if (it % GR == 0) {
#pragma unroll
      for (int u = it; u < it + GR && u < ITERS; ++u) {
        const int idx = tid + u * NT;
        const int row = idx / C4, c4 = idx - row * C4;
        cv[u] = *reinterpret_cast<const f32x4*>(ct + row * CS + (CSW ? csw_chunk(row, c4) : c4) * 4);
      }
    }
    int m, n;
    long long o;
    if constexpr (FIXED && BI == 1 && LIN) {
      m = mb + r0 + it * RSTEP;
      n = n_fix;
      o = o0 + it * ostep;
    } else if constexpr (FIXED && BI == 1) {
      // Rows2D: iteration it is the thread's base pixel + (k / TW) map rows +
      // k % TW columns, k = it RSTEP (RSTEP divides TW, r0 < RSTEP and the
      // slab starts a block row: no carry), so the compile-time steps cost an
      // add each instead of a row map per iteration (that spilled the
      // 256x256 tile)
      constexpr int TW = RM::kTW;
      static_assert(TW % RSTEP == 0, "Rows2D: whole steps per block row");
      const int k = it * RSTEP, dy = k / TW, dx = k % TW;
      m = (r2y + dy < rm.H && r2x + dx < rm.W) ? r2m + dy * rm.W + dx : 0x7fffffff;
      n = n_fix;
      o = (long long)m * g.ldc + n;
    } else {
      const int idx = tid + it * NT;
      const int row = idx / C4, c4 = idx - row * C4;
      m = rm(mb, row);
      n = n0 + c4 * 4;
      o = (long long)m * g.ldc + n;
    }
    if (m >= g.M || n >= g.N) continue;
    f32x4 v = cv[it];
    if constexpr (FIXED && (FL & EP_SCALE) != 0) v *= sc_v[BI == 1 ? 0 : it];
    if constexpr (FIXED && (FL & EP_LNFOLD) != 0) {
      // the row's rstd and tile-mean offsets d_t = mean_t - mean and the
      // tile's column sums per k tile, staged in LDS before the k-loop
      // (rows slab-relative): y = rstd (acc + sum_t d_t colsum_t).  The
      // column sums are re-read per row (an opaque offset), not held in
      // registers through the stores: 12 more there spilled the 256 x 256 tile.
      const f32x4 rd = *reinterpret_cast<const f32x4*>(ln_l + LN_ROW * (m - mb));
      const int co = ep_opaque(c40 * 4);
      f32x4 u = v;
#pragma unroll
      for (int t = 0; t < LN_TMAX; ++t) u += rd[1 + t] * *reinterpret_cast<const f32x4*>(ln_cs + t * (4 * C4) + co);
      v = u * rd[0];
    }
    if (has_bias) v += bias_v[BI == 1 ? 0 : it];
    if (has_res) v += res[it];
    if (act == 1) {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
    } else if (act == 2) {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = quick_gelu(v[e]);
    }
    if constexpr (FIXED && (FL & EP_AMAX) != 0) {
#pragma unroll
      for (int e = 0; e < 4; ++e) am = amax_acc(am, v[e]);
    }
    if (obf) {
      const bf16x4 ob = {(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
      *reinterpret_cast<bf16x4*>(reinterpret_cast<uint16_t*>(Cb) + o) = ob;
    } else if constexpr (FIXED && (FL & EP_SC1) != 0) {
      // (the s_nop: a VALU write to the data registers of a store wider than
      // 8 B needs a wait state after it, which hipcc inserts for its own
      // stores but not after an inline-asm one; without it the registers
      // were overwritten before the store read them: wrong outputs)
      asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(Cb + o), "v"(v) : "memory");
    } else {
      *reinterpret_cast<f32x4*>(Cb + o) = v;
    }
    if constexpr (FIXED && (FL & EP_STATS) != 0) {
      // the row's tile LayerNorm partials, two passes over the 256 values the
      // wave holds (row m is wave-uniform; N % 256 == 0), and its bf16 copy
      // centred on the tile mean: bf16(v - mean_t) rounds 2^-9 |v - mean_t|,
      // not 2^-9 |v|, so a row mean far from 0 costs the fold no precision
      const float mt = wave_sum((v[0] + v[1]) + (v[2] + v[3])) * (1.0f / 256.0f);
      const f32x4 dv = v - mt;
      const bf16x4 ob = {(__bf16)dv[0], (__bf16)dv[1], (__bf16)dv[2], (__bf16)dv[3]};
      *reinterpret_cast<bf16x4*>(g.c2 + o) = ob;
      const float m2 = wave_sum((dv[0] * dv[0] + dv[1] * dv[1]) + (dv[2] * dv[2] + dv[3] * dv[3]));
      // (wave-uniform: lane 0 stores)
      if ((threadIdx.x & 63) == 0) {
        const int T = (g.N + 255) >> 8;
        *reinterpret_cast<float2*>(g.stats_out + ((long long)m * T + (n0 >> 8)) * 2) = float2{mt, m2};
      }
    }
  }
}

// Stage the BM x BN accumulator tile (32x32 MFMA C/D layout: col = lane & 31,
// row = (r&3) + 8(r>>2) + 4(lane>>5)) through LDS, then write whole rows: each
// lane moves 16 B, 32 lanes cover a 512-B row run, the residual is read the
// same way, every load of a slab issued before its accumulators are staged
// (one HBM round trip per slab, overlapping the staging).  When the tile exceeds the CAPF floats of LDS it goes in P row
// slabs.  Called by every thread of the block after the k-loop's last
// barrier (the LDS is free).
template <int WM, int WN, int FM, int FN, int CAPF, bool MF16 = false, int FL = -1, class RM = RowsLinear>
__device__ __forceinline__ void epilogue_store(const GemmArgs& g, float* Cb, const f32x16 (&acc)[FM][FN], float* lds,
                                               int m0, int n0, float a_isc = 1.f, const float* ln_lds = nullptr,
                                               RM rm = RM{}) {
  // (rm: the tile's row map, RowsLinear or Rows2D; row r of the tile is output row rm(m0, r))
  // (EP_LNFOLD: ln_lds = [BM][LN_ROW] row statistics, then [LN_TMAX][BN] column sums)
  constexpr int NT = 64 * WM * WN;
  constexpr int WTM = 32 * FM, WTN = 32 * FN;
  constexpr int BM = WTM * WM, BN = WTN * WN;
  // staging row stride: padded so the accumulator writes hit distinct banks
  // (16x16 map: lanes 16 apart are 4 rows apart -> +4 floats per row; 32x32
  // map: lanes 32 apart are 4 rows apart -> +8); the row-contiguous 16-B
  // reads of store_slab stay conflict-free and aligned either way
  // (tiles whose padded slabs would not tile the waves keep unpadded rows)
  constexpr int CSP = BN + (MF16 ? 4 : 8);
  constexpr int PP0 = (BM * CSP + CAPF - 1) / CAPF;
  constexpr int PP = PP0 <= 1 ? 1 : (PP0 <= 2 ? 2 : (PP0 <= 4 ? 4 : 8));  // a divisor of WM
  constexpr bool PAD = PP <= WM && BM / PP * CSP <= CAPF;
  constexpr int CS = PAD ? CSP : BN;
  constexpr int P = PAD ? PP : (BM * BN + CAPF - 1) / CAPF;
  constexpr int SLAB = BM / P;
  constexpr int C4 = BN / 4;
  constexpr int ITERS = SLAB * C4 / NT;
  static_assert(WM % P == 0, "row slabs must align with wave rows");
  static_assert(ITERS * NT == SLAB * C4, "epilogue tiling");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const bool vec_ok = ((g.N & 3) == 0) && ((g.ldc & 3) == 0);
  float* ct = lds;  // [SLAB][CS] row-major
  // The bias columns, loaded before any store: a load issued after a store
  // may alias it, so the compiler waits vmcnt(0) for it — and vmcnt counts
  // stores too — turning every row chunk into a store round trip (32 per
  // 256x256 tile).  A thread's column is the same in every iteration when
  // NT % C4 == 0 (every configuration that stores C); otherwise one per
  // iteration.
  constexpr int BI = (NT % C4 == 0) ? 1 : ITERS;
  constexpr bool SCALED = FL >= 0 && (FL & EP_SCALE) != 0;
  static_assert(!(FL >= 0 && (FL & (EP_SCALE | EP_AMAX))) || BI == 1, "scaled epilogues: one column per thread");
  // Fixed flags without EP_RES: no residual load code at all (every launcher
  // derives its fixed flags from ep_flags(g), so g.residual is null there).
  // Row-mapped tiles needed it (the mapped addresses spilled the 2-D 256x256
  // halo tile); the raster ones gained too: the 256@14 halo 256 -> 240 VGPRs,
  // the C3 embed 67.29 / 66.74 / 66.76 -> 66.21 / 66.52 / 66.47 ms on one box
  // (profiles/r06zf_libab/)
  constexpr bool RES_C = FL < 0 || (FL & EP_RES) != 0;
  f32x4 bias_v[BI], sc_v[BI];
  float am = 0.f;
  if (vec_ok) {
#pragma unroll
    for (int it = 0; it < BI; ++it) {
      const int idx = tid + it * NT;
      const int n = n0 + (idx % C4) * 4;
      bias_v[it] = (g.bias != nullptr && n < g.N) ? *reinterpret_cast<const f32x4*>(g.bias + n)
                                                  : f32x4{0.f, 0.f, 0.f, 0.f};
      if constexpr (SCALED) sc_v[it] = (n < g.N ? *reinterpret_cast<const f32x4*>(g.col_scale + n)
                                                : f32x4{0.f, 0.f, 0.f, 0.f}) * a_isc;
    }
  }
#pragma unroll
  for (int p = 0; p < P; ++p) {
    const int rbase = p * SLAB;
    // single-slab tiles with registers to spare: the residual loads go out
    // first, their HBM round trip overlapping the LDS staging of the
    // accumulators and its barrier
    constexpr bool PREF = P == 1 && ITERS * 4 + FM * FN * 16 <= 160;
    f32x4 res[ITERS];
    if (RES_C && PREF && vec_ok && g.residual != nullptr) {
#pragma unroll
      for (int it = 0; it < ITERS; ++it) {
        const int idx = tid + it * NT;
        const int row = idx / C4, c4 = idx - row * C4;
        const int m = rm(m0 + rbase, row), n = n0 + c4 * 4;
        if (m < g.M && n < g.N) res[it] = *reinterpret_cast<const f32x4*>(g.residual + (long long)m * g.ldc + n);
      }
    }
    if (p > 0) __syncthreads();
    if (wm / (WM / P) == p) {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int row = wm * WTM + acc_row<MF16>(i, r, lane) - p * SLAB;
            const int col = wn * WTN + acc_col<MF16>(j, r, lane);
            ct[row * CS + col] = acc[i][j][r];
          }
    }
    __syncthreads();
    if (vec_ok) {
      if (RES_C && !PREF && g.residual != nullptr) {
#pragma unroll
        for (int it = 0; it < ITERS; ++it) {
          const int idx = tid + it * NT;
          const int row = idx / C4, c4 = idx - row * C4;
          const int m = rm(m0 + rbase, row), n = n0 + c4 * 4;
          if (m < g.M && n < g.N) res[it] = *reinterpret_cast<const f32x4*>(g.residual + (long long)m * g.ldc + n);
        }
      }
      // One wait for every bias / residual load, before this slab's first
      // store: once a store is in flight the compiler can only wait for a
      // load with vmcnt(0) (loads and stores retire out of order), i.e. for
      // the stores too — one store round trip per row chunk.  The empty asm
      // redefines the registers, so nothing below waits again.
#pragma unroll
      for (int it = 0; it < BI; ++it) asm volatile("" : "+v"(bias_v[it]));
      if constexpr (SCALED) {
#pragma unroll
        for (int it = 0; it < BI; ++it) asm volatile("" : "+v"(sc_v[it]));
      }
      if (RES_C && g.residual != nullptr) {
#pragma unroll
        for (int it = 0; it < ITERS; ++it) asm volatile("" : "+v"(res[it]));
      }
      store_slab<(BI == 1 ? FL : -1), P, ITERS, NT, C4, CS, BI, 0, RM>(g, Cb, ct, bias_v, res, tid, m0 + rbase, n0, sc_v,
                                                                       am, ln_lds ? ln_lds + LN_ROW * rbase : nullptr,
                                                                       ln_lds ? ln_lds + LN_ROW * BM : nullptr, rm);
    } else {
      for (int idx = tid; idx < SLAB * C4; idx += NT) {
        const int row = idx / C4, c4 = idx - row * C4;
        const int m = rm(m0 + rbase, row), n = n0 + c4 * 4;
        if (m >= g.M || n >= g.N) continue;
        const f32x4 v = *reinterpret_cast<const f32x4*>(ct + row * CS + c4 * 4);
        const long long o = (long long)m * g.ldc + n;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (n + e >= g.N) break;
          float x = v[e];
          if constexpr (SCALED) x *= g.col_scale[n + e] * a_isc;
          if (g.bias != nullptr) x += g.bias[n + e];
          if (g.residual != nullptr) x += g.residual[o + e];
          if (g.relu == 1) x = fmaxf(x, 0.f);
          else if (g.relu == 2) x = quick_gelu(x);
          if constexpr (FL >= 0 && (FL & EP_AMAX) != 0) am = amax_acc(am, x);
          if (g.out_bf16) reinterpret_cast<__bf16*>(Cb)[o + e] = (__bf16)x;
          else Cb[o + e] = x;
        }
      }
    }
  }
  if constexpr (FL >= 0 && (FL & EP_AMAX) != 0) {
    if (g.c_amax != nullptr) amax_publish(g.c_amax, am, blockIdx.x * (NT / 64) + wave);
  }
}

}  // namespace rr
