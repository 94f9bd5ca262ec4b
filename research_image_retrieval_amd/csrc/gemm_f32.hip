// gemm_f32.hip — fp32 MFMA GEMM core for gfx950 (CDNA4).
//
// C[M,N] = A[M,K] . B[N,K]^T with A and B both K-contiguous ("NT" layout).
// One core serves three reference call sites:
//   * cosine ranker  : A = gallery rows, B = query rows  (iris_evaluate.py:383)
//   * conv layers    : A = implicit im2col of an NHWC map, B = weights
//                      [Cout][KH][KW][Cin]               (networks/backbone.py:103-109)
//   * projections    : A = pooled descriptors, B = W     (networks/RetrievalNet.py:342,
//                                                         models/gem_pooling.py:68)
//
// Arithmetic: v_mfma_f32_32x32x2_f32 (exact f32 in, f32 accumulate; every
// output element is a k-ordered fmaf chain).  Within each 16-deep k chunk the
// lane half h of MFMA e supplies k = 16c + 8h + e, so the chain visits
// k = 16c+0, 16c+8, 16c+1, 16c+9, ..., 16c+7, 16c+15 — oracle/cosine_topk.c
// restates exactly this order, which makes GPU scores bit-identical to the
// oracle's.
//
// Tiling: a wave owns a 64x64 output block (2x2 MFMA tiles of 32x32, 64
// accumulator registers); a workgroup is WM x WN waves.  BK = 32: each k-tile
// of A and B is register-staged (one float4 per lane-chunk, coalesced along
// K) into a double-buffered LDS image of 128-byte rows whose 16-byte slots are
// XOR-swizzled by (row>>1)&7, which makes the fragment ds_read_b128 (lane
// groups of 16 distinct rows, same slot) bank-conflict free.  One barrier per
// k-tile; the next tile's global loads are in flight under the MFMAs.
// Block ids are remapped so consecutive tiles of one XCD share the A panel
// (the streamed gallery / activation rows) in that XCD's L2.
#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "gemm_epilogue.hpp"
#include "rr_internal.hpp"

namespace rr {

// input element type of A/B: DT_F32 (v_mfma_f32_32x32x2_f32), DT_BF16
// (v_mfma_f32_32x32x16_bf16), DT_FP8 (OCP e4m3, v_mfma_scale_f32_32x32x64_f8f6f4
// with unit block scales).
// LDS rows are 128 B for all three (32 fp32 / 64 bf16 / 128 fp8 per k-tile),
// so staging, swizzle and epilogues are shared.
template <int DT> struct ElemT { using T = float; };
template <> struct ElemT<DT_BF16> { using T = uint16_t; };
template <> struct ElemT<DT_FP8> { using T = uint8_t; };

// 16-byte-slot XOR swizzle of a [rows][BK] fp32 LDS image, conflict-free for
// the fragment ds_read_b128 (16 lanes = 16 rows distinct mod 16, one slot):
// BK = 32 (8 slots per 128-B row): slot ^ ((row >> 1) & 7);
// BK = 16 (4 slots per 64-B row):  slot ^ ((row >> 2) & 3).
template <int BK>
__device__ __forceinline__ int swz(int row, int slot) {
  if constexpr (BK == 32) return slot ^ ((row >> 1) & 7);
  else return slot ^ ((row >> 2) & 3);
}

// Pin the scheduler to alternate MFMAs with the next k-step's LDS fragment
// reads (NR reads, NM >= NR MFMAs in the region): MFMA, read, MFMA, read,
// ..., then the remaining MFMAs, so the reads' latency runs under MFMAs.
template <int NR, int NM>
__device__ __forceinline__ void interleave() {
#pragma unroll
  for (int x = 0; x < NR; ++x) {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // 1 MFMA
    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // 1 DS read
  }
  if constexpr (NM > NR) __builtin_amdgcn_sched_group_barrier(0x008, NM - NR, 0);
}

// interleave<nr, NM> with the next k-tile's LDS-DMA chunks spread among the
// MFMAs (IL sweeps): chunk c of NCH goes out before MFMA number (c * SPAN) /
// NCH of the k-tile; base = the k-tile's MFMA number of this region's first
// (base and nr constant once the caller's k-step loop is unrolled).
template <int NM, int SPAN, int NCH, int DSPER = 1>
__device__ __forceinline__ void interleave_il(int base, int nr) {
#pragma unroll
  for (int x = 0; x < NM; ++x) {
#pragma unroll
    for (int c = 0; c < NCH; ++c)
      if ((c * SPAN) / NCH == base + x) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // 1 VMEM (the DMA)
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                                      // 1 MFMA
    if (x < nr) __builtin_amdgcn_sched_group_barrier(0x100, DSPER, 0);                      // DSPER DS reads
  }
}

// Same with two DS reads per MFMA (NP pairs, NM >= NP MFMAs): the fp8 k-step
// reads 32 bytes (two ds_read_b128) per fragment.
template <int NP, int NM>
__device__ __forceinline__ void interleave2() {
  static_assert(NM >= NP, "interleave2: fewer MFMAs than read pairs");
#pragma unroll
  for (int x = 0; x < NP; ++x) {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // 1 MFMA
    __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);  // 2 DS reads
  }
  if constexpr (NM > NP) __builtin_amdgcn_sched_group_barrier(0x008, NM - NP, 0);
}

// BK = 32: 64 KB LDS per 128x128 block, 2 blocks (2 waves/SIMD) per CU.
// BK = 16: 32 KB, 3 blocks (3 waves/SIMD) per CU, twice the barriers.
// MF16 (bf16 only): each 32x32 tile of a wave's block is computed as four
// v_mfma_f32_16x16x32_bf16 tiles (same cycles per FLOP as 32x32x16; the
// 16x16 shape holds a higher clock on random operands, MI355X_MICROARCH.md
// 'DVFS give-back' item 7).  Register r of tile (i, j) then maps through
// acc_row / acc_col<true> (gemm_epilogue.hpp) instead of the 32x32 map.
// IL (LDS-DMA bf16 filter sweeps): the next k-tile's DMA is not issued as one
// burst at the top of the k-tile but chunk by chunk among the first SPAN
// MFMAs (18 of 40 on 32x32x16, 36 of 80 on 16x16x32): a burst of 9
// instructions from all 8 waves at once fills the vector-memory issue queue
// and stalls the waves' MFMAs behind it (tools/fetch_ceiling.hip, r04e:
// 0.481 -> 0.525 of peak on the bare 32x32x16 sweep loop).
template <int WM, int WN, int FM, int FN, int AMODE, int EMODE, int BK, int DT, int MINB, int GL, int MF16 = 0,
          int EPI = -1, int IL = 0>
__global__ __launch_bounds__(64 * WM * WN, MINB) void gemm_kernel(GemmArgs g, int tiles_n) {
  using ET = typename ElemT<DT>::T;
  static_assert(!MF16 || DT == DT_BF16, "MF16: bf16 only");
  static_assert(DT == DT_F32 || (AMODE == A_DENSE && BK == 32), "low-precision GEMM: dense A, 128-B rows");
  static_assert(!GL || AMODE == A_DENSE, "LDS-DMA staging: dense A/B");
  constexpr int ES = (int)sizeof(ET);
  constexpr int EPR = BK * 4 / ES;  // elements per LDS row (= k per k-tile)
  constexpr int CH = 16 / ES;       // elements per 16-byte staging chunk
  constexpr int NT = 64 * WM * WN;
  constexpr int WTM = 32 * FM, WTN = 32 * FN;  // one wave's output block
  constexpr int BM = WTM * WM, BN = WTN * WN;
  constexpr int SLOTS = BK / 4;
  constexpr int ROWS_PER_PASS = NT / SLOTS;
  constexpr int A_CH = BM / ROWS_PER_PASS;
  constexpr int B_CH = BN / ROWS_PER_PASS;
  static_assert(A_CH >= 1 && B_CH >= 1, "tile too small for block");
  static_assert(BM % ROWS_PER_PASS == 0 && BN % ROWS_PER_PASS == 0, "staging passes must tile the block");
  constexpr int BUF = (BM + BN) * BK;  // floats per LDS buffer
  // EP_LNFOLD: the tile's rows' LayerNorm (mean, rstd) beside the stages
  constexpr bool LNF = EPI >= 0 && (EPI & EP_LNFOLD) != 0;
  __shared__ __attribute__((aligned(16))) float lds[2 * BUF + (LNF ? LN_ROW * BM + LN_TMAX * BN : 0)];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM;

  // XCD-aware block -> tile order (rr_internal.hpp tile_coords)
  int tm, tn;
  tile_coords(blockIdx.x, gridDim.x, tiles_n, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;

  const int slot = tid % SLOTS;
  const int crow = tid / SLOTS;
  int K = g.K;
  long long koff = 0;
  float* const Cb = g.C + (g.k_split > 0 ? (long long)blockIdx.y * g.c_split_stride : 0LL);
  if (g.k_split > 0) {
    koff = (long long)blockIdx.y * g.k_split;
    K = (int)(g.K - koff < g.k_split ? g.K - koff : g.k_split);
  }
  if (g.sym && m0 > n0 + BN - 1) return;  // block-uniform, before any barrier
  const int nk = (K + EPR - 1) / EPR;

  // ---- per-chunk A row state ----
  const ET* a_ptr[A_CH];
  int a_ih0[A_CH], a_iw0[A_CH];
  bool a_ok[A_CH];
#pragma unroll
  for (int i = 0; i < A_CH; ++i) {
    const int m = m0 + crow + i * ROWS_PER_PASS;
    a_ok[i] = m < g.M;
    if constexpr (AMODE == A_DENSE) {
      a_ptr[i] = reinterpret_cast<const ET*>(g.A) + (long long)(a_ok[i] ? m : 0) * g.lda + koff;
      a_ih0[i] = 0;
      a_iw0[i] = 0;
    } else {
      const int mm = a_ok[i] ? m : 0;
      const int ohw = g.OH * g.OW;
      const int b = mm / ohw;
      const int rem = mm - b * ohw;
      const int oh = rem / g.OW;
      const int ow = rem - oh * g.OW;
      a_ptr[i] = reinterpret_cast<const ET*>(g.A) + (long long)b * g.H * g.W * g.Cin;
      a_ih0[i] = oh * g.stride - g.pad;
      a_iw0[i] = ow * g.stride - g.pad;
    }
  }
  const ET* b_ptr[B_CH];
  bool b_ok[B_CH];
#pragma unroll
  for (int i = 0; i < B_CH; ++i) {
    const int n = n0 + crow + i * ROWS_PER_PASS;
    b_ok[i] = n < g.N;
    b_ptr[i] = reinterpret_cast<const ET*>(g.B) + (long long)(b_ok[i] ? n : 0) * g.ldb + koff;
  }

  f32x4 ra[A_CH], rb[B_CH];

  auto load_tile = [&](int kt) {
    const int k = kt * EPR + slot * CH;
    const bool kok = k < K;
    if constexpr (AMODE == A_DENSE) {
#pragma unroll
      for (int i = 0; i < A_CH; ++i) {
        ra[i] = (a_ok[i] && kok) ? *reinterpret_cast<const f32x4*>(a_ptr[i] + k) : f32x4{0.f, 0.f, 0.f, 0.f};
      }
    } else if constexpr (AMODE == A_CONV) {
      // Cin % 32 == 0: the whole 32-deep k-tile lies in one (kh, kw) tap.
      const int k0 = kt * BK;
      const int khw = k0 / g.Cin;
      const int cin0 = k0 - khw * g.Cin;
      const int kh = khw / g.KW;
      const int kw = khw - kh * g.KW;
#pragma unroll
      for (int i = 0; i < A_CH; ++i) {
        const int ih = a_ih0[i] + kh, iw = a_iw0[i] + kw;
        const bool ok = a_ok[i] && kok && (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
        ra[i] = ok ? *reinterpret_cast<const f32x4*>(a_ptr[i] + ((long long)ih * g.W + iw) * g.Cin + cin0 + slot * 4)
                   : f32x4{0.f, 0.f, 0.f, 0.f};
      }
    } else if constexpr (AMODE == A_CONV_C4) {
      // Cin == 4 (RGB + zero pad channel): each float4 is one filter tap
      const int tap = k >> 2;
      const int kh = tap / g.KW;
      const int kw = tap - kh * g.KW;
#pragma unroll
      for (int i = 0; i < A_CH; ++i) {
        const int ih = a_ih0[i] + kh, iw = a_iw0[i] + kw;
        const bool ok = a_ok[i] && kok && (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
        ra[i] = ok ? *reinterpret_cast<const f32x4*>(a_ptr[i] + ((long long)ih * g.W + iw) * 4) : f32x4{0.f, 0.f, 0.f, 0.f};
      }
    } else {
      // generic gather (small / odd Cin)
      const int kwc = g.KW * g.Cin;
#pragma unroll
      for (int i = 0; i < A_CH; ++i) {
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int kk = k + e;
          if (a_ok[i] && kk < K) {
            const int kh = kk / kwc;
            const int r2 = kk - kh * kwc;
            const int kw = r2 / g.Cin;
            const int c = r2 - kw * g.Cin;
            const int ih = a_ih0[i] + kh, iw = a_iw0[i] + kw;
            if ((unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W)
              v[e] = a_ptr[i][((long long)ih * g.W + iw) * g.Cin + c];
          }
        }
        ra[i] = v;
      }
    }
    if constexpr (AMODE == A_CONV_GENERIC) {
      // K need not be a multiple of 4 here (stem: 7*7*3 = 147): scalar loads
#pragma unroll
      for (int i = 0; i < B_CH; ++i) {
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (b_ok[i] && k + e < K) v[e] = b_ptr[i][k + e];
        rb[i] = v;
      }
    } else {
#pragma unroll
      for (int i = 0; i < B_CH; ++i) {
        rb[i] = (b_ok[i] && kok) ? *reinterpret_cast<const f32x4*>(b_ptr[i] + k) : f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
  };

  // LDS-DMA staging (GL): global_load_lds writes a wave's 64 x 16 B lane-
  // linearly = 8 whole 128-B rows; the XOR swizzle moves to the SOURCE slot
  // (it is an involution, so the fragment reads below stay as they are).
  // Needs K % EPR == 0 (no partial k-tile to zero-fill).
  auto glds_tile = [&](int kt, int buf) {
    float* la = lds + buf * BUF;
    float* lb = la + BM * BK;
    const int wv = tid >> 6;
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const int row = crow + i * ROWS_PER_PASS;
      __builtin_amdgcn_global_load_lds(
          (const void*)(a_ptr[i] + (long long)kt * EPR + swz<BK>(row, slot) * CH),
          (__attribute__((address_space(3))) void*)(la + (i * ROWS_PER_PASS + wv * (64 / SLOTS)) * BK), 16, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      const int row = crow + i * ROWS_PER_PASS;
      __builtin_amdgcn_global_load_lds(
          (const void*)(b_ptr[i] + (long long)kt * EPR + swz<BK>(row, slot) * CH),
          (__attribute__((address_space(3))) void*)(lb + (i * ROWS_PER_PASS + wv * (64 / SLOTS)) * BK), 16, 0, 0);
    }
  };

  // IL: chunk c (A rows, then B rows) of glds_tile(kt, buf), due before MFMA
  // number idx; past the last k-tile it re-fetches the last one (an L2 hit)
  // into the drained buffer, so every iteration issues the same DMAs
  static_assert(!IL || (GL && DT != DT_F32 && (MF16 == 1 || EMODE == E_FILTER)),
                "IL: LDS-DMA bf16 / fp8 filter sweeps, or the PIPE16 tiles");
  constexpr int NCH = A_CH + B_CH;
  // (PIPE16: the chunks go among the last k-step's MFMAs, one every
  // 4 FM FN / NCH, right after the barrier that frees their buffer)
  // (fp8: the first k-step's FM FN MFMAs, one chunk each)
  constexpr int IL_SPAN = IL ? (MF16 == 2 ? 36 : MF16 == 1 ? 4 * FM * FN : DT == DT_FP8 ? FM * FN : 18) : 0;
  static_assert(IL_SPAN <= (MF16 ? 4 * FM * FN * (BK / 16) : DT == DT_FP8 ? FM * FN * (BK / 16) : FM * FN * (BK / 8)),
                "IL: every chunk before an MFMA of the k-tile");
  auto glds_due = [&](int kt, int buf, int idx) {
    if constexpr (IL) {
      const int kc = kt < nk ? kt : nk - 1;
      float* la = lds + buf * BUF;
      float* lb = la + BM * BK;
      const int wv = tid >> 6;
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        if ((c * IL_SPAN) / NCH != idx) continue;
        const bool is_a = c < A_CH;
        const int i = is_a ? c : c - A_CH;
        const int row = crow + i * ROWS_PER_PASS;
        const ET* src = (is_a ? a_ptr[is_a ? i : 0] : b_ptr[is_a ? 0 : i]) + (long long)kc * EPR + swz<BK>(row, slot) * CH;
        __builtin_amdgcn_global_load_lds((const void*)src,
                                         (__attribute__((address_space(3))) void*)((is_a ? la : lb) +
                                                                                   (i * ROWS_PER_PASS + wv * (64 / SLOTS)) * BK),
                                         16, 0, 0);
      }
    }
  };

  auto store_tile = [&](int buf) {
    float* la = lds + buf * BUF;
    float* lb = la + BM * BK;
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const int row = crow + i * ROWS_PER_PASS;
      *reinterpret_cast<f32x4*>(la + row * BK + swz<BK>(row, slot) * 4) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      const int row = crow + i * ROWS_PER_PASS;
      *reinterpret_cast<f32x4*>(lb + row * BK + swz<BK>(row, slot) * 4) = rb[i];
    }
  };

  f32x16 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  // MF16: sub-tile t = 2a + b (row half a, column half b) of tile (i, j)
  f32x4 acc4[MF16 ? FM : 1][MF16 ? FN : 1][4];
  if constexpr (MF16) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int t = 0; t < 4; ++t) acc4[i][j][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  const int lr = lane & 31, lh = lane >> 5;

  // EP_LNFOLD: each of the tile's rows combines its producer's partials once,
  // before the k-loop (the prologue's barrier publishes them to the epilogue)
  if constexpr (LNF) {
    if (tid < BM) {
      const f32x4 r = m0 + tid < g.M ? ln_row_stats(g.stats_in, m0 + tid, g.stats_k, g.ln_eps) : f32x4{0.f, 0.f, 0.f, 0.f};
      *reinterpret_cast<f32x4*>(lds + 2 * BUF + LN_ROW * tid) = r;
    }
    // the tile's column sums per k tile (colsum [T][N]), zero past N and T
    const int T = (g.stats_k + 255) >> 8;
    for (int i = tid; i < LN_TMAX * BN / 4; i += NT) {
      const int t = i / (BN / 4), c = (i - t * (BN / 4)) * 4;
      const f32x4 v = (t < T && n0 + c < g.N) ? *reinterpret_cast<const f32x4*>(g.colsum + (long long)t * g.N + n0 + c)
                                              : f32x4{0.f, 0.f, 0.f, 0.f};
      *reinterpret_cast<f32x4*>(lds + 2 * BUF + LN_ROW * BM + t * BN + c) = v;
    }
  }

  // bf16 16x16x32 with LDS-DMA: the barrier of k-tile kt sits inside its last
  // k-step, after that step's fragments are in registers: wait for tile kt+1's
  // DMA, barrier, DMA tile kt+2 into the buffer just drained, read tile kt+1's
  // first fragments, THEN the last step's MFMAs — they hide the post-barrier
  // LDS latency that otherwise idles both waves of every SIMD at each k-tile.
  constexpr bool PIPE16 = GL && MF16 == 1 && DT == DT_BF16;
  if constexpr (PIPE16) {
    constexpr int S = BK / 16;
    static_assert(S % 2 == 0, "PIPE16: an even number of k-steps per k-tile");
    const int l16 = lane & 15, lg = lane >> 4;
    bf16x8 af[2][FM][2], bf[2][FN][2];
    auto rd = [&](int buf, int st, bf16x8 (*a)[2], bf16x8 (*b)[2]) {
      const float* la = lds + buf * BUF;
      const float* lb = la + BM * BK;
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int row = wm * WTM + i * 32 + h * 16 + l16;
          a[i][h] = *reinterpret_cast<const bf16x8*>(la + row * BK + swz<BK>(row, 4 * st + lg) * 4);
        }
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int row = wn * WTN + j * 32 + h * 16 + l16;
          b[j][h] = *reinterpret_cast<const bf16x8*>(lb + row * BK + swz<BK>(row, 4 * st + lg) * 4);
        }
    };
    glds_tile(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (nk > 1) glds_tile(1, 1);
    rd(0, 0, af[0], bf[0]);
    __builtin_amdgcn_s_setprio(1);
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      auto mfmas = [&](int st) {
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
#pragma unroll
            for (int t = 0; t < 4; ++t)
              acc4[i][j][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[st & 1][i][t >> 1], bf[st & 1][j][t & 1],
                                                                      acc4[i][j][t], 0, 0, 0);
      };
#pragma unroll
      for (int st = 0; st < S; ++st) {
        if (st + 1 < S) {
          // next step's reads between this step's MFMAs
          mfmas(st);
          rd(cur, st + 1, af[(st + 1) & 1], bf[(st + 1) & 1]);
          interleave<2 * (FM + FN), 4 * FM * FN>();
        } else {
          // this step's fragments: waited for and redefined by an empty asm
          // on both paths, so the MFMAs below (one copy: two spill the
          // accumulators) wait for nothing — not for the next tile's reads
          auto settle = [&]() {
#pragma unroll
            for (int i = 0; i < FM; ++i)
#pragma unroll
              for (int h = 0; h < 2; ++h) asm volatile("" : "+v"(af[st & 1][i][h]));
#pragma unroll
            for (int j = 0; j < FN; ++j)
#pragma unroll
              for (int h = 0; h < 2; ++h) asm volatile("" : "+v"(bf[st & 1][j][h]));
          };
          __builtin_amdgcn_sched_barrier(0);  // the previous step's MFMAs stay above the wait
          settle();
          if constexpr (IL) {
            // tile kt+2's DMA chunk by chunk among this step's MFMAs, into the
            // buffer the barrier just freed.  Past the last tile it fetches the
            // last tile again (an L2 hit); in the last iteration (no barrier:
            // other waves may still read buffer cur) into buffer cur ^ 1, free
            // since the previous iteration's barrier.  The epilogue's
            // __syncthreads retires it.
            if (kt + 1 < nk) {
              asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
              __builtin_amdgcn_s_barrier();
              rd(cur ^ 1, 0, af[0], bf[0]);
            }
            // issued as one burst in the source; the scheduler spreads it
            // (interleave_il's VMEM groups: one DMA per 4 FM FN / NCH MFMAs)
            glds_tile(min(kt + 2, nk - 1), kt + 1 < nk ? cur : cur ^ 1);
            mfmas(st);
            interleave_il<4 * FM * FN, IL_SPAN, NCH>(0, 0);
          } else {
          if (kt + 1 < nk) {
            // every wave is done with buffer cur; tile kt+1's DMA has landed
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            if (kt + 2 < nk) glds_tile(kt + 2, cur);
            rd(cur ^ 1, 0, af[0], bf[0]);
          }
          mfmas(st);
          }
        }
      }
    }
    __builtin_amdgcn_s_setprio(0);
    if constexpr (IL) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the last spread DMA
    __syncthreads();  // every wave's last reads done: the epilogue reuses the LDS
  } else {
  if constexpr (GL) {
    glds_tile(0, 0);
    __syncthreads();
  } else {
    load_tile(0);
    store_tile(0);
    __syncthreads();
  }

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (!IL && kt + 1 < nk) {
      if constexpr (GL) glds_tile(kt + 1, cur ^ 1);
      else load_tile(kt + 1);
    }
    const float* la = lds + cur * BUF;
    const float* lb = la + BM * BK;
    if constexpr (DT == DT_F32) {
#pragma unroll
    for (int c2 = 0; c2 < BK / 16; ++c2) {
      f32x4 af[FM][2], bf[FN][2];
      const int s0 = c2 * 4 + 2 * lh;
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int row = wm * WTM + i * 32 + lr;
        af[i][0] = *reinterpret_cast<const f32x4*>(la + row * BK + swz<BK>(row, s0) * 4);
        af[i][1] = *reinterpret_cast<const f32x4*>(la + row * BK + swz<BK>(row, s0 + 1) * 4);
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int row = wn * WTN + j * 32 + lr;
        bf[j][0] = *reinterpret_cast<const f32x4*>(lb + row * BK + swz<BK>(row, s0) * 4);
        bf[j][1] = *reinterpret_cast<const f32x4*>(lb + row * BK + swz<BK>(row, s0 + 1) * 4);
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i][e >> 2][e & 3], bf[j][e >> 2][e & 3],
                                                             acc[i][j], 0, 0, 0);
      }
    }
    } else if constexpr (DT == DT_BF16 && MF16 == 2) {
      // MF16 = 2 (the 256x320 filter sweep on v_mfma_f32_16x16x32_bf16): one
      // fragment set per 32-deep k-step, read whole before its MFMAs (two sets
      // do not fit beside the 160 accumulator registers); the partner wave on
      // the SIMD covers the read latency.  Same lane -> k map as below.
      constexpr int S = BK / 16;
      const int l16 = lane & 15, lg = lane >> 4;
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int st = 0; st < S; ++st) {
        bf16x8 af[FM][2], bf[FN][2];
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int row = wm * WTM + i * 32 + h * 16 + l16;
            af[i][h] = *reinterpret_cast<const bf16x8*>(la + row * BK + swz<BK>(row, 4 * st + lg) * 4);
          }
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int row = wn * WTN + j * 32 + h * 16 + l16;
            bf[j][h] = *reinterpret_cast<const bf16x8*>(lb + row * BK + swz<BK>(row, 4 * st + lg) * 4);
          }
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int t = 0; t < 4; ++t) {
              glds_due(kt + 1, cur ^ 1, st * 4 * FM * FN + (j * FM + i) * 4 + t);
              acc4[i][j][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][t >> 1], bf[j][t & 1], acc4[i][j][t], 0, 0, 0);
            }
        if constexpr (IL) interleave_il<4 * FM * FN, IL_SPAN, NCH>(st * 4 * FM * FN, 0);
      }
      __builtin_amdgcn_s_setprio(0);
    } else if constexpr (DT == DT_BF16 && MF16) {
      // BK/16 k-steps of 32; lane group g = lane>>4 holds k = 32s + 8g .. +7
      // = 16-B slot 4s + g of rows (lane & 15) of each 16-row half.
      constexpr int S = BK / 16;
      const int l16 = lane & 15, lg = lane >> 4;
      bf16x8 af[2][FM][2], bf[2][FN][2];
      auto rd = [&](int st, bf16x8 (*a)[2], bf16x8 (*b)[2]) {
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int row = wm * WTM + i * 32 + h * 16 + l16;
            a[i][h] = *reinterpret_cast<const bf16x8*>(la + row * BK + swz<BK>(row, 4 * st + lg) * 4);
          }
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int row = wn * WTN + j * 32 + h * 16 + l16;
            b[j][h] = *reinterpret_cast<const bf16x8*>(lb + row * BK + swz<BK>(row, 4 * st + lg) * 4);
          }
      };
      rd(0, af[0], bf[0]);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int st = 0; st < S; ++st) {
        if (st + 1 < S) rd(st + 1, af[(st + 1) & 1], bf[(st + 1) & 1]);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
#pragma unroll
            for (int t = 0; t < 4; ++t)
              acc4[i][j][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[st & 1][i][t >> 1], bf[st & 1][j][t & 1],
                                                                      acc4[i][j][t], 0, 0, 0);
        if (st + 1 < S) interleave<2 * (FM + FN), 4 * FM * FN>();
      }
      __builtin_amdgcn_s_setprio(0);
    } else if constexpr (DT == DT_BF16) {
      // BK/8 k-steps of 16; lane half h holds k = 16s + 8h .. +7 = 16-B slot 2s + h.
      // Fragments are double-buffered in registers: step s+1's ds_reads are
      // issued before step s's MFMAs, so LDS latency hides under the MFMAs.
      constexpr int S = BK / 8;
      bf16x8 af[2][FM], bf[2][FN];
      auto rd = [&](int st, bf16x8* a, bf16x8* b) {
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const int row = wm * WTM + i * 32 + lr;
          a[i] = *reinterpret_cast<const bf16x8*>(la + row * BK + swz<BK>(row, 2 * st + lh) * 4);
        }
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int row = wn * WTN + j * 32 + lr;
          b[j] = *reinterpret_cast<const bf16x8*>(lb + row * BK + swz<BK>(row, 2 * st + lh) * 4);
        }
      };
      rd(0, af[0], bf[0]);
      // MFMA cluster at raised priority (cdna_hip_programming.md T5; measured
      // +2 % on the ViT linears and the bf16 sweep)
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int st = 0; st < S; ++st) {
        if (st + 1 < S) rd(st + 1, af[(st + 1) & 1], bf[(st + 1) & 1]);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            glds_due(kt + 1, cur ^ 1, st * FM * FN + i * FN + j);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[st & 1][i], bf[st & 1][j], acc[i][j], 0, 0, 0);
          }
        if constexpr (IL) interleave_il<FM * FN, IL_SPAN, NCH>(st * FM * FN, st + 1 < S ? FM + FN : 0);
        else if (st + 1 < S) interleave<FM + FN, FM * FN>();
      }
      __builtin_amdgcn_s_setprio(0);
    } else {
      // fp8 on the block-scaled v_mfma_scale_f32_32x32x64_f8f6f4 (e4m3 both
      // operands, every E8M0 block scale = 127 = 1.0; the per-row fp32 scales
      // stay in the epilogue): 2x the k per clock of the non-scaled
      // 32x32x16_fp8 form.  BK/16 k-steps of 64; lane half h holds the 32
      // bytes of 16-B slots 4s+2h, 4s+2h+1.  A and B fragments are read by
      // the same lane->k map, so each dot product covers every k once.
      constexpr int S = BK / 16;
      i32x8 af[2][FM], bf[2][FN];
      auto rd32 = [&](const float* base, int row, int st) {
        const i32x4 lo = *reinterpret_cast<const i32x4*>(base + row * BK + swz<BK>(row, 4 * st + 2 * lh) * 4);
        const i32x4 hi = *reinterpret_cast<const i32x4*>(base + row * BK + swz<BK>(row, 4 * st + 2 * lh + 1) * 4);
        return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      };
      auto rd = [&](int st, i32x8* a, i32x8* b) {
#pragma unroll
        for (int i = 0; i < FM; ++i) a[i] = rd32(la, wm * WTM + i * 32 + lr, st);
#pragma unroll
        for (int j = 0; j < FN; ++j) b[j] = rd32(lb, wn * WTN + j * 32 + lr, st);
      };
      rd(0, af[0], bf[0]);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int st = 0; st < S; ++st) {
        // IL: the next k-tile's DMA as one burst in the source, spread by the
        // scheduler among the first k-step's MFMAs (past the last k-tile: the
        // last one again, into the drained buffer)
        if (IL && st == 0) glds_tile(min(kt + 1, nk - 1), cur ^ 1);
        if (st + 1 < S) rd(st + 1, af[(st + 1) & 1], bf[(st + 1) & 1]);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(af[st & 1][i], bf[st & 1][j], acc[i][j],
                                                                         0, 0, 0, 127, 0, 127);
        if constexpr (IL) {
          if (st == 0) interleave_il<FM * FN, IL_SPAN, NCH, 2>(0, st + 1 < S ? FM + FN : 0);
          else if (st + 1 < S) interleave2<FM + FN, FM * FN>();
        } else if (st + 1 < S) {
          interleave2<FM + FN, FM * FN>();
        }
      }
      __builtin_amdgcn_s_setprio(0);
    }
    if constexpr (!GL) {
      if (kt + 1 < nk) store_tile(cur ^ 1);
    }
    __syncthreads();  // with GL: also the vmcnt(0) that retires the DMA
  }
  }
  if constexpr (MF16) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[i][j][4 * t + r] = acc4[i][j][t][r];
  }

  // ---- epilogue ----
  // 32x32 C/D map: col (N index) = lane & 31, row (M index) = (r&3) + 8(r>>2) + 4(lane>>5)
  // per-row dequantisation (fp8 only; bf16 / fp32 rows are unscaled — compiled
  // into those kernels, this block's 160 hoisted scale loads spilled ~150 VGPRs
  // of the 256x320 bf16 sweep tile).  Row scales one at a time, the FN column
  // scales held.
  if constexpr (!MF16 && DT == DT_FP8) {
    if (g.scale_a != nullptr || g.scale_b != nullptr) {
      float sb[FN];
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int n = n0 + wn * WTN + j * 32 + lr;
        sb[j] = (g.scale_b != nullptr && n < g.N) ? g.scale_b[n] : 1.f;
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + wm * WTM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
          const float sa = (g.scale_a != nullptr && m < g.M) ? g.scale_a[m] : 1.f;
#pragma unroll
          for (int j = 0; j < FN; ++j) acc[i][j][r] = acc[i][j][r] * sa * sb[j];
        }
    }
  }
  if constexpr (MF16 && EMODE == E_SCORES_T) {
    // sub-tile t: rows acc_row(i, 4t) .. +3 (consecutive), one column
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int n = n0 + wn * WTN + acc_col<true>(j, 4 * q, lane);
          const int mb = m0 + wm * WTM + acc_row<true>(i, 4 * q, lane);
          if (n >= g.N) continue;
          float* dst = g.C + (long long)n * g.ldc + mb;
          if (mb + 3 < g.M) {
            *reinterpret_cast<f32x4*>(dst) =
                f32x4{acc[i][j][4 * q], acc[i][j][4 * q + 1], acc[i][j][4 * q + 2], acc[i][j][4 * q + 3]};
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
              if (mb + e < g.M) dst[e] = acc[i][j][4 * q + e];
          }
        }
  } else if constexpr (MF16 && EMODE == E_FILTER) {
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int n = n0 + wn * WTN + acc_col<true>(j, 4 * b, lane);
        const bool nok = n < g.N;
        const float t = nok ? g.tau[n] : __builtin_inff();
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int r = 8 * a + 4 * b + e;
              const int m = m0 + wm * WTM + acc_row<true>(i, r, lane);
              const float v = acc[i][j][r];
              if (nok && m < g.M && !(v <= t)) {
                const int pos = atomicAdd(g.cnt + n, 1);
                if (pos < g.cap) g.cand[(long long)n * g.cap + pos] = make_key(v, (uint32_t)(g.row_offset + m));
              }
            }
      }
  } else {
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int n = n0 + wn * WTN + j * 32 + lr;
    const bool nok = n < g.N;
    if constexpr (EMODE == E_STORE) {
      // handled below through LDS
    } else if constexpr (EMODE == E_SCORES_T) {
#pragma unroll
      for (int i = 0; i < FM; ++i) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int mb = m0 + wm * WTM + i * 32 + 8 * q + 4 * lh;
          if (!nok) continue;
          float* dst = g.C + (long long)n * g.ldc + mb;
          if (mb + 3 < g.M) {
            *reinterpret_cast<f32x4*>(dst) =
                f32x4{acc[i][j][4 * q], acc[i][j][4 * q + 1], acc[i][j][4 * q + 2], acc[i][j][4 * q + 3]};
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
              if (mb + e < g.M) dst[e] = acc[i][j][4 * q + e];
          }
        }
      }
    } else {  // E_FILTER: keep only scores strictly above the query's threshold
      // (as !(v <= t): a NaN score, or every score under a NaN threshold, is
      // kept; the NaN keys rank last in select_final, see ord_f32).  Padding
      // query columns (n >= N) are excluded explicitly: a NaN gallery row gives
      // NaN there too, and no counter exists for them.
      const float t = nok ? g.tau[n] : __builtin_inff();
#pragma unroll
      for (int i = 0; i < FM; ++i) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + wm * WTM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
          const float v = acc[i][j][r];
          if (nok && m < g.M && !(v <= t)) {
            const int pos = atomicAdd(g.cnt + n, 1);
            if (pos < g.cap) g.cand[(long long)n * g.cap + pos] = make_key(v, (uint32_t)(g.row_offset + m));
          }
        }
      }
    }
  }
  }

  if constexpr (EMODE == E_STORE)
    epilogue_store<WM, WN, FM, FN, 2 * BUF, (bool)MF16, EPI>(g, Cb, acc, lds, m0, n0, 1.f, LNF ? lds + 2 * BUF : nullptr);
}

template <int WM, int WN, int FM, int FN, int AM, int EM, int BK, int DT, int MINB, int GL = 0, int MF16 = 0,
          int EPI = -1, int IL = 0>
static hipError_t launch_t1(const GemmArgs& g, hipStream_t s) {
  constexpr int BM = 32 * FM * WM, BN = 32 * FN * WN;
  const long long tiles_m = (g.M + BM - 1) / BM;
  const long long tiles_n = (g.N + BN - 1) / BN;
  const long long nblk = tiles_m * tiles_n;
  if (nblk <= 0) return hipSuccess;
  if (nblk > 0x7fffffffLL) return hipErrorInvalidValue;
  const unsigned splits = g.k_split > 0 ? (unsigned)((g.K + g.k_split - 1) / g.k_split) : 1u;
  hipLaunchKernelGGL((gemm_kernel<WM, WN, FM, FN, AM, EM, BK, DT, MINB, GL, MF16, EPI, IL>), dim3((unsigned)nblk, splits),
                     dim3(64 * WM * WN), 0, s, g, (int)tiles_n);
  return hipGetLastError();
}

// bf16 stored-C GEMMs (the ViT linears) with their epilogues compiled in:
// QKV (bias -> bf16), out-proj / fc2 (bias + residual, fp32), fc1 (bias +
// QuickGELU -> bf16); everything else reads its flags at run time.
template <int WM, int WN, int FM, int FN, int AM, int EM, int BK, int DT, int MINB, int GL = 0, int MF16 = 0, int IL = 0>
static hipError_t launch_t(const GemmArgs& g, hipStream_t s) {
  if constexpr (EM == E_STORE && DT == DT_BF16) {
    switch (ep_flags(g)) {
      case EP_BIAS | EP_BF16:
        return launch_t1<WM, WN, FM, FN, AM, EM, BK, DT, MINB, GL, MF16, EP_BIAS | EP_BF16, IL>(g, s);
      case EP_BIAS | EP_RES: return launch_t1<WM, WN, FM, FN, AM, EM, BK, DT, MINB, GL, MF16, EP_BIAS | EP_RES, IL>(g, s);
      case EP_BIAS | EP_GELU | EP_BF16:
        return launch_t1<WM, WN, FM, FN, AM, EM, BK, DT, MINB, GL, MF16, EP_BIAS | EP_GELU | EP_BF16, IL>(g, s);
      default: break;
    }
    // the ViT LayerNorm fold (256-column tiles only; rr_linear_bf16_ln forces lp_cfg 3)
    if constexpr (32 * FN * WN == 256 && MF16 == 1) {
      switch (ep_flags(g)) {
        case EP_BIAS | EP_RES | EP_STATS:
          return launch_t1<WM, WN, FM, FN, AM, EM, BK, DT, MINB, GL, MF16, EP_BIAS | EP_RES | EP_STATS, IL>(g, s);
        case EP_BIAS | EP_BF16 | EP_LNFOLD:
          return launch_t1<WM, WN, FM, FN, AM, EM, BK, DT, MINB, GL, MF16, EP_BIAS | EP_BF16 | EP_LNFOLD, IL>(g, s);
        case EP_BIAS | EP_GELU | EP_BF16 | EP_LNFOLD:
          return launch_t1<WM, WN, FM, FN, AM, EM, BK, DT, MINB, GL, MF16, EP_BIAS | EP_GELU | EP_BF16 | EP_LNFOLD,
                           IL>(g, s);
        default: break;
      }
    }
    if (g.stats_out != nullptr || g.stats_in != nullptr) return hipErrorInvalidValue;
  }
  return launch_t1<WM, WN, FM, FN, AM, EM, BK, DT, MINB, GL, MF16, -1, IL>(g, s);
}

// k-tile depth.  Measured on MI355X (same device, interleaved A/B): BK = 16
// (3 blocks per CU) is +2.5 % on the long-K, huge-grid cosine GEMM, BK = 32
// (2 blocks per CU) is +4.8 % on the ResNet convs.
static int pick_bk(int emode, const rr_handle_s::Tuning& t) {
  if (t.gemm_bk == 16 || t.gemm_bk == 32) return t.gemm_bk;
  return emode == E_STORE ? 32 : 16;
}

// Tile choice: both configs run 4 waves and 2 workgroups per CU (512 slots
// on 256 CUs).  Estimated time ~ rounds x tile area, rounds = ceil(tiles /
// 512): this charges both the padding of N (e.g. 320 queries on 128-wide
// tiles) and the last partially-filled round (wave quantization).
static int pick_cfg(const GemmArgs& g, int emode, const rr_handle_s::Tuning& tu) {
  if (tu.gemm_cfg == 22 || tu.gemm_cfg == 41) return tu.gemm_cfg;
  if (tu.gemm_cfg == 88) return (emode == E_STORE && pick_bk(emode, tu) == 32) ? 88 : 22;
  const long long slots = pick_bk(emode, tu) == 16 ? 768 : 512;
  const long long t22 = ((g.M + 127) / 128) * ((g.N + 127) / 128);
  const long long t41 = ((g.M + 255) / 256) * ((g.N + 63) / 64);
  const long long c22 = ((t22 + slots - 1) / slots) * 128 * 128;
  const long long c41 = ((t41 + slots - 1) / slots) * 256 * 64;
  // 88 (256x256, 1 block/CU) measured per R101 layer: +3-7 % on long-K GEMMs
  // without a residual (3x3 256@14, 1024->512/2048), -5..-30 % on residual
  // epilogues and short K, -40 % when the grid leaves CUs idle.  So: no
  // residual, K >= 1024, N a multiple of 256, ~a full round.
  if (emode == E_STORE && g.k_split == 0 && g.residual == nullptr && g.K >= 1024 && (g.N % 256) == 0 &&
      pick_bk(emode, tu) == 32) {
    const long long t88 = ((g.M + 255) / 256) * (g.N / 256);
    const long long c88 = ((t88 + 255) / 256) * 256 * 256;  // 1 block/CU vs 2 for 22: compare per CU
    if (t88 >= 240 && (double)c88 / 1.05 < (double)std::min(c22, c41) * 2.0) return 88;
  }
  return c41 < c22 ? 41 : 22;
}

template <int AM, int EM>
static hipError_t launch_cfg(const GemmArgs& g, hipStream_t s, const rr_handle_s::Tuning& tu) {
  const int cfg = pick_cfg(g, EM, tu);
  if (pick_bk(EM, tu) == 16) {
    if (cfg == 41) return launch_t<4, 1, 2, 2, AM, EM, 16, DT_F32, 3>(g, s);
    return launch_t<2, 2, 2, 2, AM, EM, 16, DT_F32, 3>(g, s);
  }
  if (cfg == 41) return launch_t<4, 1, 2, 2, AM, EM, 32, DT_F32, 2>(g, s);
  if constexpr (EM == E_STORE && (AM == A_DENSE || AM == A_CONV)) {
    // 88: 256x256, 8 waves of 128x64, 1 block per CU
    if (cfg == 88) return launch_t<2, 4, 4, 2, AM, EM, 32, DT_F32, 1>(g, s);
  }
  return launch_t<2, 2, 2, 2, AM, EM, 32, DT_F32, 2>(g, s);
}

// Low precision (dense A only, 128-B LDS rows).  Configs (waves WMxWN, MFMA
// tiles per wave FMxFN, blocks per CU):
//   1: 128x128, 4 waves of 64x64, 2/CU      2: 256x64, 4 waves of 64x64, 2/CU
//   3: 256x256, 8 waves of 128x64, 1/CU (128 KB LDS) — the large GEMMs
//   4: 256x320, 8 waves of 64x160, 1/CU (144 KB) — a 320-query batch in
//      one tile column: the streamed gallery is read exactly once (filter
//      and score sweeps only)
//   5: 256x256 on the 8-phase LDS-DMA pipeline of gemm_8p.hip (bf16, K %
//      128 == 0; picked for long-K filter sweeps whose query count 256-wide
//      panels tile better than 320-wide ones)
// picked by estimated rounds x tile area (rr_set_tuning(RR_TUNE_LP_CFG) forces).
// Not kept: the 8-phase pipeline for the ViT linears (2-4 %
// slower: short K) and the 256x320 tile on a 4-stage 64-B-row LDS-DMA ring
// (7.59 vs 6.94 ms per C3 sweep).
static int pick_lp(const GemmArgs& g, int emode, bool dt_bf16, const rr_handle_s::Tuning& tu) {
  if (tu.lp_cfg >= 1 && tu.lp_cfg <= 3) return tu.lp_cfg;
  if (tu.lp_cfg == 5) return emode == E_STORE ? 3 : 5;
  if (tu.lp_cfg == 4) return emode == E_STORE ? 3 : 4;
  // rounds x tile area / relative per-FLOP speed (measured, tools/lp_bench.py:
  // the 8-wave tiles run ViT linears 1.2-1.3x faster than 128x128; the
  // 320-query tile runs the bf16 d=2048 sweep 1.35x faster, but not d=512 or
  // fp8, where 4-wave tiles win)
  // (a round of `slots` resident blocks lasts ~ tile area x blocks per CU)
  auto cost = [&](long long bm, long long bn, long long slots, double speed) {
    const long long t = ((g.M + bm - 1) / bm) * ((g.N + bn - 1) / bn);
    return (double)((t + slots - 1) / slots) * bm * bn * (slots / 256) / speed;
  };
  double best = cost(128, 128, 512, 1.0);
  int cfg = 1;
  if (cost(256, 64, 512, 1.0) < best) best = cost(256, 64, 512, 1.0), cfg = 2;
  if (emode == E_STORE && cost(256, 256, 256, 1.25) < best) best = cost(256, 256, 256, 1.25), cfg = 3;
  // filter sweeps other than the long-K bf16 one (which takes 4 below):
  // the 8-wave 256x256 tile wins at >= 1024 queries (measured at 1280 queries
  // x 1.6 M rows: bf16 d = 512 3.27 -> 2.39 ms, fp8 d = 2048 11.2 -> 8.1 ms
  // per C5 step); at 320 queries the cost model keeps 128x128
  if (emode == E_FILTER && (g.K < 1024 || g.scale_a != nullptr) && cost(256, 256, 256, 1.25) < best)
    best = cost(256, 256, 256, 1.25), cfg = 3;
  if (emode != E_STORE && g.K >= 1024 && g.scale_a == nullptr && cost(256, 320, 256, 1.35) < best)
    best = cost(256, 320, 256, 1.35), cfg = 4;
  // the 8-phase 256x256 pipeline (gemm_8p.hip) on the long-K bf16 sweeps:
  // measured (tools/sweep_ab.py, random queries x 1.6 M x 2048) 1.22-1.25x the
  // 256x320 tile at 256 / 512 / 768 queries (no padded query columns), 1.03x
  // at 1280 and slower at 320 (256 + 64 padded); so it must win by padding
  if (emode != E_STORE && dt_bf16 && g.K >= 1024 && (g.K % 128) == 0 && cost(256, 256, 256, 1.35 * 1.03) < best * 0.97)
    best = cost(256, 256, 256, 1.35 * 1.03), cfg = 5;
  return cfg;
}

// bf16 runs on four v_mfma_f32_16x16x32_bf16 per 32x32 tile (MF16; measured:
// ViT-B/16 linears +4-7 %, 128x128 cosine sweeps +2-5 % over 32x32x16), except
// the 256x320 sweep tile, whose 16x16 fragments spill (180 B/lane).
template <int EM, int DT>
static hipError_t launch_lp_cfg(const GemmArgs& g, hipStream_t s, int cfg);

template <int EM, int DT>
static hipError_t launch_lp(const GemmArgs& g, hipStream_t s, const rr_handle_s::Tuning& tu) {
  constexpr int EPR = DT == DT_BF16 ? 64 : 128;  // elements per 128-B k-tile row
  int cfg = pick_lp(g, EM, DT == DT_BF16, tu);
  if (g.stats_out != nullptr || g.stats_in != nullptr) cfg = 3;  // the LayerNorm fold: 256-column tiles
  if ((cfg == 3 || cfg == 4) && (g.K % EPR) != 0) cfg = 1;  // LDS-DMA configs need whole k-tiles
  if constexpr (EM == E_FILTER && DT == DT_BF16) {
    // the hand-scheduled 16x16x32 sweep on 128-B LDS rows (sweep16.hip): the
    // pick for K >= 1024 (the C3 prefilter's 1.6 M x 2048 sweep).  Measured
    // against the 256x320 tile below (tools/prefilter_ab.py, 1280 queries,
    // profiles/r06m_*): random queries 9.57 -> 7.26 ms, near-parallel 7.39 ->
    // 7.04, and 6.86 -> 7.01 on identical queries (the bench's random-weight
    // descriptors); at K = 512 (C4) 2.43 -> 2.49 ms, so short K keeps the tile
    const int form = tu.sweep_form >= 0 ? tu.sweep_form : (g.K >= 1024 && (g.K % 64) == 0 ? 1 : 0);
    if ((form == 1 || form == 2) && sweep16_eligible(g)) return launch_sweep16(g, s, form == 1);
  }
  if constexpr (EM == E_FILTER) {
    // the 256x320 bf16 tile's default: v_mfma_f32_32x32x16_bf16 with the next
    // k-tile's DMA spread among the MFMAs (sweep_il).  On the C3 bench's own
    // descriptors (tools/e2e_ab.py, profiles/r04j_e2e_ab.txt): 7.15 -> 6.81
    // ms; the 16x16x32 form is 7.71 ms there (7.08 with the spread), though
    // it won on synthetic near-parallel queries (r04f_sweep_il_ab.txt).
    // Bit-identical rankings in every form.
    GemmArgs g2 = g;
    g2.mf16_sweep = tu.sweep_mf16 > 0;
    // (sweep_il = 1 spreads every filter sweep's DMA, the 256x256 bf16 one
    // too; the default: the 256x320 bf16 and the fp8 sweeps -- C5's fp8
    // sweeps 7.70 -> 7.53 ms per step on the bench, profiles/r04k_c5_*.json)
    g2.issue_spread = tu.sweep_il > 0 || (tu.sweep_il < 0 && ((cfg == 4 && DT == DT_BF16) || DT == DT_FP8));
    return launch_lp_cfg<EM, DT>(g2, s, cfg);
  }
  return launch_lp_cfg<EM, DT>(g, s, cfg);
}

template <int EM, int DT>
static hipError_t launch_lp_cfg(const GemmArgs& g, hipStream_t s, int cfg) {
  constexpr int MF = DT == DT_BF16 ? 1 : 0;
  if (cfg == 5) {
    if constexpr (DT != DT_F32 && EM != E_STORE) {
      if (gemm_8p_eligible(g, DT)) return launch_gemm_8p(g, EM, s, DT);
    }
    cfg = 3;
  }
  switch (cfg) {
    case 2: return launch_t<4, 1, 2, 2, A_DENSE, EM, 32, DT, 2, 0, MF>(g, s);
    case 3:
      // (the next k-tile's DMA spread among the MFMAs: sweep_il, the filter
      // sweeps; on the ViT linears' stored-C tile it made the C4 embed slower,
      // 61.3 -> 62.4 ms, profiles/r04k_e2e_c4_il.txt, and was removed)
      if constexpr (EM == E_FILTER && DT != DT_F32) {
        if (g.issue_spread) return launch_t<2, 4, 4, 2, A_DENSE, EM, 32, DT, 1, 1, MF, 1>(g, s);
      }
      return launch_t<2, 4, 4, 2, A_DENSE, EM, 32, DT, 1, 1, MF>(g, s);
    case 4:  // bf16 sweeps only (fp8: the 256x256 tile; its 256x320 form spills the dequantisation)
      if constexpr (EM == E_FILTER && DT == DT_BF16) {
        if (g.mf16_sweep && g.issue_spread) return launch_t1<4, 2, 2, 5, A_DENSE, EM, 32, DT, 1, 1, 2, -1, 1>(g, s);
        if (g.mf16_sweep) return launch_t1<4, 2, 2, 5, A_DENSE, EM, 32, DT, 1, 1, 2>(g, s);
        if (g.issue_spread) return launch_t1<4, 2, 2, 5, A_DENSE, EM, 32, DT, 1, 1, 0, -1, 1>(g, s);
      }
      if constexpr (EM != E_STORE && DT == DT_BF16) return launch_t<4, 2, 2, 5, A_DENSE, EM, 32, DT, 1, 1, 0>(g, s);
      else if constexpr (EM != E_STORE) return launch_t<2, 4, 4, 2, A_DENSE, EM, 32, DT, 1, 1, MF>(g, s);
      return hipErrorInvalidValue;
    default: return launch_t<2, 2, 2, 2, A_DENSE, EM, 32, DT, 2, 0, MF>(g, s);
  }
}

int launch_gemm(rr_handle_s* h, int amode, int emode, const GemmArgs& g, hipStream_t s, int timer_cls, int dt) {
  if (g.M < 0 || g.N < 0 || g.K <= 0) return set_error(h, RR_EINVAL, "gemm: bad shape");
  if (dt != DT_F32) {
    const int vec = dt == DT_BF16 ? 8 : 16;  // elements per 16-B staging load
    if (amode != A_DENSE) return set_error(h, RR_EINVAL, "gemm: low-precision GEMM needs dense A");
    if ((g.K % vec) || (g.lda % vec) || (g.ldb % vec))
      return set_error(h, RR_EINVAL, "gemm: low-precision K / lda / ldb must be multiples of 16 bytes");
    if (emode == E_SCORES_T && (g.ldc & 3)) return set_error(h, RR_EINVAL, "gemm: ldc must be a multiple of 4");
    if (g.M == 0 || g.N == 0) return RR_OK;
    hipError_t e = hipSuccess;
    {
      TimedLaunch tl(h, timer_cls, s);
      if (dt == DT_BF16) {
        // the ViT linears' epilogue flag sets with K <= 1024: the persistent
        // 256x256 k-stream (gemm_lpp.hip), with three A stages where the
        // fold's LDS is not needed (lp_cfg 3 forces the one-tile kernel; 6
        // the three-A-stage form for the no-fold flag sets at any K).  Per
        // block of linears 4.51 -> 4.35 ms (profiles/r05u_vitlin.txt); the C4
        // embed 62.29 -> 61.54 ms with the first form (r05q_e2e_c4.txt)
        if (emode == E_STORE && lpp3_eligible(g) && (h->tune.lp_cfg == 6 || (h->tune.lp_cfg == 0 && g.K <= 1024)))
          e = launch_lpp3(g, s, device_cu_count(h));
        else if (emode == E_STORE && (h->tune.lp_cfg == 0 || h->tune.lp_cfg == 6) && lpp_eligible(g))
          e = launch_lpp(g, s, device_cu_count(h));
        else if (emode == E_STORE) e = launch_lp<E_STORE, DT_BF16>(g, s, h->tune);
        else if (emode == E_SCORES_T) e = launch_lp<E_SCORES_T, DT_BF16>(g, s, h->tune);
        else e = launch_lp<E_FILTER, DT_BF16>(g, s, h->tune);
      } else {
        if (emode == E_STORE) e = launch_lp<E_STORE, DT_FP8>(g, s, h->tune);
        else if (emode == E_SCORES_T) e = launch_lp<E_SCORES_T, DT_FP8>(g, s, h->tune);
        else e = launch_lp<E_FILTER, DT_FP8>(g, s, h->tune);
      }
    }
    return check_hip(h, e, "gemm launch");
  }
  if (amode != A_CONV_GENERIC && (g.K & 3) != 0) return set_error(h, RR_EINVAL, "gemm: K must be a multiple of 4");
  if (amode == A_DENSE && (g.lda & 3)) return set_error(h, RR_EINVAL, "gemm: lda must be a multiple of 4");
  if (amode != A_CONV_GENERIC && (g.ldb & 3) != 0) return set_error(h, RR_EINVAL, "gemm: ldb must be a multiple of 4");
  if (emode == E_SCORES_T && (g.ldc & 3)) return set_error(h, RR_EINVAL, "gemm: ldc must be a multiple of 4");
  if (amode == A_CONV && (g.Cin % 32) != 0) return set_error(h, RR_EINVAL, "gemm: A_CONV needs Cin % 32 == 0");
  if ((g.k_split > 0 || g.sym) && (amode != A_DENSE || emode != E_STORE))
    return set_error(h, RR_EINVAL, "gemm: split-K / symmetric mode needs dense A and a stored C");
  if (g.k_split > 0 && (g.k_split % 32) != 0) return set_error(h, RR_EINVAL, "gemm: k_split must be a multiple of 32");
  if (g.M == 0 || g.N == 0) return RR_OK;
  hipError_t e = hipSuccess;
  {
    TimedLaunch tl(h, timer_cls, s);
    if (amode == A_DENSE && emode == E_STORE) e = launch_cfg<A_DENSE, E_STORE>(g, s, h->tune);
    else if (amode == A_DENSE && emode == E_SCORES_T) e = launch_cfg<A_DENSE, E_SCORES_T>(g, s, h->tune);
    else if (amode == A_DENSE && emode == E_FILTER) e = launch_cfg<A_DENSE, E_FILTER>(g, s, h->tune);
    else if (amode == A_CONV && emode == E_STORE) e = launch_cfg<A_CONV, E_STORE>(g, s, h->tune);
    else if (amode == A_CONV_GENERIC && emode == E_STORE) e = launch_cfg<A_CONV_GENERIC, E_STORE>(g, s, h->tune);
    else if (amode == A_CONV_C4 && emode == E_STORE) e = launch_cfg<A_CONV_C4, E_STORE>(g, s, h->tune);
    else return set_error(h, RR_EINVAL, "gemm: unsupported mode combination");
  }
  return check_hip(h, e, "gemm launch");
}

}  // namespace rr
