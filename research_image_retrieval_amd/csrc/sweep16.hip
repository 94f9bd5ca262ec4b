// sweep16.hip — the bf16 cosine filter sweep (iris_evaluate.py:383, the
// similarity GEMM; pass 2 of rr_cosine_topk_prefilter and the bf16
// rr_cosine_topk_lp) on v_mfma_f32_16x16x32_bf16 with a hand-placed k-loop.
//
// Why a separate kernel.  The 256x320 filter tile of gemm_f32.hip leaves its
// k-loop schedule to hipcc, which waits lgkmcnt(0) right after issuing the
// next k-step's fragment reads (their latency is exposed once per 10 MFMAs)
// and runs on v_mfma_f32_32x32x16_bf16, whose 16x16x32 form holds a higher
// clock under load (MI355X_MICROARCH.md 'DVFS give-back' item 7).  Here every
// LDS read, LDS-DMA and wait is an asm statement placed by hand and the MFMAs
// are fenced between them with sched_barrier(0):
//   * tile 256 gallery rows x 320 queries (the C3 / C4 query batch of 1280 is
//     four panels; the streamed gallery tile is read once per panel from L2);
//     NW = 8 waves (2 per SIMD) of 64 x 160 or NW = 4 waves (1 per SIMD, 512
//     VGPRs) of 128 x 160 outputs;
//   * k-steps of 32 (one 64-B LDS row per operand row), FOUR LDS stages of
//     36 KB: the LDS-DMA of k-step t + 3 goes out during step t, so a load
//     has two steps to land and the loop never waits vmcnt(0);
//   * one barrier per k-step, at its top, after this wave's DMA of step t + 1
//     has landed (a counted vmcnt: step t + 2's DMA stays in flight);
//   * the next step's fragments are read during this step, 1-2 reads after
//     each group of FI MFMAs that share one query fragment, into the register
//     that group just released (the query fragments) or the second A buffer;
//     each group waits only for its own query fragment (a counted lgkmcnt);
//   * LDS rows are 64 B, logical 16-B slot s of row r at s ^ (3 * bit 3 of r):
//     every ds_read_b128 lane group of the 16-row fragment read covers the 64
//     banks once (MI355X_MICROARCH.md §LDS, ds_read_b128 lane groups).  The
//     DMA writes rows linearly; the swizzle is applied to its source slot.
// The filter epilogue is gemm_f32.hip's: every score s' > tau[query] (as
// !(s' <= tau)) is appended as a 64-bit key with one atomic per survivor.
// The bf16 products are exact in fp32 and the accumulation order is covered
// by the prefilter's bound (prefilter.hip), so the exact ranker's output does
// not depend on which sweep ran (tests/test_gpu_rank.py).
#include "rr_internal.hpp"

namespace rr {
namespace {

typedef float sw_f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 sw_bf16x8 __attribute__((ext_vector_type(8)));

constexpr int SW_BM = 256, SW_BN = 320, SW_ROWS = SW_BM + SW_BN;
constexpr int SW_STAGE = SW_ROWS * 64;  // bytes per stage: 576 rows x 32 bf16
constexpr int SW_NST = 4;
constexpr int SW_NCH = SW_ROWS / 16;  // LDS-DMA instructions per stage (16 rows x 64 B each)
constexpr int SW_FJ = 10;             // query fragments per wave (160 queries)
constexpr int SW_D = 3;               // a query fragment is read this many groups ahead
constexpr int SW_RB = 5;              // query fragment ring slots (SW_FJ % SW_RB == 0)

// physical 16-B slot of logical slot s in LDS row r: s ^ sw_swz(r)
__device__ __forceinline__ int sw_swz(int r) { return ((r >> 3) & 1) * 3; }

template <int NW>
struct SwCfg {
  static constexpr int WM = NW / 2;           // waves along the gallery rows
  static constexpr int FI = SW_BM / WM / 16;  // gallery fragments per wave
  static constexpr int NQ = (SW_NCH + NW - 1) / NW;  // DMA chunks per wave (at most)
  // the group after which gallery fragment i of the next step is read: all
  // before the last SW_D groups, so the reads issued after those groups are
  // query fragments only (the prologue issues them in the same order)
  static constexpr int JA(int i) { return i * (SW_FJ - SW_D) / FI; }
  // the group after which DMA chunk q of the step goes out
  static constexpr int DG(int q) { return (q * SW_FJ) / NQ; }
  static constexpr int A_AFTER(int x, bool next) {
    int n = 0;
    for (int i = 0; i < FI; ++i) n += (next && JA(i) == x) ? 1 : 0;
    return n;
  }
  // LDS reads issued after query fragment (t, j) and before group j's wait:
  // the gallery reads after groups j - D .. j - 1 of this step and the query
  // reads after groups j - D + 1 .. j - 1 (B(t, j + 1) .. B(t, j + D - 1);
  // those of the next step exist only when there is one)
  static constexpr int LW(int j, bool next) {
    int n = 0;
    for (int x = (j - SW_D > 0 ? j - SW_D : 0); x < j; ++x) n += A_AFTER(x, next);
    for (int x = j - SW_D + 1; x < j; ++x) n += (x + SW_D < SW_FJ || next) ? 1 : 0;
    return n;
  }
  static constexpr bool ok() {
    for (int j = 0; j < SW_FJ; ++j)
      if (LW(j, true) > 7 || LW(j, false) > 7) return false;
    for (int i = 0; i < FI; ++i)
      if (JA(i) >= SW_FJ - SW_D) return false;
    return true;
  }
};
static_assert(SwCfg<8>::ok() && SwCfg<4>::ok(), "sweep16: read schedule");

template <int N>
__device__ __forceinline__ void sw_lgkwait(sw_bf16x8& f) {
  asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(f) : "i"(N));
}

template <int OFF>
__device__ __forceinline__ void sw_read(sw_bf16x8& f, uint32_t addr) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "+v"(f) : "v"(addr), "i"(OFF));
}

typedef int sw_i32x4 __attribute__((ext_vector_type(4)));

// 16 rows x 64 B of one operand into LDS at m0v: lane l's 16 B from byte
// soff + voff[l] of the buffer srd (rows past the operand's last valid row
// fail the descriptor's range check and land as zeros)
__device__ __forceinline__ void sw_dma(uint32_t voff, sw_i32x4 srd, uint32_t soff, uint32_t m0v) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %4\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %1, %2, %3 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(srd), "s"(soff), "s"(m0v)
      : "memory");
}

// vmcnt(n) for this wave's DMA count per step n (wave-uniform)
__device__ __forceinline__ void sw_vmwait(int n) {
  if (n == 5) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
  else if (n == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if (n == 9) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
__device__ __forceinline__ void sw_vmwait2(int n) {
  if (n == 5) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
  else if (n == 4) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if (n == 9) asm volatile("s_waitcnt vmcnt(18)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// the 16-row fragment (row block rb, k-step stage base) -> register f
template <int RB>
__device__ __forceinline__ void sw_read_rb(sw_bf16x8& f, uint32_t base) {
  sw_read<RB * 1024>(f, base);
}

// read query fragment jj (0..9) of the stage at rdB into ring slot jj % SW_RB
template <int JJ>
__device__ __forceinline__ void sw_read_b(sw_bf16x8 (&B)[SW_RB], uint32_t rdB) {
  sw_read_rb<JJ>(B[JJ % SW_RB], rdB);
}

// The filter epilogue (both kernels): lane holds rows 4 (lane >> 4) + r of
// each 16 x 16 tile, column lane & 15 (the v_mfma_f32_16x16x32 C/D map).
// Every score s' > tau[query] (as !(s' <= tau): a NaN score, or every score
// under a NaN threshold, is kept; padding columns n >= N are excluded
// explicitly) is appended to its query's candidate list as a 64-bit key.
// Survivors are counted per (wave, query column) first: the four lanes of a
// column exchange their counts (exclusive prefix by lane >> 4), the first of
// them takes the column's whole range with ONE returning atomic, the ten
// columns' atomics of a lane all in flight together, then every lane stores
// its keys at base + prefix + its own order.  The candidate order differs
// from one atomic per survivor; the lists are sets (the prefilter's rescoring
// and select_final rank them by key).
template <int FI>
__device__ __forceinline__ void sw_filter_epilogue(const GemmArgs& g, const sw_f32x4 (&acc)[FI][SW_FJ], int m_base,
                                                   int n_base, int lane, const float* tau_lds = nullptr,
                                                   int tau_off = 0) {
  const int lr = lane & 15, lg = lane >> 4;
  unsigned msk[SW_FJ];
  int pre[SW_FJ], base[SW_FJ];
#pragma unroll
  for (int j = 0; j < SW_FJ; ++j) {
    const int n = n_base + 16 * j + lr;
    const bool nok = n < g.N;
    // the thresholds: staged in LDS by the caller (+inf past N), or global
    const float tq = tau_lds != nullptr ? tau_lds[tau_off + 16 * j + lr] : (nok ? g.tau[n] : __builtin_inff());
    unsigned mk = 0u;
#pragma unroll
    for (int i = 0; i < FI; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m_base + 16 * i + 4 * lg + r;
        if (nok && m < g.M && !(acc[i][j][r] <= tq)) mk |= 1u << (4 * i + r);
      }
    msk[j] = mk;
    const int c = __builtin_popcount(mk);
    const int c0 = __shfl(c, lr, 64), c1 = __shfl(c, lr + 16, 64), c2 = __shfl(c, lr + 32, 64);
    const int c3 = __shfl(c, lr + 48, 64);
    pre[j] = (lg > 0 ? c0 : 0) + (lg > 1 ? c1 : 0) + (lg > 2 ? c2 : 0);
    const int tot = c0 + c1 + c2 + c3;
    base[j] = 0;
    if (lg == 0 && tot > 0) base[j] = atomicAdd(g.cnt + n, tot);
  }
#pragma unroll
  for (int j = 0; j < SW_FJ; ++j) {
    const int b0 = __shfl(base[j], lr, 64);
    unsigned mk = msk[j];
    if (mk == 0u) continue;
    const int n = n_base + 16 * j + lr;
    long long pos = (long long)b0 + pre[j];
#pragma unroll
    for (int i = 0; i < FI; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (mk & (1u << (4 * i + r))) {
          if (pos < g.cap)
            g.cand[(long long)n * g.cap + pos] =
                make_key(acc[i][j][r], (uint32_t)(g.row_offset + m_base + 16 * i + 4 * lg + r));
          ++pos;
        }
      }
  }
}

// One k-step: SW_FJ groups, group j = the FI MFMAs of query fragment (t, j)
// against the step's gallery fragments A[CUR][*].  After group j: the query
// fragment D groups ahead (the next step's first D past the step's end), then
// the next step's gallery fragments the JA schedule names, then the DMA
// chunks of step t + 3 the DG schedule names.  Past the last step the next
// step's reads fetch a stage nothing wrote (never used) and the DMA re-fetches
// the last step into the stage just freed: every step issues the same
// instructions, so the counted waits hold everywhere.
template <int NW, int CUR, int ABL>
__device__ __forceinline__ void sw_step(sw_bf16x8 (&A)[2][SwCfg<NW>::FI], sw_bf16x8 (&B)[SW_RB],
                                        sw_f32x4 (&acc)[SwCfg<NW>::FI][SW_FJ], uint32_t rdA_cur, uint32_t rdB_cur,
                                        uint32_t rdA_nxt, uint32_t rdB_nxt, uint32_t voffA, uint32_t voffB,
                                        sw_i32x4 srdA, sw_i32x4 srdB, uint32_t soffA, uint32_t soffB, long long lda2,
                                        long long ldb2, int has_last, uint32_t m0st, int wave) {
  using C = SwCfg<NW>;
  constexpr int FI = C::FI;
  static_assert(SW_FJ % SW_RB == 0 && SW_RB > SW_D, "sweep16: query ring");
#pragma unroll
  for (int j = 0; j < SW_FJ; ++j) {
    const int lw = C::LW(j, true);
    sw_bf16x8& bj = B[j % SW_RB];
    if constexpr (ABL & (4 | 32)) {
    } else switch (lw) {
      case 0: sw_lgkwait<0>(bj); break;
      case 1: sw_lgkwait<1>(bj); break;
      case 2: sw_lgkwait<2>(bj); break;
      case 3: sw_lgkwait<3>(bj); break;
      case 4: sw_lgkwait<4>(bj); break;
      case 5: sw_lgkwait<5>(bj); break;
      case 6: sw_lgkwait<6>(bj); break;
      default: sw_lgkwait<7>(bj); break;
    }
    if (j == 0) {
#pragma unroll
      for (int i = 0; i < FI; ++i) asm volatile("" : "+v"(A[CUR][i]));
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < FI; ++i)
      if constexpr (!(ABL & 8)) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[CUR][i], bj, acc[i][j], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
    // the query fragment D groups ahead
    if constexpr (ABL & 4) {
    } else switch (j + SW_D) {
      case 3: sw_read_b<3>(B, rdB_cur); break;
      case 4: sw_read_b<4>(B, rdB_cur); break;
      case 5: sw_read_b<5>(B, rdB_cur); break;
      case 6: sw_read_b<6>(B, rdB_cur); break;
      case 7: sw_read_b<7>(B, rdB_cur); break;
      case 8: sw_read_b<8>(B, rdB_cur); break;
      case 9: sw_read_b<9>(B, rdB_cur); break;
      case 10: sw_read_b<0>(B, rdB_nxt); break;
      case 11: sw_read_b<1>(B, rdB_nxt); break;
      default: sw_read_b<2>(B, rdB_nxt); break;
    }
#pragma unroll
    for (int i = 0; i < FI; ++i) {
      if (C::JA(i) != j || (ABL & 4)) continue;
      switch (i) {
        case 0: sw_read_rb<0>(A[CUR ^ 1][0], rdA_nxt); break;
        case 1: sw_read_rb<1>(A[CUR ^ 1][1 % FI], rdA_nxt); break;
        case 2: sw_read_rb<2>(A[CUR ^ 1][2 % FI], rdA_nxt); break;
        case 3: sw_read_rb<3>(A[CUR ^ 1][3 % FI], rdA_nxt); break;
        case 4: sw_read_rb<4>(A[CUR ^ 1][4 % FI], rdA_nxt); break;
        case 5: sw_read_rb<5>(A[CUR ^ 1][5 % FI], rdA_nxt); break;
        case 6: sw_read_rb<6>(A[CUR ^ 1][6 % FI], rdA_nxt); break;
        default: sw_read_rb<7>(A[CUR ^ 1][7 % FI], rdA_nxt); break;
      }
    }
    if constexpr (ABL & 16) {
      // DMA roles: waves 4..7 (one per SIMD) issue all 36 chunks, 9 each,
      // c = (wave - 4) + 4 q, after group q (q = 0..8)
      if (!(ABL & 1) && j < 9 && wave >= 4) {
        const int c = (wave - 4) + 4 * j;
        const uint32_t m0v = m0st + (uint32_t)c * 1024u;
        if (j < 4) sw_dma(voffA, srdA, soffA + (uint32_t)(16 * c * lda2), m0v);
        else sw_dma(voffB, srdB, soffB + (uint32_t)(16 * (c - 16) * ldb2), m0v);
      }
    } else {
#pragma unroll
    for (int q = 0; q < C::NQ; ++q) {
      if ((ABL & 256) ? j != 1 : C::DG(q) != j) continue;
      if (ABL & 1) continue;
      const int c = wave + NW * q;
      // chunks 0..15 are gallery rows, 16..35 query rows (per q a compile-
      // time fact for NW = 4 and 8: c < 16 iff NW * q + NW - 1 < 16)
      const uint32_t m0v = m0st + (uint32_t)c * 1024u;
      if (NW * q + NW - 1 < 16) {
        sw_dma(voffA, srdA, soffA + (uint32_t)(16 * c * lda2), m0v);
      } else if (q == C::NQ - 1 && C::NQ * NW > SW_NCH) {
        if (has_last) sw_dma(voffB, srdB, soffB + (uint32_t)(16 * (c - 16) * ldb2), m0v);
      } else {
        sw_dma(voffB, srdB, soffB + (uint32_t)(16 * (c - 16) * ldb2), m0v);
      }
    }
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

// ABL (tools/sweep_lab.hip ablations only; the library runs 0): 1 = no DMA
// in the loop, 2 = no vmcnt wait / barrier at the step top, 4 = no fragment
// reads in the loop, 8 = no MFMAs, 16 = DMA by waves 4..7 only, 32 = no
// lgkmcnt waits, 64 = in-kernel clock stamps (wave 0 of each block writes
// its shader-clock MHz over the k-loop to g.C[block]; diagnostic only)
template <int NW, int ABL = 0>
__global__ __launch_bounds__(64 * NW, 1) void sweep16_kernel(GemmArgs g, int tiles_n) {
  using C = SwCfg<NW>;
  constexpr int FI = C::FI, NQ = C::NQ, WTM = 16 * FI;
  static_assert(NW == 4 || NW == 8, "sweep16: 4 or 8 waves");
  static_assert(NW != 8 || (NQ == 5 && NW * 2 == 16), "sweep16: chunk layout (NW 8)");
  static_assert(NW != 4 || (NQ == 9 && NW * 4 == 16), "sweep16: chunk layout (NW 4)");
  __shared__ __attribute__((aligned(1024))) unsigned char lds[SW_NST * SW_STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave % C::WM, wn = wave / C::WM;
  int tm, tn;
  tile_coords(blockIdx.x, gridDim.x, tiles_n, tm, tn);
  const int m0 = tm * SW_BM, n0 = tn * SW_BN;
  const int nk = g.K >> 5;
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) unsigned char*)lds;

  // fragment reads: row r0 + (lane & 15), logical slot lane >> 4
  const int lr = lane & 15, lg = lane >> 4;
  const uint32_t lpart = (uint32_t)(lr * 64 + ((lg ^ sw_swz(lr)) << 4));
  const uint32_t rdA0 = lds0 + (uint32_t)(wm * WTM) * 64u + lpart;
  const uint32_t rdB0 = lds0 + (uint32_t)(SW_BM + wn * 160) * 64u + lpart;

  // LDS-DMA: chunk c = wave + NW q of a stage is its rows 16c .. 16c + 15
  // (gallery rows for c < 16, then query rows); lane l -> row 16c + (l >> 2),
  // physical slot l & 3 = logical slot (l & 3) ^ swz.  The row-in-chunk part
  // is the lane's buffer offset, the chunk and k-step parts the scalar
  // offset; each operand's descriptor covers its valid rows only.
  const int nq_w = (ABL & 16) ? (wave >= 4 ? 9 : 0) : (SW_NCH - wave + NW - 1) / NW;
  const int has_last = nq_w == C::NQ;
  const long long lda2 = g.lda * 2, ldb2 = g.ldb * 2;
  const int lrow = lane >> 2, lslot = (lane & 3) ^ sw_swz(lane >> 2);
  const uint32_t voffA = (uint32_t)(lrow * lda2) + (uint32_t)lslot * 16u;
  const uint32_t voffB = (uint32_t)(lrow * ldb2) + (uint32_t)lslot * 16u;
  auto make_srd = [](const void* base, long long bytes) {
    const unsigned long long b = (unsigned long long)base;
    return sw_i32x4{(int)(unsigned)b, (int)((unsigned)(b >> 32) & 0xffffu), (int)(unsigned)bytes, 0x00020000};
  };
  const sw_i32x4 srdA = make_srd(reinterpret_cast<const char*>(g.A) + (long long)m0 * lda2,
                                 (long long)min(g.M - m0, SW_BM) * lda2);
  const sw_i32x4 srdB = make_srd(reinterpret_cast<const char*>(g.B) + (long long)n0 * ldb2,
                                 (long long)min(g.N - n0, SW_BN) * ldb2);

  // DMA of k-step kt into stage st (all of this wave's chunks)
  auto dma_all = [&](int kt, int st) {
    const uint32_t m0st = lds0 + (uint32_t)st * SW_STAGE;
    if constexpr (ABL & 16) {
      if (wave >= 4) {
#pragma unroll
        for (int q = 0; q < 9; ++q) {
          const int c = (wave - 4) + 4 * q;
          const uint32_t m0v = m0st + (uint32_t)c * 1024u;
          if (q < 4) sw_dma(voffA, srdA, (uint32_t)(kt * 64 + 16 * c * lda2), m0v);
          else sw_dma(voffB, srdB, (uint32_t)(kt * 64 + 16 * (c - 16) * ldb2), m0v);
        }
      }
      return;
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int c = wave + NW * q;
      const uint32_t m0v = m0st + (uint32_t)c * 1024u;
      if (NW * q + NW - 1 < 16) sw_dma(voffA, srdA, (uint32_t)(kt * 64 + 16 * c * lda2), m0v);
      else if (q < nq_w) sw_dma(voffB, srdB, (uint32_t)(kt * 64 + 16 * (c - 16) * ldb2), m0v);
    }
  };

  sw_f32x4 acc[FI][SW_FJ];
#pragma unroll
  for (int i = 0; i < FI; ++i)
#pragma unroll
    for (int j = 0; j < SW_FJ; ++j) acc[i][j] = sw_f32x4{0.f, 0.f, 0.f, 0.f};
  sw_bf16x8 A[2][FI], B[SW_RB];
#pragma unroll
  for (int i = 0; i < FI; ++i) {
    A[0][i] = sw_bf16x8{};
    A[1][i] = sw_bf16x8{};
  }
#pragma unroll
  for (int j = 0; j < SW_RB; ++j) B[j] = sw_bf16x8{};

  // prologue: steps 0, 1, 2 in flight (past the last step: the last one
  // again, into a stage nothing reads), step 0 landed; step 0's gallery
  // fragments and its first D query fragments read, in the order a step
  // issues them (the gallery reads before the last D groups' query reads)
  dma_all(0, 0);
  dma_all(min(1, nk - 1), 1);
  if constexpr (ABL & 128) {
    sw_vmwait(nq_w);
  } else {
    dma_all(min(2, nk - 1), 2);
    sw_vmwait2(nq_w);
  }
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  sw_read_rb<0>(A[0][0], rdA0);
  sw_read_rb<1>(A[0][1], rdA0);
  sw_read_rb<2>(A[0][2], rdA0);
  sw_read_rb<3>(A[0][3], rdA0);
  if constexpr (FI == 8) {
    sw_read_rb<4>(A[0][4 % FI], rdA0);
    sw_read_rb<5>(A[0][5 % FI], rdA0);
    sw_read_rb<6>(A[0][6 % FI], rdA0);
    sw_read_rb<7>(A[0][7 % FI], rdA0);
  }
  sw_read_b<0>(B, rdB0);
  sw_read_b<1>(B, rdB0);
  sw_read_b<2>(B, rdB0);
  __builtin_amdgcn_sched_barrier(0);

  // step t: top = this wave's DMA of step t + 1 landed (step t + 2's in
  // flight), barrier; then the step's MFMAs with its own later query
  // fragments, step t + 1's first reads and step t + 3's DMA among them
  auto top = [&]() {
    if constexpr (!(ABL & 2)) {
      if constexpr (ABL & (1 | 128)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      else sw_vmwait(nq_w);
      asm volatile("s_barrier" ::: "memory");
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  unsigned long long clk0 = 0, rt0 = 0;
  if constexpr (ABL & 64) {
    clk0 = __builtin_amdgcn_s_memtime();
    rt0 = __builtin_amdgcn_s_memrealtime();
  }
  auto st_off = [&](int t) { return (uint32_t)((t & 3) * SW_STAGE); };
  constexpr int PD = (ABL & 128) ? 2 : 3;  // DMA prefetch distance in k-steps
  auto soff_at = [&](int t) { return (uint32_t)(min(t + PD, nk - 1) * 64); };
  auto m0_at = [&](int t) { return lds0 + (uint32_t)(((t + PD) & 3) * SW_STAGE); };
  for (int t = 0; t < nk; t += 2) {
    top();
    sw_step<NW, 0, ABL>(A, B, acc, rdA0 + st_off(t), rdB0 + st_off(t), rdA0 + st_off(t + 1), rdB0 + st_off(t + 1), voffA,
                   voffB, srdA, srdB, soff_at(t), soff_at(t), lda2, ldb2, has_last, m0_at(t), wave);
    if (t + 1 < nk) {
      top();
      sw_step<NW, 1, ABL>(A, B, acc, rdA0 + st_off(t + 1), rdB0 + st_off(t + 1), rdA0 + st_off(t + 2),
                     rdB0 + st_off(t + 2), voffA, voffB, srdA, srdB, soff_at(t + 1), soff_at(t + 1), lda2, ldb2,
                     has_last, m0_at(t + 1), wave);
    }
  }
  // the last step's reads of the (unused) next step and the trailing DMA
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (ABL & 64) {
    const unsigned long long clk1 = __builtin_amdgcn_s_memtime(), rt1 = __builtin_amdgcn_s_memrealtime();
    if (tid == 0) g.C[blockIdx.x] = (float)((double)(clk1 - clk0) / (double)(rt1 - rt0) * 100.0);
  }

  sw_filter_epilogue<FI>(g, acc, m0 + wm * WTM, n0 + wn * 160, lane);
}

// ---------------------------------------------------------------------------
// The same sweep on 128-B LDS rows (one 64-deep k-tile per row, two stages of
// 72 KB): every LDS-DMA instruction then fetches 8 whole 128-B lines instead
// of 16 half lines.  A k-tile is 20 groups (two 32-deep sub-steps of the 10
// groups above).  Two barriers per k-tile:
//   X, at its top: every wave has finished reading the other stage (k-tile
//     t - 1), so k-tile t + 1's DMA goes into it, 9 chunks per wave after
//     groups 0..8;
//   Y, after group 16's MFMAs: this wave's DMA has landed (vmcnt(0)), so the
//     reads of k-tile t + 1 start there: its gallery fragments right after Y,
//     its first D query fragments after groups 17..19.
// Reads of k-tile t's second sub-step go out during its first (gallery
// fragments after the JA groups, the query ring D groups ahead throughout).
template <int FI>
struct SwTile {
  static constexpr int NG = 2 * SW_FJ;  // groups per k-tile
  static constexpr int GY = 16;         // the group after which Y sits
  static constexpr int JA(int i) { return i * (SW_FJ - SW_D) / FI; }  // sub-step 1's gallery reads, in sub-step 0
  static constexpr int A_AFTER(int x) {
    x = ((x % NG) + NG) % NG;
    if (x == GY) return FI;  // the next k-tile's gallery fragments
    int n = 0;
    for (int i = 0; i < FI; ++i) n += JA(i) == x ? 1 : 0;
    return n;
  }
  // LDS reads issued after query fragment g and before group g's wait (every
  // group issues one query read D ahead, first, then its gallery reads)
  static constexpr int LW(int g) {
    int n = A_AFTER(g - SW_D);
    for (int x = g - SW_D + 1; x < g; ++x) n += 1 + A_AFTER(x);
    return n;
  }
  static constexpr bool ok() {
    for (int g = 0; g < NG; ++g)
      if (LW(g) > 15) return false;
    for (int i = 0; i < FI; ++i)
      if (JA(i) >= SW_FJ - SW_D) return false;
    return GY + SW_D < NG + 1 && GY <= NG - SW_D;
  }
};
static_assert(SwTile<4>::ok(), "sweep128: read schedule");

template <int N>
__device__ __forceinline__ void sw_lgkwait_n(sw_bf16x8& f) {
  if constexpr (N <= 15) asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(f) : "i"(N));
}

// fragment (row block RB) at byte base + RB * 2048 (16 rows of 128 B)
template <int RB>
__device__ __forceinline__ void sw_read128(sw_bf16x8& f, uint32_t base) {
  sw_read<RB * 2048>(f, base);
}

// (A persistent form that walked several tiles per block as one k-stream was
// built and measured: with the next tile's descriptors and the epilogue
// inside the loop it spilled 206 VGPRs and ran 5x slower; not kept.)
template <int ABL = 0, int PERS = 0>
__global__ __launch_bounds__(512, 1) void sweep128_kernel(GemmArgs g, int tiles_n, int ntiles) {
  constexpr int NW = 8, FI = 4, WTM = 64;
  using T = SwTile<FI>;
  static_assert(!PERS, "sweep128: the persistent form was retired");
  constexpr int STAGE = SW_ROWS * 128;  // 73 728 B
  // two stages, then the block's 320 query thresholds (the epilogue's)
  __shared__ __attribute__((aligned(1024))) unsigned char lds[2 * STAGE + SW_BN * 4];
  float* const tau_lds = reinterpret_cast<float*>(lds + 2 * STAGE);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave % 4, wn = wave / 4;
  const int nt = g.K >> 6;
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) unsigned char*)lds;

  // fragment reads: row r0 + (lane & 15), logical slot 4 s + (lane >> 4) at
  // physical slot (4 s + (lane >> 4)) ^ ((row >> 1) & 7) (gemm_f32.hip's
  // 128-B-row swizzle: conflict-free for this read)
  const int lr = lane & 15, lg = lane >> 4, sw = (lr >> 1) & 7;
  const uint32_t lp0 = (uint32_t)(lr * 128 + ((lg ^ sw) << 4));
  const uint32_t lp1 = (uint32_t)(lr * 128 + (((4 + lg) ^ sw) << 4));
  const uint32_t offA = (uint32_t)(wm * WTM) * 128u, offB = (uint32_t)(SW_BM + wn * 160) * 128u;

  // LDS-DMA: chunk c = wave + 8 q (q = 0..8) = stage rows 8c .. 8c + 7
  // (c < 32: gallery rows, then query rows); lane l -> row 8c + (l >> 3),
  // physical slot l & 7 = logical slot (l & 7) ^ ((row >> 1) & 7); the
  // swizzle's row bits are (c & 1) and l >> 4: fixed per wave
  const long long lda2 = g.lda * 2, ldb2 = g.ldb * 2;
  const int lrow = lane >> 3, srow = 8 * (wave & 1) + lrow;
  const int lslot = (lane & 7) ^ ((srow >> 1) & 7);
  const uint32_t voffA = (uint32_t)(lrow * lda2) + (uint32_t)lslot * 16u;
  const uint32_t voffB = (uint32_t)(lrow * ldb2) + (uint32_t)lslot * 16u;
  // a tile: its origin and the two operands' descriptors (valid rows only)
  struct Tile {
    int m0, n0;
    sw_i32x4 srdA, srdB;
  };
  auto make_srd = [](const void* base, long long bytes) {
    const unsigned long long b = (unsigned long long)base;
    return sw_i32x4{(int)(unsigned)b, (int)((unsigned)(b >> 32) & 0xffffu), (int)(unsigned)bytes, 0x00020000};
  };
  auto tile_at = [&](int v) {
    int tm, tn;
    if constexpr ((ABL & 4096) != 0) {
      // lab: one query panel per XCD (8 / tiles_n XCDs share a panel and
      // split its row blocks), so an XCD's L2 holds one 1.3 MB panel
      const int x = v & 7, w = v >> 3, per = 8 / tiles_n;
      tn = x % tiles_n;
      tm = w * per + x / tiles_n;
    } else {
      tile_coords(v, ntiles, tiles_n, tm, tn);
    }
    Tile x;
    x.m0 = tm * SW_BM;
    x.n0 = tn * SW_BN;
    x.srdA = make_srd(reinterpret_cast<const char*>(g.A) + (long long)x.m0 * lda2,
                      (long long)min(g.M - x.m0, SW_BM) * lda2);
    x.srdB = make_srd(reinterpret_cast<const char*>(g.B) + (long long)x.n0 * ldb2,
                      (long long)min(g.N - x.n0, SW_BN) * ldb2);
    return x;
  };
  auto dma_chunk = [&](int q, const Tile& x, int kt, uint32_t m0st) {
    const int c = wave + NW * q;
    const uint32_t m0v = m0st + (uint32_t)c * 1024u;
    if (q < 4) sw_dma(voffA, x.srdA, (uint32_t)(kt * 128 + 8 * c * lda2), m0v);
    else sw_dma(voffB, x.srdB, (uint32_t)(kt * 128 + 8 * (c - 32) * ldb2), m0v);
  };

  sw_f32x4 acc[FI][SW_FJ];
#pragma unroll
  for (int i = 0; i < FI; ++i)
#pragma unroll
    for (int j = 0; j < SW_FJ; ++j) acc[i][j] = sw_f32x4{0.f, 0.f, 0.f, 0.f};
  sw_bf16x8 A[2][FI], B[SW_RB];
#pragma unroll
  for (int i = 0; i < FI; ++i) {
    A[0][i] = sw_bf16x8{};
    A[1][i] = sw_bf16x8{};
  }
#pragma unroll
  for (int j = 0; j < SW_RB; ++j) B[j] = sw_bf16x8{};

  int v = blockIdx.x;  // this block's (first) tile in the grid's order
  const int vstep = PERS ? (int)gridDim.x : ntiles;
  Tile cur_t = tile_at(v);

  // prologue: the first tile's k-tile 0 landed; its first sub-step's gallery
  // fragments and first D query fragments read in the steady state's order;
  // the tile's query thresholds staged
#pragma unroll
  for (int q = 0; q < 9; ++q) dma_chunk(q, cur_t, 0, lds0);
  if (tid < SW_BN) tau_lds[tid] = cur_t.n0 + tid < g.N ? g.tau[cur_t.n0 + tid] : __builtin_inff();
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  {
    const uint32_t a0 = lds0 + offA + lp0, b0 = lds0 + offB + lp0;
    sw_read128<0>(A[0][0], a0);
    sw_read128<1>(A[0][1], a0);
    sw_read128<2>(A[0][2], a0);
    sw_read128<3>(A[0][3], a0);
    sw_read128<0>(B[0], b0);
    sw_read128<1>(B[1], b0);
    sw_read128<2>(B[2], b0);
  }
  __builtin_amdgcn_sched_barrier(0);

  unsigned long long clk0 = 0, rt0 = 0;
  if constexpr (ABL & 64) {
    clk0 = __builtin_amdgcn_s_memtime();
    rt0 = __builtin_amdgcn_s_memrealtime();
  }
  if constexpr (ABL & 1024) {
    if (wave >= 4) __builtin_amdgcn_s_setprio(1);
  }
  int kt_glob = 0;  // k-tiles done by this block (the LDS stage parity)
  for (;;) {
    const int vn = v + vstep;
    const bool more = PERS && vn < ntiles;
    const Tile nxt_t = more ? tile_at(vn) : cur_t;
    for (int t = 0; t < nt; ++t, ++kt_glob) {
      const uint32_t cur = lds0 + (uint32_t)((kt_glob & 1) * STAGE), nxt = lds0 + (uint32_t)(((kt_glob + 1) & 1) * STAGE);
      // the next k-tile: this tile's t + 1, else the next tile's first, else
      // (past the block's last) the last one again into the free stage
      const bool last = t + 1 == nt;
      const Tile& dt = (last && more) ? nxt_t : cur_t;
      const int kn = last ? (more ? 0 : nt - 1) : t + 1;
      const uint32_t aC1 = cur + offA + lp1, aN0 = nxt + offA + lp0;
      const uint32_t bC0 = cur + offB + lp0, bC1 = cur + offB + lp1, bN0 = nxt + offB + lp0;
      // X
      if constexpr (!(ABL & 2)) asm volatile("s_barrier" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int gi = 0; gi < T::NG; ++gi) {
        const int s = gi / SW_FJ, j = gi % SW_FJ;
        sw_bf16x8& bj = B[gi % SW_RB];
        if constexpr (!(ABL & 4)) {
          switch (T::LW(gi)) {
            case 0: sw_lgkwait_n<0>(bj); break;
            case 1: sw_lgkwait_n<1>(bj); break;
            case 2: sw_lgkwait_n<2>(bj); break;
            case 3: sw_lgkwait_n<3>(bj); break;
            case 4: sw_lgkwait_n<4>(bj); break;
            case 5: sw_lgkwait_n<5>(bj); break;
            case 6: sw_lgkwait_n<6>(bj); break;
            case 7: sw_lgkwait_n<7>(bj); break;
            case 8: sw_lgkwait_n<8>(bj); break;
            default: sw_lgkwait_n<9>(bj); break;
          }
        }
        if (j == 0) {
#pragma unroll
          for (int i = 0; i < FI; ++i) asm volatile("" : "+v"(A[s][i]));
        }
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (ABL & 2048) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < FI; ++i)
          if constexpr (!(ABL & 8)) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[s][i], bj, acc[i][j], 0, 0, 0);
        if constexpr (ABL & 2048) __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
        if (gi == T::GY) {
          // Y: this wave's DMA of the next k-tile landed, then every wave's
          if constexpr (!(ABL & 2)) asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
          else if constexpr (!(ABL & 1)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          __builtin_amdgcn_sched_barrier(0);
        }
        if constexpr (!(ABL & 4)) {
          // the query fragment D groups ahead
          const int gt = gi + SW_D;
          switch (gt) {
            case 3: sw_read128<3>(B[3 % SW_RB], bC0); break;
            case 4: sw_read128<4>(B[4 % SW_RB], bC0); break;
            case 5: sw_read128<5>(B[5 % SW_RB], bC0); break;
            case 6: sw_read128<6>(B[6 % SW_RB], bC0); break;
            case 7: sw_read128<7>(B[7 % SW_RB], bC0); break;
            case 8: sw_read128<8>(B[8 % SW_RB], bC0); break;
            case 9: sw_read128<9>(B[9 % SW_RB], bC0); break;
            case 10: sw_read128<0>(B[10 % SW_RB], bC1); break;
            case 11: sw_read128<1>(B[11 % SW_RB], bC1); break;
            case 12: sw_read128<2>(B[12 % SW_RB], bC1); break;
            case 13: sw_read128<3>(B[13 % SW_RB], bC1); break;
            case 14: sw_read128<4>(B[14 % SW_RB], bC1); break;
            case 15: sw_read128<5>(B[15 % SW_RB], bC1); break;
            case 16: sw_read128<6>(B[16 % SW_RB], bC1); break;
            case 17: sw_read128<7>(B[17 % SW_RB], bC1); break;
            case 18: sw_read128<8>(B[18 % SW_RB], bC1); break;
            case 19: sw_read128<9>(B[19 % SW_RB], bC1); break;
            case 20: sw_read128<0>(B[20 % SW_RB], bN0); break;
            case 21: sw_read128<1>(B[21 % SW_RB], bN0); break;
            default: sw_read128<2>(B[22 % SW_RB], bN0); break;
          }
          // gallery fragments: the second sub-step's during the first, the
          // next k-tile's first sub-step's right after Y
          if (gi == T::GY) {
            sw_read128<0>(A[0][0], aN0);
            sw_read128<1>(A[0][1], aN0);
            sw_read128<2>(A[0][2], aN0);
            sw_read128<3>(A[0][3], aN0);
          } else if (s == 0) {
#pragma unroll
            for (int i = 0; i < FI; ++i) {
              if (T::JA(i) != j) continue;
              switch (i) {
                case 0: sw_read128<0>(A[1][0], aC1); break;
                case 1: sw_read128<1>(A[1][1], aC1); break;
                case 2: sw_read128<2>(A[1][2], aC1); break;
                default: sw_read128<3>(A[1][3], aC1); break;
              }
            }
          }
        }
        // the next k-tile's DMA, chunk gi after group gi (gi < 9)
        if constexpr (!(ABL & 1)) {
          if (gi < 9) dma_chunk(gi, dt, kn, nxt);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    if (!more) break;
    // this tile's epilogue (the next tile's first fragment reads in flight:
    // their registers are not the epilogue's)
    __builtin_amdgcn_sched_barrier(0);
    sw_filter_epilogue<FI>(g, acc, cur_t.m0 + wm * WTM, cur_t.n0 + wn * 160, lane);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < FI; ++i)
#pragma unroll
      for (int j = 0; j < SW_FJ; ++j) acc[i][j] = sw_f32x4{0.f, 0.f, 0.f, 0.f};
    v = vn;
    cur_t = nxt_t;
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  if constexpr (ABL & 1024) __builtin_amdgcn_s_setprio(0);
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (ABL & 64) {
    const unsigned long long clk1 = __builtin_amdgcn_s_memtime(), rt1 = __builtin_amdgcn_s_memrealtime();
    if (tid == 0) g.C[blockIdx.x] = (float)((double)(clk1 - clk0) / (double)(rt1 - rt0) * 100.0);
  }
  sw_filter_epilogue<FI>(g, acc, cur_t.m0 + wm * WTM, cur_t.n0 + wn * 160, lane, tau_lds, wn * 160);
}

}  // namespace

bool sweep16_eligible(const GemmArgs& g) {
  return g.K > 0 && (g.K % 32) == 0 && (g.lda % 8) == 0 && (g.ldb % 8) == 0 && g.scale_a == nullptr &&
         g.scale_b == nullptr && ((uintptr_t)g.A & 15) == 0 && ((uintptr_t)g.B & 15) == 0 &&
         (long long)SW_BM * g.lda * 2 < (1LL << 31) && (long long)SW_BN * g.ldb * 2 < (1LL << 31);
}

// rows128: the 128-B-row kernel (K % 64 == 0), else the 64-B-row one
hipError_t launch_sweep16(const GemmArgs& g, hipStream_t s, int rows128) {
  const long long tiles_m = (g.M + SW_BM - 1) / SW_BM;
  const long long tiles_n = (g.N + SW_BN - 1) / SW_BN;
  const long long nblk = tiles_m * tiles_n;
  if (nblk <= 0) return hipSuccess;
  if (nblk > 0x7fffffffLL) return hipErrorInvalidValue;
  if (rows128 && (g.K % 64) == 0)
    hipLaunchKernelGGL(sweep128_kernel<0>, dim3((unsigned)nblk), dim3(512), 0, s, g, (int)tiles_n, (int)nblk);
  else
    hipLaunchKernelGGL(sweep16_kernel<8>, dim3((unsigned)nblk), dim3(512), 0, s, g, (int)tiles_n);
  return hipGetLastError();
}

}  // namespace rr
