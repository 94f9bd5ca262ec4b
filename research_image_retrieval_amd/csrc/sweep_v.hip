// sweep_v.hip — the bf16 filter sweep of the exact prefilter ranker (pass 2
// of rr_cosine_topk_prefilter: the 1.6 M-row gallery x every query, keeping
// the scores above each query's threshold; iris_evaluate.py:383's torch.mm)
// with the gallery operand loaded straight from global memory into VGPRs.
//
// The LDS-DMA tiles of gemm_f32.hip stage BOTH operands through LDS; the
// 256x320 sweep tile moves 142 FLOP per filled byte and tops out near half of
// the bf16 peak on the fill.  Here only the query panel, which
// every wave of the block reuses, goes through LDS (LDS-DMA, three stages);
// each wave owns 32 gallery rows and loads its 16x16x32 A fragments as one
// 16-B global load per lane (lane l: row l % 16 of a 16-row tile, k-chunk
// 8 (l / 16)), three stages ahead, into registers the MFMAs read directly.
// That is 256 FLOP per LDS-filled byte and no LDS traffic for the gallery.
//
// Block: 8 waves x 32 gallery rows = 256 rows, one 256-query panel; wave tile
// 32 x 256 = 2 x 16 MFMA tiles (128 accumulator VGPRs).  Stage = 64 k (two
// 32-deep k-steps): the query panel slice is 256 rows x 128 B = 32 KB, 16-B
// slots XOR-swizzled by (row >> 1) & 7 on the DMA source (conflict-free
// fragment reads, as gemm_8p.hip).  Iteration s: wait for stage s (the
// loads of s + 1 stay in flight: a counted vmcnt), one barrier (stage s
// visible to every wave; everyone done with stage s - 1, whose LDS and
// registers s + 2 now reuses), issue stage s + 2 (4 gallery loads by inline
// asm, 4 LDS-DMA instructions per wave), then 64 MFMAs on stage s.  The
// gallery loads are inline asm so hipcc keeps no scoreboard entry for them
// (with LDS-DMA in flight it would otherwise wait vmcnt(0) at their first use,
// gemm_s3.hip); the registers are laundered after the counted wait.
//
// XCD-aware bijective block remap with the query panel fastest: the panels of
// one gallery tile run together on one XCD, which fetches the tile from HBM
// once into its L2.  Filter epilogue identical to gemm_f32.hip's E_FILTER:
// keep !(s <= tau[q]) (NaN kept), one atomic slot per survivor, 64-bit keys.
// bf16 x bf16 products are exact and the accumulation is fp32 in another k
// order than gemm_f32.hip's tiles: the prefilter's bound covers any order
// (prefilter.hip), so the ranker's result is unchanged, bit for bit.
#include "gemm_epilogue.hpp"
#include "rr_internal.hpp"

namespace rr {

namespace {

constexpr int SV_BK = 64;                      // k per stage
constexpr int SV_QP = 256;                     // queries per block
constexpr int SV_ROWS = 256;                   // gallery rows per block (8 waves x 32)
constexpr int SV_STAGES = 3;
constexpr int SV_STAGE = SV_QP * SV_BK * 2;    // bytes per LDS stage (32 KB)
constexpr int SV_G_LD = 4;                     // gallery loads per lane per stage
constexpr int SV_Q_DMA = SV_STAGE / 1024 / 8;  // LDS-DMA instructions per wave per stage (4)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int sv_swz(int row, int slot) { return slot ^ ((row >> 1) & 7); }

__global__ __launch_bounds__(512, 1) void sweep_v_kernel(GemmArgs g, int tiles_n) {
  __shared__ __attribute__((aligned(16))) unsigned char lds[SV_STAGES * SV_STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l16 = lane & 15, lg = lane >> 4;

  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int tn = wgid % tiles_n, tm = wgid / tiles_n;
  const int m0 = tm * SV_ROWS, n0 = tn * SV_QP;
  const int nk = g.K / SV_BK;

  // gallery A fragments: rows m0 + 32 wave + 16 i + l16 (clamped: rows past M
  // are never kept), k-chunk 8 lg (+ 32 for the second k-step)
  const uint16_t* A = reinterpret_cast<const uint16_t*>(g.A);
  const uint16_t* ga[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) ga[i] = A + (long long)min(m0 + 32 * wave + 16 * i + l16, g.M - 1) * g.lda + 8 * lg;
  // query panel DMA: instruction j of wave w fills panel rows (8 j + w) 8 .. +7,
  // lane l -> row + l / 8, physical slot l % 8 (logical slot sv_swz of it)
  const uint16_t* B = reinterpret_cast<const uint16_t*>(g.B);
  const uint16_t* qs[SV_Q_DMA];
#pragma unroll
  for (int j = 0; j < SV_Q_DMA; ++j) {
    const int r = (j * 8 + wave) * 8 + (lane >> 3);
    qs[j] = B + (long long)min(n0 + r, g.N - 1) * g.ldb + sv_swz(r, lane & 7) * 8;
  }

  u32x4 gb[SV_STAGES][2][2];  // [stage][row tile][k-step]
  auto issue = [&](int kt, int st) {
    const long long t = (long long)min(kt, nk - 1) * SV_BK;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      asm volatile("global_load_dwordx4 %0, %2, off\n\tglobal_load_dwordx4 %1, %2, off offset:64"
                   : "=&v"(gb[st][i][0]), "=&v"(gb[st][i][1])
                   : "v"(ga[i] + t)
                   : "memory");
#pragma unroll
    for (int j = 0; j < SV_Q_DMA; ++j)
      __builtin_amdgcn_global_load_lds((const void*)(qs[j] + t),
                                       (__attribute__((address_space(3))) void*)(lds + st * SV_STAGE +
                                                                                  (j * 8 + wave) * 8 * 128),
                                       16, 0, 0);
  };
  auto launder = [&](int st) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) asm volatile("" : "+v"(gb[st][i][ks]));
  };

  f32x4 acc[2][16];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int c = 0; c < 16; ++c) acc[i][c] = f32x4{0.f, 0.f, 0.f, 0.f};

  // 32 (k-step, column tile) pairs per stage in 8 groups of 4 B fragments:
  // the reads of group q + 1 are issued before the 8 MFMAs of group q, so the
  // LDS latency hides under them (hipcc otherwise waited for each pair of
  // reads right before its MFMAs)
  auto compute = [&](int st) {
    const unsigned char* lq = lds + st * SV_STAGE;
    bf16x8 bq[2][4];
    auto rd = [&](int q) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int p = 4 * q + u, ks = p >> 4, c = p & 15;
        const int r = c * 16 + l16;
        bq[q & 1][u] = *reinterpret_cast<const bf16x8*>(lq + r * 128 + sv_swz(r, 4 * ks + lg) * 16);
      }
    };
    rd(0);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      if (q + 1 < 8) rd(q + 1);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int p = 4 * q + u, ks = p >> 4, c = p & 15;
        const bf16x8 a0 = __builtin_bit_cast(bf16x8, gb[st][0][ks]);
        const bf16x8 a1 = __builtin_bit_cast(bf16x8, gb[st][1][ks]);
        acc[0][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bq[q & 1][u], acc[0][c], 0, 0, 0);
        acc[1][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, bq[q & 1][u], acc[1][c], 0, 0, 0);
      }
      if (q + 1 < 8) {
        __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);  // the next group's 4 LDS reads
        __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);  // this group's 8 MFMAs
      }
    }
  };

  constexpr int PER = SV_G_LD + SV_Q_DMA;  // vmcnt entries per stage: 4 gallery loads + 4 DMA
  issue(0, 0);
  issue(1, 1);
  auto iter = [&](int s, int st) __attribute__((always_inline)) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER) : "memory");  // stage s landed (s + 1 in flight)
    launder(st);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    issue(s + 2, (st + 2) % SV_STAGES);
    compute(st);
  };
  for (int s = 0; s < nk; s += 3) {
    iter(s, 0);
    if (s + 1 < nk) iter(s + 1, 1);
    if (s + 2 < nk) iter(s + 2, 2);
  }
  // the clamped tail loads are still in flight: keep their registers live
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int st = 0; st < SV_STAGES; ++st) launder(st);

  // filter epilogue: acc[i][c][e] = score of gallery row m0 + 32 wave + 16 i +
  // 4 lg + e and query n0 + 16 c + l16
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    const int n = n0 + 16 * c + l16;
    const bool nok = n < g.N;
    const float t = nok ? g.tau[n] : __builtin_inff();
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + 32 * wave + 16 * i + 4 * lg + e;
        const float v = acc[i][c][e];
        if (nok && m < g.M && !(v <= t)) {
          const int pos = atomicAdd(g.cnt + n, 1);
          if (pos < g.cap) g.cand[(long long)n * g.cap + pos] = make_key(v, (uint32_t)(g.row_offset + m));
        }
      }
  }
}

}  // namespace

bool sweep_v_eligible(const GemmArgs& g) {
  return g.K > 0 && (g.K % SV_BK) == 0 && (g.lda % 8) == 0 && (g.ldb % 8) == 0 && g.scale_a == nullptr &&
         g.scale_b == nullptr && ((uintptr_t)g.A & 15) == 0 && ((uintptr_t)g.B & 15) == 0;
}

hipError_t launch_sweep_v(const GemmArgs& g, hipStream_t s) {
  const long long tiles_m = (g.M + SV_ROWS - 1) / SV_ROWS, tiles_n = (g.N + SV_QP - 1) / SV_QP;
  const long long nblk = tiles_m * tiles_n;
  if (nblk <= 0) return hipSuccess;
  if (nblk > 0x7fffffffLL) return hipErrorInvalidValue;
  hipLaunchKernelGGL(sweep_v_kernel, dim3((unsigned)nblk), dim3(512), 0, s, g, (int)tiles_n);
  return hipGetLastError();
}

}  // namespace rr
