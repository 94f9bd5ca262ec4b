// sweep_v.hip — the bf16 filter sweep of the exact prefilter ranker (pass 2
// of rr_cosine_topk_prefilter: the 1.6 M-row gallery x every query, keeping
// the scores above each query's threshold; iris_evaluate.py:383's torch.mm)
// with the gallery operand loaded straight from global memory into VGPRs.
//
// Why: the LDS-DMA tiles of gemm_f32.hip stage BOTH operands through LDS.  The
// 256x320 sweep tile (8 waves of 64x160 on 32x32x16) fills 28.8 B/clk/CU and
// reads 2 + 5 fragments per 10 MFMAs, ~90 B/clk/CU at the bf16 MFMA rate:
// ~118 of the LDS's 128 B/clk, which is where it stops (0.47-0.50 of peak,
// DESIGN.md).  The first gallery-in-VGPR form (round 3: 8 waves of 32 gallery
// rows x 256 queries) fixed the fill but read 16 query fragments per 32 MFMAs:
// 128 B/clk of fragment reads, slower still.
//
// Here: block = 256 gallery rows x 256 queries, 8 waves as 4 (gallery) x 2
// (queries); wave tile 64 rows x 128 queries = 4 x 8 v_mfma_f32_16x16x32_bf16
// tiles (128 accumulator VGPRs).  Per 32-deep k-step a wave reads 8 query
// fragments (8 KB) from LDS for 32 MFMAs: 64 B/clk/CU of reads + 16 B/clk/CU
// of query-panel fill at the MFMA rate (80 of 128).  The gallery fragments
// (lane l: row l % 16 of a 16-row tile, k-chunk 8 (l / 16)) are one 16-B
// global load per lane and row tile — one wave instruction = 16 rows x 64
// contiguous bytes — issued three stages ahead into registers the MFMAs read
// directly.  The two waves of a gallery slice load the same rows (the second
// read hits L1).
//
// Stage = one 32-deep k-step: 4 gallery loads per lane + 2 LDS-DMA
// instructions per wave (the 16 KB query slice, 256 rows x 64 B, 16-B slots
// XOR-swizzled on the DMA source as gemm_s3.hip's f16x2 BK = 32 rows:
// conflict-free 16x16x32 fragment reads).  Four stages (64 KB LDS, 64
// gallery VGPRs).  Iteration s: wait for stage s (the loads of s + 1, s + 2
// stay in flight: a counted vmcnt), one barrier (stage s visible to every
// wave; everyone done with stage s - 1, whose LDS and registers s + 3 now
// reuses), issue stage s + 3, then 32 MFMAs on stage s.  The gallery loads
// are inline asm so hipcc keeps no scoreboard entry for them (with LDS-DMA in
// flight it would otherwise wait vmcnt(0) at their first use, gemm_s3.hip);
// the registers are laundered after the counted wait.
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

constexpr int SV_QP = 256;    // queries per block (2 wave columns x 128)
constexpr int SV_ROWS = 256;  // gallery rows per block (4 wave rows x 64)
constexpr int SV_RT = 4;      // 16-row gallery tiles per wave
constexpr int SV_CT = 8;      // 16-query tiles per wave

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Per dtype: KS = k per MFMA step (= per stage), RB = bytes of one operand row
// per stage, LPT = 16-B loads per lane and 16-row tile, NST = stages.
//   bf16: v_mfma_f32_16x16x32_bf16, lane l: row l % 16, k 8 (l / 16) .. +7
//         (one 16-B slot of a 64-B row); 4 stages.
//   fp8:  v_mfma_scale_f32_16x16x128_f8f6f4 (e4m3, unit E8M0 block scales,
//         2x the bf16 k per clock; the rows' fp32 scales in the epilogue),
//         lane l: row l % 16, the 32 bytes of 16-B slots l / 16 and l / 16 + 4
//         of a 128-B row (A and B read by the same lane -> k map, so each dot
//         product covers every k once; one wave load instruction is still 16
//         rows x 64 contiguous bytes); 2 stages (32 gallery VGPRs per stage).
//         The fp8 gallery loads are plain loads into the 8-register MFMA
//         operand: two inline-asm halves needed copies that spilled the
//         kernel (87 VGPRs at 3 stages).  With two stages the k-loop waits
//         vmcnt(0) anyway, so the waits hipcc inserts for plain loads cost
//         nothing, as long as the next stage's loads are issued after the
//         stage's first use of its fragments (a sched_barrier keeps them there).
template <int DT>
struct SvT;
template <>
struct SvT<DT_BF16> {
  static constexpr int KS = 32, RB = 64, LPT = 1, NST = 4;
  typedef bf16x8 frag;
  // 64-B rows, 4 slots: conflict-free 16x16x32 reads (gemm_s3.hip pswz<32, 2>)
  static __device__ __forceinline__ int swz(int row, int slot) {
    return slot ^ ((((row >> 3) & 1) << 1) | ((row >> 4) & 1));
  }
};
template <>
struct SvT<DT_FP8> {
  static constexpr int KS = 128, RB = 128, LPT = 2, NST = 2;
  typedef i32x8 frag;
  // 128-B rows, 8 slots (gemm_f32.hip's swizzle): the reads of slots g and
  // g + 4 (g = lane / 16) by rows l % 16 hit 16 distinct bank quads per group
  static __device__ __forceinline__ int swz(int row, int slot) { return slot ^ ((row >> 1) & 7); }
};

template <int DT>
__global__ __launch_bounds__(512, 1) void sweep_v_kernel(GemmArgs g, int tiles_n) {
  typedef SvT<DT> T;
  typedef typename T::frag frag_t;
  constexpr int KS = T::KS, RB = T::RB, LPT = T::LPT, NST = T::NST;
  constexpr int STAGE = SV_QP * RB;             // LDS bytes per stage
  constexpr int Q_DMA = STAGE / 1024 / 8;       // LDS-DMA instructions per wave per stage
  constexpr int RPI = 1024 / RB;                // query rows per DMA instruction
  constexpr int SPR = RB / 16;                  // 16-B slots per row
  __shared__ __attribute__((aligned(16))) unsigned char lds[NST * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l16 = lane & 15, lg = lane >> 4;
  const int wg = wave & 3, wq = wave >> 2;

  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int tn = wgid % tiles_n, tm = wgid / tiles_n;
  const int m0 = tm * SV_ROWS, n0 = tn * SV_QP;
  const int nk = g.K / KS;  // K counted in elements (bf16) or bytes (fp8)

  // gallery A fragments: rows m0 + 64 wg + 16 i + l16 (clamped: rows past M
  // are never kept), byte 16 lg (+ 64: fp8's second slot) of the stage
  const unsigned char* A = reinterpret_cast<const unsigned char*>(g.A);
  const int esz = DT == DT_BF16 ? 2 : 1;
  const unsigned char* ga[SV_RT];
#pragma unroll
  for (int i = 0; i < SV_RT; ++i)
    ga[i] = A + ((long long)min(m0 + 64 * wg + 16 * i + l16, g.M - 1) * g.lda) * esz + 16 * lg;
  // query slice DMA: instruction j of wave w fills panel rows (8 j + w) RPI ..
  // + RPI - 1, lane l -> row + l / SPR, physical slot l % SPR (logical slot
  // swz of it)
  const unsigned char* B = reinterpret_cast<const unsigned char*>(g.B);
  const unsigned char* qs[Q_DMA];
#pragma unroll
  for (int j = 0; j < Q_DMA; ++j) {
    const int r = (j * 8 + wave) * RPI + lane / SPR;
    qs[j] = B + ((long long)min(n0 + r, g.N - 1) * g.ldb) * esz + T::swz(r, lane % SPR) * 16;
  }

  frag_t gb[NST][SV_RT];  // [stage][row tile]: the MFMA A operands
  constexpr int PER = SV_RT * LPT + Q_DMA;  // vmcnt entries per stage: gallery loads + DMA
  constexpr int AHEAD = NST - 1;            // stages in flight beyond the one computed
  auto issue = [&](int kt, int st) {
    const long long t = (long long)min(kt, nk - 1) * RB;
#pragma unroll
    for (int i = 0; i < SV_RT; ++i) {
      if constexpr (LPT == 1) {
        asm volatile("global_load_dwordx4 %0, %1, off" : "=&v"(gb[st][i]) : "v"(ga[i] + t) : "memory");
      } else {
        const u32x4 lo = *reinterpret_cast<const u32x4*>(ga[i] + t);
        const u32x4 hi = *reinterpret_cast<const u32x4*>(ga[i] + t + 64);
        gb[st][i] = __builtin_bit_cast(frag_t, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
    }
#pragma unroll
    for (int j = 0; j < Q_DMA; ++j)
      __builtin_amdgcn_global_load_lds((const void*)(qs[j] + t),
                                       (__attribute__((address_space(3))) void*)(lds + st * STAGE +
                                                                                  (j * 8 + wave) * 1024),
                                       16, 0, 0);
  };
  auto launder = [&](int st) {
    if constexpr (LPT == 1) {
#pragma unroll
      for (int i = 0; i < SV_RT; ++i) asm volatile("" : "+v"(gb[st][i]));
    }
  };

  f32x4 acc[SV_RT][SV_CT];
#pragma unroll
  for (int i = 0; i < SV_RT; ++i)
#pragma unroll
    for (int c = 0; c < SV_CT; ++c) acc[i][c] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto mfma = [&](const frag_t& a, const frag_t& b, f32x4 c) {
    if constexpr (DT == DT_BF16) return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
    else return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, 127, 0, 127);
  };
  // 8 query fragments per stage in 4 groups of 2: the reads of group q + 1
  // are issued before the 8 MFMAs of group q, so the LDS latency hides under
  // them; after group 0 (the stage's first use of every gallery fragment) the
  // loads of stage `next` are issued into the buffers freed at the barrier
  auto compute = [&](int st, int next) {
    const unsigned char* lq = lds + st * STAGE;
    const frag_t(&a)[SV_RT] = gb[st];
    frag_t bq[2][2];
    auto rd = [&](int q) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int r = 128 * wq + 16 * (2 * q + u) + l16;
        const unsigned char* row = lq + r * RB;
        if constexpr (LPT == 1) {
          bq[q & 1][u] = *reinterpret_cast<const frag_t*>(row + T::swz(r, lg) * 16);
        } else {
          const u32x4 lo = *reinterpret_cast<const u32x4*>(row + T::swz(r, lg) * 16);
          const u32x4 hi = *reinterpret_cast<const u32x4*>(row + T::swz(r, lg + 4) * 16);
          bq[q & 1][u] = __builtin_bit_cast(frag_t, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
        }
      }
    };
    rd(0);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (q + 1 < 4) rd(q + 1);
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int c = 2 * q + u;
#pragma unroll
        for (int i = 0; i < SV_RT; ++i) acc[i][c] = mfma(a[i], bq[q & 1][u], acc[i][c]);
      }
      if (q + 1 < 4) {
        __builtin_amdgcn_sched_group_barrier(0x100, 2 * LPT, 0);  // the next group's LDS reads
        __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);        // this group's 8 MFMAs
      }
      if (q == 0) {
        __builtin_amdgcn_sched_barrier(0);
        issue(next, (st + AHEAD) % NST);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };

#pragma unroll
  for (int s = 0; s < AHEAD; ++s) issue(s, s);
  auto iter = [&](int s, int st) __attribute__((always_inline)) {
    // stage s landed; the AHEAD - 1 stages after it stay in flight
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"((AHEAD - 1) * PER) : "memory");
    launder(st);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    compute(st, s + AHEAD);
  };
  for (int s = 0; s < nk; s += NST) {
    iter(s, 0);
#pragma unroll
    for (int u = 1; u < NST; ++u)
      if (s + u < nk) iter(s + u, u);
  }
  // the clamped tail loads are still in flight: keep their registers live
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int st = 0; st < NST; ++st) launder(st);

  // filter epilogue: acc[i][c][e] = score of gallery row m0 + 64 wg + 16 i +
  // 4 lg + e and query n0 + 128 wq + 16 c + l16 (fp8: times the two rows'
  // scales, as gemm_f32.hip's dequantisation: (acc * sa) * sb)
#pragma unroll
  for (int c = 0; c < SV_CT; ++c) {
    const int n = n0 + 128 * wq + 16 * c + l16;
    const bool nok = n < g.N;
    const float t = nok ? g.tau[n] : __builtin_inff();
    float sb = 1.f;
    if constexpr (DT == DT_FP8) sb = (g.scale_b != nullptr && nok) ? g.scale_b[n] : 1.f;
#pragma unroll
    for (int i = 0; i < SV_RT; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + 64 * wg + 16 * i + 4 * lg + e;
        float v = acc[i][c][e];
        if constexpr (DT == DT_FP8) {
          const float sa = (g.scale_a != nullptr && m < g.M) ? g.scale_a[m] : 1.f;
          v = v * sa * sb;
        }
        if (nok && m < g.M && !(v <= t)) {
          const int pos = atomicAdd(g.cnt + n, 1);
          if (pos < g.cap) g.cand[(long long)n * g.cap + pos] = make_key(v, (uint32_t)(g.row_offset + m));
        }
      }
  }
}

}  // namespace

bool sweep_v_eligible(const GemmArgs& g, int dt) {
  const int ks = dt == DT_FP8 ? 128 : 32, vec = dt == DT_FP8 ? 16 : 8;
  if (dt != DT_BF16 && dt != DT_FP8) return false;
  if (dt == DT_BF16 && (g.scale_a != nullptr || g.scale_b != nullptr)) return false;  // bf16 rows are unscaled
  return g.K > 0 && (g.K % ks) == 0 && (g.lda % vec) == 0 && (g.ldb % vec) == 0 && ((uintptr_t)g.A & 15) == 0 &&
         ((uintptr_t)g.B & 15) == 0;
}

hipError_t launch_sweep_v(const GemmArgs& g, hipStream_t s, int dt) {
  const long long tiles_m = (g.M + SV_ROWS - 1) / SV_ROWS, tiles_n = (g.N + SV_QP - 1) / SV_QP;
  const long long nblk = tiles_m * tiles_n;
  if (nblk <= 0) return hipSuccess;
  if (nblk > 0x7fffffffLL) return hipErrorInvalidValue;
  if (dt == DT_FP8) hipLaunchKernelGGL(sweep_v_kernel<DT_FP8>, dim3((unsigned)nblk), dim3(512), 0, s, g, (int)tiles_n);
  else hipLaunchKernelGGL(sweep_v_kernel<DT_BF16>, dim3((unsigned)nblk), dim3(512), 0, s, g, (int)tiles_n);
  return hipGetLastError();
}

}  // namespace rr
