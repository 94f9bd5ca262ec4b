// gemm_lpp.hip — the bf16 stored-C GEMM (the ViT-B/16 linears,
// networks/model.py:171-192: in-proj / out-proj / c_fc / c_proj) as a
// persistent 256x256 k-stream.
//
// The one-tile-per-block 256x256 bf16 tile (gemm_f32.hip, lp config 3) runs
// every tile as prologue (first k-tile's DMA round trip) -> 12 k-tiles at K =
// 768 -> epilogue (bias, GELU / residual, the LayerNorm partials and bf16
// copy, the fold's per-row correction; up to 640 KB of HBM traffic per tile)
// with the matrix cores idle outside the k-loop.  Here one block per CU walks
// its tiles as ONE k-stream: the LDS-DMA of both operands runs one 64-deep
// k-tile ahead across tile boundaries, so a tile's epilogue runs with the next
// tile's first k-tile already in LDS, and a tile never pays a cold prologue.
// The epilogue goes in four 64-row slabs (slab s = MFMA row tile s of every
// wave, all eight waves staging each) through the stage its last k-tile
// released; with a residual, each 32-row band's residual rows are loaded two
// bands ahead (as config 15 of gemm_s3.hip).  Same fragments, k-step order
// and per-accumulator MFMA sequence (v_mfma_f32_16x16x32_bf16, one per
// sub-tile per 32-deep k-step, k-steps in order) and the same epilogue
// arithmetic (store_slab) as the one-tile kernel: bit-identical results.
// Measured against the one-tile kernel (tools/vit_lin_ab.py, 1280 images,
// profiles/r05s_vitlin.txt): in-proj 1.101 -> 1.039 ms, out-proj 0.602 ->
// 0.577, c_fc 1.570 -> 1.509 (step 1's fragments read among step 0's MFMAs;
// without that, 1.072 / 0.589 / 1.570).  c_proj (K = 3072) ran 1.291 -> 1.343
// (r05t_vitlin_k4096.txt), so the kernel serves K <= 1024.  A ring of four
// 32-deep stages with the DMA three k-tiles ahead was slower on all four
// (c_fc 1.744, c_proj 1.498 ms, r05p_vitlin.txt): twice the barriers.
//
// Operands: A [M][K] bf16 (lda), B [N][K] bf16 (ldb), K % 64 == 0, K <= 1024,
// N % 256 == 0 (lpp_eligible).  Rows past M read row M - 1 (never stored).

#include <algorithm>

#include "gemm_epilogue.hpp"
#include "rr_internal.hpp"

namespace rr {

namespace {

// the 16-B slot swizzle of a 128-B LDS row (as gemm_f32.hip swz<32>)
__device__ __forceinline__ int lswz(int row, int slot) { return slot ^ ((row >> 1) & 7); }

__device__ __forceinline__ int lpp_opaque(int v) {
  asm volatile("" : "+v"(v));
  return v;
}

template <int EPI>
__global__ __launch_bounds__(512, 1) void gemm_lpp_kernel(GemmArgs g, int tiles_n, int ntiles) {
  constexpr int NT = 512, WM = 2, FM = 4, FN = 2, WTM = 128, WTN = 64, BM = 256, BN = 256;
  constexpr int BK = 32;                 // floats per 128-B LDS row (64 bf16 = one k-tile)
  constexpr int SLOTS = 8, RPP = NT / SLOTS;  // 16-B slots per row, rows per DMA pass (64)
  constexpr int A_CH = BM / RPP, B_CH = BN / RPP;  // DMA instructions per wave and k-tile (4 + 4)
  constexpr int EPR = 64;                // bf16 per k-tile row
  constexpr int CS = BN + 4;             // C staging row stride (floats; the 16x16 map's writes spread over banks)
  constexpr int BUF = (BM + BN) * BK;    // floats per k-tile stage
  constexpr int STG = BUF > 64 * CS ? BUF : 64 * CS;
  constexpr bool LNF = (EPI & EP_LNFOLD) != 0;
  constexpr bool RES = (EPI & EP_RES) != 0;
  __shared__ __attribute__((aligned(16))) float lds[2 * STG + (LNF ? LN_ROW * BM + LN_TMAX * BN : 0)];
  float* const lnf = lds + 2 * STG;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const int l16 = lane & 15, lg = lane >> 4;
  const int G = gridDim.x, bid = blockIdx.x;
  const int nk = g.K / EPR;
  const int my_tiles = (ntiles - bid + G - 1) / G;
  const int J = my_tiles * nk;
  // local tile tl -> origin (as gemm_s3.hip config 8 / 15: virtual block
  // bid + tl G keeps the block's XCD, then the bijective XCD remap)
  auto tile_origin = [&](int tl, int& m0, int& n0) __attribute__((always_inline)) {
    const int v = bid + tl * G;
    const int xcd = v & 7, q8 = ntiles >> 3, r8 = ntiles & 7;
    const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (v >> 3);
    const int tn = wgid % tiles_n, tm = wgid / tiles_n;
    m0 = tm * BM;
    n0 = tn * BN;
  };

  // ---- LDS-DMA of k-tile (tile tl, k-tile kt) into stage buf: lane-linear
  // destinations (8 whole 128-B rows per wave instruction), swizzle on the
  // source slot ----
  const uint16_t* const Ab = reinterpret_cast<const uint16_t*>(g.A);
  const uint16_t* const Bb = reinterpret_cast<const uint16_t*>(g.B);
  auto glds = [&](int tl, int kt, int buf) __attribute__((always_inline)) {
    int m0, n0;
    tile_origin(tl, m0, n0);
    float* la = lds + buf * STG;
    float* lb = la + BM * BK;
    const int t = lpp_opaque(tid);
    const int sl = t % SLOTS, cr = t / SLOTS;
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const int row = cr + i * RPP;
      const int m = min(m0 + row, g.M - 1);
      __builtin_amdgcn_global_load_lds(
          (const void*)(Ab + (long long)m * g.lda + kt * EPR + lswz(row, sl) * 8),
          (__attribute__((address_space(3))) void*)(la + (i * RPP + wave * (64 / SLOTS)) * BK), 16, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      const int row = cr + i * RPP;
      __builtin_amdgcn_global_load_lds(
          (const void*)(Bb + (long long)(n0 + row) * g.ldb + kt * EPR + lswz(row, sl) * 8),
          (__attribute__((address_space(3))) void*)(lb + (i * RPP + wave * (64 / SLOTS)) * BK), 16, 0, 0);
    }
  };

  // ---- MFMAs: sub-tile t = 2a + b (row half a, column half b) of each 32x32 tile ----
  f32x4 acc4[FM][FN][4];
  auto zero_acc = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int t = 0; t < 4; ++t) acc4[i][j][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  };
  zero_acc();
  // the k-tile's two 32-deep k-steps (lane group lg: k 8 lg .. +7 of slot
  // 4 st + lg); step 1's fragments are read among step 0's MFMAs (the
  // one-tile kernel's order), step 0's before them (the SIMD's other wave
  // covers that latency)
  auto compute = [&](int cur) __attribute__((always_inline)) {
    const float* la = lds + cur * STG;
    const float* lb = la + BM * BK;
    bf16x8 af[2][FM][2], bf[2][FN][2];
    auto rd = [&](int st) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int row = wm * WTM + i * 32 + h * 16 + l16;
          af[st][i][h] = *reinterpret_cast<const bf16x8*>(la + row * BK + lswz(row, 4 * st + lg) * 4);
        }
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int row = wn * WTN + j * 32 + h * 16 + l16;
          bf[st][j][h] = *reinterpret_cast<const bf16x8*>(lb + row * BK + lswz(row, 4 * st + lg) * 4);
        }
    };
    rd(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int st = 0; st < BK / 16; ++st) {
      if (st + 1 < BK / 16) rd(st + 1);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int t = 0; t < 4; ++t)
            acc4[i][j][t] =
                __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[st][i][t >> 1], bf[st][j][t & 1], acc4[i][j][t], 0, 0, 0);
      if (st + 1 < BK / 16) {
        // MFMA, read, MFMA, read, ... then the remaining MFMAs
#pragma unroll
        for (int x = 0; x < 2 * (FM + FN); ++x) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 4 * FM * FN - 2 * (FM + FN), 0);
      }
    }
    __builtin_amdgcn_s_setprio(0);
  };

  // ---- epilogue of local tile tl through stage `buf` (free) ----
  // Eight 32-row bands, band b = rows 128 (b & 1) + 32 (b >> 1) + [0, 32);
  // bands 2s, 2s + 1 form slab s (MFMA row tile s of every wave), staged together.
  constexpr int C4 = BN / 4, HITERS = 32 * C4 / NT;  // 4 row chunks per thread and band
  constexpr int NB = 2 * FM, RD = 2;                   // bands; residual look-ahead (bands)
  float am = 0.f;
  auto epilogue = [&](int tl, int buf) __attribute__((always_inline)) {
    int m0, n0;
    tile_origin(tl, m0, n0);
    const int te = lpp_opaque(tid);
    const int c40 = te % C4;
    if constexpr (LNF) {
      // the tile's rows' rstd / tile-mean offsets and its column sums per k
      // tile (as the one-tile kernel's prologue; published by stage(0)'s barrier)
      if (te < BM) {
        const f32x4 r = m0 + te < g.M ? ln_row_stats(g.stats_in, m0 + te, g.stats_k, g.ln_eps) : f32x4{0.f, 0.f, 0.f, 0.f};
        *reinterpret_cast<f32x4*>(lnf + LN_ROW * te) = r;
      }
      const int T = (g.stats_k + 255) >> 8;
      for (int i = te; i < LN_TMAX * BN / 4; i += NT) {
        const int t = i / (BN / 4), c = (i - t * (BN / 4)) * 4;
        const f32x4 v = (t < T && n0 + c < g.N) ? *reinterpret_cast<const f32x4*>(g.colsum + (long long)t * g.N + n0 + c)
                                                : f32x4{0.f, 0.f, 0.f, 0.f};
        *reinterpret_cast<f32x4*>(lnf + LN_ROW * BM + t * BN + c) = v;
      }
    }
    f32x4 bias_v[1] = {f32x4{0.f, 0.f, 0.f, 0.f}}, sc_v[1] = {f32x4{1.f, 1.f, 1.f, 1.f}};
    f32x4 res[RD + 1][HITERS];
    auto band_row0 = [&](int bb) { return (bb & 1) * 128 + (bb >> 1) * 32; };
    auto load_band = [&](int bb) __attribute__((always_inline)) {
      if constexpr (RES) {
        const int tq = lpp_opaque(tid);
        const int cq = tq % C4, rq = tq / C4;
#pragma unroll
        for (int it = 0; it < HITERS; ++it) {
          const int m = min(m0 + band_row0(bb) + rq + it * (NT / C4), g.M - 1);
          const float* p = g.residual + (long long)m * g.ldc + n0 + cq * 4;
          asm volatile("global_load_dwordx4 %0, %1, off" : "=&v"(res[bb % (RD + 1)][it]) : "v"(p) : "memory");
        }
      }
    };
    float* ct = lds + buf * STG;  // [2 bands x 32 rows][CS]
    const int le = te & 63, we = te >> 6;
    auto stage = [&](int sl) __attribute__((always_inline)) {
      float* cw = ct + ((we % WM) * 32) * CS + (we / WM) * WTN;
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int r = 4 * t + e;
            cw[acc_row<true>(0, r, le) * CS + acc_col<true>(j, r, le)] = acc4[sl][j][t][e];
          }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    };
    // the bias first, by inline asm (a plain load's use would make hipcc wait
    // vmcnt(0), the residual look-ahead included): older than every band
    if ((EPI & EP_BIAS) && g.bias != nullptr)
      asm volatile("global_load_dwordx4 %0, %1, off" : "=&v"(bias_v[0]) : "v"(g.bias + n0 + c40 * 4) : "memory");
    load_band(0);
    load_band(1);
#pragma unroll
    for (int bb = 0; bb < NB; ++bb) {
      if ((bb & 1) == 0) stage(bb >> 1);
      if (bb + RD < NB) load_band(bb + RD);
      if constexpr (RES) {
        // band bb's wait counts only the loads issued after it (loads return
        // in order among themselves; nothing is assumed about the stores)
        const int ahead = (NB - 1 - bb < RD ? NB - 1 - bb : RD);
        switch (HITERS * ahead) {
          case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
          case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
          default: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
        }
#pragma unroll
        for (int it = 0; it < HITERS; ++it) asm volatile("" : "+v"(res[bb % (RD + 1)][it]));
      } else if (bb == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      if (bb == 0) asm volatile("" : "+v"(bias_v[0]));
      store_slab<EPI, 2, HITERS, NT, C4, CS, 1>(g, g.C, ct + (bb & 1) * 32 * CS, bias_v, res[bb % (RD + 1)], te,
                                                m0 + band_row0(bb), n0, sc_v, am,
                                                LNF ? lnf + LN_ROW * band_row0(bb) : nullptr,
                                                LNF ? lnf + LN_ROW * BM : nullptr);
      if (bb & 1) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();  // every LDS read of the slab done (the last also frees `buf` and the fold's area)
        asm volatile("" ::: "memory");
      }
    }
    zero_acc();
  };

  // ---- the stream: k-tile j of the block = k-tile j % nk of local tile j / nk.
  // Iteration j: DMA of k-tile j + 1 into the other stage (released by the
  // previous iteration's barrier), k-tile j's MFMAs, wait for that DMA, barrier,
  // then after a tile's last k-tile its epilogue through stage j & 1 ----
  glds(0, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  int c_kt = 0, c_tl = 0;  // the k-tile being computed
  int n_kt = 1, n_tl = 0;  // the next one to load
  if (n_kt == nk) n_kt = 0, n_tl = 1;
  auto iter = [&](int cur, int j) __attribute__((always_inline)) {
    if (j + 1 < J) glds(n_tl, n_kt, cur ^ 1);
    if (++n_kt == nk) n_kt = 0, ++n_tl;
    compute(cur);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // k-tile j + 1 (and the previous epilogue's stores)
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (++c_kt == nk) {
      c_kt = 0;
      epilogue(c_tl++, cur);
    }
  };
  for (int j = 0; j < J; j += 2) {
    iter(0, j);
    if (j + 1 < J) iter(1, j + 1);
  }
}

// The same stream with three A stages (the DMA of A two k-tiles ahead, B's
// one: A streams from HBM at K = 3072, B stays in L2) for the flag sets
// without the LayerNorm fold: 3 x 32 KB + 2 x 32 KB = the whole 160 KB of
// LDS.  The epilogue stages a 64-row slab as two unpadded 32-row bands in the
// A and B stages the tile's last k-tile released, their 16-B chunks
// XOR-swizzled (csw_chunk) instead of padded.  Iteration j: B DMA of k-tile
// j + 1, A DMA of j + 2, k-tile j's MFMAs, wait (everything but A(j + 2)),
// barrier.  Same fragments, MFMA sequence and epilogue arithmetic as
// gemm_lpp_kernel.
template <int EPI>
__global__ __launch_bounds__(512, 1) void gemm_lpp3_kernel(GemmArgs g, int tiles_n, int ntiles) {
  static_assert((EPI & EP_LNFOLD) == 0, "three A stages: no room for the fold's LDS");
  constexpr int NT = 512, WM = 2, FM = 4, FN = 2, WTM = 128, WTN = 64, BM = 256, BN = 256;
  constexpr int BK = 32, SLOTS = 8, RPP = NT / SLOTS, A_CH = BM / RPP, B_CH = BN / RPP;
  constexpr int EPR = 64, OPS = BM * BK;  // floats per operand stage (32 KB)
  constexpr int CS = BN;                  // unpadded staging rows (swizzled chunks)
  static_assert(32 * CS <= OPS, "a 32-row band fits a stage");
  constexpr bool RES = (EPI & EP_RES) != 0;
  __shared__ __attribute__((aligned(16))) float lds[5 * OPS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const int l16 = lane & 15, lg = lane >> 4;
  const int G = gridDim.x, bid = blockIdx.x;
  const int nk = g.K / EPR;
  const int my_tiles = (ntiles - bid + G - 1) / G;
  const int J = my_tiles * nk;
  auto tile_origin = [&](int tl, int& m0, int& n0) __attribute__((always_inline)) {
    const int v = bid + tl * G;
    const int xcd = v & 7, q8 = ntiles >> 3, r8 = ntiles & 7;
    const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (v >> 3);
    const int tn = wgid % tiles_n, tm = wgid / tiles_n;
    m0 = tm * BM;
    n0 = tn * BN;
  };
  auto sa = [&](int i) { return lds + i * OPS; };        // A stages 0..2
  auto sb = [&](int i) { return lds + (3 + i) * OPS; };  // B stages 0..1
  const uint16_t* const Ab = reinterpret_cast<const uint16_t*>(g.A);
  const uint16_t* const Bb = reinterpret_cast<const uint16_t*>(g.B);
  // stream k-tile q = (tile q / nk, k-tile q % nk)
  auto glds_a = [&](int q, int buf) __attribute__((always_inline)) {
    int m0, n0;
    tile_origin(q / nk, m0, n0);
    const int kt = q % nk, t = lpp_opaque(tid), sl = t % SLOTS, cr = t / SLOTS;
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const int row = cr + i * RPP, m = min(m0 + row, g.M - 1);
      __builtin_amdgcn_global_load_lds((const void*)(Ab + (long long)m * g.lda + kt * EPR + lswz(row, sl) * 8),
                                       (__attribute__((address_space(3))) void*)(sa(buf) + (i * RPP + wave * 8) * BK),
                                       16, 0, 0);
    }
  };
  auto glds_b = [&](int q, int buf) __attribute__((always_inline)) {
    int m0, n0;
    tile_origin(q / nk, m0, n0);
    const int kt = q % nk, t = lpp_opaque(tid), sl = t % SLOTS, cr = t / SLOTS;
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      const int row = cr + i * RPP;
      __builtin_amdgcn_global_load_lds((const void*)(Bb + (long long)(n0 + row) * g.ldb + kt * EPR + lswz(row, sl) * 8),
                                       (__attribute__((address_space(3))) void*)(sb(buf) + (i * RPP + wave * 8) * BK),
                                       16, 0, 0);
    }
  };
  f32x4 acc4[FM][FN][4];
  auto zero_acc = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int t = 0; t < 4; ++t) acc4[i][j][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  };
  zero_acc();
  auto compute = [&](const float* la, const float* lb) __attribute__((always_inline)) {
    bf16x8 af[2][FM][2], bf[2][FN][2];
    auto rd = [&](int st) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int row = wm * WTM + i * 32 + h * 16 + l16;
          af[st][i][h] = *reinterpret_cast<const bf16x8*>(la + row * BK + lswz(row, 4 * st + lg) * 4);
        }
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int row = wn * WTN + j * 32 + h * 16 + l16;
          bf[st][j][h] = *reinterpret_cast<const bf16x8*>(lb + row * BK + lswz(row, 4 * st + lg) * 4);
        }
    };
    rd(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int st = 0; st < BK / 16; ++st) {
      if (st + 1 < BK / 16) rd(st + 1);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int t = 0; t < 4; ++t)
            acc4[i][j][t] =
                __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[st][i][t >> 1], bf[st][j][t & 1], acc4[i][j][t], 0, 0, 0);
      if (st + 1 < BK / 16) {
#pragma unroll
        for (int x = 0; x < 2 * (FM + FN); ++x) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 4 * FM * FN - 2 * (FM + FN), 0);
      }
    }
    __builtin_amdgcn_s_setprio(0);
  };

  constexpr int C4 = BN / 4, HITERS = 32 * C4 / NT, NB = 2 * FM, RD = 2;
  float am = 0.f;
  // epilogue of local tile tl: slab s = bands 2s (staged in A stage `ab`) and
  // 2s + 1 (B stage `bbuf`), band 2s + q = MFMA row tile s of wave row q
  auto epilogue = [&](int tl, float* ct0, float* ct1) __attribute__((always_inline)) {
    int m0, n0;
    tile_origin(tl, m0, n0);
    const int te = lpp_opaque(tid);
    const int c40 = te % C4;
    f32x4 bias_v[1] = {f32x4{0.f, 0.f, 0.f, 0.f}}, sc_v[1] = {f32x4{1.f, 1.f, 1.f, 1.f}};
    f32x4 res[RD + 1][HITERS];
    auto band_row0 = [&](int bb) { return (bb & 1) * 128 + (bb >> 1) * 32; };
    auto load_band = [&](int bb) __attribute__((always_inline)) {
      if constexpr (RES) {
        const int tq = lpp_opaque(tid);
        const int cq = tq % C4, rq = tq / C4;
#pragma unroll
        for (int it = 0; it < HITERS; ++it) {
          const int m = min(m0 + band_row0(bb) + rq + it * (NT / C4), g.M - 1);
          const float* p = g.residual + (long long)m * g.ldc + n0 + cq * 4;
          asm volatile("global_load_dwordx4 %0, %1, off" : "=&v"(res[bb % (RD + 1)][it]) : "v"(p) : "memory");
        }
      }
    };
    const int le = te & 63, we = te >> 6;
    auto stage = [&](int sl) __attribute__((always_inline)) {
      float* cw = ((we % WM) == 0 ? ct0 : ct1) + (we / WM) * WTN;
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int r = 4 * t + e, row = acc_row<true>(0, r, le), col = acc_col<true>(j, r, le) + (we / WM) * WTN;
            cw[row * CS + csw_chunk(row, col >> 2) * 4 + (col & 3) - (we / WM) * WTN] = acc4[sl][j][t][e];
          }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    };
    if ((EPI & EP_BIAS) && g.bias != nullptr)
      asm volatile("global_load_dwordx4 %0, %1, off" : "=&v"(bias_v[0]) : "v"(g.bias + n0 + c40 * 4) : "memory");
    load_band(0);
    load_band(1);
#pragma unroll
    for (int bb = 0; bb < NB; ++bb) {
      if ((bb & 1) == 0) stage(bb >> 1);
      if (bb + RD < NB) load_band(bb + RD);
      if constexpr (RES) {
        const int ahead = (NB - 1 - bb < RD ? NB - 1 - bb : RD);
        switch (HITERS * ahead) {
          case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
          case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
          default: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
        }
#pragma unroll
        for (int it = 0; it < HITERS; ++it) asm volatile("" : "+v"(res[bb % (RD + 1)][it]));
      } else if (bb == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      if (bb == 0) asm volatile("" : "+v"(bias_v[0]));
      store_slab<EPI, 2, HITERS, NT, C4, CS, 1, 1>(g, g.C, (bb & 1) ? ct1 : ct0, bias_v, res[bb % (RD + 1)], te,
                                                   m0 + band_row0(bb), n0, sc_v, am);
      if (bb & 1) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
      }
    }
    zero_acc();
  };

  // prologue: A(0), B(0), A(1); wait for all but A(1)
  glds_a(0, 0);
  glds_b(0, 0);
  if (J > 1) {
    glds_a(1, 1);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(A_CH) : "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  int c_kt = 0, c_tl = 0;
  // iteration j: A stage j % 3, B stage j % 2 (constants: unrolled by 6)
  auto iter = [&](int ja, int jb, int j) __attribute__((always_inline)) {
    if (j + 1 < J) glds_b(j + 1, jb ^ 1);
    const bool a2 = j + 2 < J;
    if (a2) glds_a(j + 2, (ja + 2) % 3);
    compute(sa(ja), sb(jb));
    // B(j + 1) and A(j + 1) landed (A(j + 2), issued last, may not have)
    if (a2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(A_CH) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (++c_kt == nk) {
      c_kt = 0;
      epilogue(c_tl++, sa(ja), sb(jb));
    }
  };
  for (int j = 0; j < J; j += 6) {
    iter(0, 0, j);
    if (j + 1 < J) iter(1, 1, j + 1);
    if (j + 2 < J) iter(2, 0, j + 2);
    if (j + 3 < J) iter(0, 1, j + 3);
    if (j + 4 < J) iter(1, 0, j + 4);
    if (j + 5 < J) iter(2, 1, j + 5);
  }
}

template <int EPI>
static hipError_t launch_lpp3_t(GemmArgs g, hipStream_t s, int n_cu) {
  const long long tiles_m = (g.M + 255) / 256, tiles_n = g.N / 256;
  const long long ntiles = tiles_m * tiles_n;
  if (ntiles <= 0) return hipSuccess;
  if (ntiles * (g.K / 64) > 0x7fffffffLL) return hipErrorInvalidValue;
  const int slots = std::max(8, n_cu & ~7);
  const int grid = ntiles <= slots ? (int)ntiles : slots;
  hipLaunchKernelGGL((gemm_lpp3_kernel<EPI>), dim3((unsigned)grid), dim3(512), 0, s, g, (int)tiles_n, (int)ntiles);
  return hipGetLastError();
}

template <int EPI>
static hipError_t launch_lpp_t(GemmArgs g, hipStream_t s, int n_cu) {
  const long long tiles_m = (g.M + 255) / 256, tiles_n = g.N / 256;
  const long long ntiles = tiles_m * tiles_n;
  if (ntiles <= 0) return hipSuccess;
  if (ntiles * (g.K / 64) > 0x7fffffffLL) return hipErrorInvalidValue;
  // one block per CU; a block that owns several tiles stays on its XCD (grid a multiple of 8)
  const int slots = std::max(8, n_cu & ~7);
  const int grid = ntiles <= slots ? (int)ntiles : slots;
  hipLaunchKernelGGL((gemm_lpp_kernel<EPI>), dim3((unsigned)grid), dim3(512), 0, s, g, (int)tiles_n, (int)ntiles);
  return hipGetLastError();
}

}  // namespace

// The ViT linears' epilogue flag sets (as gemm_f32.hip launch_t); other flag
// sets return hipErrorNotSupported (the caller runs the one-tile kernel).
bool lpp_eligible(const GemmArgs& g) {
  // (K <= 1024: c_proj, K = 3072, ran 11 % slower than the one-tile kernel)
  if (g.M <= 0 || (g.N % 256) != 0 || (g.K % 64) != 0 || g.K > 1024 || g.k_split > 0 || g.sym) return false;
  switch (ep_flags(g)) {
    case EP_BIAS | EP_BF16:
    case EP_BIAS | EP_RES:
    case EP_BIAS | EP_GELU | EP_BF16:
    case EP_BIAS | EP_RES | EP_STATS:
    case EP_BIAS | EP_BF16 | EP_LNFOLD:
    case EP_BIAS | EP_GELU | EP_BF16 | EP_LNFOLD: return true;
    default: return false;
  }
}

// The three-A-stage form: the pick for the no-fold flag sets with K <= 1024
// (out-proj 0.579 -> 0.546 ms against the two-stage form, r05u_vitlin.txt);
// at K = 3072 (c_proj) it ran 1.313 ms against the one-tile kernel's 1.257,
// so lp_cfg 6 (tests) is the only way there.
bool lpp3_eligible(const GemmArgs& g) {
  if (g.M <= 0 || (g.N % 256) != 0 || (g.K % 64) != 0 || g.k_split > 0 || g.sym) return false;
  const int f = ep_flags(g);
  return f == (EP_BIAS | EP_BF16) || f == (EP_BIAS | EP_RES) || f == (EP_BIAS | EP_GELU | EP_BF16) ||
         f == (EP_BIAS | EP_RES | EP_STATS);
}
hipError_t launch_lpp3(const GemmArgs& g, hipStream_t s, int n_cu) {
  switch (ep_flags(g)) {
    case EP_BIAS | EP_BF16: return launch_lpp3_t<EP_BIAS | EP_BF16>(g, s, n_cu);
    case EP_BIAS | EP_RES: return launch_lpp3_t<EP_BIAS | EP_RES>(g, s, n_cu);
    case EP_BIAS | EP_GELU | EP_BF16: return launch_lpp3_t<EP_BIAS | EP_GELU | EP_BF16>(g, s, n_cu);
    case EP_BIAS | EP_RES | EP_STATS: return launch_lpp3_t<EP_BIAS | EP_RES | EP_STATS>(g, s, n_cu);
    default: return hipErrorNotSupported;
  }
}

hipError_t launch_lpp(const GemmArgs& g, hipStream_t s, int n_cu) {
  switch (ep_flags(g)) {
    case EP_BIAS | EP_BF16: return launch_lpp_t<EP_BIAS | EP_BF16>(g, s, n_cu);
    case EP_BIAS | EP_RES: return launch_lpp_t<EP_BIAS | EP_RES>(g, s, n_cu);
    case EP_BIAS | EP_GELU | EP_BF16: return launch_lpp_t<EP_BIAS | EP_GELU | EP_BF16>(g, s, n_cu);
    case EP_BIAS | EP_RES | EP_STATS: return launch_lpp_t<EP_BIAS | EP_RES | EP_STATS>(g, s, n_cu);
    case EP_BIAS | EP_BF16 | EP_LNFOLD: return launch_lpp_t<EP_BIAS | EP_BF16 | EP_LNFOLD>(g, s, n_cu);
    case EP_BIAS | EP_GELU | EP_BF16 | EP_LNFOLD: return launch_lpp_t<EP_BIAS | EP_GELU | EP_BF16 | EP_LNFOLD>(g, s, n_cu);
    default: return hipErrorNotSupported;
  }
}

}  // namespace rr
