// gemm_s3.hip — fp32-accurate GEMM on the 16-bit matrix cores: the f16x2
// split core of the ResNet trunk (rr_conv2d_h2, rr_bottleneck_out_h2,
// rr_stem_pool_h2; networks/backbone.py:60-109, :305-346).
//
// gfx950 has no xf32/TF32 MFMA, and its f32-input MFMA runs at 1/16 of the
// bf16 rate (MI355X_MICROARCH.md: 157 vs 2500 TF/s dense).  Every fp32
// operand is scaled by a power of two and split into two fp16 pieces,
// x 2^e = x0 + x1 + r with |r| <= 2^-22 |x 2^e|; a.b keeps a0b0 (its own
// accumulator) + a0b1 + a1b0 (DESIGN.md, f16x2 split core): three fp16 MFMAs
// per fp32 product with exact products and fp32 accumulation, error vs
// float64 at the exact-fp32 MFMA chain's (tests/test_gpu_h2.py).
//
// The kernel templates carry the split kind SP (planes per operand).  Rounds
// 1-2 ran a three-plane bf16 split (SP 3: six bf16 MFMAs per product) here;
// it lost to f16x2 in round 3 and its instantiations and entry points
// (rr_conv2d_s3, rr_linear_s3, rr_split3_bf16) were retired in ABI 6: SP 2
// is the only split these templates compile for (static_assert).
//
// Operands: A = fp32 activations (dense rows or the implicit im2col of an
// NHWC map with Cin % 32 == 0), split in registers while staging into LDS;
// B = weights pre-split once into fp16 planes [2][N][K] (rr_split2_f16),
// copied global -> LDS by LDS-DMA (global_load_lds).  16-B slots of the LDS
// rows are XOR-swizzled so the fragment ds_read_b128 are conflict-free.
#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "gemm_epilogue.hpp"
#include "h2_common.hpp"
#include "rr_internal.hpp"

namespace rr {

// exact 3-way split of x into bf16 pieces, returned as fp32 bit patterns
// whose low 16 bits are zero
__device__ __forceinline__ void split3(float x, uint32_t& h, uint32_t& m, uint32_t& l) {
  const uint32_t hb = __float_as_uint(x) & 0xffff0000u;
  const float r1 = x - __uint_as_float(hb);
  const uint32_t mb = __float_as_uint(r1) & 0xffff0000u;
  const float r2 = r1 - __uint_as_float(mb);
  h = hb;
  m = mb;
  l = __float_as_uint(r2);
}

// two bf16 (the high halves of e0, e1) in one dword, e0 in the low half
__device__ __forceinline__ uint32_t pack2(uint32_t e0, uint32_t e1) { return __builtin_amdgcn_perm(e1, e0, 0x07060302u); }

// 32 zero bytes in global memory: the A source of padding taps and rows past M
__device__ f32x4 s3_zero_src[2];
__device__ __forceinline__ const f32x4* s3_zero_page() { return s3_zero_src; }

// Diagnostic build only (-DRR_S3_PHASES=1, tools/phase_build.sh): per-wave
// s_memtime deltas of the k-loop phases of the f16x2 kernels, summed over
// every wave into s3_phase_sum[kernel][phase] (rr_debug_phases reads them).
// Phases: 0 issue loads, 1 first MFMA part, 2 mid wait, 3 split + second
// MFMA part, 4 end wait, 5 barrier, 6 epilogue, 7 prologue (kernel 0: the
// one-tile kernels, 1: config 8).  Kernel 2 (config 15): 0 issue + first
// k-step, 1 mid wait, 2 split + second k-step, 3 end wait + barrier, 4
// epilogue staging (+ its barrier), 5 epilogue residual waits, 6 epilogue
// stores (+ barriers), 7 prologue.  Kernel 3 (the halo tile): 0 B DMA + halo
// pass issue / split, 1 MFMAs (+ fragment reads), 2 end wait, 3 barrier, 6
// epilogue, 7 prologue.  The timers cost a few % and are compiled out of the
// product library.
#ifndef RR_S3_PHASES
#define RR_S3_PHASES 0
#endif
#if RR_S3_PHASES
__device__ unsigned long long s3_phase_sum[4][8];
struct S3Phases {
  unsigned long long t, acc[8];
  __device__ __forceinline__ S3Phases() {
    t = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < 8; ++i) acc[i] = 0;
  }
  __device__ __forceinline__ void mark(int i) {
    const unsigned long long n = __builtin_amdgcn_s_memtime();
    acc[i] += n - t;
    t = n;
  }
  __device__ __forceinline__ void flush(int kernel) {
    if ((threadIdx.x & 63) == 0)
      for (int i = 0; i < 8; ++i) atomicAdd(&s3_phase_sum[kernel][i], acc[i]);
  }
};
#define RR_PH_DECL S3Phases ph_;
#define RR_PH(i) ph_.mark(i)
#define RR_PH_FLUSH(k) ph_.flush(k)
#else
#define RR_PH_DECL
#define RR_PH(i) ((void)0)
#define RR_PH_FLUSH(k) ((void)0)
#endif

// MF16 (BK = 32): each 32x32 tile is four v_mfma_f32_16x16x32_bf16
// tiles (one 32-deep k-step per k-tile instead of two 16-deep ones; the
// 16x16 shape holds a higher clock on random operands, MI355X_MICROARCH.md
// 'DVFS give-back' item 7).  The k-tile's MFMAs go in two parts around the A
// split: a0b0 + a1b1 + a0b1 + a1b0 (planes 0-1), then a0b2 + a2b0 (plane 2).
// IL (the 32x32x16 two-stage loop, dense or Cin % 32 == 0 conv A): the next
// k-tiles' B DMA and A loads are not issued as one burst at the top of the
// k-tile but one instruction group at a time among the first MFMAs of its
// first k-step (see gemm_f32.hip IL: a burst of every wave's loads at once
// fills the vector-memory issue queue and stalls the MFMAs behind it).
template <int WM, int WN, int FM, int FN, int BK, int AMODE, int MINB, int MF16 = 0, int EPI = -1, int SP = 2,
          int NSTG = 2, int POOL = 0, int ACC1 = 0, int IL = 0>
__global__ __launch_bounds__(64 * WM * WN, MINB) void gemm_s3_kernel(GemmArgs g, int tiles_n) {
  static_assert(!ACC1 || SP == 2, "one accumulator: the f16x2 split");
  static_assert(!POOL || (AMODE == A_CONV_C4 && WM * 32 * FM == 256 && SP == 2), "stem + max-pool: 256-row NHWC4 tile");
  static_assert(NSTG == 2 || (NSTG == 3 && MF16 && SP == 2), "three LDS stages: the f16x2 16x16x32 tile");
  static_assert(!IL || (!MF16 && NSTG == 2 && !POOL), "IL: the 32x32x16 two-stage loop");
  static_assert(!MF16 || BK == 32, "MF16: BK 32");
  static_assert(SP == 2, "split kind: f16x2 (the bf16x3 instantiations were retired in ABI 6)");
  static_assert(SP == 3 || (EPI >= 0 && (EPI & EP_SCALE)), "f16x2: scaled epilogue");
  typedef typename S3Frag<SP>::T frag_t;
  constexpr int NP = SP;                     // planes per operand
  constexpr int NT = 64 * WM * WN, NW = WM * WN;
  constexpr int WTM = 32 * FM, WTN = 32 * FN;
  constexpr int BM = WTM * WM, BN = WTN * WN;
  constexpr int SL = BK / 8;                 // 16-B slots per plane row
  constexpr int A_EL = NP * BM * BK;         // 16-bit elements per stage: A planes
  constexpr int BUF = A_EL + NP * BN * BK;   // 16-bit elements per stage: A + B planes
  constexpr int A_RPP = NT / SL;             // A rows staged per pass
  constexpr int A_CH = BM / A_RPP;           // A chunks (8 k each) per thread
  constexpr int B_RPI = 64 / SL;             // plane rows per LDS-DMA wave instruction
  constexpr int B_TI = NP * BN / B_RPI;      // LDS-DMA wave instructions per k-tile
  constexpr int B_INS = (B_TI + NW - 1) / NW; // ... per wave (the last round may be partial)
  static_assert(BM % A_RPP == 0 && (NP * BN) % B_RPI == 0, "staging must tile the block");
  static_assert(BK == 16 || BK == 32, "BK");
  // f16x2 at one block per CU: room for the whole fp32 C tile, so the
  // epilogue stages it in one slab (two planes leave the stages smaller)
  // (rows padded by 4 / 8 floats, epilogue_store)
  constexpr int CT_F = BM * (BN + (MF16 ? 4 : 8));
  // (the fused stem + max-pool stages its whole C tile at any MINB)
  constexpr int LDS_U16 =
      (SP == 2 && (MINB == 1 || POOL) && 2 * CT_F > NSTG * BUF && 2 * CT_F <= 80 * 1024) ? 2 * CT_F : NSTG * BUF;
  __shared__ __attribute__((aligned(16))) uint16_t lds[LDS_U16];

  // the A operand's split scale (f16x2): its max-|x| record is loaded first,
  // so it has landed by the prologue's first counted wait
  uint32_t a_amax_w = 0;
  if constexpr (SP == 2) a_amax_w = amax_load_slot(g.a_amax);

  // round stagger (GemmArgs): half of the first round's blocks start later,
  // so in every later round half the CUs run their k-loop while the other
  // half run their HBM-heavy epilogue (blocks b, b+8, ... share an XCD, so
  // (b >> 3) & 1 halves every XCD).  At two blocks per CU the later half is
  // the second resident of every CU (blocks n_cu .. 2 n_cu - 1: the
  // dispatcher fills every CU's first slot first), so each CU's two blocks
  // alternate between k-loop and epilogue.
  if (g.stagger_sleeps > 0 && (int)blockIdx.x < g.stagger_blocks &&
      (MINB >= 2 ? (int)blockIdx.x >= g.stagger_blocks / 2 : ((blockIdx.x >> 3) & 1)))
    for (int i = 0; i < g.stagger_sleeps; ++i) __builtin_amdgcn_s_sleep(32);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float a_sc = 1.f, a_isc = 1.f;
  const int wm = wave % WM, wn = wave / WM;
  const int lr = lane & 31, lh = lane >> 5;

  // XCD-aware bijective block remap (blocks b, b+8, ... share an XCD)
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int tn = wgid % tiles_n, tm = wgid / tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int nk = g.K / BK;  // K % BK == 0 (checked on the host)

  // ---- A: per-chunk row state (fp32, register-staged, split on store) ----
  const int a_slot = tid % SL, a_row = tid / SL;
  const float* a_ptr[A_CH];
  int a_ih0[A_CH], a_iw0[A_CH];
  bool a_ok[A_CH];
#pragma unroll
  for (int i = 0; i < A_CH; ++i) {
    const int m = m0 + a_row + i * A_RPP;
    a_ok[i] = m < g.M;
    const int mm = a_ok[i] ? m : 0;
    if constexpr (POOL) {
      // tile tm = (image, pr, pc); local row lr -> conv output pixel
      // (16 pr - 1 + lr / 15, 14 pc - 1 + lr % 15), lr < 255; rows outside the
      // conv map load the zero page and are left out of every window
      const int tpi = g.pool_tr * g.pool_tc;
      const int b = tm / tpi, t2 = tm - b * tpi, pr = t2 / g.pool_tc, pc = t2 - pr * g.pool_tc;
      const int tr = a_row + i * A_RPP, q = tr / 15;
      const int oh = 16 * pr - 1 + q, ow = 14 * pc - 1 + (tr - 15 * q);
      a_ok[i] = tr < 255 && (unsigned)oh < (unsigned)g.OH && (unsigned)ow < (unsigned)g.OW;
      a_ih0[i] = oh * g.stride - g.pad;
      a_iw0[i] = ow * g.stride - g.pad;
      a_ptr[i] = g.A + (((long long)b * g.H + a_ih0[i]) * g.W + a_iw0[i]) * g.Cin;
    } else if constexpr (AMODE == A_DENSE) {
      a_ptr[i] = g.A + (long long)mm * g.lda + a_slot * 8;
      a_ih0[i] = a_iw0[i] = 0;
    } else {
      const int ohw = g.OH * g.OW;
      const int b = mm / ohw, rem = mm - b * ohw;
      const int oh = rem / g.OW, ow = rem - oh * g.OW;
      a_ih0[i] = oh * g.stride - g.pad;
      a_iw0[i] = ow * g.stride - g.pad;
      // the (possibly padded, out-of-image) top-left tap pixel; a k-tile adds a
      // block-uniform offset (kh*W + kw)*Cin + cin0
      a_ptr[i] = g.A + (((long long)b * g.H + a_ih0[i]) * g.W + a_iw0[i]) * g.Cin + (AMODE == A_CONV ? a_slot * 8 : 0);
    }
  }
  // conv tap of the k-tile the A loader is at, advanced incrementally (the
  // loader requests k-tiles in non-decreasing order, one step at a time):
  // no per-tile integer divisions
  int tp_kt = 0, tp_kh = 0, tp_kw = 0, tp_cin = 0;
  long long tp_off = 0;  // (kh * W + kw) * Cin + cin0
  auto tap_to = [&](int kt) {
    while (tp_kt < kt) {
      ++tp_kt;
      tp_off += BK;
      tp_cin += BK;
      if (tp_cin == g.Cin) {
        tp_cin = 0;
        if (++tp_kw == g.KW) {
          tp_kw = 0;
          ++tp_kh;
          tp_off += (long long)(g.W - g.KW) * g.Cin;
        }
      }
    }
  };
  f32x4 ra2[2][A_CH][2];
  auto load_a = [&](int kt, int rb) {
    f32x4(&ra)[A_CH][2] = ra2[rb];
    const int k0 = kt * BK;
    if constexpr (AMODE == A_DENSE) {
#pragma unroll
      for (int i = 0; i < A_CH; ++i) {
        // every load is issued (the counted vmcnt of the k-loop assumes A_LD
        // loads per tile); out-of-range rows read the zero page, so the
        // loaded registers are used as they are, no select after the load
        // (a select right after it makes hipcc wait for the load at once)
        const f32x4* p = a_ok[i] ? reinterpret_cast<const f32x4*>(a_ptr[i] + k0) : s3_zero_page();
        s3_load2<1>(p, ra[i]);
      }
    } else if constexpr (AMODE == A_CONV_C4) {
      // NHWC4 stem (RGB + a zero channel): a k-tile is BK/4 filter taps of 4
      // channels, a thread's 8-k chunk the taps (BK/4) kt + 2 slot + {0, 1},
      // one 16-B load each; taps past KH*KW (K padded to a multiple of 32) and
      // padding pixels read the zero page
      const int tb = kt * (BK / 4), khb = tb / g.KW, kwb = tb - khb * g.KW;
      const f32x4* p[A_CH][2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        int kh = khb, kw = kwb + 2 * a_slot + e;
        while (kw >= g.KW) kw -= g.KW, ++kh;
        const bool tap_ok = kh < g.KH;
        const long long toff = (long long)(kh * g.W + kw) * 4;
#pragma unroll
        for (int i = 0; i < A_CH; ++i) {
          const int ih = a_ih0[i] + kh, iw = a_iw0[i] + kw;
          const bool ok = tap_ok && a_ok[i] && (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
          p[i][e] = ok ? reinterpret_cast<const f32x4*>(a_ptr[i] + toff) : s3_zero_page();
        }
      }
#pragma unroll
      for (int i = 0; i < A_CH; ++i) s3_load1x2<1>(p[i][0], p[i][1], ra[i]);
    } else {
      // Cin % 32 == 0: the whole k-tile lies in one (kh, kw) filter tap
      tap_to(kt);
      const int kh = tp_kh, kw = tp_kw;
      const long long toff = tp_off;
#pragma unroll
      for (int i = 0; i < A_CH; ++i) {
        const int ih = a_ih0[i] + kh, iw = a_iw0[i] + kw;
        const bool ok = a_ok[i] && (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
        const f32x4* p = ok ? reinterpret_cast<const f32x4*>(a_ptr[i] + toff) : s3_zero_page();
        s3_load2<1>(p, ra[i]);
      }
    }
  };
  // IL: chunk i of load_a(kt, rb) alone (dense or Cin % 32 == 0 conv A)
  auto load_a_chunk = [&](int kt, int rb, int i) {
    static_assert(!IL || AMODE == A_DENSE || AMODE == A_CONV, "IL: dense or Cin % 32 == 0 conv A");
    f32x4(&ra)[A_CH][2] = ra2[rb];
    if constexpr (AMODE == A_DENSE) {
      const f32x4* p = a_ok[i] ? reinterpret_cast<const f32x4*>(a_ptr[i] + kt * BK) : s3_zero_page();
      s3_load2<1>(p, ra[i]);
    } else if constexpr (AMODE == A_CONV) {
      tap_to(kt);
      const int ih = a_ih0[i] + tp_kh, iw = a_iw0[i] + tp_kw;
      const bool ok = a_ok[i] && (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
      const f32x4* p = ok ? reinterpret_cast<const f32x4*>(a_ptr[i] + tp_off) : s3_zero_page();
      s3_load2<1>(p, ra[i]);
    }
  };
  // split the staged fp32 chunks into the three packed bf16 planes
  u32x4 pk[A_CH][NP];
  auto split_a = [&](int rb) {
    const f32x4(&ra)[A_CH][2] = ra2[rb];
    if constexpr (SP == 2) {
#pragma unroll
      for (int i = 0; i < A_CH; ++i) split2h8(ra[i], a_sc, pk[i][0], pk[i][1]);
      return;
    }
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      uint32_t h[8], m[8], l[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        // scalar f32 subtractions: packed v_pk_add_f32 beside MFMAs costs
        // more issue time than two v_sub_f32 (MI355X_MICROARCH.md constants)
        const float x = ra[i][e >> 2][e & 3];
        const float r1 = x - __uint_as_float(__float_as_uint(x) & 0xffff0000u);
        const float r2 = r1 - __uint_as_float(__float_as_uint(r1) & 0xffff0000u);
        h[e] = __float_as_uint(x);  // pack2 keeps only the high halves
        m[e] = __float_as_uint(r1);
        l[e] = __float_as_uint(r2);
      }
      pk[i][0] = u32x4{pack2(h[0], h[1]), pack2(h[2], h[3]), pack2(h[4], h[5]), pack2(h[6], h[7])};
      pk[i][1] = u32x4{pack2(m[0], m[1]), pack2(m[2], m[3]), pack2(m[4], m[5]), pack2(m[6], m[7])};
      pk[i][NP - 1] = u32x4{pack2(l[0], l[1]), pack2(l[2], l[3]), pack2(l[4], l[5]), pack2(l[6], l[7])};
    }
  };
  auto write_a = [&](int buf) {
    uint16_t* la = lds + buf * BUF;
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const int row = a_row + i * A_RPP;
      const int off = row * BK + pswz<BK, SP>(row, a_slot) * 8;
#pragma unroll
      for (int p = 0; p < NP; ++p) *reinterpret_cast<u32x4*>(la + p * BM * BK + off) = pk[i][p];
    }
  };
  auto store_a = [&](int rb, int buf) {
    split_a(rb);
    write_a(buf);
  };

  // ---- B: three bf16 planes, LDS-DMA (64 lanes x 16 B = B_RPI whole plane
  // rows per instruction; the swizzle moves to the source slot) ----
  const uint16_t* b_src[B_INS];
  const uint16_t* Bp = reinterpret_cast<const uint16_t*>(g.B);
#pragma unroll
  for (int i = 0; i < B_INS; ++i) {
    const int prow = min(i * NW + wave, B_TI - 1) * B_RPI + lane / SL;
    const int p = prow / BN, r = prow - p * BN;
    const int n = min(n0 + r, g.N - 1);  // rows past N feed only unstored columns
    b_src[i] = Bp + p * g.b_plane + (long long)n * g.ldb + pswz<BK, SP>(r, lane % SL) * 8;
  }
  auto glds_b = [&](int kt, int buf) {
    uint16_t* lb = lds + buf * BUF + A_EL;
    // every wave issues B_INS (the counted vmcnt assumes it): in a partial
    // last round the surplus waves repeat the last row group (same source,
    // same LDS destination)
#pragma unroll
    for (int i = 0; i < B_INS; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(b_src[i] + (long long)kt * BK),
                                       (__attribute__((address_space(3))) void*)(lb + min(i * NW + wave, B_TI - 1) * B_RPI * BK),
                                       16, 0, 0);
  };

  auto glds_b_one = [&](int kt, int buf, int i) {
    uint16_t* lb = lds + buf * BUF + A_EL;
    __builtin_amdgcn_global_load_lds((const void*)(b_src[i] + (long long)kt * BK),
                                     (__attribute__((address_space(3))) void*)(lb + min(i * NW + wave, B_TI - 1) * B_RPI * BK),
                                     16, 0, 0);
  };
  // IL: the iteration's load groups in issue order (B DMA of kt + 1, then the
  // A chunks of kt + 2: the counted waits assume that order), group q before
  // MFMA number 2q of the first k-step, each fenced in place
  constexpr int IL_GROUPS = B_INS + A_CH;
  // every group's MFMA number exists: 0 .. FM FN - 1 (a0b0), then FM FN + 2m
  static_assert(!IL || ((FM * FN) % 2 == 0 && 2 * (IL_GROUPS - 1) < 3 * FM * FN), "IL: a slot for every load group");
  auto il_issue = [&](int kt, int cur, int idx) {
    if constexpr (IL) {
#pragma unroll
      for (int q = 0; q < IL_GROUPS; ++q) {
        if (2 * q != idx) continue;
        __builtin_amdgcn_sched_barrier(0);
        if (q < B_INS) glds_b_one(min(kt + 1, nk - 1), cur ^ 1, q);
        else load_a_chunk(min(kt + 2, nk - 1), cur, q - B_INS);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };

  f32x16 hi[FM][FN];
  f32x16 lo[ACC1 ? 1 : FM][ACC1 ? 1 : FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        hi[i][j][r] = 0.f;
        if constexpr (!ACC1) lo[i][j][r] = 0.f;
      }

  // IL, first k-step: iteration kt_il's loads go out among the MFMAs
  auto compute_st = [&](int cur, int st, int kt_il = 0) {
    const uint16_t* la = lds + cur * BUF;
    const uint16_t* lb = la + A_EL;
    {
      frag_t a[NP][FM], b[NP][FN];
#pragma unroll
      for (int p = 0; p < NP; ++p) {
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const int row = wm * WTM + i * 32 + lr;
          a[p][i] = *reinterpret_cast<const frag_t*>(la + (p * BM + row) * BK + pswz<BK, SP>(row, 2 * st + lh) * 8);
        }
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int row = wn * WTN + j * 32 + lr;
          b[p][j] = *reinterpret_cast<const frag_t*>(lb + (p * BN + row) * BK + pswz<BK, SP>(row, 2 * st + lh) * 8);
        }
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          if constexpr (IL) {
            if (st == 0) il_issue(kt_il, cur, i * FN + j);
          }
          hi[i][j] = s3_mf32<SP>(a[0][i], b[0][j], hi[i][j]);
        }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          if constexpr (IL) {
            if (st == 0) il_issue(kt_il, cur, FM * FN + 2 * (i * FN + j));
          }
          f32x16& L = ACC1 ? hi[i][j] : lo[ACC1 ? 0 : i][ACC1 ? 0 : j];
          if constexpr (SP == 3) {
            L = s3_mf32<SP>(a[1][i], b[1][j], L);
            L = s3_mf32<SP>(a[0][i], b[NP - 1][j], L);
            L = s3_mf32<SP>(a[NP - 1][i], b[0][j], L);
          }
          L = s3_mf32<SP>(a[0][i], b[1][j], L);
          L = s3_mf32<SP>(a[1][i], b[0][j], L);
        }
    }
  };
  // ---- MF16: 16x16x32 tiles, sub-tile t = 2a + b (row half a, column half b) ----
  f32x4 hi4[MF16 ? FM : 1][MF16 ? FN : 1][4], lo4[MF16 && !ACC1 ? FM : 1][MF16 && !ACC1 ? FN : 1][4];
  frag_t fa[MF16 ? NP : 1][MF16 ? FM : 1][2], fb[MF16 ? NP : 1][MF16 ? FN : 1][2];
  if constexpr (MF16) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          hi4[i][j][t] = f32x4{0.f, 0.f, 0.f, 0.f};
          if constexpr (!ACC1) lo4[i][j][t] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
  }
  // ACC1: the plane-1 products go to the a0b0 accumulator (one accumulator set)
#define RR_LO(i, j, t) (*(ACC1 ? &hi4[i][j][t] : &lo4[ACC1 ? 0 : i][ACC1 ? 0 : j][t]))
  const int l16 = lane & 15, lg = lane >> 4;
  // plane p fragments of one 32-deep k-tile: lane group lg holds k = 8lg..8lg+7
  // (16-B slot lg) of row l16 of each 16-row half
  auto rd_mf = [&](int cur, int p) {
    // three stages: the stage offset (up to 96 KB) does not fit the 16-bit
    // ds_read offset, so each stage would need its own address registers;
    // an opaque per-call base keeps one set
    const uint16_t* la = lds + (NSTG == 3 ? s3_opaque(cur * BUF) : cur * BUF);
    const uint16_t* lb = la + A_EL;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int row = wm * WTM + i * 32 + h * 16 + l16;
        fa[MF16 ? p : 0][i][h] = *reinterpret_cast<const frag_t*>(la + (p * BM + row) * BK + pswz<BK, SP>(row, lg) * 8);
      }
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int row = wn * WTN + j * 32 + h * 16 + l16;
        fb[MF16 ? p : 0][j][h] = *reinterpret_cast<const frag_t*>(lb + (p * BN + row) * BK + pswz<BK, SP>(row, lg) * 8);
      }
  };
#define RR_MF16(a, b, c) c = s3_mf16<SP>(a, b, c)
  // k-tile of MFMAs in two parts.  lo1: the plane-1 products into lo (SP 3:
  // a1b1, a0b1, a1b0; SP 2: a0b1, a1b0); rest: a0b0 into hi, then (SP 3) the
  // plane-2 products (a0b2, a2b0) into lo — the same per-accumulator order as
  // one pass — with the A split + LDS store of the next stage interleaved
  // (the plane-1 fragments are dead by then, which leaves the registers for it).
  auto mf_lo1 = [&](int cur) {
    if constexpr (MF16) {
      rd_mf(cur, 0);
      rd_mf(cur, 1);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            if constexpr (SP == 3) RR_MF16(fa[1][i][t >> 1], fb[1][j][t & 1], lo4[i][j][t]);
            RR_MF16(fa[0][i][t >> 1], fb[1][j][t & 1], RR_LO(i, j, t));
            RR_MF16(fa[1][i][t >> 1], fb[0][j][t & 1], RR_LO(i, j, t));
          }
    }
  };
  // with two A chunks per thread the plane-0 fragments are re-read for the
  // plane-2 products rather than held across the A split (holding them spills)
  constexpr bool MF_REREAD = A_CH >= 2;
  // dense A (1x1 convs, linears), SP 3: a0b0 + the plane-1 products, then the
  // split, then the plane-2 products (the order above measured slower there)
  auto mf_dense0 = [&](int cur) {
    if constexpr (MF16 && SP == 3) {
      rd_mf(cur, 0);
      rd_mf(cur, 1);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int t = 0; t < 4; ++t) RR_MF16(fa[0][i][t >> 1], fb[0][j][t & 1], hi4[i][j][t]);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            RR_MF16(fa[1][i][t >> 1], fb[1][j][t & 1], lo4[i][j][t]);
            RR_MF16(fa[0][i][t >> 1], fb[1][j][t & 1], lo4[i][j][t]);
            RR_MF16(fa[1][i][t >> 1], fb[0][j][t & 1], lo4[i][j][t]);
          }
    }
  };
  auto mf_dense1 = [&](int cur) {
    if constexpr (MF16 && SP == 3) {
      if constexpr (MF_REREAD) rd_mf(cur, 0);
      rd_mf(cur, NP - 1);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            RR_MF16(fa[0][i][t >> 1], fb[NP - 1][j][t & 1], lo4[i][j][t]);
            RR_MF16(fa[NP - 1][i][t >> 1], fb[0][j][t & 1], lo4[i][j][t]);
          }
    }
  };
  // rbn: the register buffer holding the next A k-tile; stn: the stage it goes to
  auto mf_rest = [&](int cur, int rbn, int stn) {
    if constexpr (MF16) {
      split_a(rbn);
      write_a(stn);  // that stage is free since the last barrier
      // f16x2: the conv A loader's state leaves no room to hold the plane-0
      // fragments across the split (2 registers spilled): re-read them
      // (ACC1 leaves the registers to hold them)
      if constexpr (SP == 2 && !ACC1 && (MF_REREAD || AMODE != A_DENSE)) rd_mf(cur, 0);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int t = 0; t < 4; ++t) RR_MF16(fa[0][i][t >> 1], fb[0][j][t & 1], hi4[i][j][t]);
      if constexpr (SP == 3) {
        if constexpr (MF_REREAD) rd_mf(cur, 0);
        rd_mf(cur, NP - 1);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
#pragma unroll
            for (int t = 0; t < 4; ++t) {
              RR_MF16(fa[0][i][t >> 1], fb[NP - 1][j][t & 1], lo4[i][j][t]);
              RR_MF16(fa[NP - 1][i][t >> 1], fb[0][j][t & 1], lo4[i][j][t]);
            }
#pragma unroll
        for (int x = 0; x < 3 * FM * FN * 4; ++x) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // 1 MFMA
          __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);  // 1 VALU
        }
      } else {
        // SP 2: the split's VALU (about 3 per element) two per MFMA gap
#pragma unroll
        for (int x = 0; x < FM * FN * 4; ++x) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // 1 MFMA
          __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);  // 2 VALU
        }
      }
    }
  };
#undef RR_MF16

  constexpr int A_LD = 2 * A_CH;  // A global loads per tile per thread
  {
    // Pipelined k-loop with asynchronous A loads (s3_load2<1>), two register
    // buffers: A(j) lives in buffer j&1.  Iteration kt issues the B DMA of
    // tile kt+1 and the A loads of tile kt+2 (into the buffer A(kt) left),
    // computes tile kt, then waits for everything but the A loads of kt+2
    // (so A(kt+1) and B(kt+1) have landed), splits A(kt+1) into the other
    // stage and crosses a raw barrier.  An A load thus has almost two
    // iterations to land instead of one; its split runs between the MFMAs of
    // the second 16-deep step.  The loop is unrolled by two so the stage and
    // buffer indices are constants.
    auto launder_a = [&](int rb) {
#pragma unroll
      for (int i = 0; i < A_CH; ++i) {
        s3_launder(ra2[rb][i][0]);
        s3_launder(ra2[rb][i][1]);
      }
    };
    if constexpr (NSTG == 3) {
      // Three LDS stages (config 9): the B DMA of k-tile kt+2 and the A
      // loads of kt+2 go out at the start of iteration kt, so B has two
      // iterations to land instead of one; A(kt+1) is split into stage
      // (kt+1) % 3 among the MFMAs as before.  Its counted wait also covers
      // B(kt+1) (issued before it), so the iteration ends on the barrier
      // alone.  Unrolled by six: stage (kt % 3) and register buffer (kt % 2)
      // indices are constants.
      load_a(0, 0);
      glds_b(0, 0);
      glds_b(nk > 1 ? 1 : 0, 1);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * B_INS) : "memory");  // A(0) landed
      launder_a(0);
      {
        const int e = __builtin_amdgcn_readfirstlane(h2_exp(amax_reduce(a_amax_w)));
        a_sc = __int_as_float((127 + e) << 23);
        a_isc = __int_as_float((127 - e) << 23);
      }
      store_a(0, 0);
      load_a(nk > 1 ? 1 : 0, 1);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(A_LD + B_INS) : "memory");  // B(0) landed
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      auto iter3 = [&](int kt, int cur, int rb) __attribute__((always_inline)) {
        glds_b(min(kt + 2, nk - 1), (cur + 2) % 3);
        load_a(min(kt + 2, nk - 1), rb);
        mf_lo1(cur);
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(A_LD + B_INS) : "memory");  // A(kt+1), B(kt+1) landed
        launder_a(rb ^ 1);
        mf_rest(cur, rb ^ 1, (cur + 1) % 3);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
      };
      for (int kt = 0; kt < nk; kt += 6) {
        iter3(kt, 0, 0);
        if (kt + 1 < nk) iter3(kt + 1, 1, 1);
        if (kt + 2 < nk) iter3(kt + 2, 2, 0);
        if (kt + 3 < nk) iter3(kt + 3, 0, 1);
        if (kt + 4 < nk) iter3(kt + 4, 1, 0);
        if (kt + 5 < nk) iter3(kt + 5, 2, 1);
      }
    } else {
      RR_PH_DECL
      load_a(0, 0);
      glds_b(0, 0);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(B_INS) : "memory");  // A(0) landed
      launder_a(0);
      if constexpr (SP == 2) {
        // uniform: the exponent and both powers of two stay in scalar registers
        const int e = __builtin_amdgcn_readfirstlane(h2_exp(amax_reduce(a_amax_w)));
        a_sc = __int_as_float((127 + e) << 23);
        a_isc = __int_as_float((127 - e) << 23);
      }
      store_a(0, 0);
      load_a(nk > 1 ? 1 : 0, 1);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(A_LD) : "memory");  // B(0) landed
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      auto iter = [&](int kt, int cur) __attribute__((always_inline)) {
        if constexpr (!IL) {
          glds_b(min(kt + 1, nk - 1), cur ^ 1);
          load_a(min(kt + 2, nk - 1), cur);
        }
        if constexpr (MF16 && AMODE == A_DENSE && SP == 3) {
          mf_dense0(cur);
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(A_LD + B_INS) : "memory");
          launder_a(cur ^ 1);
          split_a(cur ^ 1);
          mf_dense1(cur);
          write_a(cur ^ 1);
        } else if constexpr (MF16) {
          RR_PH(0);
          mf_lo1(cur);
          RR_PH(1);
          // A(kt+1) landed (the B DMA of kt+1 and the A loads of kt+2 may not
          // have): split and stored among the remaining MFMAs of tile kt
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(A_LD + B_INS) : "memory");
          launder_a(cur ^ 1);
          RR_PH(2);
          mf_rest(cur, cur ^ 1, cur ^ 1);
          RR_PH(3);
        } else {
          compute_st(cur, 0, kt);
          // A(kt+1) landed: its split overlaps the remaining MFMAs of tile kt
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(A_LD + B_INS) : "memory");
          launder_a(cur ^ 1);
          split_a(cur ^ 1);
        }
        if constexpr (!MF16) {
  #pragma unroll
          for (int st = 1; st < BK / 16; ++st) compute_st(cur, st);
          write_a(cur ^ 1);
        }
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(A_LD) : "memory");  // B DMA of kt+1 landed
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        RR_PH(4);
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        RR_PH(5);
      };
      RR_PH(7);
      for (int kt = 0; kt < nk; kt += 2) {
        iter(kt, 0);
        if (kt + 1 < nk) iter(kt + 1, 1);
      }
      if constexpr (SP == 2 && MF16) RR_PH_FLUSH(0);
    }
    // the clamped tail loads are still in flight: keep both buffers live
    // until they have landed, so no later value is allocated to them
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    launder_a(0);
    launder_a(1);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  if constexpr (MF16) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int e = 0; e < 4; ++e) hi[i][j][4 * t + e] = ACC1 ? hi4[i][j][t][e] : hi4[i][j][t][e] + RR_LO(i, j, t)[e];
  } else {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        if constexpr (!ACC1) hi[i][j] += lo[i][j];
  }
  if constexpr (POOL) {
    // stage the raw 256 x 64 accumulator tile, then every pooled output of
    // the tile: the max over the window's in-map conv outputs of the raw
    // accumulators, then scale, bias, ReLU once (all monotone: the same bits
    // as pooling the stored conv outputs)
    constexpr int CS = BN + (MF16 ? 4 : 8);
    static_assert(BM * CS <= LDS_U16 / 2, "stem + max-pool: the C tile must fit the LDS");
    float* ct = reinterpret_cast<float*>(lds);
    {
      const int wm = wave % WM, wn = wave / WM;
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            ct[(wm * WTM + acc_row<(bool)MF16>(i, r, lane)) * CS + wn * WTN + acc_col<(bool)MF16>(j, r, lane)] =
                hi[i][j][r];
    }
    __syncthreads();
    const int tpi = g.pool_tr * g.pool_tc;
    const int b = tm / tpi, t2 = tm - b * tpi, pr = t2 / g.pool_tc, pc = t2 - pr * g.pool_tc;
    constexpr int C4 = BN / 4;
    float am = 0.f;
    for (int it = tid; it < 56 * C4; it += NT) {
      const int qd = it / C4, c4 = it - qd * C4, pi = qd / 7, pj = qd - 7 * pi;
      const int ph = 8 * pr + pi, pw = 7 * pc + pj;
      if (ph >= g.POH || pw >= g.POW) continue;
      f32x4 mx = {-__builtin_inff(), -__builtin_inff(), -__builtin_inff(), -__builtin_inff()};
#pragma unroll
      for (int dr = -1; dr <= 1; ++dr)
#pragma unroll
        for (int dc = -1; dc <= 1; ++dc) {
          const int oh = 2 * ph + dr, ow = 2 * pw + dc;
          if ((unsigned)oh >= (unsigned)g.OH || (unsigned)ow >= (unsigned)g.OW) continue;
          const f32x4 v = *reinterpret_cast<const f32x4*>(ct + ((2 * pi + dr + 1) * 15 + 2 * pj + dc + 1) * CS + c4 * 4);
#pragma unroll
          for (int e = 0; e < 4; ++e) mx[e] = __builtin_fmaxf(mx[e], v[e]);
        }
      const f32x4 sc = *reinterpret_cast<const f32x4*>(g.col_scale + c4 * 4) * a_isc;
      const f32x4 bv = g.bias != nullptr ? *reinterpret_cast<const f32x4*>(g.bias + c4 * 4) : f32x4{0.f, 0.f, 0.f, 0.f};
      f32x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        o[e] = __builtin_fmaxf(mx[e] * sc[e] + bv[e], 0.f);
        am = amax_acc(am, o[e]);
      }
      *reinterpret_cast<f32x4*>(g.pool_out + (((long long)b * g.POH + ph) * g.POW + pw) * BN + c4 * 4) = o;
    }
    if (g.c_amax != nullptr) amax_publish(g.c_amax, am, blockIdx.x * NW + wave);
  } else {
    epilogue_store<WM, WN, FM, FN, LDS_U16 / 2, (bool)MF16, EPI>(g, g.C, hi, reinterpret_cast<float*>(lds), m0, n0,
                                                                   a_isc);
  }
}

// ---- Persistent 128x256 tile (config 8) ------------------------------------
// The config-4 tile (8 waves of 64x64, BK 32, v_mfma_f32_16x16x32_bf16, dense
// A or the Cin % 32 == 0 conv A) as one block per CU that walks its tiles as
// ONE continuous k-stream: the B DMA runs one k-tile and the A loads two
// k-tiles ahead ACROSS tile boundaries, so while a tile's epilogue runs the
// next tile's first k-tile already sits in LDS and its second is in flight
// (a fresh block pays that round trip before its first MFMA), and the
// epilogue's stores drain under the next tile's first k-tiles.  The epilogue
// stages C through the stage buffer the tile's last k-tile just released (two
// 64-row slabs of 64 KB), with every bias / residual load issued before the
// staging.  Same per-accumulator k order and epilogue arithmetic as config 4:
// the results are bit-identical to it.
// (s3_opaque: per-thread address math built from it inside a tile loop's
// epilogue / loader switch cannot be hoisted out of the loop -- its results
// would then be live through the whole k-loop and spill it)

template <int EPI, int SP = 2, int SEG2 = 0>
__global__ __launch_bounds__(512, 1) void gemm_s3p_kernel(GemmArgs g, int tiles_n, int ntiles) {
  static_assert(SP == 2, "split kind: f16x2 (the bf16x3 instantiations were retired in ABI 6)");
  static_assert(SP == 3 || (EPI & EP_SCALE), "f16x2: scaled epilogue");
  typedef typename S3Frag<SP>::T frag_t;
  constexpr int NP = SP;
  constexpr int WM = 2, FM = 2, FN = 2, BK = 32, NT = 512, NW = 8;
  constexpr int WTM = 64, WTN = 64, BM = 128, BN = 256, SL = BK / 8;
  constexpr int A_EL = NP * BM * BK, BUF = A_EL + NP * BN * BK;
  // stage stride: a stage also stages one 64-row slab of C in the epilogue
  // (rows padded by 4 floats: the 16x16 accumulator writes hit distinct banks)
  constexpr int CS = BN + 4;
  constexpr int STG = BUF > 64 * CS * 2 ? BUF : 64 * CS * 2;
  constexpr int B_INS = NP * BN / (64 / SL) / NW;  // LDS-DMA instructions per wave per k-tile (6 / 4)
  constexpr int A_LD = 2;                          // A loads per thread per k-tile
  static_assert(B_INS * NW * (64 / SL) == NP * BN, "B staging must tile the block");
  __shared__ __attribute__((aligned(16))) uint16_t lds[2 * STG];
  uint32_t a_amax_w = 0;
  if constexpr (SP == 2) a_amax_w = amax_load_slot(g.a_amax);
  if constexpr (SEG2) {  // one split scale for both segments: the larger max
    const uint32_t w2 = amax_load_slot(g.a2_amax);
    a_amax_w = w2 > a_amax_w ? w2 : a_amax_w;
  }
  float a_sc = 1.f, a_isc = 1.f, am = 0.f;

  // round stagger: every block is resident from the start, so half of them
  // (every other XCD slot) start later and the halves stay out of phase
  if (g.stagger_sleeps > 0 && ((blockIdx.x >> 3) & 1))
    for (int i = 0; i < g.stagger_sleeps; ++i) __builtin_amdgcn_s_sleep(32);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const int G = gridDim.x, bid = blockIdx.x;
  const int nk = g.K / BK;
  const int my_tiles = (ntiles - bid + G - 1) / G;
  const int J = my_tiles * nk;  // k-tiles in this block's stream
  // local tile tl -> origin: virtual block v = bid + tl*G keeps this block's
  // XCD (G % 8 == 0 whenever a block owns more than one tile), then the same
  // bijective XCD remap as the one-tile-per-block kernel
  auto tile_origin = [&](int tl, int& m0, int& n0) {
    const int v = bid + tl * G;
    const int xcd = v & 7, q8 = ntiles >> 3, r8 = ntiles & 7;
    const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (v >> 3);
    const int tn = wgid % tiles_n, tm = wgid / tiles_n;
    m0 = tm * BM;
    n0 = tn * BN;
  };

  // ---- A loader (one 8-k chunk of one row per thread), two k-tiles ahead
  // of the MFMAs; load_a() issues the loader's k-tile and advances it one
  // k-tile along the stream (into the next tile after a tile's last).  Past
  // the stream's end the loaders run on into one virtual tile v >= ntiles,
  // which the remap sends to another block's tile or past M (A then reads
  // row M - 1; B's column tile is always a real one): every address stays
  // valid, nothing reads what they stage, and every iteration issues the same
  // loads, as the counted waits assume ----
  // rows past M load row M - 1 (only their own, unstored, output rows see it)
  const float* a_ptr = g.A;
  int a_kt = 0, a_tl = 0;
  auto a_tile = [&](int tl) {
    int m0, n0;
    tile_origin(tl, m0, n0);
    const int t = s3_opaque(tid);
    const int m = min(m0 + t / SL, g.M - 1);
    a_ptr = g.A + (long long)m * g.lda + (t % SL) * 8;
  };
  // SEG2: from k-tile K1 / BK on, the row's pointer moves to its sampled
  // pixel of A2 (minus K1, so a_ptr + a_kt * BK stays the element address)
  auto a_seg2 = [&](int tl) {
    int m0, n0;
    tile_origin(tl, m0, n0);
    const int t = s3_opaque(tid);
    const int m = min(m0 + t / SL, g.M - 1);
    const int ohw = g.OH * g.OW;
    const int b = m / ohw, r = m - b * ohw, oh = r / g.OW, ow = r - oh * g.OW;
    const long long pix = ((long long)b * g.H2 + (long long)oh * g.s2) * g.W2 + (long long)ow * g.s2;
    a_ptr = g.A2 + pix * g.lda2 + (t % SL) * 8 - g.K1;
  };
  a_tile(0);
  f32x4 ra2[2][2];
  auto load_a = [&](int rb) {
    s3_load2<1>(reinterpret_cast<const f32x4*>(a_ptr + a_kt * BK), ra2[rb]);
    if (++a_kt == nk) {
      a_kt = 0;
      a_tile(++a_tl);
    } else if (SEG2 && a_kt * BK == g.K1) {
      a_seg2(a_tl);
    }
  };
  u32x4 pk[NP];
  auto split_a = [&](int rb) {
    if constexpr (SP == 2) {
      split2h8(ra2[rb], a_sc, pk[0], pk[1]);
      return;
    }
    uint32_t h[8], m[8], l[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float x = ra2[rb][e >> 2][e & 3];
      const float r1 = x - __uint_as_float(__float_as_uint(x) & 0xffff0000u);
      const float r2 = r1 - __uint_as_float(__float_as_uint(r1) & 0xffff0000u);
      h[e] = __float_as_uint(x);
      m[e] = __float_as_uint(r1);
      l[e] = __float_as_uint(r2);
    }
    pk[0] = u32x4{pack2(h[0], h[1]), pack2(h[2], h[3]), pack2(h[4], h[5]), pack2(h[6], h[7])};
    pk[1] = u32x4{pack2(m[0], m[1]), pack2(m[2], m[3]), pack2(m[4], m[5]), pack2(m[6], m[7])};
    pk[NP - 1] = u32x4{pack2(l[0], l[1]), pack2(l[2], l[3]), pack2(l[4], l[5]), pack2(l[6], l[7])};
  };
  auto write_a = [&](int buf) {
    uint16_t* la = lds + buf * STG;
    const int a_slot = tid % SL, a_row = tid / SL;
    const int off = a_row * BK + pswz<BK, SP>(a_row, a_slot) * 8;
#pragma unroll
    for (int p = 0; p < NP; ++p) *reinterpret_cast<u32x4*>(la + p * BM * BK + off) = pk[p];
  };
  auto launder_a = [&](int rb) {
    s3_launder(ra2[rb][0]);
    s3_launder(ra2[rb][1]);
  };

  // ---- B loader: instruction i of a wave DMAs plane i/2, plane rows
  // 128 (i&1) + 16 wave + lane/4 (N % 256 == 0: no row past N) ----
  const uint16_t* Bp = reinterpret_cast<const uint16_t*>(g.B);
  const int b_r = wave * (64 / SL) + lane / SL;
  const int b_sw = pswz<BK, SP>(b_r, lane % SL) * 8;  // the same for every i
  const uint16_t* b_src = Bp;
  int b_kt = 0, b_tl = 0;
  auto b_tile = [&](int tl) {
    int m0, n0;
    tile_origin(tl, m0, n0);
    b_src = Bp + (long long)(n0 + b_r) * g.ldb + b_sw;
  };
  b_tile(0);
  auto glds_b = [&](int buf) {
    uint16_t* lb = lds + buf * STG + A_EL;
#pragma unroll
    for (int i = 0; i < B_INS; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(b_src + (i >> 1) * g.b_plane + (long long)(i & 1) * (BN / 2) * g.ldb +
                                                     b_kt * BK),
                                       (__attribute__((address_space(3))) void*)(lb + (i * NW + wave) * (64 / SL) * BK),
                                       16, 0, 0);
    if (++b_kt == nk) {
      b_kt = 0;
      b_tile(++b_tl);
    }
  };

  // ---- MFMAs: four 16x16x32 sub-tiles per 32x32 tile, as config 4 ----
  f32x4 hi4[FM][FN][4], lo4[FM][FN][4];
  auto zero_acc = [&]() {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          hi4[i][j][t] = f32x4{0.f, 0.f, 0.f, 0.f};
          lo4[i][j][t] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
  };
  zero_acc();
  frag_t fa[NP][FM][2], fb[NP][FN][2];
  const int l16 = lane & 15, lg = lane >> 4;
  auto rd_mf = [&](int cur, int p) {
    const uint16_t* la = lds + cur * STG;
    const uint16_t* lb = la + A_EL;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int row = wm * WTM + i * 32 + h * 16 + l16;
        fa[p][i][h] = *reinterpret_cast<const frag_t*>(la + (p * BM + row) * BK + pswz<BK, SP>(row, lg) * 8);
      }
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int row = wn * WTN + j * 32 + h * 16 + l16;
        fb[p][j][h] = *reinterpret_cast<const frag_t*>(lb + (p * BN + row) * BK + pswz<BK, SP>(row, lg) * 8);
      }
  };
#define RR_MF16(a, b, c) c = s3_mf16<SP>(a, b, c)
  auto mf_hi = [&]() {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int t = 0; t < 4; ++t) RR_MF16(fa[0][i][t >> 1], fb[0][j][t & 1], hi4[i][j][t]);
  };
  auto mf_lo1 = [&]() {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          if constexpr (SP == 3) RR_MF16(fa[1][i][t >> 1], fb[1][j][t & 1], lo4[i][j][t]);
          RR_MF16(fa[0][i][t >> 1], fb[1][j][t & 1], lo4[i][j][t]);
          RR_MF16(fa[1][i][t >> 1], fb[0][j][t & 1], lo4[i][j][t]);
        }
  };
  auto mf_lo2 = [&]() {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          RR_MF16(fa[0][i][t >> 1], fb[NP - 1][j][t & 1], lo4[i][j][t]);
          RR_MF16(fa[NP - 1][i][t >> 1], fb[0][j][t & 1], lo4[i][j][t]);
        }
  };
#undef RR_MF16

  // ---- epilogue of local tile tl through stage buffer `buf` (free) ----
  // Two slabs by MFMA row tile i: slab s = rows 64 wm + 32 s + [0, 32) of every
  // wave, so staging slab 0 frees half of every wave's accumulators before
  // slab 1's residual is loaded (both slabs' residuals in registers at once
  // beside all accumulators spilled the k-loop).  Residual rows are loaded by
  // inline asm (rows past M clamped to M - 1; never stored), so one explicit
  // vmcnt(0) covers both slabs: slab 1's loads fly while slab 0 is staged.
  constexpr int C4 = BN / 4, HITERS = 32 * C4 / NT;  // 4 row chunks per thread and 32-row band
  auto epilogue = [&](int tl, int buf) {
    // the two accumulator tiles summed first (128 registers -> 64)
    f32x16 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[i][j][4 * t + e] = hi4[i][j][t][e] + lo4[i][j][t][e];
    int m0, n0;
    tile_origin(tl, m0, n0);
    const int te = s3_opaque(tid);
    const int c40 = te % C4, r0 = te / C4;
    f32x4 bias_v[1] = {f32x4{0.f, 0.f, 0.f, 0.f}}, sc_v[1];
    // the bias / column scales load after slab 0's residual rows go out and
    // are waited for (redefined by an empty asm) only after slab 0 is staged:
    // waited for up front, as before, they cost a full memory round trip (a
    // vmcnt(0), the next tile's prefetch included) ahead of the residual loads
    auto load_bias = [&]() {
      if ((EPI & EP_BIAS) && g.bias != nullptr) bias_v[0] = *reinterpret_cast<const f32x4*>(g.bias + n0 + c40 * 4);
      if constexpr ((EPI & EP_SCALE) != 0) sc_v[0] = *reinterpret_cast<const f32x4*>(g.col_scale + n0 + c40 * 4);
    };
    auto launder_bias = [&]() {
      asm volatile("" : "+v"(bias_v[0]));
      if constexpr ((EPI & EP_SCALE) != 0) {
        asm volatile("" : "+v"(sc_v[0]));
        sc_v[0] *= a_isc;
      }
    };
    f32x4 res[2][2][HITERS];  // [slab][band][row chunk]
    auto load_res = [&](int sl) {
      if constexpr ((EPI & EP_RES) != 0) {
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
          for (int it = 0; it < HITERS; ++it) {
            const int m = min(m0 + q * 64 + sl * 32 + r0 + it * (NT / C4), g.M - 1);
            const float* p = g.residual + (long long)m * g.ldc + n0 + c40 * 4;
            if constexpr ((EPI & EP_SC1) != 0)  // streamed (EP_SC1): nt
              asm volatile("global_load_dwordx4 %0, %1, off nt" : "=&v"(res[sl][q][it]) : "v"(p) : "memory");
            else
              asm volatile("global_load_dwordx4 %0, %1, off" : "=&v"(res[sl][q][it]) : "v"(p) : "memory");
          }
      }
    };
    float* ct = reinterpret_cast<float*>(lds + buf * STG);  // [2 bands x 32 rows][CS]
    const int le = te & 63;
    auto stage = [&](int sl) {
      float* cw = ct + (wm * 32) * CS + wn * WTN;
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) cw[acc_row<true>(0, r, le) * CS + acc_col<true>(j, r, le)] = acc[sl][j][r];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    };
    auto store = [&](int sl) {
      if constexpr ((EPI & EP_RES) != 0) {
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
          for (int it = 0; it < HITERS; ++it) asm volatile("" : "+v"(res[sl][q][it]));
      }
#pragma unroll
      for (int q = 0; q < 2; ++q)
        store_slab<EPI, 2, HITERS, NT, C4, CS, 1>(g, g.C, ct + q * 32 * CS, bias_v, res[sl][q], te,
                                                  m0 + q * 64 + sl * 32, n0, sc_v, am);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // every LDS read of the slab done
      asm volatile("" ::: "memory");
    };
    load_res(0);
    load_bias();
    stage(0);
    load_res(1);
    // every load issued so far has landed, the next tile's A(j+1) included:
    // the next iteration's skipped A wait (wait_a) relies on this explicit
    // wait, not on the one hipcc places for the plain bias / scale loads
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    launder_bias();
    store(0);
    stage(1);
    store(1);  // its barrier also frees `buf` for the next k-tiles
    zero_acc();  // here, not at the sum: 128 registers of zeros held through the stores spilled
  };

  // ---- the stream: k-tile j of the block = k-tile j % nk of local tile j / nk ----
  load_a(0);
  glds_b(0);
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(B_INS) : "memory");  // A(0) landed
  launder_a(0);
  if constexpr (SP == 2) {
    // uniform: the exponent and both powers of two stay in scalar registers
    const int e = __builtin_amdgcn_readfirstlane(h2_exp(amax_reduce(a_amax_w)));
    a_sc = __int_as_float((127 + e) << 23);
    a_isc = __int_as_float((127 - e) << 23);
  }
  split_a(0);
  write_a(0);
  load_a(1);
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(A_LD) : "memory");  // B(0) landed
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  int c_kt = 0, c_tl = 0;
  RR_PH_DECL
  // iteration j (stage cur = j & 1 holds k-tile j, register buffer cur ^ 1
  // holds A(j+1)): B DMA of j+1, A loads of j+2, the k-tile's MFMAs with the
  // split of A(j+1) among them (the dense-A order of config 4), then — after
  // the last k-tile of a tile — its epilogue through stage cur.  The
  // epilogue's stores are issued after A(j+2) and before the next loads: the
  // next A wait (vmcnt(A_LD + B_INS)) counts only loads after it, so it is
  // exact if the stores retire in order and waits longer (never shorter) if
  // they do not.
  auto iter = [&](int cur) __attribute__((always_inline)) {
    glds_b(cur ^ 1);
    load_a(cur);
    RR_PH(0);
    rd_mf(cur, 0);
    rd_mf(cur, 1);
    // (a tile's first k-tile skips the A wait: its A(j+1) was issued before
    // the previous epilogue, whose waits -- the residual's vmcnt(0), or the
    // bias / scale loads' -- covered it; waiting here would wait for that
    // epilogue's stores as well)
    const bool wait_a = c_kt != 0 || c_tl == 0;
    if constexpr (SP == 3) {
      mf_hi();
      mf_lo1();
      if (wait_a) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(A_LD + B_INS) : "memory");  // A(j+1) landed
      launder_a(cur ^ 1);
      split_a(cur ^ 1);
      rd_mf(cur, NP - 1);
      mf_lo2();
    } else {
      // f16x2: the plane-1 products, then a0b0 with the split of A(j+1) two
      // VALU per MFMA gap (same per-accumulator order as config 4)
      mf_lo1();
      RR_PH(1);
      if (wait_a) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(A_LD + B_INS) : "memory");  // A(j+1) landed
      launder_a(cur ^ 1);
      RR_PH(2);
      split_a(cur ^ 1);
      mf_hi();
#pragma unroll
      for (int x = 0; x < FM * FN * 4; ++x) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // 1 MFMA
        __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);  // 2 VALU
      }
    }
    write_a(cur ^ 1);
    RR_PH(3);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(A_LD) : "memory");  // B DMA of j+1 landed
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    RR_PH(4);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    RR_PH(5);
    if (++c_kt == nk) {
      c_kt = 0;
      epilogue(c_tl++, cur);
      RR_PH(6);
    }
  };
  RR_PH(7);
  for (int j = 0; j < J; j += 2) {
    iter(0);
    if (j + 1 < J) iter(1);
  }
  // the clamped tail loads are still in flight: keep both buffers live until
  // they have landed, so no later value is allocated to them
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  launder_a(0);
  launder_a(1);
  if constexpr ((EPI & EP_AMAX) != 0) {
    if (g.c_amax != nullptr) amax_publish(g.c_amax, am, bid * NW + wave);
  }
  if constexpr (SP == 2) RR_PH_FLUSH(1);
}

template <int EPI, int SP = 2, int SEG2 = 0>
static hipError_t launch_s3p_t(GemmArgs g, hipStream_t s, int n_cu, int stagger) {
  const long long tiles_m = (g.M + 127) / 128, tiles_n = g.N / 256;
  const long long ntiles = tiles_m * tiles_n;
  if (ntiles <= 0) return hipSuccess;
  if (ntiles * (g.K / 32) > 0x7fffffffLL) return hipErrorInvalidValue;
  // one block per CU; a block that owns several tiles must stay on its XCD
  // (grid a multiple of 8)
  const int slots = std::max(8, n_cu & ~7);
  const int grid = ntiles <= slots ? (int)ntiles : slots;
  g.stagger_blocks = grid;
  g.stagger_sleeps = ntiles > 2LL * grid ? stagger : 0;
  hipLaunchKernelGGL((gemm_s3p_kernel<EPI, SP, SEG2>), dim3((unsigned)grid), dim3(512), 0, s, g, (int)tiles_n,
                     (int)ntiles);
  return hipGetLastError();
}

// ---- Persistent 256x256 one-accumulator tile (config 15, f16x2) -----------
// Config 12 (8 waves of 128x64 on v_mfma_f32_32x32x16_f16, one accumulator
// set, BK 32, dense A) as one block per CU walking its tiles as ONE k-stream,
// as config 8 does for config 4: the B DMA one k-tile and the A loads two
// k-tiles ahead across tile boundaries, so a tile's epilogue runs with the
// next tile's first k-tile in LDS and its second in flight, and a fresh tile
// never pays the cold prologue of a new block.  The epilogue goes in four
// 64-row slabs (slab s = MFMA row tile s of every wave: rows 32 s + [0, 32)
// and 128 + 32 s + [0, 32), so all eight waves stage every slab) through the
// stage buffer the tile's last k-tile released, and slab s + 1's residual rows
// are in flight while slab s is staged and stored: one exposed residual round
// trip per tile instead of config 12's two (its two 128-row slabs each load
// their residual after staging, and only half the waves stage each slab).
// Same per-accumulator k order (per 16-deep k-step: a0b0, a0b1, a1b0) and
// epilogue arithmetic as config 12: bit-identical to it.  FN = 1: the 256x128
// form (waves of 128x32, two B DMA instructions per wave, 96 KB of LDS) for
// N = 128; FN = 1, WM = 4: the 256x64 form (waves 4 x 2 of 64x32, one B DMA
// instruction per wave spanning both planes, slabs of four 32-row bands, 80
// KB) for N = 64, with config 7's two accumulator sets (ACC2: its arithmetic
// at K = 64, where one accumulator's error passes the exact-fp32 core's).
// Every column of the 256x128 form is config 12's column bit for bit, the
// 256x64 form's output config 7's.
// Counted waits rely only on loads returning in issue order among
// themselves: each names how many younger loads may remain, and stores are
// never counted (a wait issued after stores also covers them, which makes it
// longer, never shorter); where fewer loads were issued (rows past M) the
// wait is longer, never shorter.
template <int EPI, int FN = 2, int WM = 2, int ACC2 = 0>
__global__ __launch_bounds__(512, 1) void gemm_s3q_kernel(GemmArgs g, int tiles_n, int ntiles) {
  static_assert((EPI & EP_SCALE) != 0, "f16x2: scaled epilogue");
  static_assert((WM == 2 && (FN == 1 || FN == 2)) || (WM == 4 && FN == 1), "256x256, 256x128 or 256x64");
  typedef f16x8 frag_t;
  constexpr int NP = 2, FM = 8 / WM, BK = 32, NT = 512, NW = 8, WN = NW / WM;
  constexpr int WTM = 32 * FM, WTN = 32 * FN, BM = 256, BN = WN * WTN, SL = BK / 8;
  constexpr int A_EL = NP * BM * BK, BUF = A_EL + NP * BN * BK;
  // stage stride: a stage also holds one 64-row slab of C (rows padded by 8
  // floats: the 32x32 accumulator writes hit distinct banks)
  constexpr int CS = BN + 8;
  constexpr int STG = BUF > WM * 32 * CS * 2 ? BUF : WM * 32 * CS * 2;
  constexpr int B_INS = NP * BN / (64 / SL) / NW;  // LDS-DMA instructions per wave per k-tile (4 / 2)
  constexpr int IPP = BN >= 128 ? BN / 128 : 1;     // of them per plane (64 columns: one spans both)
  constexpr int A_RPP = NT / SL, A_CH = BM / A_RPP;  // 128 rows per pass, 2 chunks per thread
  constexpr int A_LD = 2 * A_CH;                     // A loads per thread per k-tile
  static_assert(B_INS * NW * (64 / SL) == NP * BN && A_CH * A_RPP == BM, "staging must tile the block");
  __shared__ __attribute__((aligned(16))) uint16_t lds[2 * STG];
  const uint32_t a_amax_w = amax_load_slot(g.a_amax);
  float a_sc = 1.f, a_isc = 1.f, am = 0.f;

  // round stagger: every block is resident from the start, so half of them
  // (every other XCD slot) start later and the halves stay out of phase
  if (g.stagger_sleeps > 0 && ((blockIdx.x >> 3) & 1))
    for (int i = 0; i < g.stagger_sleeps; ++i) __builtin_amdgcn_s_sleep(32);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const int lr = lane & 31, lh = lane >> 5;
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);  // (scalar: the amax slot at the end)
  const int G = gridDim.x, bid = blockIdx.x;
  const int nk = g.K / BK;
  const int my_tiles = (ntiles - bid + G - 1) / G;
  const int J = my_tiles * nk;  // k-tiles in this block's stream
  // local tile tl -> origin (as config 8: virtual block bid + tl G keeps the
  // block's XCD, then the bijective XCD remap)
  auto tile_origin = [&](int tl, int& m0, int& n0) __attribute__((always_inline)) {
    const int v = bid + tl * G;
    const int xcd = v & 7, q8 = ntiles >> 3, r8 = ntiles & 7;
    const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (v >> 3);
    const int tn = wgid % tiles_n, tm = wgid / tiles_n;
    m0 = tm * BM;
    n0 = tn * BN;
  };

  // ---- A loader: two 8-k chunks per thread (rows t / 4 and 128 + t / 4),
  // two k-tiles ahead of the MFMAs, advancing along the stream; past the
  // stream's end it runs into a virtual tile whose rows clamp to M - 1 ----
  // (32-bit byte offsets from the uniform base, saddr form: 64-bit row
  // pointers spilled this kernel; the host keeps A and C below 4 GB)
  uint32_t a_off[A_CH];
  int a_kt = 0, a_tl = 0;
  auto a_tile = [&](int tl) __attribute__((always_inline)) {
    int m0, n0;
    tile_origin(tl, m0, n0);
    const int t = s3_opaque(tid);
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const int m = min(m0 + t / SL + i * A_RPP, g.M - 1);
      a_off[i] = ((uint32_t)m * (uint32_t)g.lda + (uint32_t)(t % SL) * 8u) * 4u;
    }
  };
  a_tile(0);
  f32x4 ra2[2][A_CH][2];
  auto load_a = [&](int rb) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < A_CH; ++i)
      asm volatile("global_load_dwordx4 %0, %2, %3\n\tglobal_load_dwordx4 %1, %2, %3 offset:16"
                   : "=&v"(ra2[rb][i][0]), "=&v"(ra2[rb][i][1])
                   : "v"(a_off[i] + (uint32_t)(a_kt * BK * 4)), "s"(g.A)
                   : "memory");
    if (++a_kt == nk) {
      a_kt = 0;
      a_tile(++a_tl);
    }
  };
  u32x4 pk[A_CH][NP];
  auto split_a = [&](int rb) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < A_CH; ++i) split2h8(ra2[rb][i], a_sc, pk[i][0], pk[i][1]);
  };
  auto write_a = [&](int buf) __attribute__((always_inline)) {
    uint16_t* la = lds + buf * STG;
    const int a_slot = tid % SL, a_row = tid / SL;
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const int row = a_row + i * A_RPP;
      const int off = row * BK + pswz<BK, 2>(row, a_slot) * 8;
#pragma unroll
      for (int p = 0; p < NP; ++p) *reinterpret_cast<u32x4*>(la + p * BM * BK + off) = pk[i][p];
    }
  };
  auto launder_a = [&](int rb) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      s3_launder(ra2[rb][i][0]);
      s3_launder(ra2[rb][i][1]);
    }
  };

  // ---- B loader (as config 8): instruction i of a wave DMAs plane i / IPP,
  // plane rows 128 (i % IPP) + 16 wave + lane / 4 ----
  const uint16_t* Bp = reinterpret_cast<const uint16_t*>(g.B);
  const int b_r = wave * (64 / SL) + lane / SL;
  const int b_sw = pswz<BK, 2>(b_r, lane % SL) * 8;  // the same for every i
  const uint16_t* b_src = Bp;
  int b_kt = 0, b_tl = 0;
  auto b_tile = [&](int tl) __attribute__((always_inline)) {
    int m0, n0;
    tile_origin(tl, m0, n0);
    b_src = Bp + (long long)(b_r / BN) * g.b_plane + (long long)(n0 + b_r % BN) * g.ldb + b_sw;
  };
  b_tile(0);
  auto glds_b = [&](int buf) __attribute__((always_inline)) {
    uint16_t* lb = lds + buf * STG + A_EL;
#pragma unroll
    for (int i = 0; i < B_INS; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(b_src + (i / IPP) * g.b_plane + (long long)(i % IPP) * 128 * g.ldb +
                                                     b_kt * BK),
                                       (__attribute__((address_space(3))) void*)(lb + (i * NW + wave) * (64 / SL) * BK),
                                       16, 0, 0);
    if (++b_kt == nk) {
      b_kt = 0;
      b_tile(++b_tl);
    }
  };

  // ---- MFMAs: config 12's 16-deep k-step (st = 0, 1 of the k-tile) ----
  // ACC2: config 7's two accumulator sets (a0b0 in acc, a0b1 + a1b0 in lo,
  // summed before the epilogue)
  f32x16 acc[FM][FN], lo[ACC2 ? FM : 1][ACC2 ? FN : 1];
  auto zero_acc = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          acc[i][j][r] = 0.f;
          if constexpr (ACC2) lo[i][j][r] = 0.f;
        }
  };
  zero_acc();
  auto compute_st = [&](int cur, int st) __attribute__((always_inline)) {
    const uint16_t* la = lds + cur * STG;
    const uint16_t* lb = la + A_EL;
    frag_t a[NP][FM], b[NP][FN];
#pragma unroll
    for (int p = 0; p < NP; ++p) {
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int row = wm * WTM + i * 32 + lr;
        a[p][i] = *reinterpret_cast<const frag_t*>(la + (p * BM + row) * BK + pswz<BK, 2>(row, 2 * st + lh) * 8);
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int row = wn * WTN + j * 32 + lr;
        b[p][j] = *reinterpret_cast<const frag_t*>(lb + (p * BN + row) * BK + pswz<BK, 2>(row, 2 * st + lh) * 8);
      }
    }
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = s3_mf32<2>(a[0][i], b[0][j], acc[i][j]);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        f32x16& L = ACC2 ? lo[ACC2 ? i : 0][ACC2 ? j : 0] : acc[i][j];
        L = s3_mf32<2>(a[0][i], b[1][j], L);
        L = s3_mf32<2>(a[1][i], b[0][j], L);
      }
  };

  // ---- epilogue of local tile tl through stage buffer `buf` (free) ----
  // Eight 32-row bands, band b = rows 128 (b & 1) + 32 (b >> 1) + [0, 32);
  // bands 2s and 2s + 1 form slab s (MFMA row tile s of every wave), staged
  // together.  Band b's residual rows are loaded two bands ahead (issued
  // before band b - 2 is stored): at most three bands (48 registers) in
  // flight -- a whole slab ahead (64) spilled the k-loop.
  constexpr int C4 = BN / 4, HITERS = 32 * C4 / NT;  // 4 / 2 / 1 row chunks per thread and band
  static_assert(HITERS * 2 <= 16 && (HITERS == 1 || HITERS % 2 == 0), "the counted waits' immediates");
  constexpr int NB = WM * FM, RD = 2;                  // bands, residual look-ahead (bands)
  RR_PH_DECL
  auto epilogue = [&](int tl, int buf) __attribute__((always_inline)) {
    int m0, n0;
    tile_origin(tl, m0, n0);
    const int te = s3_opaque(tid);
    const int c40 = te % C4;
    f32x4 bias_v[1] = {f32x4{0.f, 0.f, 0.f, 0.f}}, sc_v[1];
    f32x4 res[RD + 1][HITERS];  // ring of bands
    auto band_row0 = [&](int bb) { return (bb % WM) * WTM + (bb / WM) * 32; };
    auto load_band = [&](int bb) __attribute__((always_inline)) {
      if constexpr ((EPI & EP_RES) != 0) {
        // (addresses from an opaque thread index per band: hoisted, every
        // band's addresses would be live through the epilogue and spill)
        const int tq = s3_opaque(tid);
        const int cq = tq % C4, rq = tq / C4;
#pragma unroll
        for (int it = 0; it < HITERS; ++it) {
          const int m = min(m0 + band_row0(bb) + rq + it * (NT / C4), g.M - 1);
          const uint32_t o = ((uint32_t)m * (uint32_t)g.ldc + (uint32_t)(n0 + cq * 4)) * 4u;
          if constexpr ((EPI & EP_SC1) != 0)  // streamed: nt
            asm volatile("global_load_dwordx4 %0, %1, %2 nt" : "=&v"(res[bb % (RD + 1)][it]) : "v"(o), "s"(g.residual) : "memory");
          else
            asm volatile("global_load_dwordx4 %0, %1, %2" : "=&v"(res[bb % (RD + 1)][it]) : "v"(o), "s"(g.residual) : "memory");
        }
      }
    };
    float* ct = reinterpret_cast<float*>(lds + buf * STG);  // [2 bands x 32 rows][CS]
    // (wave and lane from the opaque index too: the staging addresses are
    // loop-invariant and would otherwise be held through the k-loop)
    const int le = te & 63, we = te >> 6;
    auto stage = [&](int sl) __attribute__((always_inline)) {
      float* cw = ct + ((we % WM) * 32) * CS + (we / WM) * WTN;
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          cw[acc_row<false>(0, r, le) * CS + acc_col<false>(j, r, le)] =
              ACC2 ? acc[sl][j][r] + lo[ACC2 ? sl : 0][ACC2 ? j : 0][r] : acc[sl][j][r];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      RR_PH(4);
    };
    // the bias / column scales first, by inline asm as well (a plain load's
    // use would make hipcc wait vmcnt(0), the look-ahead bands included):
    // older than every band, so band 0's wait covers them
    if ((EPI & EP_BIAS) && g.bias != nullptr)
      asm volatile("global_load_dwordx4 %0, %1, off" : "=&v"(bias_v[0]) : "v"(g.bias + n0 + c40 * 4) : "memory");
    asm volatile("global_load_dwordx4 %0, %1, off" : "=&v"(sc_v[0]) : "v"(g.col_scale + n0 + c40 * 4) : "memory");
    load_band(0);
    load_band(1);
    // band bb's wait: vmcnt(the loads issued after it: bands bb + 1 ..
    // bb + RD, HITERS each).  The stores issued after it (bands bb - RD ..
    // bb - 1) are not counted: loads return in order among themselves, but
    // nothing is assumed about stores against loads, so the wait also covers
    // those stores (measured free: 0.584 vs 0.590 ms counting them,
    // profiles/r05j_probe.txt)
#pragma unroll
    for (int bb = 0; bb < NB; ++bb) {
      if (bb % WM == 0) stage(bb / WM);
      if (bb + RD < NB) load_band(bb + RD);
      if constexpr ((EPI & EP_RES) != 0) {
        const int ahead = (NB - 1 - bb < RD ? NB - 1 - bb : RD);
        const int younger = HITERS * ahead;
        // (s_waitcnt needs an immediate: the few values this unrolled loop produces)
        switch (younger) {
#define RR_VMW(n) \
  case n: asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory"); break;
          RR_VMW(0) RR_VMW(1) RR_VMW(2) RR_VMW(3) RR_VMW(4) RR_VMW(6) RR_VMW(8) RR_VMW(10) RR_VMW(12) RR_VMW(14)
#undef RR_VMW
          default: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
        }
#pragma unroll
        for (int it = 0; it < HITERS; ++it) asm volatile("" : "+v"(res[bb % (RD + 1)][it]));
      } else if (bb == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      RR_PH(5);
      if (bb == 0) {
        asm volatile("" : "+v"(bias_v[0]));
        asm volatile("" : "+v"(sc_v[0]));
        sc_v[0] *= a_isc;
      }
      store_slab<EPI, 2, HITERS, NT, C4, CS, 1>(g, g.C, ct + (bb % WM) * 32 * CS, bias_v, res[bb % (RD + 1)], te,
                                                m0 + band_row0(bb), n0, sc_v, am);
      if (bb % WM == WM - 1) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();  // every LDS read of the slab done (the last also frees `buf`)
        asm volatile("" ::: "memory");
      }
      RR_PH(6);
    }
    zero_acc();
  };

  // ---- the stream: k-tile j of the block = k-tile j % nk of local tile j / nk ----
  load_a(0);
  glds_b(0);
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(B_INS) : "memory");  // A(0) landed
  launder_a(0);
  {
    // uniform: the exponent and both powers of two stay in scalar registers
    const int e = __builtin_amdgcn_readfirstlane(h2_exp(amax_reduce(a_amax_w)));
    a_sc = __int_as_float((127 + e) << 23);
    a_isc = __int_as_float((127 - e) << 23);
  }
  split_a(0);
  write_a(0);
  load_a(1);
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(A_LD) : "memory");  // B(0) landed
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  int c_kt = 0, c_tl = 0;
  // iteration j (stage cur = j & 1 holds k-tile j, register buffer cur ^ 1
  // holds A(j+1)): B DMA of j+1, A loads of j+2, the first k-step, the split
  // of A(j+1) under the second, then -- after a tile's last k-tile -- its
  // epilogue through stage cur.  A(j+1) of a tile's first k-tile was issued
  // before the previous epilogue, whose waits already covered it: that
  // iteration skips the A wait (it would wait for the epilogue's stores).
  auto iter = [&](int cur, int j) __attribute__((always_inline)) {
    glds_b(cur ^ 1);
    load_a(cur);
    compute_st(cur, 0);
    RR_PH(0);
    if (c_kt != 0 || c_tl == 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(A_LD + B_INS) : "memory");  // A(j+1) landed
    launder_a(cur ^ 1);
    RR_PH(1);
    split_a(cur ^ 1);
    compute_st(cur, 1);
    write_a(cur ^ 1);
    RR_PH(2);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(A_LD) : "memory");  // B DMA of j+1 landed
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    RR_PH(3);
    if (++c_kt == nk) {
      c_kt = 0;
      epilogue(c_tl++, cur);
    }
    // the stream's last k-tile: the clamped tail loads (into buffer cur) are
    // still in flight; that buffer stays live until they have landed, so no
    // later value is allocated to it (laundering both buffers after the loop
    // instead kept 32 registers live through every epilogue and spilled)
    if (j == J - 1) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      launder_a(cur);
    }
  };
  RR_PH(7);
  for (int j = 0; j < J; j += 2) {
    iter(0, j);
    if (j + 1 < J) iter(1, j + 1);
  }
  RR_PH_FLUSH(2);
  if constexpr ((EPI & EP_AMAX) != 0) {
    if (g.c_amax != nullptr) amax_publish(g.c_amax, am, bid * NW + wave_u);
  }
}

// config 15 addresses A and the residual by 32-bit byte offsets
static bool s3q_fits(const GemmArgs& g) {
  const long long lim = 1LL << 32;
  return (long long)g.M * g.lda * 4 < lim && (long long)g.M * g.ldc * 4 < lim;
}

template <int EPI, int FN = 2, int WM = 2, int ACC2 = 0>
static hipError_t launch_s3q_t(GemmArgs g, hipStream_t s, int n_cu, int stagger) {
  const long long tiles_m = (g.M + 255) / 256, tiles_n = g.N / (32 * FN * (8 / WM));
  const long long ntiles = tiles_m * tiles_n;
  if (ntiles <= 0) return hipSuccess;
  if (ntiles * (g.K / 32) > 0x7fffffffLL) return hipErrorInvalidValue;
  // 32-bit byte offsets (checked by the caller, s3q_fits)
  const int slots = std::max(8, n_cu & ~7);
  const int grid = ntiles <= slots ? (int)ntiles : slots;
  g.stagger_blocks = grid;
  g.stagger_sleeps = ntiles > 2LL * grid ? stagger : 0;
  hipLaunchKernelGGL((gemm_s3q_kernel<EPI, FN, WM, ACC2>), dim3((unsigned)grid), dim3(512), 0, s, g, (int)tiles_n, (int)ntiles);
  return hipGetLastError();
}

// f16x2 epilogue flag sets: the scale, the max-|C| record (skipped at run
// time when c_amax is NULL) and the bias (zeros when NULL) always compiled
// in; residual and ReLU select the instance
constexpr int H2_EP = EP_SCALE | EP_AMAX | EP_BIAS;

// ---- Halo-staged A for stride-1 3x3 convolutions (config 13, f16x2) -------
// The implicit-GEMM A loader of gemm_s3_kernel fetches every input pixel once
// per filter tap: nine fetches of each activation on a 3x3 conv.  Every tile
// here on this chip is bound by the bytes each CU fetches per MFMA cycle
// (the per-CU fill rate), and on the 3x3 256@14 layer the A operand
// is half of them: per output, 4 K / Nt B of A plus 4 K / Mt B of B planes =
// 36 + 36 B at the 256x256 tile.  Here a 256-row tile (256 consecutive output
// pixels in NHWC raster order) loads, per 32-channel slice of Cin, the raster
// range of input pixels its nine taps can touch — 256 + 2 (W + 1) rows, one
// fetch each — splits it once into the two fp16 planes of an LDS halo buffer,
// and runs the slice's nine k-tiles (one per tap) on it: output row r reads
// halo row r + kh W + kw, or a zero row when the tap falls outside its image
// (padding) or r is past M.  A fetch per output drops to (256 + 2W + 2) / 256
// x 4 Cin / Nt (4.5 B at 256@14), the split VALU to one per slice instead of
// one per k-tile.  k order: slice-major, tap-minor (k-tile (c, t) = weight
// columns t Cin + 32 c ..); B planes by LDS-DMA one k-tile ahead as config 12;
// 256x256 tile, 8 waves of 128x64 on v_mfma_f32_32x32x16_f16, one accumulator
// set (ACC1, config 12's arithmetic per product); the next slice's halo goes
// to the other buffer one 128-row pass per k-tile during the slice's first
// four.  Instances (waves WM x WN of FM x FN 32x32 tiles, halo rows HR):
//   <2, 4, 4, 2, 288>  256x256, N % 256 == 0, W <= 15 (the 14x14 / 7x7 layers)
//   <4, 2, 2, 2, 320>  256x128, N % 128 == 0, W <= 31 (28x28, N = 128)
//   <4, 2, 2, 1, 384>  256x64,  N % 64 == 0,  W <= 63 (56x56, N = 64), three
//                      taps per k-step (and barrier): its 12 MFMAs per wave
//                      and tap are too few to carry a barrier each
// Row HR of each halo plane is the zero row.
// Halo rows are read 32 at a time from any row offset r0 + kh W + kw, not from
// 32-aligned groups, so the row-group swizzle of the other tiles (pswz<32, 2>)
// conflicts there (PMC: 3.5e7 SQ_LDS_BANK_CONFLICT on the 3x3 256@14 layer,
// profiles/r03pmc_layer3_sq_counters.txt).  slot ^ ((row >> 2) & 3) keeps every
// ds_read_b128 lane group on 16 distinct bank quads for every offset: the four
// rows of a group that share row & 3 differ by {0, 12, 20, 24} or {4, 8, 16,
// 28}, whose (row >> 2) & 3 are four distinct values whatever the offset.
__device__ __forceinline__ int hswz(int row, int slot) { return slot ^ ((row >> 2) & 3); }

// MF = 1: v_mfma_f32_16x16x32_f16 (one 32-deep k-step per k-tile; each 32x32
// tile of a wave is four 16x16 sub-tiles, the acc_row / acc_col<true> map),
// which the chip holds at a higher clock than 32x32x16 in MFMA-dense loops
// (MI355X_MICROARCH.md 'DVFS give-back' item 7; profiles/r04b_fetch_ceiling.txt:
// register-only 0.875 vs 0.725 of the bf16 peak at two waves per SIMD).  A row
// half's A fragments are read once, the B fragments once per row half.
// IL (16x16x32, one tap per barrier): the next k-tile's B DMA goes out one
// instruction at a time among the k-tile's first MFMAs instead of as one
// burst before them (the halo pass load stays at the top: it comes from HBM).
// T2 (round 6): 2-D block tiles for maps too wide for a raster halo.  The
// tile is TH x T2 output pixels of one image (TH = BM / T2); its halo is the
// (TH + 2) x (T2 + 2) input block around them, out-of-image pixels loaded as
// zeros, so every tap of an in-map row is live (no tap masks) and output row
// r = (oy, ox) reads halo row (oy + kh)(T2 + 2) + ox + kw; rows outside the
// map are neither computed from (the zero row) nor stored (Rows2D).  Same
// products in the same order as the raster tile: bit-identical to it.
template <int EPI, int WM, int WN, int FM, int FN, int HALO_HR, int TPK = 1, int MF = 0, int IL = 0, int PERS = 0,
          int T2 = 0>
__global__ __launch_bounds__(512, 1) void gemm_h2_halo_kernel(GemmArgs g, int tiles_n) {
  constexpr int NP = 2, BK = 32, NT = 512, NW = 8;
  constexpr int WTM = 32 * FM, WTN = 32 * FN, BM = WTM * WM, BN = WTN * WN, SL = BK / 8;
  static_assert(WM * WN == NW && (BM == 256 || BM == 512), "8 waves, 256- or 512-row tiles");
  // SB (the 512-row tile): ONE halo buffer.  The next slice's passes wait in
  // registers through the slice's taps and are split into the buffer at the
  // top of the next slice, behind a barrier of their own.
  // (PERS 2: the one-tile form with one halo buffer at 256 rows too: room for
  // three taps' B stages per barrier where two halo buffers left none)
  constexpr bool SB = BM == 512 || PERS == 2;
  constexpr bool PST = PERS == 1;  // the persistent stream
  static_assert(!SB || (!PST && !IL && (BM == 256 || !MF)), "single-buffer halo: the one-tile form");
  constexpr int NHB = SB ? 1 : 2;  // halo buffers
  constexpr int TH = T2 ? BM / T2 : 1, HWD = T2 + 2;  // T2: the tile's output rows, the halo's width
  constexpr int NHR = T2 ? (TH + 2) * HWD : HALO_HR;   // halo rows a tile loads
  static_assert(!T2 || (BM % T2 == 0 && T2 % (MF ? 16 : 32) == 0 && NHR <= HALO_HR && !PST && !IL), "2-D tile");
  constexpr int HRA = HALO_HR + 1;                  // rows per A plane (+ the zero row)
  constexpr int A_EL = NP * HRA * BK;               // u16 per halo buffer
  constexpr int B_TAP = NP * BN * BK;               // u16 of one tap's B planes
  constexpr int B_EL = TPK * B_TAP;                 // u16 per B stage (TPK taps per barrier)
  constexpr int B_RPI = 64 / SL;                    // plane rows per LDS-DMA wave instruction
  constexpr int B_INS = NP * BN / B_RPI / NW;       // LDS-DMA instructions per wave per k-tile (4 / 2 / 1)
  constexpr int A_PASS = (HALO_HR + NT / SL - 1) / (NT / SL);  // 128-row passes over the halo (3)
  constexpr int LDS_U16 = NHB * A_EL + 2 * B_EL;
  static_assert(B_INS * NW * B_RPI == NP * BN, "B staging must tile the block");
  __shared__ __attribute__((aligned(16))) uint16_t lds[LDS_U16];
  typedef f16x8 frag_t;

  const uint32_t a_amax_w = amax_load_slot(g.a_amax);
  float a_sc = 1.f, a_isc = 1.f;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const int lr = lane & 31, lh = lane >> 5;

  static_assert(!PST || (TPK > 1 && !IL), "persistent halo tile: the all-passes-at-once instance");
  const int nwg = gridDim.x, bid = blockIdx.x;
  // PERS: one block per CU walks the row tiles bid + t nwg (tiles_n == 1, so
  // the weights never change), remapped per virtual block as config 8 / 15
  const int ntiles = PST ? (g.M + BM - 1) / BM * tiles_n : nwg;
  auto tile_m0 = [&](int tl) __attribute__((always_inline)) {
    const int v = bid + tl * nwg;
    const int xcd = v & 7, q8 = ntiles >> 3, r8 = ntiles & 7;
    const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (v >> 3);
    return (wgid / tiles_n) * BM;
  };
  int m0, n0;
  {
    const int xcd = bid & 7, q8 = ntiles >> 3, r8 = ntiles & 7;
    const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    m0 = (wgid / tiles_n) * BM;
    n0 = (wgid % tiles_n) * BN;
  }
  // 3x3 only (h2_halo_rows): the tap -> (kh, kw) split and the group count
  // are compile-time constants
  const int W = g.W, H = g.H;
  constexpr int KW = 3, KH = 3, ntap = KH * KW;
  const int nch = g.Cin / BK, ngrp = ntap / TPK, nk = nch * ngrp;  // k-step kt = (slice, group of TPK taps)
  const int hoff = g.pad * W + g.pad;  // halo row 0 = input raster index m0 - hoff
  // T2: the tile's image (its first output row) and top-left output pixel
  int t_img = 0, t_y0 = 0, t_x0 = 0;
  if constexpr (T2 != 0) {
    const int mt = m0 / BM, tx_n = (W + T2 - 1) / T2, tpi = (H + TH - 1) / TH * tx_n;
    const int im = mt / tpi, rem = mt - im * tpi, ty = rem / tx_n;
    t_img = im * H * W;
    t_y0 = ty * TH;
    t_x0 = (rem - ty * tx_n) * T2;
  }
  // the halo row (tap (0, 0)) of tile row rb + l (rb a multiple of the
  // fragment height, l below it, so l stays an offset: T2 % 32 == 0 for the
  // 32x32 fragments), and the halo-row step of kh
  auto hrow = [&](int rb, int l) __attribute__((always_inline)) { return T2 ? (rb / T2) * HWD + rb % T2 + l : rb + l; };
  const int tstep = T2 ? HWD : W;

  // ---- halo loader: thread -> (row t / 4 + 128 pass, 16-B slot pair t % 4);
  // one 128-row pass at a time (8 registers), so the halo of the next slice
  // never holds more than one pass beside the accumulators ----
  // (TPK > 1: the narrow tiles have the registers to hold every pass at once)
  const int a_slot = tid % SL, a_row = tid / SL;
  constexpr int RA_N = (TPK == 1 && !SB) ? 1 : A_PASS;
  f32x4 ra[RA_N][2];
  auto load_pass_to = [&](int c, int p, f32x4(&r)[2], int mb) {
    const int hr = a_row + p * (NT / SL);
    long long q;
    bool ok;
    if constexpr (T2 != 0) {
      // (from an opaque row: hoisted out of the k-loop, the three passes'
      // addresses and bounds would be held beside the accumulators)
      const int ho = s3_opaque(hr), hy = ho / HWD, iy = t_y0 - 1 + hy, ix = t_x0 - 1 + (ho - hy * HWD);
      q = (long long)t_img + iy * W + ix;
      ok = hr < NHR && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
    } else {
      q = (long long)mb - hoff + hr;
      ok = hr < HALO_HR && q >= 0 && q < g.M;
    }
    const f32x4* src = ok ? reinterpret_cast<const f32x4*>(g.A + q * g.Cin + c * BK + a_slot * 8) : s3_zero_page();
    s3_load2<1>(src, r);
  };
  auto load_pass = [&](int c, int p) { load_pass_to(c, p, ra[RA_N == 1 ? 0 : p], m0); };
  auto launder_pass = [&]() {
#pragma unroll
    for (int p = 0; p < RA_N; ++p) {
      s3_launder(ra[p][0]);
      s3_launder(ra[p][1]);
    }
  };
  auto store_pass_from = [&](int buf, int p, const f32x4(&r)[2]) {
    const int hr = a_row + p * (NT / SL);
    u32x4 p0, p1;
    split2h8(r, a_sc, p0, p1);
    if (hr < HALO_HR) {
      uint16_t* la = lds + buf * A_EL;
      const int off = hr * BK + hswz(hr, a_slot) * 8;
      *reinterpret_cast<u32x4*>(la + off) = p0;
      *reinterpret_cast<u32x4*>(la + HRA * BK + off) = p1;
    }
  };
  auto store_pass = [&](int buf, int p) { store_pass_from(buf, p, ra[RA_N == 1 ? 0 : p]); };

  // ---- B planes: LDS-DMA, instruction i of a wave fills plane rows
  // prow = (i NW + wave) B_RPI + lane / 4 of the [2][BN] stage (N % BN == 0:
  // every row real).  256 columns: plane i / 2, rows 128 (i & 1) + prow % 128
  // off one pointer (rows r and r + 128 share their swizzle); narrower tiles
  // keep a pointer per instruction ----
  const int b_r = wave * B_RPI + lane / SL;
  const uint16_t* Bp = reinterpret_cast<const uint16_t*>(g.B);
  static_assert(NW * B_RPI == 128, "one DMA round = 128 plane rows");
  const uint16_t* b_src[BN == 256 ? 1 : B_INS];
  if constexpr (BN == 256) {
    b_src[0] = Bp + (long long)(n0 + b_r) * g.ldb + pswz<BK, 2>(b_r, lane % SL) * 8;
  } else {
#pragma unroll
    for (int i = 0; i < B_INS; ++i) {
      const int prow = i * 128 + b_r, p = prow / BN, r = prow - p * BN;
      b_src[i] = Bp + p * g.b_plane + (long long)(n0 + r) * g.ldb + pswz<BK, 2>(r, lane % SL) * 8;
    }
  }
  auto glds_b = [&](int kt, int buf) {
    const int c = kt / ngrp, t0 = (kt - c * ngrp) * TPK;
#pragma unroll
    for (int u = 0; u < TPK; ++u) {
      const long long koff = (long long)(t0 + u) * g.Cin + c * BK;
      uint16_t* lb = lds + NHB * A_EL + buf * B_EL + u * B_TAP;
#pragma unroll
      for (int i = 0; i < B_INS; ++i) {
        const uint16_t* src = BN == 256 ? b_src[0] + (i >> 1) * g.b_plane + (long long)(i & 1) * (BN / 2) * g.ldb
                                        : b_src[BN == 256 ? 0 : i];
        __builtin_amdgcn_global_load_lds((const void*)(src + koff),
                                         (__attribute__((address_space(3))) void*)(lb + (i * NW + wave) * B_RPI * BK),
                                         16, 0, 0);
      }
    }
  };

  static_assert(!IL || (MF && TPK == 1 && B_INS <= FM * FN), "IL: the 16x16x32 one-tap-per-barrier tile");
  // IL: DMA instruction i of glds_b(kt, buf), before a0b0 MFMA number
  // i * IL_STEP of the k-tile's first (row half, column half) block
  constexpr int IL_STEP = (FM * FN) / B_INS;
  auto glds_b_due = [&](int kt, int buf, int idx) {
    if constexpr (IL) {
      const int c = kt / ngrp, t0 = kt - c * ngrp;
      const long long koff = (long long)t0 * g.Cin + c * BK;
      uint16_t* lb = lds + NHB * A_EL + buf * B_EL;
#pragma unroll
      for (int i = 0; i < B_INS; ++i) {
        if (i * IL_STEP != idx) continue;
        const uint16_t* src = BN == 256 ? b_src[0] + (i >> 1) * g.b_plane + (long long)(i & 1) * (BN / 2) * g.ldb
                                        : b_src[BN == 256 ? 0 : i];
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_global_load_lds((const void*)(src + koff),
                                         (__attribute__((address_space(3))) void*)(lb + (i * NW + wave) * B_RPI * BK),
                                         16, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };

  // ---- the lanes' fragment rows: a 9-bit mask of the taps that stay inside
  // the row's image (bit kh KW + kw), empty past M ----
  // (MF: the lane's rows are i * 32 + 16 a + (lane & 15), a = 0, 1)
  constexpr int RPT = MF ? 2 : 1;
  const int l16 = lane & 15, lg = lane >> 4;
  int tmask[FM][RPT];
  auto masks = [&](int mb) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int a = 0; a < RPT; ++a) {
        const int m = mb + wm * WTM + i * 32 + (MF ? 16 * a + l16 : lr);
        if constexpr (T2 != 0) {
          // every tap reads the halo (zeros off the image); rows off the map
          // compute from it too, finite, and are not stored (Rows2D)
          tmask[i][a] = (1 << ntap) - 1;
          continue;
        }
        const int rem = m % (H * W), oh = rem / W, ow = rem - oh * W;
        int mk = 0;
        for (int kh = 0; kh < KH; ++kh)
          for (int kw = 0; kw < KW; ++kw)
            if ((unsigned)(oh + kh - g.pad) < (unsigned)H && (unsigned)(ow + kw - g.pad) < (unsigned)W)
              mk |= 1 << (kh * KW + kw);
        tmask[i][a] = m < g.M ? mk : 0;
      }
  };
  masks(m0);

  f32x16 acc[FM][FN];
  f32x4 acc4[MF ? FM : 1][MF ? FN : 1][4];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  if constexpr (MF) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int t = 0; t < 4; ++t) acc4[i][j][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  // one k-tile: tap t of halo buffer hb, B stage bs; two 16-deep k-steps, each
  // a0b0 first, then a0b1 + a1b0 (config 12's per-accumulator order)
  // kt_next: the k-tile whose B DMA an IL tile issues among these MFMAs
  auto compute = [&](int hb, int bs, int t, int u, int kt_next = 0) {
    const int kh = t / KW, kw = t - kh * KW;
    const uint16_t* la = lds + hb * A_EL;
    const uint16_t* lb = lds + NHB * A_EL + bs * B_EL + u * B_TAP;
    if constexpr (MF) {
      // one 32-deep k-step: lane group lg holds k 8 lg .. +7 (16-B slot lg)
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        frag_t fa[NP][FM];
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const int ar = ((tmask[i][a] >> t) & 1) ? hrow(wm * WTM + i * 32 + 16 * a, l16) + kh * tstep + kw : HALO_HR;
#pragma unroll
          for (int p = 0; p < NP; ++p)
            fa[p][i] = *reinterpret_cast<const frag_t*>(la + (p * HRA + ar) * BK + hswz(ar, lg) * 8);
        }
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          frag_t fb[NP][FN];
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            const int row = wn * WTN + j * 32 + 16 * b + l16;
#pragma unroll
            for (int p = 0; p < NP; ++p)
              fb[p][j] = *reinterpret_cast<const frag_t*>(lb + (p * BN + row) * BK + pswz<BK, 2>(row, lg) * 8);
          }
          // config 12's per-accumulator order: a0b0, then a0b1 + a1b0
#pragma unroll
          for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j) {
              if constexpr (IL) {
                if (a == 0 && b == 0) glds_b_due(kt_next, bs ^ 1, i * FN + j);
              }
              acc4[i][j][2 * a + b] = s3_mf16<2>(fa[0][i], fb[0][j], acc4[i][j][2 * a + b]);
            }
#pragma unroll
          for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j) {
              acc4[i][j][2 * a + b] = s3_mf16<2>(fa[0][i], fb[1][j], acc4[i][j][2 * a + b]);
              acc4[i][j][2 * a + b] = s3_mf16<2>(fa[1][i], fb[0][j], acc4[i][j][2 * a + b]);
            }
        }
      }
      return;
    }
    int ar[FM];
#pragma unroll
    for (int i = 0; i < FM; ++i)
      ar[i] = ((tmask[i][0] >> t) & 1) ? hrow(wm * WTM + i * 32, lr) + kh * tstep + kw : HALO_HR;
#pragma unroll
    for (int st = 0; st < BK / 16; ++st) {
      frag_t a[NP][FM], b[NP][FN];
#pragma unroll
      for (int p = 0; p < NP; ++p) {
#pragma unroll
        for (int i = 0; i < FM; ++i)
          a[p][i] = *reinterpret_cast<const frag_t*>(la + (p * HRA + ar[i]) * BK + hswz(ar[i], 2 * st + lh) * 8);
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int row = wn * WTN + j * 32 + lr;
          b[p][j] = *reinterpret_cast<const frag_t*>(lb + (p * BN + row) * BK + pswz<BK, 2>(row, 2 * st + lh) * 8);
        }
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = s3_mf32<2>(a[0][i], b[0][j], acc[i][j]);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          acc[i][j] = s3_mf32<2>(a[0][i], b[1][j], acc[i][j]);
          acc[i][j] = s3_mf32<2>(a[1][i], b[0][j], acc[i][j]);
        }
    }
  };

  // ---- prologue: the zero rows, slice 0's halo (pass by pass), k-tile 0's B ----
  RR_PH_DECL
  if (tid < 8 * NHB) {
    // row HALO_HR of both planes of every halo buffer: 64 B per plane, 16 B per thread
    const int buf = tid >> 3, p = (tid >> 2) & 1, sl = tid & 3;
    *reinterpret_cast<u32x4*>(lds + buf * A_EL + (p * HRA + HALO_HR) * BK + sl * 8) = u32x4{0u, 0u, 0u, 0u};
  }
  glds_b(0, 0);
  {
    // slice 0's halo: every pass's loads first, one wait (three waits in
    // turn cost a tile three HBM round trips before its first MFMA); the
    // accumulators are still constant zeros here, so the registers are free
    f32x4 rp[A_PASS][2];
#pragma unroll
    for (int p = 0; p < A_PASS; ++p) load_pass_to(0, p, rp[p], m0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int p = 0; p < A_PASS; ++p) {
      s3_launder(rp[p][0]);
      s3_launder(rp[p][1]);
    }
    {
      // the record's wave max, with shuffle addresses from an opaque lane id:
      // amax_reduce's would be shared with the epilogue's amax_publish and held
      // (spilled) through the whole k-loop
      uint32_t u = a_amax_w;
      const int lo = s3_opaque(lane);
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const uint32_t v = (uint32_t)__builtin_amdgcn_ds_bpermute((lo ^ o) << 2, (int)u);
        u = v > u ? v : u;
      }
      const int e = __builtin_amdgcn_readfirstlane(h2_exp(__uint_as_float(u)));
      a_sc = __int_as_float((127 + e) << 23);
      a_isc = __int_as_float((127 - e) << 23);
    }
#pragma unroll
    for (int p = 0; p < A_PASS; ++p) store_pass_from(0, p, rp[p]);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  // ---- k-loop: k-tile kt = (slice c, tap t); B stage kt & 1, halo buffer c & 1.
  // The next slice's halo: pass p loaded in tap p's k-tile (after its B DMA,
  // landed by the end-of-tile wait) and split into the other buffer at the
  // start of tap p + 1's (that buffer's last reader was slice c - 1) ----
  static_assert(A_PASS < 9, "the halo passes must fit in one slice's taps");
  if constexpr (PST) {
    // ---- the persistent stream: k-step q of the block = k-step q % nk of
    // local tile q / nk, B stage q & 1, halo buffer sg & 1 (sg: the block's
    // slice counter).  The next slice -- the tile's next, or after the
    // tile's last the next tile's slice 0 -- loads in a slice's first group
    // and splits into the other buffer in its second (with that buffer's
    // zero rows: an epilogue may have staged C over them); the next k-step's
    // B DMA may belong to the next tile (the same weights).  After a tile's
    // last k-step its epilogue stages C through the halo buffer that slice
    // released, in 128-row slabs ----
    const int my_tiles = (ntiles - bid + nwg - 1) / nwg;
    const int Q = my_tiles * nk;
    // the group whose top splits the next slice into the other buffer: the
    // slice's third (its passes, loaded in the first group, then have two
    // groups' MFMAs to arrive from HBM; the first group's end waits only for
    // the B DMA issued before them), or the second with fewer groups
    const int st_g = ngrp >= 3 ? 2 : 1;
    int tl = 0, c = 0, tg = 0, kt = 0, sg = 0;
    int m_next = my_tiles > 1 ? tile_m0(1) : m0;
    for (int q = 0; q < Q; ++q) {
      const bool last_slice = c + 1 == nch;
      const bool more = !last_slice || tl + 1 < my_tiles;
      if (q + 1 < Q) glds_b(kt + 1 == nk ? 0 : kt + 1, (q + 1) & 1);
      if (more && tg == st_g) {
        const int nb = (sg + 1) & 1;
#pragma unroll
        for (int p = 0; p < A_PASS; ++p) store_pass(nb, p);
        if (tid < 8) {
          const int pl = tid >> 2, sl = tid & 3;
          *reinterpret_cast<u32x4*>(lds + nb * A_EL + (pl * HRA + HALO_HR) * BK + sl * 8) = u32x4{0u, 0u, 0u, 0u};
        }
      }
      if (more && tg == 0) {
#pragma unroll
        for (int p = 0; p < A_PASS; ++p) load_pass_to(last_slice ? 0 : c + 1, p, ra[p], last_slice ? m_next : m0);
      }
#pragma unroll
      for (int u = 0; u < TPK; ++u) compute(sg & 1, q & 1, tg * TPK + u, u);
      if (more && tg == 0 && st_g == 2)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * A_PASS) : "memory");  // the next B (older than the passes)
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the next B (and the next slice's passes)
      launder_pass();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (++tg == ngrp) {
        tg = 0;
        ++c;
        ++sg;
      }
      if (++kt == nk) {
        if constexpr (MF) {
#pragma unroll
          for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j)
#pragma unroll
              for (int t = 0; t < 4; ++t)
#pragma unroll
                for (int e = 0; e < 4; ++e) acc[i][j][4 * t + e] = acc4[i][j][t][e];
        }
        epilogue_store<WM, WN, FM, FN, A_EL / 2, (bool)MF, EPI>(
            g, g.C, acc, reinterpret_cast<float*>(lds + ((sg - 1) & 1) * A_EL), m0, n0, a_isc);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) {
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
            if constexpr (MF) {
#pragma unroll
              for (int t = 0; t < 4; ++t) acc4[i][j][t] = f32x4{0.f, 0.f, 0.f, 0.f};
            }
          }
        kt = 0;
        c = 0;
        ++tl;
        m0 = m_next;
        m_next = tl + 1 < my_tiles ? tile_m0(tl + 1) : m0;
        masks(m0);
      }
    }
    return;
  }
  int c = 0, tg = 0;
  RR_PH(7);
  for (int kt = 0; kt < nk; ++kt) {
    const bool more = c + 1 < nch;
    if constexpr (!IL) glds_b(min(kt + 1, nk - 1), (kt + 1) & 1);
    if constexpr (TPK == 1 && !SB) {
      if (more && tg >= 1 && tg <= A_PASS) store_pass((c + 1) & 1, tg - 1);
      if (more && tg < A_PASS) load_pass(c + 1, tg);
    } else if constexpr (SB) {
      // one halo buffer: slice c's passes (loaded during slice c - 1) split
      // into it once every wave is done with slice c - 1 (the last group's
      // barrier), then a barrier before any tap reads them
      if (c > 0 && tg == 0) {
#pragma unroll
        for (int p = 0; p < A_PASS; ++p) store_pass(0, p);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
      }
      if (more && tg == 0) {
#pragma unroll
        for (int p = 0; p < A_PASS; ++p) load_pass(c + 1, p);
      }
    } else {
      // every pass loaded in the slice's first group, split in its second
      if (more && tg == 1) {
#pragma unroll
        for (int p = 0; p < A_PASS; ++p) store_pass((c + 1) & 1, p);
      }
      if (more && tg == 0) {
#pragma unroll
        for (int p = 0; p < A_PASS; ++p) load_pass(c + 1, p);
      }
    }
    RR_PH(0);
#pragma unroll
    for (int u = 0; u < TPK; ++u) compute(SB ? 0 : (c & 1), kt & 1, tg * TPK + u, u, min(kt + 1, nk - 1));
    RR_PH(1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the next B (and a halo pass)
    launder_pass();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    RR_PH(2);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    RR_PH(3);
    if (++tg == ngrp) {
      tg = 0;
      ++c;
    }
  }
  __syncthreads();
  if constexpr (MF) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[i][j][4 * t + e] = acc4[i][j][t][e];
  }
  if constexpr (T2 != 0)
    epilogue_store<WM, WN, FM, FN, LDS_U16 / 2, (bool)MF, EPI, Rows2D<T2>>(
        g, g.C, acc, reinterpret_cast<float*>(lds), 0, n0, a_isc, nullptr, Rows2D<T2>{t_img, t_y0, t_x0, H, W});
  else
    epilogue_store<WM, WN, FM, FN, LDS_U16 / 2, (bool)MF, EPI>(g, g.C, acc, reinterpret_cast<float*>(lds), m0, n0,
                                                               a_isc);
  RR_PH(6);
  RR_PH_FLUSH(3);
}

// config 13 serves: f16x2, conv A, 3x3 stride 1 pad 1 (output = input size),
// Cin % 32 == 0, N % 64 == 0 and W within the instance's halo (see above),
// the ResNet's f16x2 flag sets.  Returns the halo rows of the instance that
// serves g, 0 if none.
static int h2_halo_rows(const GemmArgs& g) {
  if (!(g.KH == 3 && g.KW == 3 && g.stride == 1 && g.pad == 1 && g.OH == g.H && g.OW == g.W && (g.Cin % 32) == 0 &&
        g.K == 9 * g.Cin && g.col_scale != nullptr && g.a_amax != nullptr))
    return 0;
  const int need = 256 + 2 * (g.W + 1);
  if ((g.N % 256) == 0) return need <= 288 ? 288 : 0;
  if ((g.N % 128) == 0) return need <= 320 ? 320 : 0;
  if ((g.N % 64) == 0) return need <= 384 ? 384 : 0;
  return 0;
}
template <int EPI, int WM, int WN, int FM, int FN, int HR, int TPK, int MF, int IL = 0, int PERS = 0, int T2 = 0>
static hipError_t launch_h2_halo_t(const GemmArgs& g, hipStream_t s, int n_cu = 256) {
  constexpr int BN = 32 * FN * WN, BM = 32 * FM * WM;
  // (T2: images x row blocks x column blocks of the map)
  const long long tiles_m = T2 ? (long long)(g.M / (g.H * g.W)) * ((g.H + BM / T2 - 1) / (BM / T2)) * ((g.W + T2 - 1) / T2)
                               : (g.M + BM - 1) / BM,
                  tiles_n = g.N / BN;
  const long long nblk = tiles_m * tiles_n;
  if (nblk <= 0) return hipSuccess;
  if (nblk > 0x7fffffffLL) return hipErrorInvalidValue;
  // PERS: one block per CU walking the row tiles (tiles_n == 1; a block that
  // owns several stays on its XCD: grid a multiple of 8)
  const int slots = std::max(8, n_cu & ~7);
  const long long grid = PERS == 1 ? (nblk <= slots ? nblk : slots) : nblk;
  hipLaunchKernelGGL((gemm_h2_halo_kernel<EPI, WM, WN, FM, FN, HR, TPK, MF, IL, PERS, T2>), dim3((unsigned)grid), dim3(512),
                     0, s, g, (int)tiles_n);
  return hipGetLastError();
}
template <int WM, int WN, int FM, int FN, int HR, int TPK, int MF, int IL = 0, int PERS = 0>
static hipError_t launch_h2_halo_ep(const GemmArgs& g, hipStream_t s, int n_cu = 256) {
  switch (ep_flags(g) & (EP_RES | EP_RELU)) {
    case EP_RELU: return launch_h2_halo_t<H2_EP | EP_RELU, WM, WN, FM, FN, HR, TPK, MF, IL, PERS>(g, s, n_cu);
    case EP_RES | EP_RELU: return launch_h2_halo_t<H2_EP | EP_RES | EP_RELU, WM, WN, FM, FN, HR, TPK, MF, IL, PERS>(g, s, n_cu);
    case EP_RES: return launch_h2_halo_t<H2_EP | EP_RES, WM, WN, FM, FN, HR, TPK, MF, IL, PERS>(g, s, n_cu);
    default: return launch_h2_halo_t<H2_EP, WM, WN, FM, FN, HR, TPK, MF, IL, PERS>(g, s, n_cu);
  }
}
// mf: 1 = the 16x16x32 form (s3_cfg 14 forces it); pers: the N = 64 instance
// as a persistent stream (one column tile)
static hipError_t launch_h2_halo(const GemmArgs& g, hipStream_t s, int hr, int mf, bool pers = false, int n_cu = 256) {
  // N = 64 (the 64@56 layers): the 512-row single-buffer tile, 8 waves of
  // 64 x 64, wherever its 640-row halo holds the map (W <= 63): every wave
  // reads 64 + 64 fragment rows per tap for 24 MFMAs instead of 64 + 32 for
  // 12, and the taps of a barrier carry 72 MFMAs per wave instead of 36.
  // 1.193 -> 1.059 ms at 1280 images, bit-identical
  // (profiles/r06r_halo512_ab.txt).  halo_mf 3 forces the persistent
  // 256-row stream (round 5's default), 2 the 512-row tile.
  if (hr == 384 && g.N == 64 && (mf == 2 || (mf == 0 && pers)) && 512 + 2 * (g.W + 1) <= 640)
    return launch_h2_halo_ep<8, 1, 2, 2, 640, 3, 0>(g, s);
  // N = 128 on 16x16x32: one halo buffer and three taps per barrier (the
  // LDS the second halo buffer held now holds three taps' B stages): 0.924 ->
  // 0.897 ms at 128@28, bit-identical (profiles/r06z2_halo128_sb_ab.txt);
  // halo_mf 4 keeps the two-buffer one-tap form for A/Bs
  if (hr == 320 && mf == 4) return launch_h2_halo_ep<4, 2, 2, 2, 320, 1, 1>(g, s);
  if (hr == 320 && mf == 1) return launch_h2_halo_ep<4, 2, 2, 2, 320, 3, 1, 0, 2>(g, s);
  if (mf >= 2) {
    pers = pers || mf == 3;
    mf = mf == 4 ? 1 : 0;
  }
  if (hr == 384 && !mf && pers && g.N == 64) return launch_h2_halo_ep<4, 2, 2, 1, 384, 3, 0, 0, 1>(g, s, n_cu);
  // (the 16x16x32 256x256 form with its B DMA spread among the MFMAs: conv_il)
  if (hr == 288 && mf && g.issue_spread) return launch_h2_halo_ep<2, 4, 4, 2, 288, 1, 1, 1>(g, s);
  if (hr == 288) return mf ? launch_h2_halo_ep<2, 4, 4, 2, 288, 1, 1>(g, s) : launch_h2_halo_ep<2, 4, 4, 2, 288, 1, 0>(g, s);
  if (hr == 320) return mf ? launch_h2_halo_ep<4, 2, 2, 2, 320, 1, 1>(g, s) : launch_h2_halo_ep<4, 2, 2, 2, 320, 1, 0>(g, s);
  return mf ? launch_h2_halo_ep<4, 2, 2, 1, 384, 3, 1>(g, s) : launch_h2_halo_ep<4, 2, 2, 1, 384, 3, 0>(g, s);
}

// The 2-D block tiles (T2) for the stride-1 3x3 layers of maps too wide for a
// raster halo (C2's 1024-px layers 1-3: W 256 / 128 / 64): the tile's halo is
// (TH + 2)(T2 + 2) rows whatever W is.  Instances: 16 x 16 outputs, 18 x 18 =
// 324 halo rows, on the 256x256 (N % 256) and 256x128 single-buffer three-tap
// (N = 128) tiles; 16 x 32 outputs, 18 x 34 = 612 rows, on the 512-row N = 64
// tile.  No residual epilogue (the trunk's 3x3s have none).  Returns whether
// one serves g.
static bool h2_halo_2d_ok(const GemmArgs& g) {
  if (!(g.KH == 3 && g.KW == 3 && g.stride == 1 && g.pad == 1 && g.OH == g.H && g.OW == g.W && (g.Cin % 32) == 0 &&
        g.K == 9 * g.Cin && g.col_scale != nullptr && g.a_amax != nullptr && g.H > 0 && g.W > 0 &&
        (g.M % (g.H * g.W)) == 0 && (ep_flags(g) & EP_RES) == 0))
    return false;
  if (g.N == 128) {
    // the N = 128 tile needs a block per CU: below that config 11's
    // 128-column tiles spread further (a batch-1 128@75x100 crop, 35 blocks:
    // 0.040 -> 0.045 ms; 64 images of 128@128x96: 0.811 -> 0.685 ms;
    // profiles/r06zb_halo2d_ab.txt)
    const long long blocks = (long long)(g.M / (g.H * g.W)) * ((g.H + 15) / 16) * ((g.W + 15) / 16);
    return blocks >= 256 || g.halo_2d == 1;
  }
  return (g.N % 256) == 0 || g.N == 64;
}
template <int WM, int WN, int FM, int FN, int HR, int TPK, int MF, int PERS, int T2>
static hipError_t launch_h2_halo_2d_ep(const GemmArgs& g, hipStream_t s) {
  if ((ep_flags(g) & EP_RELU) != 0) return launch_h2_halo_t<H2_EP | EP_RELU, WM, WN, FM, FN, HR, TPK, MF, 0, PERS, T2>(g, s);
  return launch_h2_halo_t<H2_EP, WM, WN, FM, FN, HR, TPK, MF, 0, PERS, T2>(g, s);
}
static hipError_t launch_h2_halo_2d(const GemmArgs& g, hipStream_t s) {
  if (g.N == 64) return launch_h2_halo_2d_ep<8, 1, 2, 2, 640, 3, 0, 0, 32>(g, s);
  if (g.N == 128) return launch_h2_halo_2d_ep<4, 2, 2, 2, 324, 3, 1, 2, 16>(g, s);
  return launch_h2_halo_2d_ep<2, 4, 4, 2, 324, 1, 1, 0, 16>(g, s);
}

// config 8 serves dense A (1x1 convs), N % 256 == 0 and the ResNet's flag
// sets (conv + BN + ReLU, + residual + ReLU, the projection conv; f16x2: any
// residual / ReLU combination); the rest falls back to the library's pick
template <int SP>
static bool s3_persist_ok(const GemmArgs& g, int amode) {
  const int f = ep_flags(g);
  if ((g.N % 256) != 0 || amode != A_DENSE) return false;
  if constexpr (SP == 2) return true;
  return f == (EP_BIAS | EP_RELU) || f == (EP_BIAS | EP_RES | EP_RELU) || f == EP_BIAS;
}
template <int SP>
static hipError_t launch_s3p(const GemmArgs& g, hipStream_t s, int n_cu, int st) {
  if constexpr (SP == 2) {
    // residual epilogues streamed (EP_SC1, as config 15's): 128->512 + residual
    // x3 0.908 -> 0.877 ms, 64->256 x2 1.701 -> 1.707; the embed 69.09 -> 69.06
    // ms (profiles/r05k_sweep.txt, r05k_e2e.txt)
    switch (ep_flags(g) & (EP_RES | EP_RELU)) {
      case EP_RELU: return launch_s3p_t<H2_EP | EP_RELU, 2>(g, s, n_cu, st);
      case EP_RES | EP_RELU: return launch_s3p_t<H2_EP | EP_RES | EP_RELU | EP_SC1, 2>(g, s, n_cu, st);
      case EP_RES: return launch_s3p_t<H2_EP | EP_RES | EP_SC1, 2>(g, s, n_cu, st);
      default: return launch_s3p_t<H2_EP, 2>(g, s, n_cu, st);
    }
  } else {
    static_assert(SP == 2, "launch_s3p: the f16x2 split only (ABI 6)");
  }
}

template <int WM, int WN, int FM, int FN, int BK, int AM, int MINB, int MF16 = 0, int EPI = -1, int SP = 2,
          int NSTG = 2, int POOL = 0, int ACC1 = 0, int IL = 0>
static hipError_t launch_s3_t(GemmArgs g, hipStream_t s, int n_cu, int stagger) {
  constexpr int BM = 32 * FM * WM, BN = 32 * FN * WN;
  const long long tiles_m = (g.M + BM - 1) / BM, tiles_n = (g.N + BN - 1) / BN;
  const long long nblk = tiles_m * tiles_n;
  if (nblk <= 0) return hipSuccess;
  if (nblk > 0x7fffffffLL) return hipErrorInvalidValue;
  // resident blocks per CU: MINB is the launch bound's minimum waves per SIMD
  constexpr int PER_CU = (MINB * 4) / (WM * WN) > 1 ? (MINB * 4) / (WM * WN) : 1;
  g.stagger_blocks = n_cu * PER_CU;
  g.stagger_sleeps = nblk > 2LL * n_cu * PER_CU ? stagger : 0;  // only grids of several rounds
  hipLaunchKernelGGL((gemm_s3_kernel<WM, WN, FM, FN, BK, AM, MINB, MF16, EPI, SP, NSTG, POOL, ACC1, IL>), dim3((unsigned)nblk),
                     dim3(64 * WM * WN), 0, s, g, (int)tiles_n);
  return hipGetLastError();
}

// Tile configs (waves WMxWN, MFMA tiles per wave FMxFN, BK, blocks per CU;
// LDS of the bf16x3 split, two thirds of it for f16x2):
//   1: 128x128, 4 waves of 64x64, BK 16, 2/CU (48 KB LDS)
//   2: 128x128, 4 waves of 64x64, BK 32, 1/CU (96 KB)
//   3: 256x128, 8 waves of 64x64, BK 32, 1/CU (144 KB)
//   4: 128x256, 8 waves of 64x64, BK 32, 1/CU (144 KB), v_mfma_f32_16x16x32_{bf16,f16}
//   5: 256x64,  4 waves of 64x64, BK 32, 1/CU (120 KB)
//   6: 256x64,  4 waves of 64x64, BK 16, 2/CU (60 KB)
//   7: 256x64,  8 waves of 32x64, BK 16, 2/CU (60 KB), 4 waves per SIMD
//      (<= 128 registers): the picked 256x64 tile (the N = 64 layers and the
//      stem 2-7 % faster than 6, profiles/r02f_s3_cfg7.txt; f16x2 dense N = 64
//      now takes config 15's 256x64 form, profiles/r05ah_s3q64_ab/)
//   8: config 4 as a persistent k-stream (gemm_s3p_kernel): dense A, N % 256
//      == 0 — the picked tile for the 1x1 layers it serves
//   9: config 4 with three LDS stages (f16x2 only, 144 KB): the B DMA two
//      k-tiles ahead
//  10: config 4 with one accumulator set (f16x2 only, ACC1: the plane-1
//      products accumulate with a0b0; error vs float64 still at the exact-fp32
//      core's, profiles/r03j_acc1_ab.txt; 196 instead of 254 VGPRs)
//  11: 128x128, 4 waves of 64x64, BK 32, 2/CU (64 KB), 16x16x32, ACC1 (f16x2
//      only): the picked tile for N == 128 (dense K >= 256: config 15's
//      256x128 form)
//  12: 256x256, 8 waves of 128x64, BK 32, 1/CU (128 KB), 32x32x16, ACC1 (f16x2
//      only; 254 VGPRs — two accumulator sets do not fit this tile): half the
//      operand bytes per FLOP of config 4, the picked tile for N % 256 == 0
//      except the K < 256 residual expansions
//  15: config 12 as a persistent k-stream (gemm_s3q_kernel, f16x2, dense A,
//      config 12's shapes; the pick there): the next tile's first k-tiles load under
//      the epilogue, which runs in four slabs with the residual two 32-row
//      bands ahead; bit-identical to config 12.  Its 256x128 form serves
//      dense N == 128, K >= 256, its 256x64 form dense N == 64, K >= 64
// (all others on v_mfma_f32_32x32x16_{bf16,f16}).  The f16x2 split is built
// for configs 3, 4, 7, 8, 9, 10 and 11 (a forced 1, 2, 5 or 6 runs the pick).
// Measured per R101 layer at 320 images (round 2's tools/s3_bench.py): 3 is the fastest
// wherever N >= 128 (1.1-1.3x config 1 per FLOP); 4 on 16x16x32 runs every
// N % 256 == 0 layer 3-14 % faster than 3 (the 16x16 shape holds a higher
// clock on random operands, MI355X_MICROARCH.md 'DVFS give-back' item 7; the
// same shape is slower in the one-wave-per-SIMD configs 2 and 5 and spills in
// 3).  Not kept: an all-DMA ring with the A split at fragment-read
// time (10-15 % slower), a one-wave-per-SIMD 256x128 variant (1.16x slower), a
// single accumulator for all six terms (less accurate than exact fp32).
// rr_set_tuning(RR_TUNE_S3_CFG) forces a config (tests, tools).
static int pick_s3(const GemmArgs& g, int forced) {
  if (forced >= 1 && forced <= 8) return forced;
  if ((g.N % 256) == 0) return 4;
  // rounds of resident blocks x tile area per CU / relative per-FLOP speed
  auto cost = [&](long long bm, long long bn, long long per_cu, double speed) {
    const long long slots = 256 * per_cu;
    const long long t = ((g.M + bm - 1) / bm) * ((g.N + bn - 1) / bn);
    return (double)((t + slots - 1) / slots) * bm * bn * per_cu / speed;
  };
  double best = cost(128, 128, 2, 1.0);
  int cfg = 1;
  if (cost(256, 128, 1, 1.15) < best) best = cost(256, 128, 1, 1.15), cfg = 3;
  if (cost(256, 64, 2, 1.0) < best) best = cost(256, 64, 2, 1.0), cfg = 7;
  return cfg;
}
// f16x2: config 1 (no f16x2 build) -> 3 where it tiles no worse than 7
static int pick_h2(const GemmArgs& g, int forced) {
  if (forced == 9) return (g.N % 256) == 0 ? 9 : pick_h2(g, 0);
  if (forced == 10) return (g.N % 256) == 0 ? 10 : pick_h2(g, 0);
  if (forced == 11) return (g.N % 128) == 0 ? 11 : pick_h2(g, 0);
  if (forced == 12) return (g.N % 256) == 0 ? 12 : pick_h2(g, 0);
  // N == 128: two 128x128 blocks per CU (config 11) run the R101 N = 128
  // layers 4-7 % faster than the 256x128 tile (profiles/r03l_h2_cfg_sweep.txt);
  // the dense K >= 256 ones take config 15's persistent 256x128 form before
  // this pick (profiles/r05ae_s3q128_ab/)
  if (forced == 0 && g.N == 128) return 11;
  int cfg = pick_s3(g, forced);
  if (cfg == 3 || cfg == 4 || cfg == 7 || cfg == 8) return cfg;
  cfg = pick_s3(g, 0);
  if (cfg == 1) cfg = (g.N % 128) == 0 ? 3 : 7;
  return cfg;
}

// The picked configs (3, 4, 7) with the ResNet's epilogues compiled in:
// conv + BN + ReLU, + residual + ReLU, projection conv + BN (f16x2: the four
// residual / ReLU combinations of H2_EP).
template <int WM, int WN, int FM, int FN, int BK, int AM, int MINB, int MF16 = 0, int SP = 2, int NSTG = 2,
          int ACC1 = 0, int IL = 0>
static hipError_t launch_s3_ep(const GemmArgs& g, hipStream_t s, int n_cu, int st) {
  if constexpr (SP == 2) {
    switch (ep_flags(g) & (EP_RES | EP_RELU)) {
      case EP_RELU:
        return launch_s3_t<WM, WN, FM, FN, BK, AM, MINB, MF16, H2_EP | EP_RELU, 2, NSTG, 0, ACC1, IL>(g, s, n_cu, st);
      case EP_RES | EP_RELU:
        return launch_s3_t<WM, WN, FM, FN, BK, AM, MINB, MF16, H2_EP | EP_RES | EP_RELU, 2, NSTG, 0, ACC1, IL>(g, s,
                                                                                                             n_cu, st);
      case EP_RES:
        return launch_s3_t<WM, WN, FM, FN, BK, AM, MINB, MF16, H2_EP | EP_RES, 2, NSTG, 0, ACC1, IL>(g, s, n_cu, st);
      default: return launch_s3_t<WM, WN, FM, FN, BK, AM, MINB, MF16, H2_EP, 2, NSTG, 0, ACC1, IL>(g, s, n_cu, st);
    }
  } else {
    static_assert(SP == 2, "launch_s3_ep: the f16x2 split only (ABI 6)");
  }
}

template <int AM>
static hipError_t launch_h2_am(const GemmArgs& g, hipStream_t s, int forced, int n_cu, int st) {
  // the N = 64 halo tile as a persistent stream: the default (s3_cfg 13
  // forces the one-tile form); 64@56 3x3 1.212 -> 1.161 ms, bit-identical
  // (profiles/r05w_sweep.txt; the embed 68.26 / 68.22 ms, r05w_e2e.txt)
  const bool hpers = forced == 0;
  // dense A past config 15's 32-bit byte offsets (A or C of 4 GB or more:
  // C2's 1024-px gallery batches at layer 1, 6.4 GB at batch 128) ran config
  // 7 / 11 instead: the GEMM now goes in row chunks that fit, each a config-15
  // launch on offset pointers (chunks of 256-row multiples keep the one-launch
  // tiling, so every row is the one launch's).  256->64 at 128 x 256 x 192:
  // 1.738 -> 1.575 ms, 256->128 2.204 -> 2.136 (profiles/r06ze_dense4gb_ab.txt)
  if constexpr (AM == A_DENSE) {
    const bool q_shape = ((g.N % 256) == 0 && g.K >= 256) || (g.N == 128 && g.K >= 256) || (g.N == 64 && g.K >= 64);
    if ((forced == 15 || forced == 0) && q_shape && !s3q_fits(g)) {
      const long long per = ((1LL << 32) - 1) / (4LL * std::max(g.lda, g.ldc)) / 256 * 256;
      if (per >= 256) {
        for (long long m0 = 0; m0 < g.M; m0 += per) {
          GemmArgs c = g;
          c.M = (int)std::min<long long>(per, g.M - m0);
          c.A = g.A + m0 * g.lda;
          c.C = g.C + m0 * g.ldc;
          if (g.residual != nullptr) c.residual = g.residual + m0 * g.ldc;
          if (const hipError_t e = launch_h2_am<AM>(c, s, forced, n_cu, st)) return e;
        }
        return hipSuccess;
      }
    }
  }
  // config 15 (config 12 as a persistent k-stream): the pick for dense A
  // with config 12's shape condition (forced 15: the same, every other GEMM
  // on the library's pick; forced 12 runs config 12).  Measured at 1280
  // images (profiles/r05f_cfg15_sweep.txt, interleaved): 256->1024 + residual
  // x22 0.704 -> 0.569 ms, 512->2048 0.513 -> 0.432, 1024->256 0.409 ->
  // 0.384, 2048->512 0.357 -> 0.351; the bench's embed 70.49 -> 69.05 ms
  // (r05f_cfg15_e2e.txt; residual layers only: 69.17)
  if (forced == 15 || forced == 0) {
    if constexpr (AM == A_DENSE) {
      if ((g.N % 256) == 0 && g.K >= 256 && s3q_fits(g)) {
        // residual epilogues streamed (EP_SC1): output stores sc1, residual
        // loads nt -- neither keeps XCD L2 lines the row tile's other column
        // tiles still re-read (256->1024 + residual 0.604 -> 0.579 ms, 512->2048
        // 0.470 -> 0.466; the embed 69.82 -> 69.47 ms with every config-15
        // layer streamed).  Without a residual the plain policy stays: streamed
        // stores there ran 1024->256 0.395 -> 0.406 ms (profiles/r05i_sweep.txt,
        // r05j_probe2.txt)
        switch (ep_flags(g) & (EP_RES | EP_RELU)) {
          case EP_RELU: return launch_s3q_t<H2_EP | EP_RELU>(g, s, n_cu, st);
          case EP_RES | EP_RELU: return launch_s3q_t<H2_EP | EP_RES | EP_RELU | EP_SC1>(g, s, n_cu, st);
          case EP_RES: return launch_s3q_t<H2_EP | EP_RES | EP_SC1>(g, s, n_cu, st);
          default: return launch_s3q_t<H2_EP>(g, s, n_cu, st);
        }
      }
      if (g.N == 128 && g.K >= 256 && s3q_fits(g)) {
        switch (ep_flags(g) & (EP_RES | EP_RELU)) {
          case EP_RELU: return launch_s3q_t<H2_EP | EP_RELU, 1>(g, s, n_cu, st);
          case EP_RES | EP_RELU: return launch_s3q_t<H2_EP | EP_RES | EP_RELU | EP_SC1, 1>(g, s, n_cu, st);
          case EP_RES: return launch_s3q_t<H2_EP | EP_RES | EP_SC1, 1>(g, s, n_cu, st);
          default: return launch_s3q_t<H2_EP, 1>(g, s, n_cu, st);
        }
      }
      if (g.N == 64 && g.K >= 64 && s3q_fits(g)) {
        switch (ep_flags(g) & (EP_RES | EP_RELU)) {
          case EP_RELU: return launch_s3q_t<H2_EP | EP_RELU, 1, 4, 1>(g, s, n_cu, st);
          case EP_RES | EP_RELU: return launch_s3q_t<H2_EP | EP_RES | EP_RELU | EP_SC1, 1, 4, 1>(g, s, n_cu, st);
          case EP_RES: return launch_s3q_t<H2_EP | EP_RES | EP_SC1, 1, 4, 1>(g, s, n_cu, st);
          default: return launch_s3q_t<H2_EP, 1, 4, 1>(g, s, n_cu, st);
        }
      }
    }
    if (forced == 15) forced = 0;
  }
  // the halo-A tile (configs 13 / 14) is the pick for N % 256 == 0 and N == 64: the 3x3
  // 256@14 and 512@7 layers 2.7 % / 1.6 % faster than config 12 at 1280
  // images (profiles/r03t_h2_cfg_sweep.txt)
  if constexpr (AM == A_CONV) {
    // (N == 64 too: the 256x64 instance with three taps per barrier runs the
    // 64@56 3x3 layers 1.455 -> 1.297 ms; the 256x128 one lost on 128@28,
    // 0.888 -> 0.922 ms, and stays opt-in; profiles/r03w_h2_cfg_sweep.txt)
    // The 256x256 instance (hr 288, the N % 256 layers) runs on
    // v_mfma_f32_16x16x32_f16 by default: 256@14 0.716 -> 0.675 ms, 512@7
    // 0.671 -> 0.606; the 256x64 one lost on 64@56 (1.225 -> 1.334 ms) and
    // keeps the 32x32x16 form (profiles/r04c_h2_cfg_sweep.txt).  Forcing 13
    // selects the 32x32x16 form everywhere, 14 the 16x16x32 form everywhere.
    // Round 6: N = 128 too (the 256x128 instance on 16x16x32): 128@28 1.035 ->
    // 0.931 ms against config 11 at 1280 images, after the halo tiles' taps
    // became compile-time (profiles/r06w_halo128_ab.txt)
    // halo_2d: the 2-D block tiles where no raster halo holds the map (-1),
    // wherever one serves (1), never (0)
    if (forced == 0 && g.halo_2d != 0 && h2_halo_2d_ok(g) && (g.halo_2d == 1 || !h2_halo_rows(g)))
      return launch_h2_halo_2d(g, s);
    if (forced == 13 || forced == 14 || (forced == 0 && ((g.N % 256) == 0 || g.N == 64 || g.N == 128))) {
      if (const int hr = h2_halo_rows(g))
        return launch_h2_halo(g, s, hr,
                              forced == 14 ? 1 : forced == 13 ? 0 : g.halo_mf >= 0 ? g.halo_mf : (hr == 288 || hr == 320 ? 1 : 0),
                              hpers, n_cu);
    }
  }
  if (forced == 13 || forced == 14) forced = 0;
  int cfg = pick_h2(g, forced);
  // (dense A: config 15 above, config 12 as a persistent k-stream)
  // N % 256 == 0: the 256x256 one-accumulator tile (config 12) everywhere but
  // the short-K residual expansions (K < 256: their epilogue dominates and the
  // persistent k-stream, config 8, hides part of it).  Measured per R101 layer
  // at 1280 images (profiles/r03p_h2_cfg_sweep.txt): 3x3 256@14 0.848 -> 0.794
  // ms, 1024->256 0.432 -> 0.400, 512@7 0.778 -> 0.707, 2048->512 0.393 ->
  // 0.350, 256->1024 (residual) 0.690 -> 0.676; 128->512 / 64->256 (residual,
  // K 128 / 64) 17 % / 8 % slower, so those keep config 8.  K < 256 without a
  // residual keeps the two-accumulator tiles too: on a K = 64 conv the single
  // accumulator's max error (2.7e-7 Sigma|ab|) exceeded the exact-fp32 core's
  // (2.2e-7), the bar of tests/test_gpu_h2.py (no such layer in the R101
  // trunk: its K = 64 projection runs fused, rr_bottleneck_out_h2).
  const bool big = (g.N % 256) == 0 && g.K >= 256;
  if (forced == 0 && big) cfg = 12;
  else if (forced == 0 && AM == A_DENSE && s3_persist_ok<2>(g, AM)) cfg = 8;
  if (cfg == 8) {
    if constexpr (AM == A_DENSE) {
      if (s3_persist_ok<2>(g, AM)) return launch_s3p<2>(g, s, n_cu, st);
    }
    cfg = pick_h2(g, 0);
  }
  switch (cfg) {
    case 4: return launch_s3_ep<2, 4, 2, 2, 32, AM, 1, 1, 2>(g, s, n_cu, st);
    case 9: return launch_s3_ep<2, 4, 2, 2, 32, AM, 1, 1, 2, 3>(g, s, n_cu, st);
    case 10: return launch_s3_ep<2, 4, 2, 2, 32, AM, 1, 1, 2, 2, 1>(g, s, n_cu, st);
    case 11: return launch_s3_ep<2, 2, 2, 2, 32, AM, 2, 1, 2, 2, 1>(g, s, n_cu, st);
    case 12:
      if constexpr (AM != A_CONV_C4) {
        if (g.issue_spread) return launch_s3_ep<2, 4, 4, 2, 32, AM, 1, 0, 2, 2, 1, 1>(g, s, n_cu, st);
      }
      return launch_s3_ep<2, 4, 4, 2, 32, AM, 1, 0, 2, 2, 1>(g, s, n_cu, st);
    case 7: return launch_s3_ep<8, 1, 1, 2, 16, AM, 4, 0, 2>(g, s, n_cu, st);
    default: return launch_s3_ep<4, 2, 2, 2, 32, AM, 1, 0, 2>(g, s, n_cu, st);
  }
}

int launch_gemm_h2_seg2(rr_handle_s* h, const GemmArgs& g, hipStream_t s, int timer_cls) {
  if (g.M < 0 || g.N <= 0 || g.K <= 0 || g.K1 <= 0 || g.K1 >= g.K || (g.K % 32) || (g.K1 % 32) || (g.N % 256))
    return set_error(h, RR_EINVAL, "gemm_h2_seg2: K1, K - K1 multiples of 32 and N % 256 == 0");
  if ((g.lda & 3) || (g.lda2 & 3) || ((uintptr_t)g.A & 15) || ((uintptr_t)g.A2 & 15) || g.OH <= 0 || g.OW <= 0 ||
      g.s2 <= 0 || (long long)(g.OH - 1) * g.s2 >= g.H2 || (long long)(g.OW - 1) * g.s2 >= g.W2)
    return set_error(h, RR_EINVAL, "gemm_h2_seg2: bad A / A2 layout");
  if (g.col_scale == nullptr || g.a_amax == nullptr || g.a2_amax == nullptr || g.residual != nullptr ||
      g.relu != 1 || g.out_bf16 || (g.ldb & 7) || (g.b_plane & 7) || ((uintptr_t)g.B & 15) ||
      ((uintptr_t)g.col_scale & 15))
    return set_error(h, RR_EINVAL, "gemm_h2_seg2: ReLU epilogue, scales and both max-|x| records");
  if (g.M == 0) return RR_OK;
  hipError_t e;
  {
    TimedLaunch tl(h, timer_cls, s);
    e = launch_s3p_t<H2_EP | EP_RELU, 2, 1>(g, s, device_cu_count(h), h->tune.s3_stagger >= 0 ? h->tune.s3_stagger : 0);
  }
  return check_hip(h, e, "gemm_h2_seg2 launch");
}

// ---- The stem (7x7 / 2, pad 3, NHWC4) + ReLU + 3x3 / 2 max-pool as a halo
// tile (f16x2) ---------------------------------------------------------------
// The implicit-GEMM stem reads each input pixel's 16 B once per filter tap
// that covers it (~12x at stride 2) plus the 64 x 224 weight planes for every
// 256-row tile (more bytes than the tile's whole input patch).  Here one
// persistent block per CU keeps both weight planes resident in LDS (loaded
// once) and, per tile, stages the tile's input patch once: the tile is the
// same 17 x 15 patch of conv outputs (8 x 7 pooled outputs plus their window
// halo) as the fused config-7 stem, so its input is a 39 x 35-pixel patch,
// fetched once (one 16-B load per pixel, zero outside the image) and split
// into two fp16 planes of 4 channels (8 B per pixel).  The k-loop then reads
// only LDS and has no barrier: k-step s = taps 4s .. 4s + 3 (16 k), lane half
// h supplies taps 4s + 2h, 4s + 2h + 1 (one ds_read_b64 each per plane), taps
// past 49 read a zero pixel (their weight columns are zero as well).  Same
// per-accumulator products and order as the fused config-7 stem (a0b0 into
// one set; a0b1, a1b0 into the other; 32x32x16 f16) over taps 0..51 instead of
// 0..55 (the four dropped k-steps add exact zeros).  The next tile's patch is
// loaded into registers under the k-loop; the pool epilogue stages the raw
// accumulators through LDS exactly as the config-7 stem does.
// Round 6 (PMC on this launch alone, profiles/r06y_halo_stem_pmc.txt: MFMA
// busy 0.36, 3.3 LDS bank-conflict cycles per MFMA, four barriers per tile):
//  - the C staging has its own LDS region (B 58 KB + patch 22 KB + C 68 KB),
//    so tile i's pool epilogue (its LDS reads, the max / scale / bias / ReLU
//    and the stores) runs inside tile i + 1's k-loop, between its k-steps,
//    instead of after it with the matrix cores idle; two barriers per tile;
//  - patch row hr keeps its even columns in slots 0..17 and its odd ones in
//    18..34 (row stride 36 slots): a lane row reads every other pixel of a
//    patch row, so consecutive lanes now read consecutive 8-B slots, where
//    the raster layout put them 16 B apart (two lanes per bank pair).
// Same products, order and epilogue arithmetic: bit-identical output.
// NW = 4: four waves of 64 rows x 64 columns instead of eight of 32 x 64
// (every wave reads the whole B operand each k-step: 32 KB of fragments per
// k-step through LDS instead of 48 KB for the same MFMAs).  Bit-identical, and
// measured slower: 2.20 vs 1.68 ms at 1280 images (one wave per SIMD leaves
// nothing to cover the LDS latency; profiles/r06m_stem_4wave_ab.txt), so the
// launch keeps NW = 8.
// BREG: the weights in registers instead of LDS.  8 waves as 4 row groups of
// 64 rows x 2 column groups of 32: a wave's B fragments for all 13 k-steps
// (its 32 columns, both planes: 104 VGPRs) are loaded once per block, so the
// k-loop reads only the patch from LDS, 4 KB of fragments per wave and k-step
// instead of 6 KB for the same six MFMAs.  Same products and order per
// accumulator: bit-identical.  BREG 1 spills (33 VGPRs; 16 even with the
// pool items out of the k-loop).  BREG 2, the launch's form: only the high
// plane in registers (52 VGPRs; it feeds two of the three products), the low
// plane still read from LDS, 5 KB per wave and k-step; 256 VGPRs, no spill.
// 1.759 -> 1.715 ms at 1280 images, bit-identical
// (profiles/r06zd_stem_breg_ab.txt).
template <int EPI, int NW = 8, int BREG = 0>
__global__ __launch_bounds__(64 * NW, 1) void stem_pool_halo_kernel(GemmArgs g, int ntiles) {
  constexpr int NT = 64 * NW, BN = 64, HR = 39, HC = 35, HP = HR * HC;  // 1365 patch pixels
  constexpr int WR = BREG ? 64 : 256 / NW, FM = WR / 32;  // rows per wave, 32-row MFMA tiles per wave
  constexpr int JN = BREG ? 1 : 2;                        // 32-column MFMA tiles per wave
  static_assert(NW == 8 || (NW == 4 && !BREG), "8 waves of 32 rows or 4 of 64");
  constexpr int HS = 36, HPS = HR * HS;       // patch slots per row / in all (even | odd columns), zero slot HPS
  constexpr int KP = 224, BS = KP + 8;        // weight row (k) length; LDS row stride (u16, padded)
  constexpr int NKS = 13;                     // k-steps of 4 taps (taps 0..51)
  constexpr int B_U16 = BREG == 1 ? 0 : 2 * BN * BS;  // both weight planes
  constexpr int A_U16 = 2 * (HPS + 1) * 4;    // both patch planes + the zero slot
  constexpr int CS = BN + 4;                  // C staging row stride (floats)
  constexpr int C_U16 = 256 * CS * 2;
  constexpr int A_PASS = (HP + NT - 1) / NT;  // 3
  constexpr int C4 = BN / 4, NPOOL = 56 * C4;  // pool work items per tile (896)
  constexpr int QI = (NPOOL + NT - 1) / NT;     // pool items per thread (2 / 4), the last one partial
  constexpr int PS = NKS / QI;                  // k-steps between them
  __shared__ __attribute__((aligned(16))) uint16_t lds[B_U16 + A_U16 + C_U16];
  uint16_t* lb = lds;
  uint16_t* la = lds + B_U16;
  float* ct = reinterpret_cast<float*>(lds + B_U16 + A_U16);
  typedef f16x8 frag_t;
  typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 31, lh = lane >> 5;
  const int wrg = BREG ? wave % 4 : wave, wn = BREG ? wave / 4 : 0;  // the wave's row / column group
  const uint32_t a_amax_w = amax_load_slot(g.a_amax);
  float a_sc, a_isc;
  {
    uint32_t u = a_amax_w;
    const int lo = s3_opaque(lane);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const uint32_t v = (uint32_t)__builtin_amdgcn_ds_bpermute((lo ^ o) << 2, (int)u);
      u = v > u ? v : u;
    }
    const int e = __builtin_amdgcn_readfirstlane(h2_exp(__uint_as_float(u)));
    a_sc = __int_as_float((127 + e) << 23);
    a_isc = __int_as_float((127 - e) << 23);
  }

  // ---- both weight planes into LDS, once: [plane][n][k], rows padded
  // (BREG: the wave's own fragments into registers) ----
  constexpr int BRP = BREG == 1 ? 2 : 1;  // weight planes in registers
  frag_t breg[BREG ? NKS : 1][BRP];
  if constexpr (BREG != 0) {
    const uint16_t* Bp = reinterpret_cast<const uint16_t*>(g.B) + (long long)(32 * wn + lr) * g.ldb + 8 * lh;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
      for (int p = 0; p < BRP; ++p) breg[ks][p] = *reinterpret_cast<const frag_t*>(Bp + p * g.b_plane + 16 * ks);
  }
  if constexpr (BREG != 1) {
    const uint16_t* Bp = reinterpret_cast<const uint16_t*>(g.B);
    for (int i = tid; i < 2 * BN * (KP / 8); i += NT) {
      const int row = i / (KP / 8), c8 = i - row * (KP / 8);  // row = plane * 64 + n
      const int p = row / BN, n = row - p * BN;
      *reinterpret_cast<u32x4*>(lb + row * BS + c8 * 8) =
          *reinterpret_cast<const u32x4*>(Bp + p * g.b_plane + (long long)n * g.ldb + c8 * 8);
    }
  }

  const int tpi = g.pool_tr * g.pool_tc;
  // the patch of tile tl: pixel p -> input (32 pr - 5 + p / 35, 28 pc - 5 + p % 35)
  f32x4 px[A_PASS];
  auto load_patch = [&](int tl) {
    const int b = tl / tpi, t2 = tl - b * tpi, pr = t2 / g.pool_tc, pc = t2 - pr * g.pool_tc;
#pragma unroll
    for (int q = 0; q < A_PASS; ++q) {
      const int p = tid + q * NT, hr = p / HC, hc = p - hr * HC;
      const int ih = 32 * pr - 5 + hr, iw = 28 * pc - 5 + hc;
      const bool ok = tl < ntiles && p < HP && (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
      const f32x4* src = ok ? reinterpret_cast<const f32x4*>(g.A + (((long long)b * g.H + ih) * g.W + iw) * 4)
                            : s3_zero_page();
      asm volatile("global_load_dwordx4 %0, %1, off" : "=&v"(px[q]) : "v"(src) : "memory");
    }
  };
  auto store_patch = [&]() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int q = 0; q < A_PASS; ++q) {
      asm volatile("" : "+v"(px[q]));
      const int p = tid + q * NT, hr = p / HC, hc = p - hr * HC;
      const int slot = hr * HS + (hc & 1) * (HS / 2) + (hc >> 1);
      const f32x4 v = px[q] * a_sc;
      const f16x4 hi = __builtin_convertvector(v, f16x4);
      const f16x4 lo = __builtin_convertvector(v - __builtin_convertvector(hi, f32x4), f16x4);
      if (p < HP) {
        *reinterpret_cast<f16x4*>(la + slot * 4) = hi;
        *reinterpret_cast<f16x4*>(la + (HPS + 1) * 4 + slot * 4) = lo;
      }
    }
    if (tid < 2) *reinterpret_cast<uint2*>(la + tid * (HPS + 1) * 4 + HPS * 4) = uint2{0u, 0u};  // the zero slot
  };

  // lane rows: wave w owns tile rows WR w .. +WR-1 (MFMA row tile i: WR w + 32 i
  // + lane & 31); row r -> conv output (q, c) = (r / 15, r % 15) of the patch,
  // input pixel of tap (kh, kw) = (2q + kh, 2c + kw), slot (2q + kh) 36 +
  // (kw & 1) 18 + c + (kw >> 1)
  int sbase[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int row = wrg * WR + 32 * i + lr, rq = row / 15, rc = row - rq * 15;
    sbase[i] = row < 255 ? (2 * rq) * HS + rc : -1;
  }

  // ---- pool work item `it` of tile tl (C staged in ct): the pooled output
  // (8 pr + it / 16 / 7, 7 pc + it / 16 % 7), channels 4 (it % 16) .. +3: max
  // over the window's in-map conv outputs of the raw accumulators, then
  // scale, bias, ReLU (all monotone) ----
  float am = 0.f;
  auto pool_item = [&](int tl, int it) __attribute__((always_inline)) {
    const int b = tl / tpi, t2 = tl - b * tpi, pr = t2 / g.pool_tc, pc = t2 - pr * g.pool_tc;
    const int qd = it / C4, c4 = it - qd * C4, pi = qd / 7, pj = qd - 7 * pi;
    const int ph = 8 * pr + pi, pw = 7 * pc + pj;
    if (ph >= g.POH || pw >= g.POW) return;
    f32x4 mx = {-__builtin_inff(), -__builtin_inff(), -__builtin_inff(), -__builtin_inff()};
#pragma unroll
    for (int dr = -1; dr <= 1; ++dr)
#pragma unroll
      for (int dc = -1; dc <= 1; ++dc) {
        const int oh = 2 * ph + dr, ow = 2 * pw + dc;
        if ((unsigned)oh >= (unsigned)g.OH || (unsigned)ow >= (unsigned)g.OW) continue;
        const f32x4 v = *reinterpret_cast<const f32x4*>(ct + ((2 * pi + dr + 1) * 15 + 2 * pj + dc + 1) * CS + c4 * 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) mx[e] = __builtin_fmaxf(mx[e], v[e]);
      }
    const f32x4 sc = *reinterpret_cast<const f32x4*>(g.col_scale + c4 * 4) * a_isc;
    const f32x4 bv = g.bias != nullptr ? *reinterpret_cast<const f32x4*>(g.bias + c4 * 4) : f32x4{0.f, 0.f, 0.f, 0.f};
    f32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      o[e] = __builtin_fmaxf(mx[e] * sc[e] + bv[e], 0.f);
      am = amax_acc(am, o[e]);
    }
    *reinterpret_cast<f32x4*>(g.pool_out + (((long long)b * g.POH + ph) * g.POW + pw) * BN + c4 * 4) = o;
  };

  const int G = gridDim.x;
  int tl = blockIdx.x;
  int prev = -1;  // the tile whose C is staged in ct (its pool still to run)
  load_patch(tl);
  store_patch();
  __syncthreads();
  for (; tl < ntiles; tl += G) {
    load_patch(tl + G);  // the next tile's patch lands under this tile's k-loop
    f32x16 hi[FM][JN], lo[FM][JN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < JN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) hi[i][j][r] = lo[i][j][r] = 0.f;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      frag_t a[2][FM], b[2][2];
      const int t0 = 4 * ks + 2 * lh;
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        int pix[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int t = t0 + u, kh = t / 7, kw = t - kh * 7;
          pix[u] = (sbase[i] >= 0 && t < 49) ? sbase[i] + kh * HS + (kw & 1) * (HS / 2) + (kw >> 1) : HPS;
        }
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          const uint16_t* pl = la + p * (HPS + 1) * 4;
          const f16x4 x0 = *reinterpret_cast<const f16x4*>(pl + pix[0] * 4);
          const f16x4 x1 = *reinterpret_cast<const f16x4*>(pl + pix[1] * 4);
          a[p][i] = __builtin_shufflevector(x0, x1, 0, 1, 2, 3, 4, 5, 6, 7);
        }
      }
#pragma unroll
      for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int j = 0; j < JN; ++j)
          b[p][j] = (BREG == 1 || (BREG == 2 && p == 0))
                        ? breg[ks][BREG == 1 ? p : 0]
                        : *reinterpret_cast<const frag_t*>(lb + (p * BN + 32 * (j + wn) + lr) * BS + 16 * ks + 8 * lh);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < JN; ++j) hi[i][j] = s3_mf32<2>(a[0][i], b[0][j], hi[i][j]);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < JN; ++j) {
          lo[i][j] = s3_mf32<2>(a[0][i], b[1][j], lo[i][j]);
          lo[i][j] = s3_mf32<2>(a[1][i], b[0][j], lo[i][j]);
        }
      // the previous tile's pool epilogue, one work item at a time, among the MFMAs
      if (prev >= 0) {
#pragma unroll
        for (int q = 0; q < QI; ++q)
          if (ks == q * PS + PS / 2 && tid + q * NT < NPOOL) pool_item(prev, tid + q * NT);
      }
    }
    __syncthreads();  // every wave done with the patch and with ct's previous tile
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < JN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          ct[(wrg * WR + 32 * i + acc_row<false>(0, r, lane)) * CS + 32 * wn + acc_col<false>(j, r, lane)] =
              hi[i][j][r] + lo[i][j][r];
    store_patch();
    prev = tl;
    __syncthreads();
  }
  if (prev >= 0) {  // the last tile's pool
#pragma unroll
    for (int q = 0; q < QI; ++q)
      if (tid + q * NT < NPOOL) pool_item(prev, tid + q * NT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if constexpr ((EPI & EP_AMAX) != 0) {
    if (g.c_amax != nullptr) amax_publish(g.c_amax, am, blockIdx.x * NW + wave);
  }
}

int launch_stem_pool_h2(rr_handle_s* h, const GemmArgs& g, hipStream_t s, int timer_cls) {
  if (g.N != 64 || g.Cin != 4 || g.K % 32 || g.K < g.KH * g.KW * 4 || g.relu != 1 || g.residual != nullptr ||
      g.col_scale == nullptr || g.a_amax == nullptr || g.pool_out == nullptr || g.POH <= 0 || g.POW <= 0 ||
      g.pool_tr != (g.POH + 7) / 8 || g.pool_tc != (g.POW + 6) / 7 || ((uintptr_t)g.A & 15) || (g.ldb & 7) ||
      (g.b_plane & 7) || ((uintptr_t)g.B & 15) || ((uintptr_t)g.col_scale & 15) || ((uintptr_t)g.pool_out & 15))
    return set_error(h, RR_EINVAL, "stem_pool_h2: NHWC4 input, 64 output channels, ReLU, aligned operands");
  GemmArgs q = g;
  const long long tiles = (long long)(g.M / ((long long)g.OH * g.OW)) * g.pool_tr * g.pool_tc;
  if (tiles * 256 > 0x7fffffffLL) return set_error(h, RR_EINVAL, "stem_pool_h2: too many tiles");
  if (tiles == 0) return RR_OK;
  q.M = (int)(tiles * 256);  // 256 rows per tile (255 used)
  hipError_t e;
  {
    TimedLaunch tl(h, timer_cls, s);
    // the halo stem (7x7 / 2, pad 3; s3_cfg 7 forces the implicit-GEMM one)
    if (h->tune.s3_cfg != 7 && g.KH == 7 && g.KW == 7 && g.stride == 2 && g.pad == 3 && g.K == 224 && g.ldb == 224) {
      const int grid = (int)std::min<long long>(tiles, device_cu_count(h));
      hipLaunchKernelGGL((stem_pool_halo_kernel<H2_EP | EP_RELU, 8, 2>), dim3((unsigned)grid), dim3(512), 0, s, g, (int)tiles);
      e = hipGetLastError();
    } else {
      e = launch_s3_t<8, 1, 1, 2, 16, A_CONV_C4, 4, 0, H2_EP | EP_RELU, 2, 2, 1>(q, s, device_cu_count(h), 0);
    }
  }
  return check_hip(h, e, "stem_pool_h2 launch");
}

int launch_gemm_s3(rr_handle_s* h, int amode, const GemmArgs& g, hipStream_t s, int timer_cls, int sp) {
  if (g.M < 0 || g.N <= 0 || g.K <= 0) return set_error(h, RR_EINVAL, "gemm_s3: bad shape");
  if (g.K % 32) return set_error(h, RR_EINVAL, "gemm_s3: K must be a multiple of 32");
  if (amode == A_DENSE && ((g.lda & 3) || ((uintptr_t)g.A & 15)))
    return set_error(h, RR_EINVAL, "gemm_s3: dense A needs lda % 4 == 0 and 16-B alignment");
  if (amode == A_CONV && (g.Cin % 32)) return set_error(h, RR_EINVAL, "gemm_s3: conv A needs Cin % 32 == 0");
  if (amode == A_CONV_C4 && (g.Cin != 4 || g.K < g.KH * g.KW * 4 || ((uintptr_t)g.A & 15)))
    return set_error(h, RR_EINVAL, "gemm_s3: NHWC4 A needs Cin == 4, K >= KH*KW*4, 16-B alignment");
  if (amode != A_DENSE && amode != A_CONV && amode != A_CONV_C4)
    return set_error(h, RR_EINVAL, "gemm_s3: unsupported A mode");
  if ((g.ldb & 7) || (g.b_plane & 7) || ((uintptr_t)g.B & 15))
    return set_error(h, RR_EINVAL, "gemm_s3: B planes need ldb % 8 == 0, plane stride % 8 == 0, 16-B alignment");
  if (sp != 2) return set_error(h, RR_EINVAL, "gemm_h2: the f16x2 split (the bf16x3 core was retired in ABI 6)");
  if (g.col_scale == nullptr || g.a_amax == nullptr || ((uintptr_t)g.col_scale & 15))
    return set_error(h, RR_EINVAL, "gemm_h2: needs 16-B aligned column scales and the A max-|x| record");
  if (g.relu == 2 || g.out_bf16 || (g.N & 3) || (g.ldc & 3))
    return set_error(h, RR_EINVAL, "gemm_h2: fp32 output, ReLU or none, N % 4 == 0");
  if (g.M == 0) return RR_OK;
  // default stagger: the residual layers only (their 256 KB-per-tile epilogue
  // is the HBM-heavy phase): 256->1024 x23 -5 %, the other residual layers
  // -1 %, the rest neutral to +2 % (tools/ab_trunk.sh stagger, profiles/r02f_s3_stagger.txt)
  const int st = h->tune.s3_stagger >= 0 ? h->tune.s3_stagger : (g.residual != nullptr ? 8 : 0);
  hipError_t e;
  {
    TimedLaunch tl(h, timer_cls, s);
    const int f = (g.residual != nullptr && h->tune.s3_cfg_res > 0) ? h->tune.s3_cfg_res : h->tune.s3_cfg;
    const int n_cu = device_cu_count(h);
    {
      // conv_il (opt-in): every R101 layer the 256x256 tile serves ran 1-3 %
      // faster alone at 1280 images (256->1024 0.681 -> 0.668 ms; profiles/
      // r04g_h2_cfg_il.txt, r04h_h2_cfg_il.txt), but the bench's whole embed
      // ran 0.5 % slower with it (71.77 -> 72.11 ms, r04j_e2e_ab.txt; limited
      // to the GEMMs without a residual, 1.0 % slower, r04s_e2e_conv_il.txt).
      // It also selects the halo tile's 16x16x32 form with its B DMA spread.
      GemmArgs g2 = g;
      g2.issue_spread = h->tune.conv_il == 1;
      g2.halo_mf = h->tune.halo_mf;
      g2.halo_2d = h->tune.halo_2d;
      e = amode == A_DENSE ? launch_h2_am<A_DENSE>(g2, s, f, n_cu, st)
          : amode == A_CONV ? launch_h2_am<A_CONV>(g2, s, f, n_cu, st)
                            : launch_h2_am<A_CONV_C4>(g2, s, f, n_cu, st);
    }
  }
  return check_hip(h, e, "gemm_h2 launch");
}

// ---- weight split, f16x2: row n of w [rows][k] at scale 2^e_n (h2_exp of
// the row's max |w|) -> planes [2][rows][kpad] (zero past k), iscale[n] ----
__global__ __launch_bounds__(256) void split2h_kernel(const float* __restrict__ w, int rows, int k, int kpad,
                                                      uint16_t* __restrict__ planes, float* __restrict__ iscale) {
  __shared__ float red[4];
  const int n = blockIdx.x, tid = threadIdx.x;
  const float* wr = w + (long long)n * k;
  float am = 0.f;
  for (int i = tid; i < k; i += 256) am = amax_acc(am, wr[i]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) am = fmaxf(am, __shfl_xor(am, o));
  if ((tid & 63) == 0) red[tid >> 6] = am;
  __syncthreads();
  am = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  const int e = h2_exp(am);
  const float sc = __builtin_amdgcn_ldexpf(1.f, e);
  if (tid == 0) iscale[n] = __builtin_amdgcn_ldexpf(1.f, -e);
  const long long plane = (long long)rows * kpad;
  uint16_t* p0 = planes + (long long)n * kpad;
  for (int i = tid; i < kpad; i += 256) {
    const float v = i < k ? wr[i] * sc : 0.f;
    const _Float16 hi = (_Float16)v;
    const _Float16 lo = (_Float16)(v - (float)hi);
    p0[i] = __builtin_bit_cast(uint16_t, hi);
    p0[plane + i] = __builtin_bit_cast(uint16_t, lo);
  }
}

int launch_split2h(rr_handle_s* h, const float* w, int rows, int k, int kpad, uint16_t* planes, float* iscale,
                   hipStream_t s) {
  if (rows <= 0) return RR_OK;
  hipLaunchKernelGGL(split2h_kernel, dim3((unsigned)rows), dim3(256), 0, s, w, rows, k, kpad, planes, iscale);
  return check_hip(h, hipGetLastError(), "split2h launch");
}

// ---- max |x| of a tensor into its RR_AMAX_SLOTS-word record ----
__global__ __launch_bounds__(256) void amax_kernel(const float* __restrict__ x, long long n, uint32_t* slots) {
  float am = 0.f;
  const long long gs = (long long)gridDim.x * blockDim.x;
  const long long i0 = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (((uintptr_t)x & 15) == 0) {
    const long long n4 = n >> 2;
    const f32x4* x4 = reinterpret_cast<const f32x4*>(x);
    for (long long i = i0; i < n4; i += gs) {
      const f32x4 v = x4[i];
      am = amax_acc(amax_acc(am, v[0]), v[1]);
      am = amax_acc(amax_acc(am, v[2]), v[3]);
    }
    for (long long i = (n4 << 2) + i0; i < n; i += gs) am = amax_acc(am, x[i]);
  } else {
    for (long long i = i0; i < n; i += gs) am = amax_acc(am, x[i]);
  }
  amax_publish(slots, am, blockIdx.x * 4 + (threadIdx.x >> 6));
}

int launch_amax(rr_handle_s* h, const float* x, long long n, uint32_t* slots, hipStream_t s) {
  if (n <= 0) return RR_OK;
  const long long blocks = std::min<long long>((n / 4 + 255) / 256 + 1, 2048);
  hipLaunchKernelGGL(amax_kernel, dim3((unsigned)blocks), dim3(256), 0, s, x, n, slots);
  return check_hip(h, hipGetLastError(), "amax launch");
}

#if RR_S3_PHASES
// diagnostic build: read and clear the phase sums ([4][8] cycles)
int debug_phases(unsigned long long* out) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(s3_phase_sum), sizeof(s3_phase_sum)) != hipSuccess) return RR_EHIP;
  unsigned long long z[4][8] = {};
  return hipMemcpyToSymbol(HIP_SYMBOL(s3_phase_sum), z, sizeof(z)) == hipSuccess ? RR_OK : RR_EHIP;
}
#endif

}  // namespace rr

#if RR_S3_PHASES
extern "C" int rr_debug_phases(unsigned long long* out) { return rr::debug_phases(out); }
#endif
