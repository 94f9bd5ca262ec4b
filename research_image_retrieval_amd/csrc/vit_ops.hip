// vit_ops.hip — CLIP-style ViT pieces for gfx950 (networks/model.py:157-243):
// LayerNorm (fp32, :157-163), patchify for the 16x16/16 patch conv (:223),
// class/positional token assembly (:226-227) and a fused multi-head
// attention (nn.MultiheadAttention inside ResidualAttentionBlock, :171-188).
// The projections (QKV, out-proj, MLP with QuickGELU, ln_post @ proj) run on
// the fp32 MFMA GEMM core (gemm_f32.hip).
#include "rr_internal.hpp"

namespace rr {

// softmax exp on the hardware exp2 (v_exp_f32, ~1 ulp; the libm expf costs
// ~15 VALU per score, 7 G scores per C4 step): x <= 0 here (score - row max)
__device__ __forceinline__ float fast_exp(float x) { return __builtin_amdgcn_exp2f(x * 1.4426950408889634f); }


typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// One wave per row: y = (x - mean) / sqrt(var + eps) * gamma + beta, biased
// variance, two-pass over the row held in registers (D <= 64 * 64).  The row
// body is shared with the generic-width fused token assembly below.
template <int PER_LANE, typename OutT>
__device__ __forceinline__ void ln_row(const float (&v)[PER_LANE], int lane, int D, const float* __restrict__ gamma,
                                       const float* __restrict__ beta, float eps, OutT* __restrict__ yr) {
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < PER_LANE; ++i) s += v[i];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  const float mean = s / (float)D;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < PER_LANE; ++i) {
    const int c = lane + 64 * i;
    const float d = c < D ? v[i] - mean : 0.f;
    q = fmaf(d, d, q);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) q += __shfl_xor(q, off, 64);
  const float rstd = 1.0f / sqrtf(q / (float)D + eps);
#pragma unroll
  for (int i = 0; i < PER_LANE; ++i) {
    const int c = lane + 64 * i;
    if (c < D) yr[c] = (OutT)((v[i] - mean) * rstd * gamma[c] + beta[c]);
  }
}

template <int PER_LANE, typename OutT>
__global__ __launch_bounds__(256) void layernorm_kernel(const float* __restrict__ x, long long ldx, int M, int D,
                                                        const float* __restrict__ gamma,
                                                        const float* __restrict__ beta, float eps,
                                                        OutT* __restrict__ y) {
  const int row = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (row >= M) return;
  const float* xr = x + (long long)row * ldx;
  float v[PER_LANE];
#pragma unroll
  for (int i = 0; i < PER_LANE; ++i) {
    const int c = lane + 64 * i;
    v[i] = c < D ? xr[c] : 0.f;
  }
  ln_row<PER_LANE>(v, lane, D, gamma, beta, eps, y + (long long)row * D);
}

// Token assembly with ln_pre fused for any width <= 4096 (the 512 / 768
// vectorised forms are vit_tokens_ln_kernel below): the row (cls or patch
// embedding, + positional embedding) is formed in registers and normalised
// there, with layernorm_kernel's row body — the same bits as assembling the
// tokens and normalising them in a separate pass, without writing y twice.
template <int PER_LANE>
__global__ __launch_bounds__(256) void vit_tokens_ln_generic_kernel(const float* __restrict__ patches, int B, int NP,
                                                                    int D, const float* __restrict__ cls,
                                                                    const float* __restrict__ pos,
                                                                    const float* __restrict__ gamma,
                                                                    const float* __restrict__ beta, float eps,
                                                                    float* __restrict__ y) {
  const long long t = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (t >= (long long)B * (NP + 1)) return;
  const int l = (int)(t % (NP + 1));
  const long long b = t / (NP + 1);
  const float* src = l == 0 ? cls : patches + (b * NP + (l - 1)) * D;
  const float* pr = pos + (long long)l * D;
  float v[PER_LANE];
#pragma unroll
  for (int i = 0; i < PER_LANE; ++i) {
    const int c = lane + 64 * i;
    v[i] = c < D ? src[c] + pr[c] : 0.f;
  }
  ln_row<PER_LANE>(v, lane, D, gamma, beta, eps, y + t * D);
}

// Same, vectorised for D % 256 == 0 and 16-B aligned rows (ViT width 768):
// lane l holds the float4s at columns 4l + 256i, so every load and store is
// one 1-KB (fp32) or 512-B (bf16) coalesced wave instruction.
// The row body is shared with the fused token-assembly kernel below so both
// give bit-identical rows.
template <int NV, typename OutT>
__device__ __forceinline__ void ln_row_vec(const f32x4 (&v)[NV], int lane, const float* __restrict__ gamma,
                                           const float* __restrict__ beta, float eps, OutT* __restrict__ yr) {
  constexpr int D = 256 * NV;
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) s += (v[i][0] + v[i][1]) + (v[i][2] + v[i][3]);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  const float mean = s / (float)D;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float d = v[i][e] - mean;
      q = fmaf(d, d, q);
    }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) q += __shfl_xor(q, off, 64);
  const float rstd = 1.0f / sqrtf(q / (float)D + eps);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = 4 * lane + 256 * i;
    const f32x4 gm = *reinterpret_cast<const f32x4*>(gamma + c);
    const f32x4 bt = *reinterpret_cast<const f32x4*>(beta + c);
    f32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = (v[i][e] - mean) * rstd * gm[e] + bt[e];
    if constexpr (sizeof(OutT) == 4) {
      *reinterpret_cast<f32x4*>(yr + c) = o;
    } else {
      typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
      *reinterpret_cast<bf16x4*>(yr + c) = bf16x4{(__bf16)o[0], (__bf16)o[1], (__bf16)o[2], (__bf16)o[3]};
    }
  }
}

template <int NV, typename OutT>
__global__ __launch_bounds__(256) void layernorm_vec_kernel(const float* __restrict__ x, long long ldx, int M,
                                                            const float* __restrict__ gamma,
                                                            const float* __restrict__ beta, float eps,
                                                            OutT* __restrict__ y) {
  const int row = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (row >= M) return;
  const float* xr = x + (long long)row * ldx;
  f32x4 v[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) v[i] = *reinterpret_cast<const f32x4*>(xr + 4 * lane + 256 * i);
  ln_row_vec<NV>(v, lane, gamma, beta, eps, y + (long long)row * (256 * NV));
}

// The LayerNorm partials of rr_linear_bf16_ln for rows no GEMM produced: one
// wave per (row, 256-column tile), the same arithmetic as the GEMM epilogue's
// EP_STATS (gemm_epilogue.hpp store_slab): bf16 copy, tile mean, then
// M2 = sum (x - mean)^2, each a 64-lane butterfly sum of per-lane 4-sums.
__global__ __launch_bounds__(256) void ln_partials_kernel(const float* __restrict__ x, int M, int D,
                                                          uint16_t* __restrict__ xb, float* __restrict__ st) {
  typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
  const int T = D >> 8;
  const long long w = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (w >= (long long)M * T) return;
  const long long row = w / T;
  const int t = (int)(w - row * T);
  const long long o = row * D + 256 * t + 4 * lane;
  const f32x4 v = *reinterpret_cast<const f32x4*>(x + o);
  const float mt = wave_sum((v[0] + v[1]) + (v[2] + v[3])) * (1.0f / 256.0f);
  const f32x4 dv = v - mt;
  // the bf16 rows are centred on their tile's mean (see rr_linear_bf16_ln)
  *reinterpret_cast<bf16x4*>(xb + o) = bf16x4{(__bf16)dv[0], (__bf16)dv[1], (__bf16)dv[2], (__bf16)dv[3]};
  const float m2 = wave_sum((dv[0] * dv[0] + dv[1] * dv[1]) + (dv[2] * dv[2] + dv[3] * dv[3]));
  if (lane == 0) *reinterpret_cast<float2*>(st + w * 2) = float2{mt, m2};
}

// Token assembly with ln_pre fused (:226-229): one wave per token row, the
// row (cls or patch embedding, + positional embedding) is formed in registers
// and normalised there, so the un-normalised tokens never reach HBM.  Same
// adds and the same LN body as vit_tokens_kernel + layernorm_vec_kernel.
template <int NV>
__global__ __launch_bounds__(256) void vit_tokens_ln_kernel(const float* __restrict__ patches, int B, int NP,
                                                            const float* __restrict__ cls,
                                                            const float* __restrict__ pos,
                                                            const float* __restrict__ gamma,
                                                            const float* __restrict__ beta, float eps,
                                                            float* __restrict__ y) {
  constexpr int Wd = 256 * NV;
  const long long t = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (t >= (long long)B * (NP + 1)) return;
  const int l = (int)(t % (NP + 1));
  const long long b = t / (NP + 1);
  const float* src = l == 0 ? cls : patches + (b * NP + (l - 1)) * Wd;
  const float* pr = pos + (long long)l * Wd;
  f32x4 v[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = 4 * lane + 256 * i;
    v[i] = *reinterpret_cast<const f32x4*>(src + c) + *reinterpret_cast<const f32x4*>(pr + c);
  }
  ln_row_vec<NV>(v, lane, gamma, beta, eps, y + t * Wd);
}

// Vectorised patchify for (P*C) % 4 == 0, (W*C) % 4 == 0 and 16-B aligned
// buffers (224x224x3, P = 16): each thread moves 4 consecutive outputs, which
// lie in one (kh) row of the patch and are contiguous in the NHWC input too,
// so the index math runs once per float4.  OutT = __bf16 writes the rows the
// bf16 patch GEMM reads directly (RNE, as rr_quantize_rows rounds).
template <typename OutT>
__global__ void patchify_vec_kernel(const float* __restrict__ x, int B, int H, int W, int C, int P,
                                    OutT* __restrict__ y) {
  const int gh = H / P, gw = W / P;
  const int pc = P * C;
  const int kdim4 = P * pc / 4;
  const long long total4 = (long long)B * gh * gw * kdim4;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x; q < total4; q += stride) {
    const long long patch = q / kdim4;
    const int k = 4 * (int)(q - patch * kdim4);
    const int kh = k / pc;
    const int r = k - kh * pc;
    const int b = (int)(patch / (gh * gw));
    const int pp = (int)(patch - (long long)b * gh * gw);
    const int ph = pp / gw, pw = pp - ph * gw;
    const f32x4 v =
        *reinterpret_cast<const f32x4*>(x + (((long long)b * H + ph * P + kh) * W + pw * P) * C + r);
    if constexpr (sizeof(OutT) == 4) {
      *reinterpret_cast<f32x4*>(y + 4 * q) = v;
    } else {
      typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
      *reinterpret_cast<bf16x4*>(y + 4 * q) = bf16x4{(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
    }
  }
}

// NHWC [B][H][W][C] -> patch rows [B*(H/P)*(W/P)][P*P*C] in (kh, kw, c) order,
// which matches conv weights permuted to [Cout][P][P][C].
template <typename OutT>
__global__ void patchify_kernel(const float* __restrict__ x, int B, int H, int W, int C, int P,
                                OutT* __restrict__ y) {
  const int gh = H / P, gw = W / P;
  const long long kdim = (long long)P * P * C;
  const long long total = (long long)B * gh * gw * kdim;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long o = (long long)blockIdx.x * blockDim.x + threadIdx.x; o < total; o += stride) {
    const long long patch = o / kdim;
    const int k = (int)(o - patch * kdim);
    const int kh = k / (P * C);
    const int r = k - kh * P * C;
    const int kw = r / C;
    const int c = r - kw * C;
    const int b = (int)(patch / (gh * gw));
    const int pp = (int)(patch - (long long)b * gh * gw);
    const int ph = pp / gw, pw = pp - (pp / gw) * gw;
    y[o] = (OutT)x[(((long long)b * H + ph * P + kh) * W + pw * P + kw) * C + c];
  }
}

// tokens[b][0] = cls + pos[0]; tokens[b][1+p] = patches[b][p] + pos[1+p]
__global__ void vit_tokens_kernel(const float* __restrict__ patches, int B, int NP, int Wd,
                                  const float* __restrict__ cls, const float* __restrict__ pos,
                                  float* __restrict__ y) {
  const long long total = (long long)B * (NP + 1) * Wd;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long o = (long long)blockIdx.x * blockDim.x + threadIdx.x; o < total; o += stride) {
    const int c = (int)(o % Wd);
    const long long t = o / Wd;
    const int l = (int)(t % (NP + 1));
    const long long b = t / (NP + 1);
    const float v = l == 0 ? cls[c] : patches[(b * NP + (l - 1)) * Wd + c];
    y[o] = v + pos[(long long)l * Wd + c];
  }
}

// ---------------------------------------------------------------------------
// Fused attention, head_dim 64, fp32 MFMA (v_mfma_f32_32x32x2_f32).
// Workgroup = one (batch, head); wave w owns queries [32w, 32w+32).
// K and V of the head are staged in LDS once (zero rows past seq).
//  1. S^T = K . Q^T for all NC*32 keys, kept in NC accumulator tiles: lane =
//     query, registers = keys (row map (r&3) + 8(r>>2) + 4(lane>>5)).
//  2. exact softmax per query: max / exp / sum over the lane's registers plus
//     the partner lane (lane ^ 32); padded keys masked to -inf.
//  3. O = P . V with the S^T accumulator used directly as the A operand:
//     lane (query, h) supplies P[query][key(r, h)] for MFMA step r, and the V
//     fragment is read from LDS at that same key.  O /= rowsum; store.
// Q is pre-scaled by 1/sqrt(64) = 0.125 (exact).
template <int NC, typename OutT>
__global__ __launch_bounds__(64 * NC) void attention_kernel(const float* __restrict__ qkv, int B, int L, int NH,
                                                            OutT* __restrict__ out) {
  constexpr int HD = 64;
  constexpr int LP = NC * 32;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* Ks = smem;            // [LP][HD], 16-B slots XOR-swizzled by (row & 15)
  float* Vs = smem + LP * HD;  // [LP][HD] row-major
  const int bh = blockIdx.x;
  const int b = bh / NH, h = bh - (bh / NH) * NH;
  const int width = NH * HD;
  const long long ld = 3LL * width;
  const float* base = qkv + (long long)b * L * ld;
  const int tid = threadIdx.x;
  // stage K and V: every thread's NIT = 8 groups, all loads issued before the
  // first LDS store (as attention_bf16_kernel)
  constexpr int NIT = LP * (HD / 4) / (64 * NC);
  static_assert(NIT * 64 * NC == LP * (HD / 4), "staging groups must tile the block");
  {
    f32x4 kv[NIT], vv[NIT];
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int idx = tid + it * 64 * NC;
      const int row = idx / (HD / 4), s4 = idx - row * (HD / 4);
      kv[it] = vv[it] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (row < L) {
        kv[it] = *reinterpret_cast<const f32x4*>(base + (long long)row * ld + width + h * HD + s4 * 4);
        vv[it] = *reinterpret_cast<const f32x4*>(base + (long long)row * ld + 2 * width + h * HD + s4 * 4);
      }
    }
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int idx = tid + it * 64 * NC;
      const int row = idx / (HD / 4), s4 = idx - row * (HD / 4);
      *reinterpret_cast<f32x4*>(Ks + row * HD + ((s4 ^ (row & 15)) * 4)) = kv[it];
      *reinterpret_cast<f32x4*>(Vs + row * HD + s4 * 4) = vv[it];
    }
  }
  const int wave = tid >> 6, lane = tid & 63;
  const int lr = lane & 31, lh = lane >> 5;
  const int q0 = wave * 32;
  // Q fragment: lane (j, h) holds Q[q0 + j][16c + 8h + e], c < 4, e < 8
  float qf[4][8];
  {
    const int q = q0 + lr;
    const bool ok = q < L;
    const float* qp = base + (long long)(ok ? q : 0) * ld + h * HD;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      f32x4 a = *reinterpret_cast<const f32x4*>(qp + 16 * c + 8 * lh);
      f32x4 bq = *reinterpret_cast<const f32x4*>(qp + 16 * c + 8 * lh + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        qf[c][e] = ok ? a[e] * 0.125f : 0.f;
        qf[c][4 + e] = ok ? bq[e] * 0.125f : 0.f;
      }
    }
  }
  __syncthreads();
  // 1. scores
  f32x16 st[NC];
#pragma unroll
  for (int kc = 0; kc < NC; ++kc) {
#pragma unroll
    for (int r = 0; r < 16; ++r) st[kc][r] = 0.f;
    const int krow = kc * 32 + lr;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int s0 = 4 * c + 2 * lh;
      const f32x4 k0 = *reinterpret_cast<const f32x4*>(Ks + krow * HD + ((s0 ^ (krow & 15)) * 4));
      const f32x4 k1 = *reinterpret_cast<const f32x4*>(Ks + krow * HD + (((s0 + 1) ^ (krow & 15)) * 4));
#pragma unroll
      for (int e = 0; e < 4; ++e) st[kc] = __builtin_amdgcn_mfma_f32_32x32x2f32(k0[e], qf[c][e], st[kc], 0, 0, 0);
#pragma unroll
      for (int e = 0; e < 4; ++e)
        st[kc] = __builtin_amdgcn_mfma_f32_32x32x2f32(k1[e], qf[c][4 + e], st[kc], 0, 0, 0);
    }
  }
  // 2. softmax over keys (registers x partner lane)
  float mx = -__builtin_inff();
#pragma unroll
  for (int kc = 0; kc < NC; ++kc)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int key = kc * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
      if (key >= L) st[kc][r] = -__builtin_inff();
      mx = fmaxf(mx, st[kc][r]);
    }
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  float sum = 0.f;
#pragma unroll
  for (int kc = 0; kc < NC; ++kc)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float p = fast_exp(st[kc][r] - mx);
      st[kc][r] = p;
      sum += p;
    }
  sum += __shfl_xor(sum, 32, 64);
  const float inv = 1.0f / sum;
  // 3. O = P V  (two 32-wide output tiles over head_dim 64)
  f32x16 o[2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[t][r] = 0.f;
#pragma unroll
  for (int kc = 0; kc < NC; ++kc) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int key = kc * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
      const float v0 = Vs[key * HD + lr];
      const float v1 = Vs[key * HD + 32 + lr];
      o[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(st[kc][r], v0, o[0], 0, 0, 0);
      o[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(st[kc][r], v1, o[1], 0, 0, 0);
    }
  }
  // normalise (1/sum lives in the query's lane) and store: lane = d, regs = queries
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int qi = (r & 3) + 8 * (r >> 2) + 4 * lh;
    const float iq = __shfl(inv, qi, 64);
    const int q = q0 + qi;
    if (q < L) {
      OutT* op = out + ((long long)b * L + q) * width + h * HD;
      op[lr] = (OutT)(o[0][r] * iq);
      op[32 + lr] = (OutT)(o[1][r] * iq);
    }
  }
}

// ---------------------------------------------------------------------------
// Fused attention on bf16 MFMA (v_mfma_f32_32x32x16_bf16), fp32 softmax: the
// C4 (bf16) ViT.  Same structure as attention_kernel: workgroup = (batch,
// head), wave w owns queries [32w, 32w+32), S^T = K . Q^T in NC accumulator
// tiles (lane = query, registers = keys), exact fp32 softmax in registers,
// then O = P . V with P packed to bf16 straight from the accumulator.  For PV
// MFMA step (key tile kc, half s) lane half lh supplies the keys
// kc*32 + 16s + 4lh + {0..3} and + 8 + {0..3} (the accumulator's own key
// order); V is staged transposed (Vt[d][key], 520-B rows: row d starts at
// bank 2d, so a lane group's ds_read_b64 of 32 d-rows is conflict-free) and
// read at exactly those keys.  K rows are 128 B with 16-B slots swizzled by
// (row >> 1) & 7 (conflict-free fragment reads, as the GEMM core).
// QKV rows come as fp32 (converted here, RNE) or already bf16 (InT = __bf16:
// the QKV linear's epilogue rounded them the same way, so the result is
// bit-identical and the kernel reads half the bytes)
template <typename InT>
__device__ __forceinline__ f32x4 ld4f(const InT* p) {
  if constexpr (sizeof(InT) == 4) {
    return *reinterpret_cast<const f32x4*>(p);
  } else {
    typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
    const bf16x4 v = *reinterpret_cast<const bf16x4*>(p);
    return f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
  }
}

template <int NC, typename OutT, typename InT>
__global__ __launch_bounds__(64 * NC, 2) void attention_bf16_kernel(const InT* __restrict__ qkv, int B, int L, int NH,
                                                                 OutT* __restrict__ out) {
  constexpr int HD = 64, LP = NC * 32, VS = 260;
  extern __shared__ __attribute__((aligned(16))) uint16_t sm16[];
  uint16_t* Ks = sm16;            // [LP][HD] bf16
  uint16_t* Vt = sm16 + LP * HD;  // [HD][VS] bf16
  const int bh = blockIdx.x;
  const int b = bh / NH, h = bh - (bh / NH) * NH;
  const int width = NH * HD;
  const long long ld = 3LL * width;
  const InT* base = qkv + (long long)b * L * ld;
  const int tid = threadIdx.x;
  // K / V staging: every thread handles exactly NIT = LP * 16 / (64 NC) = 8
  // four-element groups.  All 2 NIT loads are issued before the first LDS
  // store (one HBM round trip per block instead of NIT serialised ones: the
  // loop form waited for each iteration's loads before its stores)
  constexpr int NIT = LP * (HD / 4) / (64 * NC);
  static_assert(NIT * 64 * NC == LP * (HD / 4), "staging groups must tile the block");
  f32x4 kv[NIT], vv[NIT];
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int idx = tid + it * 64 * NC;
    const int row = idx / (HD / 4), s4 = idx - row * (HD / 4);
    kv[it] = vv[it] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (row < L) {
      kv[it] = ld4f(base + (long long)row * ld + width + h * HD + s4 * 4);
      vv[it] = ld4f(base + (long long)row * ld + 2 * width + h * HD + s4 * 4);
    }
  }
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int idx = tid + it * 64 * NC;
    const int row = idx / (HD / 4), s4 = idx - row * (HD / 4);
    typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
    const bf16x4 kb = {(__bf16)kv[it][0], (__bf16)kv[it][1], (__bf16)kv[it][2], (__bf16)kv[it][3]};
    *reinterpret_cast<bf16x4*>(Ks + row * HD + (((s4 >> 1) ^ ((row >> 1) & 7)) * 8) + (s4 & 1) * 4) = kb;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const __bf16 v = (__bf16)vv[it][e];
      Vt[(s4 * 4 + e) * VS + row] = __builtin_bit_cast(uint16_t, v);
    }
  }
  const int wave = tid >> 6, lane = tid & 63;
  const int lr = lane & 31, lh = lane >> 5;
  const int q0 = wave * 32;
  // Q^T fragment (B operand): lane (query, lh) holds Q[query][16c + 8lh + e] / 8
  bf16x8 qf[4];
  {
    const int q = q0 + lr;
    const bool ok = q < L;
    const InT* qp = base + (long long)(ok ? q : 0) * ld + h * HD;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const f32x4 a = ld4f(qp + 16 * c + 8 * lh);
      const f32x4 bq = ld4f(qp + 16 * c + 8 * lh + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        qf[c][e] = (__bf16)(ok ? a[e] * 0.125f : 0.f);
        qf[c][4 + e] = (__bf16)(ok ? bq[e] * 0.125f : 0.f);
      }
    }
  }
  __syncthreads();
  // Two passes over the key chunks, one 32x32 score tile live at a time (the
  // one-pass form held all NC tiles: 222 VGPRs, one workgroup per CU; now two
  // fit, so one workgroup's K/V staging overlaps the other's MFMAs).  Pass 1:
  // the row max; pass 2: the same scores again (deterministic), p = exp(s -
  // max) summed in the one-pass order, P packed to bf16, O += P V.  Output
  // bit-identical to the one-pass kernel.
  auto s_chunk = [&](int kc) {
    f32x16 st;
#pragma unroll
    for (int r = 0; r < 16; ++r) st[r] = 0.f;
    const int krow = kc * 32 + lr;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const bf16x8 kf =
          *reinterpret_cast<const bf16x8*>(Ks + krow * HD + (((2 * c + lh) ^ ((krow >> 1) & 7)) * 8));
      st = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[c], st, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int key = kc * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
      if (key >= L) st[r] = -__builtin_inff();
    }
    return st;
  };
  float mx = -__builtin_inff();
#pragma unroll 1
  for (int kc = 0; kc < NC; ++kc) {
    const f32x16 st = s_chunk(kc);
#pragma unroll
    for (int r = 0; r < 16; ++r) mx = fmaxf(mx, st[r]);
  }
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  float sum = 0.f;
  f32x16 o[2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[t][r] = 0.f;
  typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
#pragma unroll 1
  for (int kc = 0; kc < NC; ++kc) {
    f32x16 st = s_chunk(kc);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float p = fast_exp(st[r] - mx);
      st[r] = p;
      sum += p;
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      bf16x8 pf;
#pragma unroll
      for (int e = 0; e < 8; ++e) pf[e] = (__bf16)st[8 * s2 + e];
      const int k0 = kc * 32 + 16 * s2 + 4 * lh;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const uint16_t* vr = Vt + (32 * t + lr) * VS + k0;
        // (element-wise assembly from two u16x4 through bit_cast miscompiles
        // to a broadcast of element 0 under hipcc -O3: concatenate instead)
        const bf16x4 va = *reinterpret_cast<const bf16x4*>(vr);
        const bf16x4 vb = *reinterpret_cast<const bf16x4*>(vr + 8);
        const bf16x8 vf = __builtin_shufflevector(va, vb, 0, 1, 2, 3, 4, 5, 6, 7);
        o[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pf, vf, o[t], 0, 0, 0);
      }
    }
  }
  sum += __shfl_xor(sum, 32, 64);
  const float inv = 1.0f / sum;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int qi = (r & 3) + 8 * (r >> 2) + 4 * lh;
    const float iq = __shfl(inv, qi, 64);
    const int q = q0 + qi;
    if (q < L) {
      OutT* op = out + ((long long)b * L + q) * width + h * HD;
      op[lr] = (OutT)(o[0][r] * iq);
      op[32 + lr] = (OutT)(o[1][r] * iq);
    }
  }
}

template <int NC, typename OutT, typename InT>
static hipError_t launch_attn_bf16(const InT* qkv, int B, int L, int NH, OutT* out, hipStream_t s) {
  const size_t lds = ((size_t)NC * 32 * 64 + 64 * 260) * 2;
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute((const void*)attention_bf16_kernel<NC, OutT, InT>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL((attention_bf16_kernel<NC, OutT, InT>), dim3((unsigned)(B * NH)), dim3(64 * NC), lds, s, qkv, B,
                     L, NH, out);
  return hipGetLastError();
}

template <typename OutT, typename InT>
static hipError_t launch_attn_bf16_nc(int nc, const InT* qkv, int b, int seq, int heads, OutT* out,
                                      hipStream_t s) {
  switch (nc) {
    case 1: return launch_attn_bf16<1>(qkv, b, seq, heads, out, s);
    case 2: return launch_attn_bf16<2>(qkv, b, seq, heads, out, s);
    case 3: return launch_attn_bf16<3>(qkv, b, seq, heads, out, s);
    case 4: return launch_attn_bf16<4>(qkv, b, seq, heads, out, s);
    case 5: return launch_attn_bf16<5>(qkv, b, seq, heads, out, s);
    case 6: return launch_attn_bf16<6>(qkv, b, seq, heads, out, s);
    case 7: return launch_attn_bf16<7>(qkv, b, seq, heads, out, s);
    default: return launch_attn_bf16<8>(qkv, b, seq, heads, out, s);
  }
}

static dim3 grid_for(long long n, int block) {
  long long g = (n + block - 1) / block;
  if (g > 256 * 16) g = 256 * 16;
  if (g < 1) g = 1;
  return dim3((unsigned)g);
}

template <int NC, typename OutT>
static hipError_t launch_attn(const float* qkv, int B, int L, int NH, OutT* out, hipStream_t s) {
  const size_t lds = (size_t)2 * NC * 32 * 64 * 4;
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute((const void*)attention_kernel<NC, OutT>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL((attention_kernel<NC, OutT>), dim3((unsigned)(B * NH)), dim3(64 * NC), lds, s, qkv, B, L, NH,
                     out);
  return hipGetLastError();
}

template <typename OutT>
static hipError_t launch_attn_nc(int nc, const float* qkv, int b, int seq, int heads, OutT* out, hipStream_t s) {
  switch (nc) {
    case 1: return launch_attn<1>(qkv, b, seq, heads, out, s);
    case 2: return launch_attn<2>(qkv, b, seq, heads, out, s);
    case 3: return launch_attn<3>(qkv, b, seq, heads, out, s);
    case 4: return launch_attn<4>(qkv, b, seq, heads, out, s);
    case 5: return launch_attn<5>(qkv, b, seq, heads, out, s);
    case 6: return launch_attn<6>(qkv, b, seq, heads, out, s);
    case 7: return launch_attn<7>(qkv, b, seq, heads, out, s);
    default: return launch_attn<8>(qkv, b, seq, heads, out, s);
  }
}

template <typename OutT>
static void launch_ln(int per, dim3 grid, hipStream_t s, const float* x, long long ldx, int m, int d,
                      const float* gamma, const float* beta, float eps, OutT* y) {
  const bool vec = (ldx & 3) == 0 && (((uintptr_t)x | (uintptr_t)gamma | (uintptr_t)beta | (uintptr_t)y) & 15) == 0;
  if (vec && d == 768) {
    hipLaunchKernelGGL((layernorm_vec_kernel<3, OutT>), grid, dim3(256), 0, s, x, ldx, m, gamma, beta, eps, y);
    return;
  }
  if (vec && d == 512) {
    hipLaunchKernelGGL((layernorm_vec_kernel<2, OutT>), grid, dim3(256), 0, s, x, ldx, m, gamma, beta, eps, y);
    return;
  }
  if (per <= 4)
    hipLaunchKernelGGL((layernorm_kernel<4, OutT>), grid, dim3(256), 0, s, x, ldx, m, d, gamma, beta, eps, y);
  else if (per <= 12)
    hipLaunchKernelGGL((layernorm_kernel<12, OutT>), grid, dim3(256), 0, s, x, ldx, m, d, gamma, beta, eps, y);
  else if (per <= 16)
    hipLaunchKernelGGL((layernorm_kernel<16, OutT>), grid, dim3(256), 0, s, x, ldx, m, d, gamma, beta, eps, y);
  else
    hipLaunchKernelGGL((layernorm_kernel<64, OutT>), grid, dim3(256), 0, s, x, ldx, m, d, gamma, beta, eps, y);
}

}  // namespace rr

using namespace rr;

extern "C" int rr_layernorm(rr_handle_t h, const float* x, long long ldx, int m, int d, const float* gamma,
                            const float* beta, float eps, float* y, void* stream) {
  return rr_layernorm_ex(h, x, ldx, m, d, gamma, beta, eps, 0, y, stream);
}

extern "C" int rr_layernorm_ex(rr_handle_t h, const float* x, long long ldx, int m, int d, const float* gamma,
                               const float* beta, float eps, int out_dtype, void* y, void* stream) {
  RR_ENTRY(h);
  if (!x || !y || !gamma || !beta || m < 0 || d <= 0 || d > 4096 || ldx < d || (out_dtype != 0 && out_dtype != 1))
    return set_error(h, RR_EINVAL, "rr_layernorm: bad argument (d <= 4096, ldx >= d, out_dtype 0|1)");
  if (m == 0) return RR_OK;
  hipStream_t s = (hipStream_t)stream;
  TimedLaunch tl(h, kTimeElem, s);
  const dim3 grid((unsigned)(((long long)m * 64 + 255) / 256));
  const int per = (d + 63) / 64;
  if (out_dtype == 1)
    launch_ln<__bf16>(per, grid, s, x, ldx, m, d, gamma, beta, eps, (__bf16*)y);
  else
    launch_ln<float>(per, grid, s, x, ldx, m, d, gamma, beta, eps, (float*)y);
  return check_hip(h, hipGetLastError(), "layernorm launch");
}

extern "C" int rr_ln_partials_bf16(rr_handle_t h, const float* x, int m, int d, void* xb, float* stats,
                                   void* stream) {
  RR_ENTRY(h);
  if (!x || !xb || !stats || m < 0 || d <= 0 || (d % 256) || (((uintptr_t)x | (uintptr_t)xb) & 15) ||
      ((uintptr_t)stats & 7))
    return set_error(h, RR_EINVAL, "rr_ln_partials_bf16: bad argument (d % 256 == 0, 16-B aligned rows)");
  if (m == 0) return RR_OK;
  hipStream_t s = (hipStream_t)stream;
  TimedLaunch tl(h, kTimeElem, s);
  const long long waves = (long long)m * (d / 256);
  hipLaunchKernelGGL(ln_partials_kernel, dim3((unsigned)((waves * 64 + 255) / 256)), dim3(256), 0, s, x, m, d,
                     (uint16_t*)xb, stats);
  return check_hip(h, hipGetLastError(), "ln_partials launch");
}

extern "C" int rr_patchify(rr_handle_t h, const float* x, int b, int hgt, int wid, int c, int patch, float* y,
                           void* stream) {
  return rr_patchify_ex(h, x, b, hgt, wid, c, patch, 0, y, stream);
}

template <typename OutT>
static void launch_patchify(const float* x, int b, int hgt, int wid, int c, int patch, OutT* y, long long total,
                            hipStream_t s) {
  const bool vec = (patch * c) % 4 == 0 && (wid * c) % 4 == 0 && (((uintptr_t)x | (uintptr_t)y) & 15) == 0;
  if (vec)
    hipLaunchKernelGGL((patchify_vec_kernel<OutT>), grid_for(total / 4, 256), dim3(256), 0, s, x, b, hgt, wid, c,
                       patch, y);
  else
    hipLaunchKernelGGL((patchify_kernel<OutT>), grid_for(total, 256), dim3(256), 0, s, x, b, hgt, wid, c, patch, y);
}

extern "C" int rr_patchify_ex(rr_handle_t h, const float* x, int b, int hgt, int wid, int c, int patch,
                              int out_dtype, void* y, void* stream) {
  RR_ENTRY(h);
  if (!x || !y || b < 0 || c <= 0 || patch <= 0 || hgt % patch || wid % patch || (out_dtype != 0 && out_dtype != 1))
    return set_error(h, RR_EINVAL,
                     "rr_patchify: bad argument (H, W must be multiples of the patch, out_dtype 0|1)");
  const long long total = (long long)b * hgt * wid * c;
  if (total == 0) return RR_OK;
  hipStream_t s = (hipStream_t)stream;
  TimedLaunch tl(h, kTimeElem, s);
  if (out_dtype == 1)
    launch_patchify<__bf16>(x, b, hgt, wid, c, patch, (__bf16*)y, total, s);
  else
    launch_patchify<float>(x, b, hgt, wid, c, patch, (float*)y, total, s);
  return check_hip(h, hipGetLastError(), "patchify launch");
}

extern "C" int rr_vit_tokens(rr_handle_t h, const float* patches, int b, int npatch, int width, const float* cls,
                             const float* pos, float* y, void* stream) {
  return rr_vit_tokens_ex(h, patches, b, npatch, width, cls, pos, nullptr, nullptr, 0.f, y, stream);
}

extern "C" int rr_vit_tokens_ex(rr_handle_t h, const float* patches, int b, int npatch, int width, const float* cls,
                                const float* pos, const float* gamma, const float* beta, float eps, float* y,
                                void* stream) {
  RR_ENTRY(h);
  if (!patches || !cls || !pos || !y || b < 0 || npatch <= 0 || width <= 0 || (!gamma) != (!beta) ||
      (gamma && width > 4096))
    return set_error(h, RR_EINVAL, "rr_vit_tokens: bad argument (gamma and beta both or neither, width <= 4096)");
  const long long rows = (long long)b * (npatch + 1);
  const long long total = rows * width;
  if (total == 0) return RR_OK;
  hipStream_t s = (hipStream_t)stream;
  TimedLaunch tl(h, kTimeElem, s);
  const bool vec = (((uintptr_t)patches | (uintptr_t)cls | (uintptr_t)pos | (uintptr_t)y | (uintptr_t)gamma |
                     (uintptr_t)beta) & 15) == 0;
  const dim3 grid((unsigned)((rows * 64 + 255) / 256));
  if (gamma && vec && width == 768) {
    hipLaunchKernelGGL(vit_tokens_ln_kernel<3>, grid, dim3(256), 0, s, patches, b, npatch, cls, pos, gamma, beta,
                       eps, y);
  } else if (gamma && vec && width == 512) {
    hipLaunchKernelGGL(vit_tokens_ln_kernel<2>, grid, dim3(256), 0, s, patches, b, npatch, cls, pos, gamma, beta,
                       eps, y);
  } else {
    if (!gamma) {
      hipLaunchKernelGGL(vit_tokens_kernel, grid_for(total, 256), dim3(256), 0, s, patches, b, npatch, width, cls,
                         pos, y);
    } else {
      // other widths: assemble and normalise each row in registers (no
      // in-place pass over y: x and y of layernorm_kernel are __restrict__)
      const int per = (width + 63) / 64;
      if (per <= 4)
        hipLaunchKernelGGL(vit_tokens_ln_generic_kernel<4>, grid, dim3(256), 0, s, patches, b, npatch, width, cls,
                           pos, gamma, beta, eps, y);
      else if (per <= 12)
        hipLaunchKernelGGL(vit_tokens_ln_generic_kernel<12>, grid, dim3(256), 0, s, patches, b, npatch, width, cls,
                           pos, gamma, beta, eps, y);
      else if (per <= 16)
        hipLaunchKernelGGL(vit_tokens_ln_generic_kernel<16>, grid, dim3(256), 0, s, patches, b, npatch, width, cls,
                           pos, gamma, beta, eps, y);
      else
        hipLaunchKernelGGL(vit_tokens_ln_generic_kernel<64>, grid, dim3(256), 0, s, patches, b, npatch, width, cls,
                           pos, gamma, beta, eps, y);
    }
  }
  return check_hip(h, hipGetLastError(), "vit_tokens launch");
}

extern "C" int rr_attention(rr_handle_t h, const float* qkv, int b, int seq, int heads, int head_dim, float* out,
                            void* stream) {
  return rr_attention_ex(h, qkv, b, seq, heads, head_dim, 0, out, stream);
}

extern "C" int rr_attention_ex(rr_handle_t h, const float* qkv, int b, int seq, int heads, int head_dim,
                               int out_dtype, void* out, void* stream) {
  RR_ENTRY(h);
  if (!qkv || !out || b < 0 || heads <= 0 || head_dim != 64 || seq <= 0 || seq > 256 ||
      (out_dtype != 0 && out_dtype != 1))
    return set_error(h, RR_EINVAL, "rr_attention: supports head_dim == 64, 1 <= seq <= 256, out_dtype 0|1");
  if (b == 0) return RR_OK;
  hipStream_t s = (hipStream_t)stream;
  TimedLaunch tl(h, kTimeAttn, s);
  const int nc = (seq + 31) / 32;
  const hipError_t e = out_dtype == 1 ? launch_attn_nc<__bf16>(nc, qkv, b, seq, heads, (__bf16*)out, s)
                                      : launch_attn_nc<float>(nc, qkv, b, seq, heads, (float*)out, s);
  return check_hip(h, e, "attention launch");
}

static int attention_bf16_any(rr_handle_t h, const void* qkv, int qkv_bf16, int b, int seq, int heads, int head_dim,
                              int out_dtype, void* out, void* stream, const char* what) {
  RR_ENTRY(h);
  if (!qkv || !out || b < 0 || heads <= 0 || head_dim != 64 || seq <= 0 || seq > 256 ||
      (out_dtype != 0 && out_dtype != 1))
    return set_error(h, RR_EINVAL, std::string(what) + ": supports head_dim == 64, 1 <= seq <= 256, out_dtype 0|1");
  if (b == 0) return RR_OK;
  hipStream_t s = (hipStream_t)stream;
  TimedLaunch tl(h, kTimeAttn, s);
  const int nc = (seq + 31) / 32;
  hipError_t e;
  if (qkv_bf16) {
    const __bf16* q = (const __bf16*)qkv;
    e = out_dtype == 1 ? launch_attn_bf16_nc(nc, q, b, seq, heads, (__bf16*)out, s)
                       : launch_attn_bf16_nc(nc, q, b, seq, heads, (float*)out, s);
  } else {
    const float* q = (const float*)qkv;
    e = out_dtype == 1 ? launch_attn_bf16_nc(nc, q, b, seq, heads, (__bf16*)out, s)
                       : launch_attn_bf16_nc(nc, q, b, seq, heads, (float*)out, s);
  }
  return check_hip(h, e, "attention_bf16 launch");
}

extern "C" int rr_attention_bf16(rr_handle_t h, const float* qkv, int b, int seq, int heads, int head_dim,
                                 int out_dtype, void* out, void* stream) {
  return attention_bf16_any(h, qkv, 0, b, seq, heads, head_dim, out_dtype, out, stream, "rr_attention_bf16");
}

extern "C" int rr_attention_bf16_qkv16(rr_handle_t h, const void* qkv_bf16, int b, int seq, int heads, int head_dim,
                                       int out_dtype, void* out, void* stream) {
  return attention_bf16_any(h, qkv_bf16, 1, b, seq, heads, head_dim, out_dtype, out, stream,
                            "rr_attention_bf16_qkv16");
}
