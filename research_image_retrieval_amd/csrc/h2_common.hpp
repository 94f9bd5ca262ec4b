// h2_common.hpp — pieces of the split-core GEMM kernels (gemm_s3.hip):
// vector types, the f16x2 MFMA wrappers (and the retired bf16x3 ones the
// SP-templated kernels still name), the f16x2
// split of an 8-k chunk, the plane-row slot swizzle and the asynchronous
// (inline-asm) A loads with their register laundering.
#pragma once

#include "gemm_epilogue.hpp"
#include "rr_internal.hpp"

namespace rr {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));

// Split kinds (template SP = planes per operand):
//   3: bf16 x3 (gemm_s3.hip header), six bf16 MFMAs per product;
//   2: fp16 x2 at a power-of-two scale, three fp16 MFMAs per product.  An
//      operand scaled so its max |x| lies in [2^14, 2^15) (h2_exp) splits as
//      x 2^e = x0 + x1 + r, x0 = RNE16(x 2^e), x1 = RNE16(x 2^e - x0) (the
//      difference is exact in fp32), |r| <= 2^-22 |x 2^e|: fp16 carries 11
//      significant bits to bf16's 8, so two pieces hold 22 bits.  a.b keeps
//      a0b0 (own accumulator) + a0b1 + a1b0; dropped: a1b1 and the two
//      remainders, each <= 2^-22 |a||b| with random sign, so their sum over a
//      long dot product stays below the fp32 accumulation's own rounding.
//      Products of fp16 pieces are exact in the fp32 accumulator, and the
//      scales are powers of two: the epilogue's acc * 2^-(ea + eb_n) is exact.
//      Values below 2^-18 of their tensor's max lose relative precision (an
//      absolute error <= 2^-40 of that max).  Same k-loop, LDS layout and
//      epilogues as SP 3 with two planes per operand instead of three.
template <int SP>
struct S3Frag {
  typedef bf16x8 T;
};
template <>
struct S3Frag<2> {
  typedef f16x8 T;
};
template <int SP>
__device__ __forceinline__ f32x4 s3_mf16(const typename S3Frag<SP>::T& a, const typename S3Frag<SP>::T& b, f32x4 c) {
  if constexpr (SP == 2) return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  else return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
template <int SP>
__device__ __forceinline__ f32x16 s3_mf32(const typename S3Frag<SP>::T& a, const typename S3Frag<SP>::T& b, f32x16 c) {
  if constexpr (SP == 2) return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
  else return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// fp16 x2 split of 8 fp32 values (one 8-k chunk) at scale sc into two packed
// planes: hi = RNE16(x sc), lo = RNE16(x sc - hi)
__device__ __forceinline__ void split2h8(const f32x4 (&r)[2], float sc, u32x4& p0, u32x4& p1) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const f32x2 v = f32x2{r[q >> 1][2 * (q & 1)], r[q >> 1][2 * (q & 1) + 1]} * sc;
    const f16x2 h = __builtin_convertvector(v, f16x2);
    const f16x2 l = __builtin_convertvector(v - __builtin_convertvector(h, f32x2), f16x2);
    p0[q] = __builtin_bit_cast(uint32_t, h);
    p1[q] = __builtin_bit_cast(uint32_t, l);
  }
}

// 16-B slot swizzle of a plane row of BK 16-bit values.  A ds_read_b128 is
// serviced in four lane groups of 16 lanes, one LDS cycle each when their 16-B
// accesses hit 16 distinct bank quads; the groups are {0-3,12-15,20-27},
// {4-11,16-19,28-31} and the same +32 (MI355X_MICROARCH.md, LDS), not runs of
// 16 consecutive lanes.  BK = 32 (64-B rows, 4 slots; a row's bank quad is
// 4 (row & 3) + slot): slot ^ (2 ((row >> 3) & 1) + ((row >> 4) & 1)) is
// conflict-free for both fragment reads, 16x16x32 (lane l: row l & 15, slot
// l >> 4) and 32x32x16 (row l & 31, slot 2 step + (l >> 5)) — the earlier
// slot ^ ((row >> 2) & 3) was 2-way on every 16x16x32 read (checked by
// enumeration, tools/lds_swizzle_check.py).  BK = 16 (32-B rows, 2 slots):
// slot ^ ((row >> 3) & 1).  ds_write_b128 groups (8 contiguous lanes = two
// rows) are conflict-free under any per-row permutation.  The bf16x3 split
// (SP 3) keeps the earlier form: its config-4 conv kernels sit at the register
// limit and the new one's address arithmetic spilled them.
template <int BK, int SP>
__device__ __forceinline__ int pswz(int row, int slot) {
  if constexpr (BK == 32 && SP == 2) return slot ^ ((((row >> 3) & 1) << 1) | ((row >> 4) & 1));
  else if constexpr (BK == 32) return slot ^ ((row >> 2) & 3);
  else return slot ^ ((row >> 3) & 1);
}


// Two consecutive 16-B loads.  ASYNC: issued by inline asm, so hipcc keeps no
// scoreboard entry for them: with LDS-DMA in flight it otherwise waits
// vmcnt(0) at the first use of any plain load's result (mixed VMEM event
// types make it treat the counter as out of order), which drains the A
// prefetch every iteration.  The caller waits with a counted vmcnt and
// launders the registers (s3_launder) before using them.
template <int ASYNC>
__device__ __forceinline__ void s3_load2(const f32x4* p, f32x4 (&r)[2]) {
  if constexpr (ASYNC) {
    asm volatile("global_load_dwordx4 %0, %2, off\n\tglobal_load_dwordx4 %1, %2, off offset:16"
                 : "=&v"(r[0]), "=&v"(r[1])
                 : "v"(p)
                 : "memory");
  } else {
    r[0] = p[0];
    r[1] = p[1];
  }
}
// two 16-B loads from unrelated addresses (the NHWC4 stem's two taps)
template <int ASYNC>
__device__ __forceinline__ void s3_load1x2(const f32x4* p0, const f32x4* p1, f32x4 (&r)[2]) {
  if constexpr (ASYNC) {
    asm volatile("global_load_dwordx4 %0, %2, off\n\tglobal_load_dwordx4 %1, %3, off"
                 : "=&v"(r[0]), "=&v"(r[1])
                 : "v"(p0), "v"(p1)
                 : "memory");
  } else {
    r[0] = *p0;
    r[1] = *p1;
  }
}
// a fresh definition of v after the preceding (volatile) wait: nothing that
// reads v can be scheduled above it
__device__ __forceinline__ void s3_launder(f32x4& v) { asm volatile("" : "+v"(v)); }
// a fresh, opaque copy of v: address math built from it cannot be folded or
// hoisted (see its uses)
__device__ __forceinline__ int s3_opaque(int v) {
  asm volatile("" : "+v"(v));
  return v;
}


}  // namespace rr
