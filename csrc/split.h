// fp32-accurate matrix products on the bf16 matrix cores (gfx950): the "split" precision mode.
//
// An fp32 value x is carried as a pair of bf16 planes  hi = bf16(x),  lo = bf16(x - hi)
// (16-17 significant bits together; |x - hi - lo| <= 2^-17 |x|), and a product of two split
// operands is taken in three bf16 MFMA passes with fp32 accumulation:
//
//     a.b  ~=  a_lo.b_hi + a_hi.b_lo + a_hi.b_hi        (the a_lo.b_lo term, <= 2^-18 |a||b|,
//                                                        is dropped; small terms first)
//
// Relative error per product ~1e-5 (vs ~6e-8 for fp32 FMA, ~1e-3 for the TF32 path PyTorch uses
// for convolutions on other vendors' GPUs by default), at 3x the bf16 MFMA cost -- 5.3x faster
// than the gfx950 fp32 MFMA (v_mfma_f32_32x32x2_f32 runs at 1/16 of the bf16 rate,
// MI355X_MICROARCH.md "Matrix cores").  An operand that is exact in bf16 (the uint8 frames: integers 0..255)
// needs no lo plane: its products take two passes.  Everything that is not an MFMA operand stays
// plain fp32 (master weights, optimizer moments, cell state, gates, Q values, TD math, gradients).
//
// Storage convention ("split tensor"): a (2, *shape) bf16 tensor, plane 0 = hi, plane 1 = lo; a
// kernel receives the two plane pointers.  Producers write both planes in their epilogues, so no
// consumer ever converts.
#pragma once
#include "common.h"

__device__ __forceinline__ void sp_split(float x, bf16& hi, bf16& lo) {
  hi = (bf16)x;
  lo = (bf16)(x - (float)hi);
}
__device__ __forceinline__ bf16 sp_lo(float x) { return (bf16)(x - (float)(bf16)x); }
__device__ __forceinline__ float sp_join(bf16 hi, bf16 lo) { return (float)hi + (float)lo; }

// acc += a.b over split operands (3 passes)
__device__ __forceinline__ f32x16 mfma32_x3(const bf16x8& ah, const bf16x8& al, const bf16x8& bh,
                                            const bf16x8& bl, f32x16 acc) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma16_x3(const bf16x8& ah, const bf16x8& al, const bf16x8& bh,
                                           const bf16x8& bl, f32x4 acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, acc, 0, 0, 0);
}
// acc += a.b with `a` exact in bf16 and b split (2 passes)
__device__ __forceinline__ f32x16 mfma32_x2(const bf16x8& a, const bf16x8& bh, const bf16x8& bl,
                                            f32x16 acc) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bl, acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bh, acc, 0, 0, 0);
}

// 8 fp32 -> hi / lo bf16x8 fragments
__device__ __forceinline__ void sp_split8(const float* v, bf16x8& hi, bf16x8& lo) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    hi[e] = (bf16)v[e];
    lo[e] = (bf16)(v[e] - (float)hi[e]);
  }
}
