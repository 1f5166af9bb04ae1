// Shared helpers for the gfx950 (MI355X, CDNA4) kernels of pytorch_r2d2_amd.
//
// Conventions used by every kernel in csrc/kernels:
//  * wave = 64 lanes; blocks are multiples of 64 threads.
//  * bf16 is the clang native __bf16 (fptrunc lowers to v_cvt_pk_bf16_f32 on gfx950).
//  * MFMA tile = v_mfma_f32_32x32x16_bf16.  Lane l holds A[m=l&31][k=8*(l>>5)+j] and
//    B[k=8*(l>>5)+j][n=l&31] (j=0..7); accumulator register r holds
//    C[m=(r&3)+8*(r>>2)+4*(l>>5)][n=l&31].
//  * every launcher is `extern "C"`, takes raw device pointers and a hipStream_t, never
//    allocates or synchronises (safe under hipGraph stream capture).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

#define R2_WAVE 64

#define R2_CHECK_LAUNCH() \
  do { hipError_t e__ = hipGetLastError(); if (e__ != hipSuccess) return (int)e__; } while (0)

__device__ __forceinline__ f32x16 mfma32(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// Activations on the hardware reciprocal (v_rcp_f32, 1 ulp) instead of an IEEE division: the
// division expands to ~10 dependent VALU ops (div_scale / div_fmas / div_fixup) and sat on the
// LSTM recurrence's critical path (10 of them per thread per step).
__device__ __forceinline__ float fast_rcp(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ __forceinline__ float sigmoidf_(float x) { return fast_rcp(1.f + __expf(-x)); }
__device__ __forceinline__ float tanhf_(float x) {
  // tanh via exp; saturates cleanly for large |x| (e -> 0)
  const float e = __expf(-2.f * fabsf(x));
  return copysignf((1.f - e) * fast_rcp(1.f + e), x);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
// All-lane wave sum on the VALU: DPP exchanges inside each 16-lane row (xor 1, xor 2, the other
// quad of the 8, the other half of the row: every lane of a row then holds the same row sum,
// adds are commutative) and v_readlane of the four row sums, added as (r0 + r1) + (r2 + r3).
// ~10 dependent VALU ops instead of wave_sum's six ds_bpermute round trips through the LDS unit;
// a different (fixed) association than wave_sum, so kernels that must agree bit for bit (the
// dueling forward in head.hip and td.hip) both use this one.
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float wave_sum_x(float v) {
  v += dpp_mov<0xB1>(v);    // quad_perm [1,0,3,2]: xor 1
  v += dpp_mov<0x4E>(v);    // quad_perm [2,3,0,1]: xor 2
  v += dpp_mov<0x141>(v);   // row_half_mirror: the other quad of the 8
  v += dpp_mov<0x140>(v);   // row_mirror: the other half of the row
  const float r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
  const float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
  const float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
  const float r3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
  return (r0 + r1) + (r2 + r3);
}
__device__ __forceinline__ float wave_max_x(float v) {
  v = fmaxf(v, dpp_mov<0xB1>(v));
  v = fmaxf(v, dpp_mov<0x4E>(v));
  v = fmaxf(v, dpp_mov<0x141>(v));
  v = fmaxf(v, dpp_mov<0x140>(v));
  const float r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
  const float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
  const float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
  const float r3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
  return fmaxf(fmaxf(r0, r1), fmaxf(r2, r3));
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// 8 unsigned bytes (two dwords) -> 8 bf16 (exact: integers 0..255 are representable)
__device__ __forceinline__ bf16x8 u8x8_to_bf16(uint32_t lo, uint32_t hi) {
  bf16x8 r;
  r[0] = (bf16)(float)(lo & 0xff);
  r[1] = (bf16)(float)((lo >> 8) & 0xff);
  r[2] = (bf16)(float)((lo >> 16) & 0xff);
  r[3] = (bf16)(float)(lo >> 24);
  r[4] = (bf16)(float)(hi & 0xff);
  r[5] = (bf16)(float)((hi >> 8) & 0xff);
  r[6] = (bf16)(float)((hi >> 16) & 0xff);
  r[7] = (bf16)(float)(hi >> 24);
  return r;
}

// counter-based RNG (splitmix64 finaliser) -> uniform float in [0,1)
__device__ __forceinline__ uint64_t r2_mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ float r2_uniform(uint64_t seed, uint64_t ctr, uint64_t idx) {
  uint64_t z = r2_mix64(seed ^ r2_mix64(ctr * 0x100000001B3ull + idx));
  return (float)(z >> 40) * (1.0f / 16777216.0f);
}

// a[i] for a wave-uniform index through the scalar (constant) path: s_load + lgkmcnt instead of a
// vector load whose vmcnt wait would also wait for every older outstanding load / store
__device__ __forceinline__ int ld_uniform_i32(const int* a, int i) {
  return ((const __attribute__((address_space(4))) int*)a)[i];
}

// Workgroup barrier that orders LDS only.  __syncthreads() also emits s_waitcnt vmcnt(0), which
// drains every outstanding global load -- including a next-frame register prefetch that is meant to
// stay in flight across the barrier.  Use this where only LDS traffic must be ordered.
__device__ __forceinline__ void lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Software-pipelined MFMA chain: acc += sum_s A(s) . B(s) for s < N with the operand loads of
// step s+D issued before the MFMA of step s (register ring of depth D), so LDS latency overlaps
// the matrix pipe instead of serialising every step on lgkmcnt(0).  `lda`/`ldb` are called with
// compile-time step indices after unrolling (addresses fold to base + immediate).
template <int N, int D, class FA, class FB>
__device__ __forceinline__ void mfma_pipe(f32x16& acc, FA lda, FB ldb) {
  bf16x8 ra[D], rb[D];
#pragma unroll
  for (int i = 0; i < D; ++i)
    if (i < N) { ra[i] = lda(i); rb[i] = ldb(i); }
#pragma unroll
  for (int s = 0; s < N; ++s) {
    const bf16x8 a = ra[s % D], b = rb[s % D];
    if (s + D < N) { ra[s % D] = lda(s + D); rb[s % D] = ldb(s + D); }
    __builtin_amdgcn_sched_barrier(0);
    acc = mfma32(a, b, acc);
  }
}
// Two accumulators sharing the A operand (two N tiles of one weight-gradient row block).
template <int N, int D, class FA, class FB0, class FB1>
__device__ __forceinline__ void mfma_pipe2(f32x16& acc0, f32x16& acc1, FA lda, FB0 ldb0, FB1 ldb1) {
  bf16x8 ra[D], rb0[D], rb1[D];
#pragma unroll
  for (int i = 0; i < D; ++i)
    if (i < N) { ra[i] = lda(i); rb0[i] = ldb0(i); rb1[i] = ldb1(i); }
#pragma unroll
  for (int s = 0; s < N; ++s) {
    const bf16x8 a = ra[s % D], b0 = rb0[s % D], b1 = rb1[s % D];
    if (s + D < N) { ra[s % D] = lda(s + D); rb0[s % D] = ldb0(s + D); rb1[s % D] = ldb1(s + D); }
    __builtin_amdgcn_sched_barrier(0);
    acc0 = mfma32(a, b0, acc0);
    acc1 = mfma32(a, b1, acc1);
  }
}
