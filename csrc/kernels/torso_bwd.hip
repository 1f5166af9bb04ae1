// Fused Atari conv-torso BACKWARD for gfx950 (MI355X).
//
// Replaces the library path (3x convolution_backward on MIOpen + ReLU-mask elementwise kernels +
// NCHW/NHWC transposes + bias reductions + a uint8->bf16 frame expansion: ~0.6 ms per learner
// step at B=64 x 40 learning steps) with ONE kernel + one slab reduction.  Per learning frame,
// entirely in LDS (150 KB, 512 threads, one workgroup per CU, grid-stride over frames):
//
//   g3  = dX3 * (out3 > 0)                              (ReLU backward from the saved output)
//   dW3 += g3 (co x px) . im2col^T(act2)                 MFMA, K = 49 px (padded 64)
//   g2  = convT(g3, W3) * (act2 > 0)                      MFMA, M = 81 px, K = (kh,kw,co) = 288
//   dW2 += g2 . im2col^T(act1)                            MFMA, K = 81 px in 3 chunks of 32
//   g1  = convT_s2(g2, W2) * (act1 > 0)                   MFMA, stride-2 transposed conv split into
//                                                         its 4 output phases: only the 4 (kh,kw)
//                                                         taps that hit a phase are multiplied
//                                                         (K = 128 instead of 512 with 3/4 zeros)
//   dW1 += g1 . im2col^T(frame u8)                        MFMA, K = 400 px in 7 chunks of 64; the
//                                                         uint8 pixels are exact in bf16, 1/255 is
//                                                         applied once in the reduction
//   db_l = sum over pixels of g_l                          (MFMA epilogues / one row pass)
//
// Weight-gradient accumulators stay in MFMA registers across all frames of a workgroup
// (dW1: 1, dW2: 2, dW3: <=2 32x32 tiles per wave); at the end each workgroup writes one fp32
// slab and ``r2_torso_grad_reduce`` sums the slabs straight into the flat gradient buffer
// (deterministic; torch layout via an index map).
//
// MFMA operands: A = g (rows = output channel co, 8 consecutive pixels per lane from a CHW tile),
// B = im2col^T (rows = k, 8 consecutive pixels) built per frame in LDS with 16-byte source reads;
// the transposed convs read g channels-last (8 consecutive co) and pre-packed data-grad weight
// layouts conv3_dg[ci][kh][kw][co] / conv2_dg[phase][ci][khi][kwi][co] (engine/layout.py).
#include "../common.h"

namespace tb {
constexpr int NT = 512;
constexpr int P1 = 400, P2 = 81, P3 = 49;
constexpr int IN_BYTES = 4 * 84 * 84;
constexpr int G3C_S = 72, G2C_S = 104, G1C_S = 456;  // bf16 row strides (16-B aligned, bank-spread)
constexpr int X3_S = 72, X2_S = 40, X1_S = 72;
constexpr int FR = 0;
constexpr int A1 = FR + IN_BYTES;        // act1 hwc [400][32] bf16
constexpr int A2 = A1 + P1 * 32 * 2;     // act2 hwc [81][32]
constexpr int G3H = A2 + P2 * 32 * 2;    // g3 hwc [49][32]
constexpr int G3C = G3H + P3 * 32 * 2;   // g3 chw [32][72]
constexpr int G2H = G3C + 32 * G3C_S * 2;  // g2 hwc [81][32]
constexpr int G2C = G2H + P2 * 32 * 2;     // g2 chw [32][104]
constexpr int G1C = G2C + 32 * G2C_S * 2;  // g1 chw [32][456]
constexpr int XT = G1C + 32 * G1C_S * 2;   // im2col^T scratch
constexpr int XT_BYTES = 288 * X3_S * 2;   // largest of the three builds
constexpr int LDS = XT + XT_BYTES;         // 149248
constexpr int SLAB = 32 * 256 + 32 * 512 + 32 * 288 + 96;  // 33888 floats per workgroup
constexpr int OFF_W2 = 32 * 256, OFF_W3 = OFF_W2 + 32 * 512, OFF_B = OFF_W3 + 32 * 288;
}  // namespace tb

struct TBArgs {
  const uint8_t* frames;
  const int* rows;     // replay rows of the N learning frames
  const bf16* act1;    // (N, 400, 32) channels-last, from the forward kernel
  const bf16* act2;    // (N, 81, 32)
  const bf16* dx3;     // (N, 1568) dL/d(torso output), CHW flatten
  const bf16* out3;    // (N, 1568) torso output (ReLU mask)
  const bf16* w3dg;    // (32 ci, 288 = (kh,kw,co))
  const bf16* w2dg;    // (4 phases, 32 ci, 128 = (khi,kwi,co))
  float* slab;         // (gridDim.x, SLAB)
  int n;
};

__device__ __forceinline__ bf16x8 ld8(const bf16* p) { return *(const bf16x8*)p; }

__global__ __launch_bounds__(512) void torso_bwd_kernel(const TBArgs a) {
  using namespace tb;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  uint8_t* fr = lds + FR;
  bf16* a1 = (bf16*)(lds + A1);
  bf16* a2 = (bf16*)(lds + A2);
  bf16* g3h = (bf16*)(lds + G3H);
  bf16* g3c = (bf16*)(lds + G3C);
  bf16* g2h = (bf16*)(lds + G2H);
  bf16* g2c = (bf16*)(lds + G2C);
  bf16* g1c = (bf16*)(lds + G1C);
  bf16* xt = (bf16*)(lds + XT);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int l32 = lane & 31, half = lane >> 5;
  const bf16x8 zero8 = {};

  // zero the CHW gradient tiles once: their pad columns stay zero for every frame
  for (int i = tid; i < 32 * G3C_S * 2 / 16; i += NT) ((u32x4*)(lds + G3C))[i] = u32x4{0, 0, 0, 0};
  for (int i = tid; i < 32 * G2C_S * 2 / 16; i += NT) ((u32x4*)(lds + G2C))[i] = u32x4{0, 0, 0, 0};
  for (int i = tid; i < 32 * G1C_S * 2 / 16; i += NT) ((u32x4*)(lds + G1C))[i] = u32x4{0, 0, 0, 0};
  f32x16 acc1 = {}, acc2a = {}, acc2b = {}, acc3a = {}, acc3b = {};
  float db1p = 0.f, db2p = 0.f, db3p = 0.f;
  __syncthreads();

  for (int f = blockIdx.x; f < a.n; f += gridDim.x) {
    // ---- stage 0: this frame's inputs -> LDS
    {
      const u32x4* src = (const u32x4*)(a.frames + (size_t)a.rows[f] * IN_BYTES);
      for (int c = tid; c < IN_BYTES / 16; c += NT) ((u32x4*)fr)[c] = src[c];
      const u32x4* s1 = (const u32x4*)(a.act1 + (size_t)f * P1 * 32);
      for (int c = tid; c < P1 * 4; c += NT) ((u32x4*)a1)[c] = s1[c];
      const u32x4* s2 = (const u32x4*)(a.act2 + (size_t)f * P2 * 32);
      for (int c = tid; c < P2 * 4; c += NT) ((u32x4*)a2)[c] = s2[c];
      for (int c = tid; c < 196; c += NT) {  // g3 = dx3 * (out3 > 0): 1568 = 196 x 8
        const bf16x8 dx = ld8(a.dx3 + (size_t)f * 1568 + c * 8);
        const bf16x8 o3 = ld8(a.out3 + (size_t)f * 1568 + c * 8);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int i = c * 8 + e, co = i / P3, p = i % P3;
          const bf16 v = ((float)o3[e] > 0.f) ? dx[e] : (bf16)0.f;
          g3c[co * G3C_S + p] = v;
          g3h[p * 32 + co] = v;
        }
      }
    }
    __syncthreads();
    // ---- db3 (one row pass) and im2col^T of act2 for dW3: XT3[(kh,kw,ci)][p], p < 64
    if (wave == 0 && lane < 32) {
      float s = 0.f;
      for (int p = 0; p < P3; ++p) s += (float)g3c[lane * G3C_S + p];
      db3p += s;
    }
    for (int it = tid; it < 9 * 4 * 64; it += NT) {
      const int p = it & 63, r = it >> 6, cg = r & 3, khkw = r >> 2;
      const int kh = khkw / 3, kw = khkw % 3;
      bf16x8 v = zero8;
      if (p < P3) {
        const int oy = p / 7, ox = p % 7;
        v = ld8(a2 + ((oy + kh) * 9 + ox + kw) * 32 + cg * 8);
      }
      bf16* d = xt + (khkw * 32 + cg * 8) * X3_S + p;
#pragma unroll
      for (int e = 0; e < 8; ++e) d[e * X3_S] = v[e];
    }
    __syncthreads();
    // ---- dW3 (waves 0-4, 9 N tiles) || dact2 -> g2 (waves 5-7, 3 M tiles)
    if (wave < 5) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int nt = wave + q * 5;
        if (nt < 9) {
          f32x16 acc = q == 0 ? acc3a : acc3b;
#pragma unroll
          for (int s = 0; s < 4; ++s)
            acc = mfma32(ld8(g3c + l32 * G3C_S + s * 16 + half * 8),
                         ld8(xt + (nt * 32 + l32) * X3_S + s * 16 + half * 8), acc);
          if (q == 0) acc3a = acc; else acc3b = acc;
        }
      }
    } else {
      const int mt = wave - 5;
      const int q = mt * 32 + l32, qc = q < P2 ? q : P2 - 1;
      const int qy = qc / 9, qx = qc % 9;
      f32x16 acc = {};
#pragma unroll 2
      for (int s = 0; s < 18; ++s) {
        const int k0 = s * 16 + half * 8, khkw = k0 >> 5, co0 = k0 & 31;
        const int oy = qy - khkw / 3, ox = qx - khkw % 3;
        const bool ok = q < P2 && oy >= 0 && oy < 7 && ox >= 0 && ox < 7;
        const bf16x8 av = ok ? ld8(g3h + (oy * 7 + ox) * 32 + co0) : zero8;
        acc = mfma32(av, ld8(a.w3dg + l32 * 288 + k0), acc);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int qq = mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
        if (qq < P2) {
          const bf16 v = ((float)a2[qq * 32 + l32] > 0.f) ? (bf16)acc[r] : (bf16)0.f;
          g2h[qq * 32 + l32] = v;
          g2c[l32 * G2C_S + qq] = v;
          db2p += (float)v;
        }
      }
    }
    __syncthreads();
    // ---- dW2 over 3 pixel chunks of 32 (wave w owns N tiles w and w+8)
    for (int ch = 0; ch < 3; ++ch) {
      for (int it = tid; it < 16 * 4 * 32; it += NT) {
        const int pc = it & 31, r = it >> 5, cg = r & 3, khkw = r >> 2;
        const int kh = khkw >> 2, kw = khkw & 3, p = ch * 32 + pc;
        bf16x8 v = zero8;
        if (p < P2) {
          const int oy = p / 9, ox = p % 9;
          v = ld8(a1 + ((2 * oy + kh) * 20 + 2 * ox + kw) * 32 + cg * 8);
        }
        bf16* d = xt + (khkw * 32 + cg * 8) * X2_S + pc;
#pragma unroll
        for (int e = 0; e < 8; ++e) d[e * X2_S] = v[e];
      }
      __syncthreads();
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 av = ld8(g2c + l32 * G2C_S + ch * 32 + s * 16 + half * 8);
        acc2a = mfma32(av, ld8(xt + (wave * 32 + l32) * X2_S + s * 16 + half * 8), acc2a);
        acc2b = mfma32(av, ld8(xt + ((wave + 8) * 32 + l32) * X2_S + s * 16 + half * 8), acc2b);
      }
      __syncthreads();
    }
    // ---- dact1 -> g1: stride-2 transposed conv by output phase (16 jobs, 2 per wave)
#pragma unroll 1
    for (int jj = 0; jj < 2; ++jj) {
      const int job = wave * 2 + jj, phase = job >> 2, mt = job & 3;
      const int py = phase >> 1, px = phase & 1;
      const int m = mt * 32 + l32, mc = m < 100 ? m : 99;
      const int ay = mc / 10, bx = mc % 10;
      f32x16 acc = {};
#pragma unroll 2
      for (int s = 0; s < 8; ++s) {
        const int k0 = s * 16 + half * 8, tap = k0 >> 5, co0 = k0 & 31;
        const int oy = ay - (tap >> 1), ox = bx - (tap & 1);
        const bool ok = m < 100 && oy >= 0 && oy < 9 && ox >= 0 && ox < 9;
        const bf16x8 av = ok ? ld8(g2h + (oy * 9 + ox) * 32 + co0) : zero8;
        acc = mfma32(av, ld8(a.w2dg + (phase * 32 + l32) * 128 + k0), acc);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int mm = mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
        if (mm < 100) {
          const int qpix = (2 * (mm / 10) + py) * 20 + 2 * (mm % 10) + px;
          const bf16 v = ((float)a1[qpix * 32 + l32] > 0.f) ? (bf16)acc[r] : (bf16)0.f;
          g1c[l32 * G1C_S + qpix] = v;
          db1p += (float)v;
        }
      }
    }
    __syncthreads();
    // ---- dW1 over 7 pixel chunks of 64 from the uint8 frame (wave w owns N tile w)
    for (int ch = 0; ch < 7; ++ch) {
      for (int it = tid; it < 4 * 8 * 64; it += NT) {
        const int pc = it & 63, r = it >> 6, kh = r & 7, ci = r >> 3, p = ch * 64 + pc;
        bf16x8 v = zero8;
        if (p < P1) {
          const int oy = p / 20, ox = p % 20;
          const uint32_t* q = (const uint32_t*)(fr + ci * 7056 + (4 * oy + kh) * 84 + 4 * ox);
          v = u8x8_to_bf16(q[0], q[1]);
        }
        bf16* d = xt + ((ci * 8 + kh) * 8) * X1_S + pc;
#pragma unroll
        for (int e = 0; e < 8; ++e) d[e * X1_S] = v[e];
      }
      __syncthreads();
#pragma unroll
      for (int s = 0; s < 4; ++s)
        acc1 = mfma32(ld8(g1c + l32 * G1C_S + ch * 64 + s * 16 + half * 8),
                      ld8(xt + (wave * 32 + l32) * X1_S + s * 16 + half * 8), acc1);
      __syncthreads();
    }
  }

  // ---- epilogue: this workgroup's partial gradients -> slab
  float* sl = a.slab + (size_t)blockIdx.x * SLAB;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int co = (r & 3) + 8 * (r >> 2) + 4 * half;
    sl[co * 256 + wave * 32 + l32] = acc1[r];
    sl[OFF_W2 + co * 512 + wave * 32 + l32] = acc2a[r];
    sl[OFF_W2 + co * 512 + (wave + 8) * 32 + l32] = acc2b[r];
    if (wave < 5) sl[OFF_W3 + co * 288 + wave * 32 + l32] = acc3a[r];
    if (wave < 4) sl[OFF_W3 + co * 288 + (wave + 5) * 32 + l32] = acc3b[r];
  }
  float* red = (float*)(lds + XT);
  __syncthreads();
  if (tid < 96) red[tid] = 0.f;
  __syncthreads();
  atomicAdd(&red[l32], db1p);                       // conv1 bias (every wave ran dact1 jobs)
  if (wave >= 5) atomicAdd(&red[32 + l32], db2p);   // conv2 bias
  if (wave == 0 && lane < 32) atomicAdd(&red[64 + lane], db3p);
  __syncthreads();
  if (tid < 96) sl[OFF_B + tid] = red[tid];
}

// grad[dst[e]] = scale[e] * sum_g slab[g][e]
__global__ void torso_grad_reduce_kernel(const float* __restrict__ slab, int G,
                                         const int* __restrict__ dst, const float* __restrict__ scale,
                                         float* __restrict__ grad) {
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < tb::SLAB; e += gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int g = 0; g < G; ++g) s += slab[(size_t)g * tb::SLAB + e];
    grad[dst[e]] = s * scale[e];
  }
}

extern "C" int r2_torso_bwd(const uint8_t* frames, const int* rows, int n, const bf16* act1,
                            const bf16* act2, const bf16* dx3, const bf16* out3, const bf16* w3dg,
                            const bf16* w2dg, float* slab, int grid, const int* dst,
                            const float* scale, float* grad, void* stream) {
  if (n <= 0) return 0;
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)torso_bwd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                        tb::LDS);
    attr = true;
  }
  if (grid <= 0 || grid > n) grid = n < 256 ? n : 256;
  TBArgs a{frames, rows, act1, act2, dx3, out3, w3dg, w2dg, slab, n};
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(torso_bwd_kernel, dim3(grid), dim3(tb::NT), tb::LDS, s, a);
  hipLaunchKernelGGL(torso_grad_reduce_kernel, dim3((tb::SLAB + 255) / 256), dim3(256), 0, s, slab,
                     grid, dst, scale, grad);
  R2_CHECK_LAUNCH();
  return 0;
}

extern "C" int r2_torso_bwd_slab_floats() { return tb::SLAB; }
