// Fused Atari conv torso forward for gfx950 (MI355X).
//
// Reference: model.py:12-22,44-46 -- Conv2d(4,32,8,s4)-ReLU-Conv2d(32,32,4,s2)-ReLU-
// Conv2d(32,32,3,s1)-ReLU on (N,4,84,84) float frames that the replay first expands from uint8
// (replay_memory.py:236-256, state/255 then H2D).  Here one kernel does all of it:
//
//  * frames are read as uint8 straight from the HBM replay ring through a row-index list
//    (the replay "gather" and the /255 normalisation are fused; integers 0..255 are exact in
//    bf16 and the 1/255 is applied to the fp32 conv1 accumulator);
//  * every convolution is an implicit GEMM on MFMA (v_mfma_f32_32x32x16_bf16) with
//    M = 32 output channels, N = 32 output pixels, K = Cin*kh*kw;
//  * activations never leave LDS: conv1 output (20x20x32) and conv2 output (9x9x32) are kept
//    channels-last (HWC, 80-byte padded pixel rows -> 16-byte aligned, bank-spread
//    ds_read_b128 fragment loads);
//  * conv2/conv3 weights live in LDS (padded rows), conv1 weights in VGPRs (64 regs);
//  * the frame is converted u8->bf16 once, when it is written to LDS, so the conv1 MFMA loop
//    issues no conversion VALU; it is stored SPACE-TO-DEPTH: (21,21,64) with channel
//    c = ci*16 + dy*4 + dx, which turns the 8x8/s4 conv1 into a 2x2/s1 conv whose B fragments
//    (8 consecutive c) are single aligned ds_read_b128 (the plain CHW image needs two 8-byte
//    reads per fragment, half the LDS rate); the next frame's 28 KB is prefetched into
//    registers while the current frame computes;
//  * two-phase software pipeline per frame: phase A = conv1(f) on all waves || conv3(f-1) on
//    waves 2,3 (tiles dealt so every SIMD issues ~64 MFMAs); phase B = conv2(f) on waves 0..2
//    || next frame -> LDS and conv1 activations saved by waves 3..7; two barriers per frame;
//  * output is bf16 in PyTorch's (C,H,W) flatten order, ready for the LSTM input GEMM.
//  * optional: conv1/conv2 activations are written channels-last for the backward pass
//    (torch channels_last NCHW tensors), so backward does not recompute the forward.
//
// One 512-thread workgroup per CU (151 KB LDS), grid-stride over frames.
#include "../common.h"

// Frame geometry of the fused forward (template parameter): CIN uint8 planes of H x W (H, W
// multiples of 4), Conv(CIN,32,8,s4) -> Conv(32,32,4,s2) -> Conv(32,32,3,s1).  Instantiated for
// the Atari stack (4x84x84: 20x20 -> 9x9 -> 7x7) and DMLab-30 RGB (3x72x96: 17x23 -> 7x10 -> 5x8).
template <int CIN_, int H_, int W_>
struct TGeo {
  static constexpr int CIN = CIN_, H = H_, W = W_;
  static constexpr int IN_BYTES = CIN * H * W;
  static constexpr int IN_CHUNKS = IN_BYTES / 16;
  static constexpr int NT = 512;                      // threads
  static constexpr int PF = (IN_CHUNKS + 319) / 320;  // prefetch chunks per thread of waves 3..7
  static constexpr int H1 = (H - 8) / 4 + 1, W1 = (W - 8) / 4 + 1;
  static constexpr int H2 = (H1 - 4) / 2 + 1, W2 = (W1 - 4) / 2 + 1;
  static constexpr int H3 = H2 - 2, W3 = W2 - 2;
  static constexpr int P1 = H1 * W1, P2 = H2 * W2, P3 = H3 * W3;
  static constexpr int OUT = 32 * P3;                 // torso features per frame
  static constexpr int H4 = H / 4, W4 = W / 4;        // space-to-depth image
  static constexpr int K1S = 4 * CIN;                 // conv1 K steps of 16
  static constexpr int ACTS = 40;                     // bf16 per pixel row in LDS (32 + 8 pad) = 80 B
  static constexpr int W2S = 512 + 8;                 // bf16 per conv2 weight row (1040 B)
  static constexpr int W3S = 288 + 8;                 // bf16 per conv3 weight row (592 B)
  static constexpr int S2DS = 16 * CIN + 8;           // bf16 per space-to-depth pixel (+8 pad)
  static constexpr int OFF_IN = 0;                    // frame, bf16 space-to-depth [H4*W4][S2DS]
  static constexpr int OFF_A1 = OFF_IN + H4 * W4 * S2DS * 2;
  // act1: 64-B pixel rows, 16-B chunks row-XOR swizzled (tf_a1_off) -- conflict-lighter stride-2
  // conv2 reads than the 80-B padded rows, and 6.4 KB smaller; act2 keeps the padded rows
  static constexpr int A1_BYTES = ((P1 + 3) / 4) * 256;
  static constexpr int OFF_A2 = OFF_A1 + A1_BYTES;
  static constexpr int OFF_W2 = OFF_A2 + P2 * ACTS * 2;
  static constexpr int OFF_W3 = OFF_W2 + 32 * W2S * 2;
  static constexpr int OFF_B23 = OFF_W3 + 32 * W3S * 2;   // conv2 / conv3 biases, fp32 [2][32]
  static constexpr int LDS_BYTES = OFF_B23 + 64 * 4;
  static_assert(H % 4 == 0 && W % 4 == 0 && IN_BYTES % 16 == 0, "geometry");
  static_assert((P1 + 31) / 32 == 13 && (P2 + 31) / 32 == 3 && (P3 + 31) / 32 == 2, "tile deal");
  static_assert(OFF_A1 % 16 == 0 && LDS_BYTES <= 160 * 1024, "LDS");
};
using GeoAtari = TGeo<4, 84, 84>;    // 154464 B LDS
using GeoDmlab = TGeo<3, 72, 96>;
namespace torso {   // Atari constants used by the helper kernels below
constexpr int IN_BYTES = GeoAtari::IN_BYTES;
}

// 16 uint8 of the CHW frame (chunk c) -> bf16 space-to-depth image (the only u8->bf16
// conversion of a frame).  Every dword is 4 consecutive x of one row: (ci, y, X) -> s2d pixel
// (y/4, X), channels ci*16 + (y%4)*4 + 0..3, one 8-byte store.
// act1 pixel P, 16-byte chunk c (channels 8c .. 8c+7) -> byte offset in the act1 image
__device__ __forceinline__ int tf_a1_off(int P, int c) {
  return ((P >> 2) << 8) + (((((P & 3) << 2) | c) ^ ((P >> 2) & 15)) << 4);
}

// lane -> frame chunk inside each wave's block of 64 chunks: lane l takes chunk (25 l) mod 64, so
// the 16 lanes of a ds_write_b64 group land on more distinct banks of the space-to-depth image
// (modelled 8-byte store conflicts: 1328 -> 887 group-cycles per frame, ideal 448)
__device__ __forceinline__ int tf_chunk(int t) { return (t & ~63) | ((t * 25) & 63); }

template <class Gm>
__device__ __forceinline__ void torso_store_chunk(bf16* s2d, int c, const u32x4& v) {
  constexpr int RD = Gm::W / 4, PD = Gm::H * RD;   // dwords per row / per plane
  int d = 4 * c;                 // first dword of the chunk
  int ci = d / PD, r = d - ci * PD;
  int y = r / RD, X = r - y * RD;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const uint32_t w = v[e];
    bf16x4 o;
    o[0] = (bf16)(float)(w & 0xff);
    o[1] = (bf16)(float)((w >> 8) & 0xff);
    o[2] = (bf16)(float)((w >> 16) & 0xff);
    o[3] = (bf16)(float)(w >> 24);
    *(bf16x4*)(s2d + ((y >> 2) * Gm::W4 + X) * Gm::S2DS + ci * 16 + (y & 3) * 4) = o;
    if (++X == RD) {
      X = 0;
      if (++y == Gm::H) { y = 0; ++ci; }
    }
  }
}

// Phase A of the frame pipeline: conv1 of frame f over 13 pixel tiles, while conv3 of frame
// f-1 runs on waves 2 and 3.  Tiles are dealt so each SIMD (wave % 4) issues ~64 MFMAs:
//   SIMD0 (w0,w4) 4 conv1 tiles, SIMD1 (w1,w5) 4, SIMD2 (w2,w6) 3 + conv3, SIMD3 (w3,w7) 2 + conv3.
__constant__ int c_t1_begin[8] = {0, 2, 4, 5, 5, 7, 9, 11};
__constant__ int c_t1_count[8] = {2, 2, 1, 0, 2, 2, 2, 2};

// One launch can run up to TF_MAX_JOBS frame lists (e.g. the online and the target net's frames
// of one time chunk): the workers are split between the jobs in proportion to their frame
// counts, so each workgroup loads ONE weight set.  With reserve_slots > 0 the blocks of the
// last reserve_slots dispatch slots of XCDs 0..reserve_xcds-1 exit at once, leaving those CUs to a
// concurrently running persistent LSTM chunk (blocks are dealt to XCDs round-robin: b % 8).
#define TF_MAX_JOBS 4
struct TFJob {
  const int* rows;
  const bf16* w1; const float* b1;
  const bf16* w2; const float* b2;
  const bf16* w3; const float* b3;
  bf16* out; bf16* save1; bf16* save2;
  int n, wbegin, wcount, pad_;
};
struct TFArgs {
  const uint8_t* frames;
  TFJob job[TF_MAX_JOBS];
  int njobs, reserve_xcds, reserve_slots, pad_;
  long long* dbg;
  long long row_bytes;   // replay row stride (>= the frame's CIN*H*W bytes)
};

__device__ __forceinline__ int tf_worker(int reserve_xcds, int reserve_slots) {
  const int b = blockIdx.x;
  if (reserve_slots <= 0) return b;
  const int x = b & 7, s = b >> 3, keep = 32 - reserve_slots;
  if (s < keep) return b;
  if (x < reserve_xcds) return -1;
  return keep * 8 + (s - keep) * (8 - reserve_xcds) + (x - reserve_xcds);
}

template <class Gm>
__global__ __launch_bounds__(512) void torso_fwd_kernel(const TFArgs args) {
  constexpr int NT = Gm::NT, PF = Gm::PF, IN_CHUNKS = Gm::IN_CHUNKS;
  constexpr int P1 = Gm::P1, P2 = Gm::P2, P3 = Gm::P3, ACTS = Gm::ACTS;
  constexpr int W2S = Gm::W2S, W3S = Gm::W3S, S2DS = Gm::S2DS, K1S = Gm::K1S;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  bf16* in_bf = (bf16*)(lds + Gm::OFF_IN);
  bf16* act1 = (bf16*)(lds + Gm::OFF_A1);
  bf16* act2 = (bf16*)(lds + Gm::OFF_A2);
  bf16* lw2 = (bf16*)(lds + Gm::OFF_W2);
  bf16* lw3 = (bf16*)(lds + Gm::OFF_W3);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int half = lane >> 5, l32 = lane & 31;
  const int wk = tf_worker(args.reserve_xcds, args.reserve_slots);
  if (wk < 0) return;
  int ji = 0;
#pragma unroll
  for (int i = 1; i < TF_MAX_JOBS; ++i)
    if (i < args.njobs && wk >= args.job[i].wbegin) ji = i;
  const TFJob& J = args.job[ji];
  const int stride = J.wcount;
  if (wk - J.wbegin >= stride) return;
  const uint8_t* __restrict__ frames = args.frames;
  const long long rb = args.row_bytes;
  const int* __restrict__ rows = J.rows;
  const int n_frames = J.n;
  const bf16* __restrict__ w1 = J.w1; const float* __restrict__ b1 = J.b1;
  const bf16* __restrict__ w2 = J.w2; const float* __restrict__ b2 = J.b2;
  const bf16* __restrict__ w3 = J.w3; const float* __restrict__ b3 = J.b3;
  bf16* __restrict__ out = J.out;
  bf16* __restrict__ save1 = J.save1;
  bf16* __restrict__ save2 = J.save2;
  long long* __restrict__ dbg = args.dbg;

  // ---- weights -> LDS (conv2, conv3) with padded rows; conv1 fragments -> VGPRs
  for (int i = tid; i < 32 * 64; i += NT) {   // conv2: 32 rows x 64 chunks of 8 bf16
    const int r = i >> 6, c = i & 63;
    *(bf16x8*)(lw2 + r * W2S + c * 8) = *(const bf16x8*)(w2 + r * 512 + c * 8);
  }
  for (int i = tid; i < 32 * 36; i += NT) {   // conv3: 32 rows x 36 chunks
    const int r = i / 36, c = i % 36;
    *(bf16x8*)(lw3 + r * W3S + c * 8) = *(const bf16x8*)(w3 + r * 288 + c * 8);
  }
  bf16x8 wf1[K1S];
#pragma unroll
  for (int s = 0; s < K1S; ++s) wf1[s] = *(const bf16x8*)(w1 + l32 * (16 * K1S) + s * 16 + half * 8);
  float bias1[16];
  const bool conv3_wave = (wave == 2 || wave == 3), conv2_wave = wave < 3;
#pragma unroll
  for (int r = 0; r < 16; ++r) bias1[r] = b1[(r & 3) + 8 * (r >> 2) + 4 * half];
  float* lb23 = (float*)(lds + Gm::OFF_B23);   // epilogue biases of conv2 / conv3 (LDS broadcast)
  if (tid < 64) lb23[tid] = tid < 32 ? b2[tid] : b3[tid - 32];
  const int t1b = c_t1_begin[wave], t1n = c_t1_count[wave];

  int f = wk - J.wbegin;
  if (f >= n_frames) return;
  // ---- prologue: first frame -> LDS (bf16)
  {
    const size_t row = rows ? (size_t)ld_uniform_i32(rows, f) : (size_t)f;
    const u32x4* src = (const u32x4*)(frames + row * rb);
    for (int t = tid; t < ((IN_CHUNKS + 63) & ~63); t += NT) {
      const int c = tf_chunk(t);
      if (c < IN_CHUNKS) torso_store_chunk<Gm>(in_bf, c, src[c]);
    }
  }
  __syncthreads();

  int fprev = -1, it_dbg = 0;
#define TF_TRACE(k) \
  if (dbg && wk == 0 && tid == 0 && it_dbg < 16) dbg[it_dbg * 8 + (k)] = clock64();
  // replay row of the next frame, read one frame ahead so the prefetch never waits on its address
  int row_nx = f + stride < n_frames ? (rows ? ld_uniform_i32(rows, f + stride) : f + stride) : 0;
  for (;;) {
    const bool have = f < n_frames;
    const int fn = f + stride;
    const int fnn = fn + stride;
    const int row_nn = fnn < n_frames ? (rows ? ld_uniform_i32(rows, fnn) : fnn) : 0;
    u32x4 pf[PF];
    TF_TRACE(0);
    // =================== phase A: conv1(f) || conv3(f-1)
    if (have) {
      // waves 3..7 prefetch frame f+stride into registers (lands while the convolutions run);
      // they convert it into LDS during phase B while waves 0..2 run conv2
      if (fn < n_frames && wave >= 3) {
        const u32x4* src = (const u32x4*)(frames + (size_t)row_nx * rb);
#pragma unroll
        for (int q = 0; q < PF; ++q) {
          const int c = tf_chunk(tid - 192 + q * 320);
          if (c < IN_CHUNKS) pf[q] = src[c];
        }
      }
      for (int i = 0; i < t1n; ++i) {
        const int pt = t1b + i;
        const int p = pt * 32 + l32;
        const int pc = p < P1 ? p : P1 - 1;
        const int oy = pc / Gm::W1, ox = pc % Gm::W1;
        // K step s: s2d block (by, bx) = (s / 2CIN, (s / CIN) & 1), channels ci*16 + 8*half .. +8
        const bf16* base = in_bf + (oy * Gm::W4 + ox) * S2DS + half * 8;
        f32x16 acc = {};
        mfma_pipe<K1S, 4>(acc, [&](int s) { return wf1[s]; }, [&](int s) {
          const int by = s / (2 * Gm::CIN), bx = (s / Gm::CIN) & 1, ci = s % Gm::CIN;
          return *(const bf16x8*)(base + (by * Gm::W4 + bx) * S2DS + ci * 16);
        });
        if (p < P1) {
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            bf16x4 v;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float x = acc[4 * g + e] * (1.f / 255.f) + bias1[4 * g + e];
              v[e] = (bf16)fmaxf(x, 0.f);
            }
            *(bf16x4*)((uint8_t*)act1 + tf_a1_off(p, g) + 8 * half) = v;
          }
        }
      }
    }
    if (fprev >= 0 && conv3_wave) {
      // conv3(f-1): 2 pixel tiles, K = 288 = (kh 3, kw 3, ci 32)
      const int p = (wave - 2) * 32 + l32;
      const int pc = p < P3 ? p : P3 - 1;
      const int oy = pc / Gm::W3, ox = pc % Gm::W3;
      const bf16* abase = lw3 + l32 * W3S + half * 8;
      const bf16* bbase = act2 + (oy * Gm::W2 + ox) * ACTS + half * 8;
      f32x16 acc = {};
      mfma_pipe<18, 3>(acc, [&](int s) { return *(const bf16x8*)(abase + s * 16); }, [&](int s) {
        const int khkw = s >> 1, kh = khkw / 3, kw = khkw % 3;
        return *(const bf16x8*)(bbase + (kh * Gm::W2 + kw) * ACTS + (s & 1) * 16);
      });
      if (p < P3) {
        bf16* o = out + (size_t)fprev * Gm::OUT + p;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int co = (r & 3) + 8 * (r >> 2) + 4 * half;
          o[co * P3] = (bf16)fmaxf(acc[r] + lb23[32 + co], 0.f);
        }
      }
    }
    TF_TRACE(1);
    lds_sync();
    TF_TRACE(2);
    if (!have) break;

    // =================== phase B: conv2(f) on waves 0..2; frame f+stride -> LDS; save act1(f)
    if (conv2_wave) {
      const int p = wave * 32 + l32;
      const int pc = p < P2 ? p : P2 - 1;
      const int oy = pc / Gm::W2, ox = pc % Gm::W2;
      const bf16* abase = lw2 + l32 * W2S + half * 8;
      int oz;
      asm volatile("v_mov_b32 %0, 0" : "=v"(oz));
      const int P0 = (2 * oy) * Gm::W1 + 2 * ox + oz;   // (+oz: offsets computed per step, not hoisted)
      const uint8_t* a1b = (const uint8_t*)act1;
      f32x16 acc = {};
      mfma_pipe<32, 3>(acc, [&](int s) { return *(const bf16x8*)(abase + s * 16); }, [&](int s) {
        const int khkw = s >> 1, kh = khkw >> 2, kw = khkw & 3;
        return *(const bf16x8*)(a1b + tf_a1_off(P0 + kh * Gm::W1 + kw, (s & 1) * 2 + half));
      });
      TF_TRACE(4);
      if (p < P2) {
        bf16* d2 = save2 ? save2 + ((size_t)f * P2 + p) * 32 : nullptr;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          bf16x4 v;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int co = 4 * half + 8 * g + e;
            v[e] = (bf16)fmaxf(acc[4 * g + e] + lb23[co], 0.f);
          }
          *(bf16x4*)(act2 + p * ACTS + 8 * g + 4 * half) = v;
          if (d2) *(bf16x4*)(d2 + 8 * g + 4 * half) = v;
        }
      }
    } else if (save1 != nullptr) {
      // waves 3..7 copy the channels-last conv1 activations out for the backward pass
      const int t5 = tid - 192;  // 0..319
      bf16* d1 = save1 + (size_t)f * P1 * 32;
      for (int i = t5; i < P1 * 4; i += 320) {   // linear LDS chunks -> (pixel, chunk)
        const int row = i >> 4, pcv = (i & 15) ^ (row & 15);
        const int px = row * 4 + (pcv >> 2), q = pcv & 3;
        if (px < P1) *(bf16x8*)(d1 + px * 32 + q * 8) = *(const bf16x8*)((const uint8_t*)act1 + i * 16);
      }
    }
    TF_TRACE(5);
    // conv1(f) finished reading in_bf before the barrier above
    if (fn < n_frames && wave >= 3) {
#pragma unroll
      for (int q = 0; q < PF; ++q) {
        const int c = tf_chunk(tid - 192 + q * 320);
        if (c < IN_CHUNKS) torso_store_chunk<Gm>(in_bf, c, pf[q]);
      }
    }
    TF_TRACE(6);
    lds_sync();
    TF_TRACE(3);
    fprev = f;
    f = fn;
    row_nx = row_nn;
    ++it_dbg;
  }
}

// Expand uint8 frames (selected rows) to bf16/255 NCHW for the conv1 weight-gradient pass.
__global__ void frames_to_bf16_kernel(const uint8_t* __restrict__ frames, const int* __restrict__ rows,
                                      int n_frames, bf16* __restrict__ out) {
  const int f = blockIdx.y;
  const size_t row = rows ? (size_t)ld_uniform_i32(rows, f) : (size_t)f;
  const uint8_t* src = frames + row * torso::IN_BYTES;
  bf16* dst = out + (size_t)f * torso::IN_BYTES;
  for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < torso::IN_BYTES / 8;
       c += gridDim.x * blockDim.x) {
    const u32x2 v = ((const u32x2*)src)[c];
    bf16x8 o = u8x8_to_bf16(v[0], v[1]);
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (bf16)((float)o[e] * (1.f / 255.f));
    ((bf16x8*)dst)[c] = o;
  }
}

// Same, channels-last (N, 84, 84, 4) so the library conv1 weight-gradient pass needs no transpose.
__global__ void frames_to_bf16_nhwc_kernel(const uint8_t* __restrict__ frames,
                                           const int* __restrict__ rows, int n_frames,
                                           bf16* __restrict__ out) {
  const int f = blockIdx.y;
  const size_t row = rows ? (size_t)ld_uniform_i32(rows, f) : (size_t)f;
  const uint8_t* src = frames + row * torso::IN_BYTES;
  bf16x4* dst = (bf16x4*)(out + (size_t)f * torso::IN_BYTES);
  constexpr int PIX = 84 * 84;
  for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < PIX; p += gridDim.x * blockDim.x) {
    bf16x4 o;
#pragma unroll
    for (int c = 0; c < 4; ++c) o[c] = (bf16)((float)src[c * PIX + p] * (1.f / 255.f));
    dst[p] = o;
  }
}

// Any frame geometry (the library conv path, e.g. DMLab 3x72x96): gather replay rows of C
// uint8 planes of HW pixels and write channels-last bf16 (N, H, W, C) * scale in one pass --
// replaces index_select + dtype cast + channels-last copy (three full passes over the batch).
__global__ void frames_gather_nhwc_kernel(const uint8_t* __restrict__ frames, int64_t row_bytes,
                                          const int* __restrict__ rows, int C, int HW, float scale,
                                          bf16* __restrict__ out) {
  const int f = blockIdx.y;
  const size_t row = rows ? (size_t)ld_uniform_i32(rows, f) : (size_t)f;
  const uint8_t* src = frames + row * row_bytes;
  bf16* dst = out + (size_t)f * HW * C;
  for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < HW; p += gridDim.x * blockDim.x)
    for (int c = 0; c < C; ++c) dst[(size_t)p * C + c] = (bf16)((float)src[(size_t)c * HW + p] * scale);
}

// Vector form for C <= 4 planes and HW % 4 == 0: a thread moves 4 pixels -- one 4-byte load
// per plane, C 8-byte stores of the 4 x C interleaved bf16 (the scalar form issues byte loads
// and 2-byte stores: 180 us for a DMLab batch of 5440 frames).
template <int C>
__global__ void frames_gather_nhwc4_kernel(const uint8_t* __restrict__ frames, int64_t row_bytes,
                                           const int* __restrict__ rows, int HW, float scale,
                                           bf16* __restrict__ out) {
  const int f = blockIdx.y;
  const size_t row = rows ? (size_t)ld_uniform_i32(rows, f) : (size_t)f;
  const uint8_t* src = frames + row * row_bytes;
  bf16* dst = out + (size_t)f * HW * C;
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < HW / 4; q += gridDim.x * blockDim.x) {
    uint32_t v[C];
#pragma unroll
    for (int c = 0; c < C; ++c) v[c] = *(const uint32_t*)(src + (size_t)c * HW + 4 * q);
    bf16 o[4 * C];
#pragma unroll
    for (int px = 0; px < 4; ++px)
#pragma unroll
      for (int c = 0; c < C; ++c) o[px * C + c] = (bf16)((float)((v[c] >> (8 * px)) & 0xff) * scale);
#pragma unroll
    for (int i = 0; i < C; ++i)
      ((bf16x4*)(dst + (size_t)4 * q * C))[i] = bf16x4{o[4 * i], o[4 * i + 1], o[4 * i + 2], o[4 * i + 3]};
  }
}

extern "C" int r2_frames_gather_nhwc(const uint8_t* frames, int64_t row_bytes, const int* rows,
                                     int n_frames, int C, int HW, float scale, bf16* out,
                                     void* stream) {
  if (n_frames <= 0) return 0;
  if (n_frames > 65535 * 16 || C < 1 || HW < 1 || (int64_t)C * HW > row_bytes) return -1;
  const bool vec = C <= 4 && HW % 4 == 0 && row_bytes % 4 == 0 && ((uintptr_t)frames & 3) == 0 &&
                   ((uintptr_t)out & 7) == 0;
  const int work = vec ? HW / 4 : HW;
  const int bx = (work + 255) / 256 < 64 ? (work + 255) / 256 : 64;
  for (int f0 = 0; f0 < n_frames; f0 += 65535) {   // grid.y limit
    const int nf = n_frames - f0 < 65535 ? n_frames - f0 : 65535;
    const uint8_t* fr = rows ? frames : frames + (size_t)f0 * row_bytes;
    const int* rw = rows ? rows + f0 : nullptr;
    bf16* o = out + (size_t)f0 * HW * C;
    hipStream_t s = (hipStream_t)stream;
    const dim3 g(bx, nf), b(256);
    if (vec && C == 1) hipLaunchKernelGGL(frames_gather_nhwc4_kernel<1>, g, b, 0, s, fr, row_bytes, rw, HW, scale, o);
    else if (vec && C == 2) hipLaunchKernelGGL(frames_gather_nhwc4_kernel<2>, g, b, 0, s, fr, row_bytes, rw, HW, scale, o);
    else if (vec && C == 3) hipLaunchKernelGGL(frames_gather_nhwc4_kernel<3>, g, b, 0, s, fr, row_bytes, rw, HW, scale, o);
    else if (vec && C == 4) hipLaunchKernelGGL(frames_gather_nhwc4_kernel<4>, g, b, 0, s, fr, row_bytes, rw, HW, scale, o);
    else hipLaunchKernelGGL(frames_gather_nhwc_kernel, g, b, 0, s, fr, row_bytes, rw, C, HW, scale, o);
  }
  R2_CHECK_LAUNCH();
  return 0;
}

// x = relu(x + bias[c]) in place on a channels-last bf16 activation (C % 8 == 0): the library
// conv path's bias add + ReLU in one pass (MIOpen's separate bias op + a clamp pass were two).
__global__ void bias_relu_nhwc_kernel(bf16* __restrict__ x, const float* __restrict__ bias, int C,
                                      int64_t n8) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n8; i += stride) {
    bf16x8 v = ((bf16x8*)x)[i];
    const int c0 = (int)((i * 8) % C);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = (bf16)fmaxf((float)v[e] + bias[c0 + e], 0.f);
    ((bf16x8*)x)[i] = v;
  }
}

extern "C" int r2_bias_relu_nhwc_bf16(bf16* x, const float* bias, int C, int64_t n, void* stream) {
  if (n <= 0) return 0;
  if (C % 8 || n % C || ((uintptr_t)x & 15)) return -1;
  int64_t blocks = (n / 8 + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(bias_relu_nhwc_kernel, dim3((unsigned)blocks), dim3(256), 0,
                     (hipStream_t)stream, x, bias, C, n / 8);
  R2_CHECK_LAUNCH();
  return 0;
}

// grad * (act > 0) on bf16 tensors with identical memory layout (ReLU backward from output)
__global__ void relu_mask_bf16_kernel(const bf16* __restrict__ g, const bf16* __restrict__ act,
                                      bf16* __restrict__ out, int64_t n8) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n8; i += stride) {
    bf16x8 gv = ((const bf16x8*)g)[i];
    const bf16x8 av = ((const bf16x8*)act)[i];
#pragma unroll
    for (int e = 0; e < 8; ++e) gv[e] = ((float)av[e] > 0.f) ? gv[e] : (bf16)0.f;
    ((bf16x8*)out)[i] = gv;
  }
}

extern "C" int r2_frames_to_bf16_nhwc(const uint8_t* frames, const int* rows, int n_frames,
                                      bf16* out, void* stream) {
  if (n_frames <= 0) return 0;
  hipLaunchKernelGGL(frames_to_bf16_nhwc_kernel, dim3(7, n_frames), dim3(1024), 0,
                     (hipStream_t)stream, frames, rows, n_frames, out);
  R2_CHECK_LAUNCH();
  return 0;
}

extern "C" int r2_relu_mask_bf16(const bf16* g, const bf16* act, bf16* out, int64_t n,
                                 void* stream) {
  if (n <= 0) return 0;
  if ((n & 7) || (((uintptr_t)g | (uintptr_t)act | (uintptr_t)out) & 15)) return -1;
  int64_t blocks = (n / 8 + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(relu_mask_bf16_kernel, dim3((unsigned)blocks), dim3(256), 0,
                     (hipStream_t)stream, g, act, out, n / 8);
  R2_CHECK_LAUNCH();
  return 0;
}


static long long* g_tf_dbg = nullptr;
extern "C" int r2_torso_fwd_set_debug(long long* p) { g_tf_dbg = p; return 0; }

template <class Gm>
static void tf_launch(const TFArgs& a, int grid, hipStream_t s) {
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute((const void*)torso_fwd_kernel<Gm>, hipFuncAttributeMaxDynamicSharedMemorySize,
                        Gm::LDS_BYTES);
    attr_set = true;
  }
  hipLaunchKernelGGL(torso_fwd_kernel<Gm>, dim3(grid), dim3(Gm::NT), Gm::LDS_BYTES, s, a);
}

// jobs: njobs x 12 int64 {rows, n, w1, b1, w2, b2, w3, b3, out, save1, save2, 0}.
// grid 0 = one block per CU (256); reserve_slots > 0 (grid must then be 256) keeps the last
// reserve_slots dispatch slots of XCDs 0..reserve_xcds-1 free (see tf_worker).
// geom: (cin, h, w) of the frame = 4x84x84 (Atari) or 3x72x96 (DMLab-30); row_bytes: the replay
// row stride (0 = the frame's bytes).
extern "C" int r2_torso_fwd_geom(const uint8_t* frames, long long row_bytes, const int64_t* jobs,
                                 int njobs, int grid, int reserve_xcds, int reserve_slots, int cin,
                                 int h, int w, void* stream) {
  if (njobs < 1 || njobs > TF_MAX_JOBS) return -1;
  if (reserve_slots < 0 || reserve_slots >= 32 || reserve_xcds < 0 || reserve_xcds > 8) return -2;
  const bool atari = cin == 4 && h == 84 && w == 84, dm = cin == 3 && h == 72 && w == 96;
  if (!atari && !dm) return -6;
  const long long fb = (long long)cin * h * w;
  if (row_bytes <= 0) row_bytes = fb;
  if (row_bytes < fb || row_bytes % 16) return -7;
  TFArgs a{};
  a.frames = frames;
  a.row_bytes = row_bytes;
  a.njobs = 0;
  a.reserve_xcds = reserve_xcds;
  a.reserve_slots = reserve_slots;
  a.dbg = g_tf_dbg;
  int64_t total = 0;
  for (int i = 0; i < njobs; ++i) total += jobs[12 * i + 1] > 0 ? jobs[12 * i + 1] : 0;
  if (total <= 0) return 0;
  if (reserve_slots > 0) grid = 256;
  if (grid <= 0) grid = 256;
  const int nw = reserve_slots > 0 ? (32 - reserve_slots) * 8 + reserve_slots * (8 - reserve_xcds)
                                   : grid;
  // workers in proportion to frame counts (>= 1 each, never more than the job's frames)
  int wb = 0;
  int64_t seen = 0;
  for (int i = 0; i < njobs; ++i) {
    const int64_t* p = jobs + 12 * i;
    if (p[1] <= 0) continue;
    seen += p[1];
    int end = (int)((seen * nw + total - 1) / total);
    if (end > nw) end = nw;
    int cnt = end - wb;
    if (cnt < 1) cnt = 1;
    if (cnt > p[1]) cnt = (int)p[1];
    TFJob& J = a.job[a.njobs++];
    J.rows = (const int*)p[0]; J.n = (int)p[1];
    J.w1 = (const bf16*)p[2]; J.b1 = (const float*)p[3];
    J.w2 = (const bf16*)p[4]; J.b2 = (const float*)p[5];
    J.w3 = (const bf16*)p[6]; J.b3 = (const float*)p[7];
    J.out = (bf16*)p[8]; J.save1 = (bf16*)p[9]; J.save2 = (bf16*)p[10];
    J.wbegin = wb; J.wcount = cnt; J.pad_ = 0;
    wb += cnt;
  }
  if (wb > nw) return -3;   // more jobs than workers
  if (reserve_slots <= 0 && grid > wb) grid = wb;
  if (atari) tf_launch<GeoAtari>(a, grid, (hipStream_t)stream);
  else tf_launch<GeoDmlab>(a, grid, (hipStream_t)stream);
  R2_CHECK_LAUNCH();
  return 0;
}

extern "C" int r2_torso_fwd_multi(const uint8_t* frames, const int64_t* jobs, int njobs,
                                  int grid, int reserve_xcds, int reserve_slots, void* stream) {
  return r2_torso_fwd_geom(frames, 0, jobs, njobs, grid, reserve_xcds, reserve_slots, 4, 84, 84,
                           stream);
}

extern "C" int r2_torso_fwd(const uint8_t* frames, const int* rows, int n_frames,
                            const bf16* w1, const float* b1, const bf16* w2, const float* b2,
                            const bf16* w3, const float* b3, bf16* out, bf16* save1, bf16* save2,
                            int max_blocks, void* stream) {
  if (n_frames <= 0) return 0;
  const int64_t job[12] = {(int64_t)rows, n_frames, (int64_t)w1, (int64_t)b1, (int64_t)w2,
                           (int64_t)b2, (int64_t)w3, (int64_t)b3, (int64_t)out, (int64_t)save1,
                           (int64_t)save2, 0};
  return r2_torso_fwd_multi(frames, job, 1, max_blocks, 0, 0, stream);
}

extern "C" int r2_frames_to_bf16(const uint8_t* frames, const int* rows, int n_frames, bf16* out,
                                 void* stream) {
  if (n_frames <= 0) return 0;
  hipLaunchKernelGGL(frames_to_bf16_kernel, dim3(4, n_frames), dim3(256), 0, (hipStream_t)stream,
                     frames, rows, n_frames, out);
  R2_CHECK_LAUNCH();
  return 0;
}
