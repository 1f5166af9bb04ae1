// Fused Atari conv-torso BACKWARD for gfx950 (MI355X).
//
// Replaces the library path (3x convolution_backward on MIOpen + ReLU-mask elementwise kernels +
// NCHW/NHWC transposes + bias reductions + a uint8->bf16 frame expansion) with ONE kernel + one
// slab reduction.  Reference semantics: model.py:12-22 (the conv stack) differentiated by
// learner.py:118-120 (loss.backward()).  Per learning frame, entirely in LDS (151 KB, 512
// threads, one workgroup per CU, grid-stride over frames, next frame prefetched in registers):
//
//   S0  frame u8 -> bf16 CHW image; act1/act2 (HWC) copied in; g3 = dX3 * (out3 > 0)
//   S1  g2 = convT(g3, W3) * (act2>0) (waves 5-7, W3 from LDS)
//       (dW3 += g3 . im2col(act2) and db3 run in the light torso_dw3_kernel straight from global
//       dX3/out3/act2: keeping their 2 accumulator tiles here would push the fused kernel past 256
//       VGPRs, and its spill reloads would wait (in-order vmcnt) on the next-frame prefetch)
//   S2  dW2 += g2 . im2col(act1)      (2 N tiles per wave)
//       g1 = convT_s2(g2, W2) * (act1>0): the stride-2 transposed conv split into its 4 output
//            phases (only the 4 taps that hit a phase are multiplied; each wave keeps its phase's
//            W2 slice in VGPRs)
//   S3  dW1 += g1 . im2col(frame)     (1 N tile per wave, K = 400 pixels in 25 steps)
//
// No im2col is ever materialised: the weight-gradient B operands (rows = pixels, columns =
// (kh,kw,ci) or (ci,kh,kw)) are gathered straight from the HWC activation images / the CHW frame
// image with ds_read_b64_tr_b16 -- each lane names one 4-element row piece of the im2col matrix
// and the hardware transpose hands every lane its 8-pixel column fragment.  conv1's pixels run in
// 4x4 blocks (K step s = block (s/5, s%5)), so every tr-read address is a per-lane base plus an
// immediate; the A operand g1 is stored in that same K order.  Weight-gradient accumulators stay
// in MFMA registers across all frames (dW1: 1, dW2: 2, dW3: <=2 32x32 tiles per wave); each
// workgroup finally writes one fp32 slab and torso_grad_reduce_kernel sums the slabs straight
// into the flat gradient buffer (deterministic; torch layout via an index map,
// engine/layout.py torso_grad_map).
#include "../common.h"
#include "../slab_reduce.h"

// Geometry of the fused backward (template parameter): CIN uint8 planes of H x W (multiples of
// 4); instantiated for the Atari stack 4x84x84 and DMLab-30 RGB 3x72x96.
template <int CIN_, int H_, int W_>
struct TBGeo {
  static constexpr int CIN = CIN_, H = H_, W = W_;
  static constexpr int NT = 512;
  static constexpr int H1 = (H - 8) / 4 + 1, W1 = (W - 8) / 4 + 1;     // conv1 output
  static constexpr int H2 = (H1 - 4) / 2 + 1, W2 = (W1 - 4) / 2 + 1;   // conv2 output
  static constexpr int H3 = H2 - 2, W3 = W2 - 2;                       // conv3 output
  static constexpr int P1 = H1 * W1, P2 = H2 * W2, P3 = H3 * W3, OUT = 32 * P3;
  static constexpr int IN_BYTES = CIN * H * W;
  static constexpr int IN_CHUNKS = IN_BYTES / 16;
  // bordered gradient images: g3 (border 2, convT by W3), g2 (border 1; also covers the phase
  // grid of the stride-2 transposed conv: act1 pixel (2ay+py, 2bx+px) reads g2 (ay+1-khi, ..))
  static constexpr int PHH = (H1 + 1) / 2, PHW = (W1 + 1) / 2;          // phase grid
  static constexpr int G3H = H3 + 4, G3W = W3 + 4;
  static constexpr int G2H = (H2 + 2 > PHH + 1 ? H2 + 2 : PHH + 1), G2W = (W2 + 2 > PHW + 1 ? W2 + 2 : PHW + 1);
  static constexpr int G3N = G3H * G3W, G2N = G2H * G2W;
  // conv1 pixels in 4x4 blocks (padded to whole blocks; padded rows of g1 stay zero)
  static constexpr int BH = (H1 + 3) / 4, BW = (W1 + 3) / 4, NB1 = BH * BW;
  static constexpr int K2S = (P2 + 15) / 16, K3S = (P3 + 15) / 16;     // dW2 / dW3 K steps
  static constexpr int T1 = 2 * CIN;                                    // dW1 column tiles
  static constexpr int G3C_S = 72;                                      // g3 chw row stride (dw3)
  static constexpr int W3S = 288 + 8;                                   // conv3_dg rows in LDS
  static constexpr int FRB = 0;                                         // frame bf16 CHW
  static constexpr int A1 = FRB + IN_BYTES * 2;                         // act1 hwc [P1][32]
  static constexpr int A2 = A1 + P1 * 32 * 2;                           // act2 hwc [P2][32]
  static constexpr int G3P = A2 + P2 * 32 * 2;                          // g3 [G3N][32]
  static constexpr int G2P = G3P + G3N * 32 * 2;                        // g2 [G2N + trash][32]
  static constexpr int G1H = G2P + (G2N + 1) * 32 * 2;                  // g1 [16 NB1 + trash][32]
  static constexpr int W3L = G1H + (16 * NB1 + 6) * 32 * 2;             // conv3_dg [32][296]
  static constexpr int TBL2 = W3L + 32 * W3S * 2;                       // dW2 gather int2 [2 K2S][64]
  static constexpr int TE1 = TBL2 + 2 * K2S * 64 * 8;                   // dact1 epilogue rows [128]
  static constexpr int TE2 = TE1 + 128 * 4;                             // dact2 epilogue rows [96]
  static constexpr int LDS = TE2 + 96 * 4;
  static constexpr int G2_TRASH = G2N, G1_TRASH = 16 * NB1;
  static constexpr int PF1 = (P1 * 4 + NT - 1) / NT;                    // act1 prefetch chunks / thread
  static constexpr int PFF = (IN_CHUNKS + NT - 1) / NT;                 // frame prefetch chunks / thread
  static constexpr int OFF_W2 = 32 * CIN * 64, OFF_W3 = OFF_W2 + 32 * 512, OFF_B = OFF_W3 + 32 * 288;
  static constexpr int SLAB = OFF_B + 96;                               // floats per workgroup
  static_assert(LDS <= 160 * 1024, "LDS");
  static_assert(P2 <= 96 && PHH * PHW <= 128 && P3 <= 64 && OUT % 8 == 0 && OUT / 8 <= 512, "tiles");
  static_assert(16 * NB1 + 6 < (1 << 13) && P1 < (1 << 13), "epilogue table fields");
};
using BGeoAtari = TBGeo<4, 84, 84>;
using BGeoDmlab = TBGeo<3, 72, 96>;
namespace tb {   // the Atari slab (shared with the split-precision backward, torso_sp.hip)
constexpr int SLAB = BGeoAtari::SLAB;   // 33888
}

struct TBArgs {
  const uint8_t* frames;
  const int* rows;     // replay rows of the N learning frames
  const bf16* act1;    // (N, P1, 32) channels-last, from the forward kernel
  const bf16* act2;    // (N, P2, 32)
  const bf16* dx3;     // (N, OUT) dL/d(torso output), CHW flatten
  const bf16* out3;    // (N, OUT) torso output (ReLU mask)
  const bf16* w3dg;    // (32 ci, 288 = (kh,kw,co))
  const bf16* w2dg;    // (4 phases, 32 ci, 128 = (khi,kwi,co))
  float* slab;         // (gridDim.x, SLAB)
  int n;
  long long* dbg;      // optional phase clock trace of workgroup 0 (tools/torso_probe.py)
  long long row_bytes; // replay row stride
};

typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) i16x4 lds_i16x4;

__device__ __forceinline__ bf16x8 ld8(const bf16* p) { return *(const bf16x8*)p; }
// two hardware-transposed LDS reads -> one 8-pixel B fragment (T10: ds_read_b64_tr_b16)
__device__ __forceinline__ bf16x8 tr8(const bf16* p0, const bf16* p1) {
  const i16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)p0);
  const i16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)p1);
  return __builtin_bit_cast(bf16x8, __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7));
}

// im2col row address (pixel part, bf16 elements) of the tr-read lane for K step s, read r:
// pixel P = 16s + 8*half + 4r + q (clamped: padded pixels meet zero g columns)
template <class Gb>
__device__ __forceinline__ int im2col_off3(int s, int r, int half, int q, int colb) {
  int P = 16 * s + 8 * half + 4 * r + q;
  P = P < Gb::P3 ? P : Gb::P3 - 1;
  return ((P / Gb::W3) * Gb::W2 + P % Gb::W3) * 32 + colb;
}

template <class Gb>
__global__ __launch_bounds__(512) void torso_bwd_kernel(const TBArgs a) {
  constexpr int NT = Gb::NT, P1 = Gb::P1, P2 = Gb::P2, P3 = Gb::P3, W1 = Gb::W1, W2 = Gb::W2;
  constexpr int PF1 = Gb::PF1, PFF = Gb::PFF, IN_CHUNKS = Gb::IN_CHUNKS, W3S = Gb::W3S;
  constexpr int G3W = Gb::G3W, G2W = Gb::G2W, PHW = Gb::PHW;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;

  // ---- once per workgroup: zero the bordered gradient images and g1 (borders and padded
  // pixels stay zero), conv3_dg -> LDS, the dW2 gather-offset table, this wave's conv2_dg phase
  // slice -> VGPRs
  for (int i = tid; i < (Gb::W3L - Gb::G3P) / 16; i += NT) ((u32x4*)(lds + Gb::G3P))[i] = u32x4{0, 0, 0, 0};
  for (int i = tid; i < 32 * 36; i += NT) {
    const int r = i / 36, c = i % 36;
    *(bf16x8*)((bf16*)(lds + Gb::W3L) + r * W3S + c * 8) = ld8(a.w3dg + r * 288 + c * 8);
  }
  for (int i = tid; i < 2 * Gb::K2S * 64; i += NT) {
    // K step s, read r, lane l: pixel P = 16s + 8h + 4r + q of the conv2 output (raster)
    const int sr = i >> 6, l = i & 63, sS = sr >> 1, r = sr & 1;
    const int h = l >> 5, qq = (l >> 2) & 3, cb = 16 * ((l >> 4) & 1) + 4 * (l & 3);
    const int P = 16 * sS + 8 * h + 4 * r + qq, Pc = P < P2 ? P : P2 - 1;
    const int arow = P < P2 ? (Pc / W2 + 1) * G2W + Pc % W2 + 1 : 0;   // a zero border row
    ((int2*)(lds + Gb::TBL2))[i] = make_int2(arow * 32 + cb, ((2 * (Pc / W2)) * W1 + 2 * (Pc % W2)) * 32 + cb);
  }
  // epilogue row tables: an accumulator row's pixel depends on (tile, lane half, register) only,
  // so its index math is done once here.  dact1: mask pixel | g1 row << 16 | odd-row-phase valid
  // << 29 | odd-column-phase valid << 30 | in-grid << 31.  dact2: mask pixel | g2 row << 16 | valid.
  for (int i = tid; i < 128 + 96; i += NT) {
    const int j = i < 128 ? i : i - 128, mt = j >> 5, h = (j >> 4) & 1, r = j & 15;
    const int m = mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
    uint32_t e;
    if (i < 128) {  // phase pixel (ay, bx) -> act1 pixel (2ay, 2bx) and 4x4-block g1 row
      const bool in = m < Gb::PHH * PHW;
      const int mv = in ? m : Gb::PHH * PHW - 1, ay = mv / PHW, bx = mv % PHW;
      const int kb = 16 * (Gb::BW * (ay >> 1) + (bx >> 1)) + 8 * (ay & 1) + 2 * (bx & 1);
      e = (uint32_t)((2 * ay) * W1 + 2 * bx) | (uint32_t)(in ? kb : Gb::G1_TRASH) << 16 |
          (uint32_t)(2 * ay + 1 < Gb::H1) << 29 | (uint32_t)(2 * bx + 1 < W1) << 30 | (uint32_t)in << 31;
    } else {        // dact2: conv2 output pixel -> act2 pixel and bordered g2 row
      const int qv = m < P2 ? m : P2 - 1;
      e = (uint32_t)qv | (uint32_t)(m < P2 ? (qv / W2 + 1) * G2W + qv % W2 + 1 : Gb::G2_TRASH) << 16 |
          (uint32_t)(m < P2) << 31;
    }
    ((uint32_t*)(lds + Gb::TE1))[i] = e;
  }
  bf16x8 w2f[8];
  {
    const int l32 = lane & 31, half = lane >> 5;
#pragma unroll
    for (int s = 0; s < 8; ++s) w2f[s] = ld8(a.w2dg + ((wave >> 1) * 32 + l32) * 128 + s * 16 + half * 8);
  }

  f32x16 acc1 = {}, acc2a = {}, acc2b = {};
  float db1p = 0.f, db2p = 0.f;

  // ---- register prefetch of one frame's inputs
  u32x4 pfr[PFF], pa1[PF1], pa2, pdx, po3;
  auto prefetch_frame = [&](int row) {
    const u32x4* src = (const u32x4*)(a.frames + (size_t)row * a.row_bytes);
#pragma unroll
    for (int k = 0; k < PFF; ++k) {
      const int c = tid + k * NT;
      if (c < IN_CHUNKS) pfr[k] = src[c];
    }
  };
  auto prefetch_acts = [&](int f) {
    const u32x4* s1 = (const u32x4*)(a.act1 + (size_t)f * P1 * 32);
#pragma unroll
    for (int k = 0; k < PF1; ++k) {
      const int c = tid + k * NT;
      if (c < P1 * 4) pa1[k] = s1[c];
    }
    if (tid < P2 * 4) pa2 = ((const u32x4*)(a.act2 + (size_t)f * P2 * 32))[tid];
    if (tid < Gb::OUT / 8) {
      pdx = ((const u32x4*)(a.dx3 + (size_t)f * Gb::OUT))[tid];
      po3 = ((const u32x4*)(a.out3 + (size_t)f * Gb::OUT))[tid];
    }
  };
  if (blockIdx.x < a.n) {
    prefetch_frame(ld_uniform_i32(a.rows, blockIdx.x));
    prefetch_acts(blockIdx.x);
  }
  // replay row of the frame after next is read one frame ahead, so issuing a prefetch never
  // waits a memory round trip for its own address
  int row_nx = blockIdx.x + gridDim.x < a.n ? ld_uniform_i32(a.rows, blockIdx.x + gridDim.x) : 0;
  __syncthreads();

  int it_dbg = 0;
#define TB_TRACE(k)                                                                  \
  if (a.dbg && blockIdx.x == 0 && tid == 0 && it_dbg < 16) a.dbg[it_dbg * 8 + (k)] = clock64();
  for (int f = blockIdx.x; f < a.n; f += gridDim.x) {
    TB_TRACE(0);
    // Re-derive the LDS region pointers and lane roles from an opaque zero each frame: otherwise
    // the compiler hoists every frame-invariant fragment address (dozens per lane) out of the
    // frame loop and spills them.
    int oz;
    asm volatile("s_mov_b32 %0, 0" : "=s"(oz));
    bf16* frb = (bf16*)(lds + Gb::FRB + oz);
    bf16* a1 = (bf16*)(lds + Gb::A1 + oz);
    bf16* a2 = (bf16*)(lds + Gb::A2 + oz);
    bf16* g3p = (bf16*)(lds + Gb::G3P + oz);
    bf16* g2p = (bf16*)(lds + Gb::G2P + oz);
    bf16* g1h = (bf16*)(lds + Gb::G1H + oz);
    bf16* w3l = (bf16*)(lds + Gb::W3L + oz);
    const int2* tbl2 = (const int2*)(lds + Gb::TBL2 + oz);
    // transposed-read lane roles: group grp of 16 lanes, row q (pixel within a quad), column
    // piece pp; colb = first of the lane's 4 im2col columns in a tile
    const int lane_f = lane + oz;
    const int l32 = lane_f & 31, half = lane_f >> 5;
    const int grp = lane_f >> 4, q = (lane_f >> 2) & 3, pp = lane_f & 3;
    const int colb = 16 * (grp & 1) + 4 * pp;
    // dW1 (tile = wave < 2 CIN): columns (ci, kh, kw) with ci = wave/2, kh = 4(wave&1) + 2(grp&1) + pp/2
    const int kh1 = 4 * (wave & 1) + 2 * (grp & 1) + (pp >> 1);
    const bf16* fb0 = frb + (wave >> 1) * (Gb::H * Gb::W) + kh1 * Gb::W + 4 * (pp & 1) +
                      (4 * (2 * half)) * Gb::W + 4 * q;
    const bf16* fb1 = fb0 + 4 * Gb::W;

    // ======== S0: prefetched inputs -> LDS
    const int row_nn = f + 2 * (int)gridDim.x < a.n ? ld_uniform_i32(a.rows, f + 2 * gridDim.x) : 0;
#pragma unroll
    for (int k = 0; k < PFF; ++k) {
      const int c = tid + k * NT;
      if (c < IN_CHUNKS) {
        ((bf16x8*)(frb + c * 16))[0] = u8x8_to_bf16(pfr[k][0], pfr[k][1]);
        ((bf16x8*)(frb + c * 16))[1] = u8x8_to_bf16(pfr[k][2], pfr[k][3]);
      }
    }
#pragma unroll
    for (int k = 0; k < PF1; ++k) {
      const int c = tid + k * NT;
      if (c < P1 * 4) ((u32x4*)a1)[c] = pa1[k];
    }
    if (tid < P2 * 4) ((u32x4*)a2)[tid] = pa2;
    if (tid < Gb::OUT / 8) {  // g3 = dx3 * (out3 > 0): OUT = 8 per thread (CHW) -> bordered HWC
      const bf16x8 dx = __builtin_bit_cast(bf16x8, pdx), o3 = __builtin_bit_cast(bf16x8, po3);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int i = tid * 8 + e, co = i / P3, p = i % P3;
        const bf16 v = ((float)o3[e] > 0.f) ? dx[e] : (bf16)0.f;
        g3p[((p / Gb::W3 + 2) * G3W + p % Gb::W3 + 2) * 32 + co] = v;
      }
    }
    lds_sync();
    TB_TRACE(1);

    // ======== S1: dact2 -> g2 (waves 5-7); dW3/db3 run in torso_dw3_kernel
    if (wave >= 5) {
      const int mt = wave - 5;
      const int qq0 = mt * 32 + l32, qc = qq0 < P2 ? qq0 : P2 - 1;
      // A row of tap (kh,kw) = bordered pixel (qy-kh, qx-kw): lane base + per-step immediate
      const bf16* ab = g3p + (((qc / W2) + 2) * G3W + qc % W2 + 2) * 32 + half * 8;
      f32x16 acc = {};
      mfma_pipe<18, 3>(acc, [&](int s) {
        const int khkw = s >> 1;
        return ld8(ab - ((khkw / 3) * G3W + khkw % 3) * 32 + (s & 1) * 16);
      }, [&](int s) { return ld8(w3l + l32 * W3S + s * 16 + half * 8); });
      // epilogue: all 16 ReLU-mask reads issued before any use; rows past the conv2 pixels go
      // to a trash row (branch-free)
      const uint32_t* te = (const uint32_t*)(lds + Gb::TE2 + oz) + mt * 32 + half * 16;
#pragma unroll
      for (int r0 = 0; r0 < 16; r0 += 8) {
        uint32_t e[8];
        bf16 mk[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) e[r] = te[r0 + r];
#pragma unroll
        for (int r = 0; r < 8; ++r) mk[r] = a2[(e[r] & 0xffff) * 32 + l32];
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          const bf16 v = ((float)mk[r] > 0.f) ? (bf16)acc[r0 + r] : (bf16)0.f;
          g2p[((e[r] >> 16) & 0x1fff) * 32 + l32] = v;
          db2p += (e[r] >> 31) ? (float)v : 0.f;
        }
      }
    }
    lds_sync();
    TB_TRACE(2);

    // ======== S2: dW2 (tiles wave, wave+8) and dact1 -> g1 (jobs 2w, 2w+1)
    // the next frame's u8 frame starts loading here and its activations/gradients at the end of
    // S2: S2+S3 cover the latency, and the 28 activation VGPRs are not live across dact1
    const bool more = f + (int)gridDim.x < a.n;
    if (more) prefetch_frame(row_nx);
    row_nx = row_nn;
    TB_TRACE(5);
    {
      const int nt = wave;  // (kh, kw) = (nt>>2, nt&3); tile nt+8 is kh+2
      const bf16* b = a1 + ((nt >> 2) * W1 + (nt & 3)) * 32;
      const int2* tl = tbl2 + lane_f;
      // A = g2 (co x pixel) and B = im2col(act1) (pixel x ci), both by transposed reads
      mfma_pipe2<Gb::K2S, 2>(acc2a, acc2b, [&](int s) {
                               return tr8(g2p + tl[(2 * s) * 64].x, g2p + tl[(2 * s + 1) * 64].x);
                             },
                             [&](int s) { return tr8(b + tl[(2 * s) * 64].y, b + tl[(2 * s + 1) * 64].y); },
                             [&](int s) {
                               return tr8(b + 2 * W1 * 32 + tl[(2 * s) * 64].y, b + 2 * W1 * 32 + tl[(2 * s + 1) * 64].y);
                             });
    }
    TB_TRACE(6);
    {
      const int phase = wave >> 1, py = phase >> 1, px = phase & 1;
#pragma unroll 1
      for (int jj = 0; jj < 2; ++jj) {
        const int mt = (wave & 1) * 2 + jj;
        const int m = mt * 32 + l32, mc = m < Gb::PHH * PHW ? m : Gb::PHH * PHW - 1;
        // A row of tap t = bordered g2 pixel (ay - t/2, bx - t%2): lane base + immediate
        const bf16* ab = g2p + ((mc / PHW + 1) * G2W + mc % PHW + 1) * 32 + half * 8;
        f32x16 acc = {};
        mfma_pipe<8, 3>(acc, [&](int s) {
          const int tap = s >> 1;
          return ld8(ab - ((tap >> 1) * G2W + (tap & 1)) * 32 + (s & 1) * 16);
        }, [&](int s) { return w2f[s]; });
        // epilogue: mask reads batched, destinations in the 4x4-block K order of the conv1
        // weight-gradient pass, rows past the phase grid -> trash row (branch-free); a phase
        // pixel past the conv1 output (odd phases of an odd extent) writes a zero
        const uint32_t* te = (const uint32_t*)(lds + Gb::TE1 + oz) + mt * 32 + half * 16;
        const int moff = (py * W1 + px) * 32 + l32, koff = (4 * py + px) * 32 + l32;
        const uint32_t need = (1u << 31) | (uint32_t)py << 29 | (uint32_t)px << 30;
#pragma unroll
        for (int r0 = 0; r0 < 16; r0 += 8) {
          uint32_t e[8];
          bf16 mk[8];
#pragma unroll
          for (int r = 0; r < 8; ++r) e[r] = te[r0 + r];
#pragma unroll
          for (int r = 0; r < 8; ++r) mk[r] = a1[min((int)(e[r] & 0xffff) * 32 + moff, P1 * 32 - 1)];
#pragma unroll
          for (int r = 0; r < 8; ++r) {
            const bool ok = (e[r] & need) == need;
            const bf16 v = (ok && (float)mk[r] > 0.f) ? (bf16)acc[r0 + r] : (bf16)0.f;
            g1h[((e[r] >> 16) & 0x1fff) * 32 + koff] = v;
            db1p += ok ? (float)v : 0.f;
          }
        }
      }
    }
    TB_TRACE(7);
    if (more) prefetch_acts(f + gridDim.x);
    lds_sync();
    TB_TRACE(3);

    // ======== S3: dW1, K = NB1 steps of one 4x4 pixel block each (addresses = base + immediate)
    if (wave < Gb::T1) {
      mfma_pipe<Gb::NB1, 3>(acc1, [&](int s) {
        const int r0 = (16 * s + 8 * half + q) * 32 + colb;
        return tr8(g1h + r0, g1h + r0 + 4 * 32);
      }, [&](int s) {
        const int blk = (16 * (s / Gb::BW)) * Gb::W + 16 * (s % Gb::BW);
        return tr8(fb0 + blk, fb1 + blk);
      });
    }
    lds_sync();
    TB_TRACE(4);
    ++it_dbg;
  }

  // ---- epilogue: this workgroup's partial gradients -> slab (dW3/db3: torso_dw3_kernel)
  const int l32 = lane & 31, half = lane >> 5;
  float* sl = a.slab + (size_t)blockIdx.x * Gb::SLAB;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int co = (r & 3) + 8 * (r >> 2) + 4 * half;
    if (wave < Gb::T1) sl[co * (64 * Gb::CIN) + wave * 32 + l32] = acc1[r];
    sl[Gb::OFF_W2 + co * 512 + wave * 32 + l32] = acc2a[r];
    sl[Gb::OFF_W2 + co * 512 + (wave + 8) * 32 + l32] = acc2b[r];
  }
  // bias partials: per-lane values -> LDS, summed in a fixed order (deterministic, unlike LDS
  // float atomics): conv1 bias from every wave (all ran dact1 jobs), conv2 bias from waves 5..7
  float* red = (float*)(lds + Gb::G1H);
  red[tid] = db1p;
  red[512 + tid] = wave >= 5 ? db2p : 0.f;
  __syncthreads();
  if (tid < 64) {
    const int part = tid >> 5, c = tid & 31;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < 8; ++w) v += red[part * 512 + w * 64 + c] + red[part * 512 + w * 64 + 32 + c];
    sl[Gb::OFF_B + tid] = v;
  }
}

// dW3 += g3 . im2col(act2) and db3, straight from global dX3 / out3 / act2 (all written by
// earlier kernels): 9 N tiles (wave w: tile w; wave 0 also tile 8), K = conv3 pixels padded to
// 16s, B operand by transposed reads of the HWC act2 image.  Next frame prefetched in registers.
// Writes the dW3 and db3 parts of each workgroup's slab (same grid as torso_bwd_kernel).
template <class Gb>
__global__ __launch_bounds__(512) void torso_dw3_kernel(const TBArgs a) {
  constexpr int NT = Gb::NT, P2 = Gb::P2, P3 = Gb::P3, G3C_S = Gb::G3C_S;
  __shared__ __attribute__((aligned(16))) bf16 g3c[32 * G3C_S];
  __shared__ __attribute__((aligned(16))) bf16 a2[P2 * 32];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int l32 = lane & 31, half = lane >> 5;
  const int grp = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
  const int colb = 16 * (grp & 1) + 4 * pp;
  for (int i = tid; i < 32 * G3C_S * 2 / 16; i += NT) ((u32x4*)g3c)[i] = u32x4{0, 0, 0, 0};
  f32x16 acc = {}, acc8 = {};
  float db3p = 0.f;
  u32x4 pa2, pdx, po3;
  auto prefetch = [&](int f) {
    if (tid < P2 * 4) pa2 = ((const u32x4*)(a.act2 + (size_t)f * P2 * 32))[tid];
    if (tid < Gb::OUT / 8) {
      pdx = ((const u32x4*)(a.dx3 + (size_t)f * Gb::OUT))[tid];
      po3 = ((const u32x4*)(a.out3 + (size_t)f * Gb::OUT))[tid];
    }
  };
  if (blockIdx.x < a.n) prefetch(blockIdx.x);
  __syncthreads();
  const bf16* b0 = a2 + ((wave / 3) * Gb::W2 + wave % 3) * 32;
  const bf16* b8 = a2 + (2 * Gb::W2 + 2) * 32;
  for (int f = blockIdx.x; f < a.n; f += gridDim.x) {
    if (tid < P2 * 4) ((u32x4*)a2)[tid] = pa2;
    if (tid < Gb::OUT / 8) {
      const bf16x8 dx = __builtin_bit_cast(bf16x8, pdx), o3 = __builtin_bit_cast(bf16x8, po3);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int i = tid * 8 + e, co = i / P3, p = i % P3;
        g3c[co * G3C_S + p] = ((float)o3[e] > 0.f) ? dx[e] : (bf16)0.f;
      }
    }
    if (f + (int)gridDim.x < a.n) prefetch(f + gridDim.x);
    lds_sync();
    auto lda = [&](int s) { return ld8(g3c + l32 * G3C_S + s * 16 + half * 8); };
    auto ldb = [&](const bf16* b, int s) {
      return tr8(b + im2col_off3<Gb>(s, 0, half, q, colb), b + im2col_off3<Gb>(s, 1, half, q, colb));
    };
    if (wave == 0)
      mfma_pipe2<Gb::K3S, 2>(acc, acc8, lda, [&](int s) { return ldb(b0, s); }, [&](int s) { return ldb(b8, s); });
    else
      mfma_pipe<Gb::K3S, 3>(acc, lda, [&](int s) { return ldb(b0, s); });
    if (wave == 7) {  // db3[co] = sum_p g3[co][p] (pad columns are zero)
      float sum = 0.f;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const bf16x8 v = ld8(g3c + l32 * G3C_S + half * 32 + c * 8);
#pragma unroll
        for (int e = 0; e < 8; ++e) sum += (float)v[e];
      }
      sum += __shfl_xor(sum, 32, 64);
      db3p += sum;
    }
    lds_sync();
  }
  float* sl = a.slab + (size_t)blockIdx.x * Gb::SLAB;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int co = (r & 3) + 8 * (r >> 2) + 4 * half;
    sl[Gb::OFF_W3 + co * 288 + wave * 32 + l32] = acc[r];
    if (wave == 0) sl[Gb::OFF_W3 + co * 288 + 8 * 32 + l32] = acc8[r];
  }
  if (wave == 7 && lane < 32) sl[Gb::OFF_B + 64 + lane] = db3p;
}

// grad[dst[e]] = scale[e] * sum_g slab[g][e] (slab_reduce.h: 64 columns x 4 row-groups a block;
// ~1200 blocks fill the chip).  At world 1 the learner folds this into the optimizer launch
// instead (rms_pack.h torso section).
__global__ __launch_bounds__(256) void torso_grad_reduce_kernel(
    const float* __restrict__ slab, int G, int SL, const int* __restrict__ dst,
    const float* __restrict__ scale, float* __restrict__ grad) {
  __shared__ float part[4][64];
  const float s = slab_column_sum(slab, G, SL, blockIdx.x, part);
  const int e = blockIdx.x * 64 + threadIdx.x;
  if (threadIdx.x < 64 && e < SL) grad[dst[e]] = s * scale[e];
}

static long long* g_tb_dbg = nullptr;
extern "C" int r2_torso_bwd_set_debug(long long* p) { g_tb_dbg = p; return 0; }

template <class Gb>
static void tb_launch(const TBArgs& a, int grid, const int* dst, const float* scale, float* grad,
                      hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)torso_bwd_kernel<Gb>, hipFuncAttributeMaxDynamicSharedMemorySize,
                        Gb::LDS);
    attr = true;
  }
  hipLaunchKernelGGL(torso_bwd_kernel<Gb>, dim3(grid), dim3(Gb::NT), Gb::LDS, s, a);
  hipLaunchKernelGGL(torso_dw3_kernel<Gb>, dim3(grid), dim3(Gb::NT), 0, s, a);
  hipLaunchKernelGGL(torso_grad_reduce_kernel, dim3((Gb::SLAB + 63) / 64), dim3(256), 0, s, a.slab,
                     grid, Gb::SLAB, dst, scale, grad);
}

// geometry (cin, h, w): 4x84x84 or 3x72x96; row_bytes: replay row stride (0 = frame bytes);
// slab: grid x r2_torso_bwd_slab_floats_geom(cin, h, w) floats
extern "C" int r2_torso_bwd_geom(const uint8_t* frames, long long row_bytes, const int* rows, int n,
                                 const bf16* act1, const bf16* act2, const bf16* dx3,
                                 const bf16* out3, const bf16* w3dg, const bf16* w2dg, float* slab,
                                 int grid, const int* dst, const float* scale, float* grad, int cin,
                                 int h, int w, void* stream) {
  if (n <= 0) return 0;
  const bool atari = cin == 4 && h == 84 && w == 84, dm = cin == 3 && h == 72 && w == 96;
  if (!atari && !dm) return -6;
  const long long fb = (long long)cin * h * w;
  if (row_bytes <= 0) row_bytes = fb;
  if (row_bytes < fb || row_bytes % 16) return -7;
  if (grid <= 0 || grid > n) grid = n < 256 ? n : 256;
  TBArgs a{frames, rows, act1, act2, dx3, out3, w3dg, w2dg, slab, n, g_tb_dbg, row_bytes};
  hipStream_t s = (hipStream_t)stream;
  if (atari) tb_launch<BGeoAtari>(a, grid, dst, scale, grad, s);
  else tb_launch<BGeoDmlab>(a, grid, dst, scale, grad, s);
  R2_CHECK_LAUNCH();
  return 0;
}

extern "C" int r2_torso_bwd(const uint8_t* frames, const int* rows, int n, const bf16* act1,
                            const bf16* act2, const bf16* dx3, const bf16* out3, const bf16* w3dg,
                            const bf16* w2dg, float* slab, int grid, const int* dst,
                            const float* scale, float* grad, void* stream) {
  return r2_torso_bwd_geom(frames, 0, rows, n, act1, act2, dx3, out3, w3dg, w2dg, slab, grid, dst,
                           scale, grad, 4, 84, 84, stream);
}

extern "C" int r2_torso_bwd_slab_floats_geom(int cin, int h, int w) {
  if (cin == 4 && h == 84 && w == 84) return BGeoAtari::SLAB;
  if (cin == 3 && h == 72 && w == 96) return BGeoDmlab::SLAB;
  return -1;
}

extern "C" int r2_torso_bwd_slab_floats() { return tb::SLAB; }

// slab reduction alone (used by the split-precision backward, torso_sp.hip; Atari slab)
extern "C" int r2_torso_grad_reduce(const float* slab, int grid, const int* dst, const float* scale,
                                    float* grad, void* stream) {
  hipLaunchKernelGGL(torso_grad_reduce_kernel, dim3((tb::SLAB + 63) / 64), dim3(256), 0,
                     (hipStream_t)stream, slab, grid, tb::SLAB, dst, scale, grad);
  R2_CHECK_LAUNCH();
  return 0;
}
