// Fused Atari conv torso, fp32-accurate ("split precision", csrc/split.h) -- forward and backward.
//
// Reference op: model.py:12-22 (Conv2d(4,32,8,s4)-ReLU-Conv2d(32,32,4,s2)-ReLU-Conv2d(32,32,3,s1)-
// ReLU in fp32) and its autograd backward (learner.py:118-120).  Same decomposition as the bf16
// kernels of torso.hip / torso_bwd.hip (implicit GEMMs on v_mfma_f32_32x32x16_bf16, activations
// resident in LDS, one 512-thread workgroup per CU, grid-stride over frames), re-laid out for hi /
// lo operand pairs, which double every image that feeds an MFMA:
//
// Forward (torso_fwd_sp2_kernel, LDS 159.8 KB), per frame in two phases:
//   * phase A: conv1(f) on the int8 matrix cores (the uint8 frame, staged in LDS, is exact as
//     int8 after a -128 shift; W1 = s (d0 + d1/128 + d2/16384) as three int8 digit fragments in
//     VGPRs; exact int32 sums, one fp32 combine) on 7 waves || conv3(f-1) (3 bf16 passes over
//     act2 hi / lo, W3 in VGPRs) on wave 2; the next frame is loaded into registers meanwhile;
//   * phase B: conv2(f) (W2 hi / lo and act1 hi / lo images in LDS, 3 passes, 32x32x16 tiles) on
//     waves 0..2 || next frame -> LDS and the act1 save on the others.
//   * outputs: torso features (PyTorch CHW flatten) as hi / lo planes (the x-projection GEMM's A
//     operand), optional channels-last act1 / act2 hi / lo planes for the backward.
//   Rejected rebalancings and their numbers: profiles/r04_torso_fwd_v3_probe.txt (v3: pipelined
//   roles, W2 in registers) and profiles/r05_torso_fwd_v4_rejected.txt (v4: conv2 on all waves as
//   16x16x32 blocks -- conv2 is LDS-bound); their code is gone.
//
// Backward (torso_bwd_sp_kernel / torso_dw3_sp_kernel, LDS 145.7 KB): see the comment there.
#include <type_traits>

#include "../common.h"
#include "../split.h"

namespace tsp {
constexpr int IN_BYTES = 4 * 84 * 84;    // 28224
constexpr int NT = 512;
constexpr int P1 = 400, P2 = 81, P3 = 49;
}  // namespace tsp

#define TS_MAX_JOBS 4
#define TS_JOB_WORDS 20
struct TSJob {
  const int* rows;
  const bf16* w1; const bf16* w1l; const float* b1;
  const bf16* w2; const bf16* w2l; const float* b2;
  const bf16* w3; const bf16* w3l; const float* b3;
  bf16* out; bf16* out_l;          // (n, 1568) hi / lo planes
  bf16* s1; bf16* s1l;             // optional (n, 400, 32) channels-last act1 hi / lo
  bf16* s2; bf16* s2l;             // optional (n, 81, 32)
  // frame queue (job words 17 / 18; null = the static grid-stride deal).  qmode 1 (the hoisted
  // target-net frames beside the BPTT): frames q[0]++ until q[0] >= n or the stop word q[2] is set;
  // a taken frame is always finished, so [0, min(q[0], n)) is done once the qmode-1 launch ends.
  // qmode 2 (the same job's remainder in the next step's launch): frames [min(q[0], n), n) dealt
  // with the static stride over the job's workgroups (their number set on the device, TSArgs::dyn).
  unsigned* q;
  int n, wbegin, wcount, qmode;
  int pad_j[2];                    // (job word 19: reserved, 0)
};
struct TSArgs {
  const uint8_t* frames;
  TSJob job[TS_MAX_JOBS];
  int njobs, dbg;            // dbg: timing-probe bits (r2_torso_sp_debug), 0 in production
  int dyn;                   // dyn: workgroups dealt on the device (a qmode-2 job's size is q-dependent)
  int pad_;
  long long* trace;          // optional per-phase clock stamps (r2_torso_sp_trace), null in production
};

// Frame of a qmode-1 queue job (one thread; the workgroup's first two frames -- later ones are
// taken with the round trips hidden under phase A, in the frame loop): n once the job is
// exhausted or the stop word is set.
__device__ __forceinline__ int ts_grab(const TSJob& J) {
  unsigned* q = J.q;
  if (__hip_atomic_load(q + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) return J.n;
  const unsigned g = __hip_atomic_fetch_add(q, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return g < (unsigned)J.n ? (int)g : J.n;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t ts_rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, 0, bytes, 0x00020000);
}

// ============================================================================================
// Forward v2 (the only forward): the v1 profile (tools/sp_micro.py probe, profiles/archive/r02_torso_sp_*)
// showed conv1's B fragments (two 4-byte buffer loads per K step from L1 / L2) and conv3's W3
// fragments (L2, re-read by two waves per frame: 72 KB / frame) latency-bound, the next-frame
// warm-up waited on inside phase B, and 2-3-way bank conflicts on the padded act1 image.  v2:
//   * the raw uint8 frame lives in LDS (28 KB): waves 3..7 load frame f+1 into registers at the
//     start of phase A(f) (nothing else of theirs waits on vmcnt there) and store it in phase B(f);
//     conv1 reads its B fragments with two conflict-free ds_read_b32 per K step;
//   * act1 hi / lo unpadded (64 B per pixel) with a row-XOR swizzle (round 5: the space-to-depth a1_off2): the stride-2 conv2
//     reads drop from ~2.8 to ~1.8 LDS cycles per group and the image shrinks by 12.8 KB, which is
//     what makes room for the frame (LDS 159.3 KB);
//   * conv3 runs on wave 2 alone, both pixel tiles sharing every A fragment, with W3 hi / lo held
//     in the registers the conv1 waves use for W1 (steps 16-17 from L2): no W3 traffic per frame;
//   * tiles: conv1 2,2,0,2 | 2,2,1,2 per wave (SIMD2 = conv3 108 MFMAs + one conv1 tile).
namespace tsp2 {
using tsp::NT; using tsp::IN_BYTES; using tsp::P1; using tsp::P2; using tsp::P3;
constexpr int OFF_FR = 0;                                  // uint8 [4][84][84]
constexpr int OFF_A1H = OFF_FR + 4 * 84 * 84;             // 28224: [100 rows][16 x 16 B]
constexpr int OFF_A1L = OFF_A1H + 400 * 64;                // 53824
constexpr int OFF_A2H = OFF_A1L + 400 * 64;                // 79424: [81][40] bf16 (padded)
constexpr int OFF_A2L = OFF_A2H + 81 * 40 * 2;             // 85904
constexpr int OFF_W2H = OFF_A2L + 81 * 40 * 2;             // 92384: [32][520] bf16
constexpr int OFF_W2L = OFF_W2H + 32 * 520 * 2;            // 125664
constexpr int OFF_B = OFF_W2L + 32 * 520 * 2;              // 158944: biases conv2, conv3, conv1
constexpr int OFF_W3T = OFF_B + 96 * 4;                    // 159328: W3[:, 256:288] hi, lo
constexpr int LDS_BYTES = OFF_W3T + 2 * 32 * 32 * 2;       // 163424
constexpr int OFF_SC = LDS_BYTES;                          // int8 conv1: row corrections [2][32] int32
constexpr int LDS_BYTES_I8 = OFF_SC + 2 * 32 * 4;          // 163680
constexpr int IN_CHUNKS2 = 4 * 84 * 84 / 16;               // 1764
constexpr int PF = (IN_CHUNKS2 + 319) / 320;               // 6 chunks per prefetch thread
static_assert(LDS_BYTES <= 160 * 1024 && LDS_BYTES_I8 <= 160 * 1024, "LDS");
}  // namespace tsp2

// act1 image (one plane): space-to-depth blocks.  Pixel (y, x) of the 20 x 20 map lives in block
// (y >> 1, x >> 1) (10 x 10 blocks of 2 x 2 pixels = 256 B = one LDS bank row), sub-pixel
// s = 2 (y & 1) + (x & 1); its 16-byte chunk c (channels 8c .. 8c+7) sits at slot (4 s + c) ^
// a1_m(block).  A conv2 K step (kh, kw, chunk) reads ONE sub-pixel and chunk in every lane, so the
// slot is const ^ a1_m(block) and a ds_read_b128 lane group is conflict-free when its 16 output
// pixels map to 16 distinct a1_m: conv2's lanes take 4 x 4 squares of output pixels (and the
// column / row left over).  a1_m was searched over the affine family (a by + b bx + c (bx >> 2) +
// d (by >> 2)) mod 4 per 2-bit half jointly with conv1's epilogue stores (c1_pix order):
// conv2 reads 1.17 LDS cycles per lane group (round-2 row-XOR layout: 1.83), conv1's 8-byte
// stores at the 2-way floor of a fixed 8-byte half (profiles/r05_torso_act1_s2d.txt).
__device__ __forceinline__ int a1_m(int by, int bx) {
  return (((bx + (by >> 2)) & 3) << 2) | ((by + 2 * bx + (bx >> 2) + 2 * (by >> 2)) & 3);
}
// conv1 tile position n (32 per tile, 16 per half) -> act1 pixel: 16-pixel row segments x < 16 of
// rows 0..19, then the x = 16..19 strip as 4 rows x 4 pixels per half tile (the order that keeps
// each 16-lane epilogue store group at 2 ways); n >= 400: padding (clamped, not stored)
__device__ __forceinline__ void c1_pix(int n, int& y, int& x) {
  n = min(n, tsp::P1 - 1);
  if (n < 320) {
    y = n >> 4;
    x = n & 15;
  } else {
    const int j = n - 320;
    y = 4 * (j >> 4) + ((j >> 2) & 3);
    x = 16 + (j & 3);
  }
}
__device__ __forceinline__ int a1_off2(int y, int x, int c) {
  const int by = y >> 1, bx = x >> 1;
  return ((by * 10 + bx) << 8) + (((((2 * (y & 1) + (x & 1)) << 2) | c) ^ a1_m(by, bx)) << 4);
}
// conv2 lane -> output pixel: the 16 lanes of each ds_read_b128 group (l32 in {0-3, 12-15,
// 20-27} = set 0, the rest = set 1) take one of 6 pixel sets: the four 4 x 4 squares of the 8 x 8
// corner, the column x = 8 (9 pixels), the row y = 8 (8); lanes past a set's end repeat its last
// pixel (dup: computed, not stored)
__device__ __forceinline__ void c2_pixel(int wave, int l32, int& oy, int& ox, bool& dup) {
  const int g = (l32 >= 4 && l32 < 12) || (l32 >= 16 && l32 < 20) || l32 >= 28;
  const int i = l32 < 4 ? l32 : l32 < 12 ? l32 - 4 : l32 < 20 ? l32 - 8 : l32 < 28 ? l32 - 12 : l32 - 16;
  const int S = 2 * wave + g;
  dup = false;
  if (S < 4) {
    oy = 4 * (S >> 1) + (i >> 2);
    ox = 4 * (S & 1) + (i & 3);
  } else if (S == 4) {
    dup = i >= 9;
    oy = min(i, 8);
    ox = 8;
  } else {
    dup = i >= 8;
    oy = 8;
    ox = min(i, 7);
  }
}

typedef int i32x4_t __attribute__((ext_vector_type(4)));
typedef short s16x4_t __attribute__((ext_vector_type(4)));

// conv1 on the int8 matrix cores (the default v2 path).  The uint8 frame is exact as int8 after a
// -128 shift (one XOR per 4 bytes; the conversion to bf16 cost ~12 VALU per 8 bytes and made the
// conv1 phase issue-bound), and W1 (= hi + lo, the split pair the bf16 path multiplies) becomes
// three int8 digits under ONE scale s = max|W1| / 127:  W1 ~= s (d0 + d1 / 128 + d2 / 16384),
// |error| <= s / 32768 (2.4e-7 max|W1|, below the split pair's own rounding).  Products and sums
// are exact in int32 (|sum| <= 256 * 127 * 255); the shift comes back exactly through the per-row
// digit sums (x 128), so the only rounding is the final fp32 combine.  v_mfma_i32_16x16x64_i8
// takes the cycles of the bf16 16x16x32 form at twice the K: 3 digit products per 64 K vs the
// bf16 path's 2 (hi, lo) per 32 K -- 25 % fewer MFMA cycles and no conversion VALU.
//
// Once per workgroup, all 512 threads: 16 weights each (row t / 16, K 16 (t % 16) ..) -> digit
// images dig[d][32][256] int8 in LDS (the act1 region, free until the first conv1), per-row
// corrections 128 S0, 128 (128 S1 + S2) of the digit row sums S_d -> sc[2][32] (int32), block max
// through red[8].  Returns s / 255 (the
// epilogue's scale).  The caller synchronises, then c1_frags() loads each conv1 lane's fragments.
__device__ __forceinline__ float c1_digits(const bf16* w1, const bf16* w1l, int tid, uint8_t* dig,
                                           int* sc, float* red) {
  const int lane = tid & 63, wave = tid >> 6;
  const bf16x8 h0 = *(const bf16x8*)(w1 + tid * 16), h1 = *(const bf16x8*)(w1 + tid * 16 + 8);
  const bf16x8 l0 = *(const bf16x8*)(w1l + tid * 16), l1 = *(const bf16x8*)(w1l + tid * 16 + 8);
  float w[16];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    w[e] = (float)h0[e] + (float)l0[e];
    w[8 + e] = (float)h1[e] + (float)l1[e];
  }
  float m = 0.f;
#pragma unroll
  for (int e = 0; e < 16; ++e) m = fmaxf(m, fabsf(w[e]));
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if (lane == 0) red[wave] = m;
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 8; ++i) m = fmaxf(m, red[i]);
  const float inv = m > 0.f ? 127.f / m : 0.f;
  uint32_t pk[3][4] = {};
  int sum[3] = {0, 0, 0};
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const float q = w[e] * inv;
    const float d0 = rintf(q), r1 = (q - d0) * 128.f;
    const float d1 = rintf(r1), d2 = rintf((r1 - d1) * 128.f);
    const int dd[3] = {(int)d0, (int)d1, (int)d2};
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      sum[d] += dd[d];
      pk[d][e >> 2] |= ((uint32_t)dd[d] & 0xffu) << (8 * (e & 3));
    }
  }
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    *(u32x4*)(dig + d * 8192 + tid * 16) = u32x4{pk[d][0], pk[d][1], pk[d][2], pk[d][3]};
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) sum[d] += __shfl_xor(sum[d], o, 64);
  }
  if ((tid & 15) == 0) {   // row corrections: 128 S0 and 128 (128 S1 + S2) (|.| < 2^29)
    sc[tid >> 4] = 128 * sum[0];
    sc[32 + (tid >> 4)] = 128 * (128 * sum[1] + sum[2]);
  }
  return m * (1.f / 127.f) * (1.f / 255.f);
}

// conv1 lane (row l16, k group g): rows 16c + l16 (c = 0, 1), K steps s = 4 KB + g (KB 0..3), 16 K
// values each (K = 16 s + 4 dy + dx, the bf16 path's order); digit fragment (c, KB, d) -> slot
// 12 c + 3 KB + d of wfh[0..15] ++ wfl[0..7]
__device__ __forceinline__ void c1_frags(const uint8_t* dig, int lane, bf16x8 (&wfh)[16],
                                         bf16x8 (&wfl)[16]) {
  const int l16 = lane & 15, g = lane >> 4;
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int d = 0; d < 3; ++d) {
        const int slot = 12 * c + 3 * kb + d;
        const bf16x8 v = *(const bf16x8*)(dig + d * 8192 + (16 * c + l16) * 256 + (4 * kb + g) * 16);
        if (slot < 16) wfh[slot & 15] = v;
        else wfl[(slot - 16) & 15] = v;
      }
}

__constant__ int c_s2_begin[8] = {0, 2, 4, 4, 6, 8, 10, 11};
__constant__ int c_s2_count[8] = {2, 2, 0, 2, 2, 2, 1, 2};

// QUEUE: the hoisted launch's qmode-1 queue job (frames taken one by one); false: every job on
// the static grid-stride deal (the frame loop as before the queue existed -- its register
// allocation and schedule do not carry the queue's code)
template <bool QUEUE>
__global__ __launch_bounds__(512) void torso_fwd_sp2_kernel(const TSArgs args) {
  using namespace tsp2;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  uint8_t* fr = lds + OFF_FR;
  uint8_t* a1h = lds + OFF_A1H;
  uint8_t* a1l = lds + OFF_A1L;
  bf16* a2h = (bf16*)(lds + OFF_A2H);
  bf16* a2l = (bf16*)(lds + OFF_A2L);
  bf16* w2h = (bf16*)(lds + OFF_W2H);
  bf16* w2l = (bf16*)(lds + OFF_W2L);
  float* lb = (float*)(lds + OFF_B);
  uint8_t* w3t = lds + OFF_W3T;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int half = lane >> 5, l32 = lane & 31;
  const int wk = blockIdx.x;
  int ji = 0, wbeg = 0, wcnt = 0;
  if (args.dyn) {
    // the host's deal (r2_torso_fwd_sp_multi) with a qmode-2 job counted at its remaining frames
    // n - min(q[0], n): every workgroup computes the same table from the same words
    int ne[TS_MAX_JOBS];
    int64_t nw_[TS_MAX_JOBS];
    int64_t total = 0;
#pragma unroll
    for (int i = 0; i < TS_MAX_JOBS; ++i) {
      const TSJob& Ji = args.job[i];
      int v = i < args.njobs ? Ji.n : 0;
      if (i < args.njobs && Ji.qmode == 2)
        v -= (int)min(__hip_atomic_load(Ji.q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), (unsigned)Ji.n);
      ne[i] = v;
      nw_[i] = v > 0 ? v : 0;
      total += nw_[i];
    }
    const int nw = gridDim.x;
    int wb = 0, left = 0;
#pragma unroll
    for (int i = 0; i < TS_MAX_JOBS; ++i) left += ne[i] > 0;
    int64_t seen = 0;
    ji = -1;
#pragma unroll
    for (int i = 0; i < TS_MAX_JOBS; ++i) {
      if (ne[i] <= 0) continue;
      --left;   // non-empty jobs after this one: each keeps at least one workgroup (nw >= njobs)
      seen += nw_[i];
      int end = (int)((seen * nw + total - 1) / total);
      end = min(end, nw - left);
      const int cnt = min(max(end - wb, 1), ne[i]);
      if (wk >= wb && wk < wb + cnt) {
        ji = i;
        wbeg = wb;
        wcnt = cnt;
      }
      wb += cnt;
    }
    if (ji < 0) return;
  } else {
#pragma unroll
    for (int i = 1; i < TS_MAX_JOBS; ++i)
      if (i < args.njobs && wk >= args.job[i].wbegin) ji = i;
    wbeg = args.job[ji].wbegin;
    wcnt = args.job[ji].wcount;
  }
  const TSJob& J = args.job[ji];
  const int stride = wcnt;
  if (wk - wbeg >= stride) return;
  const int n_frames = J.n;
  // qmode 1 frames come from the queue; a qmode-2 job deals the frames the qmode-1 launch left,
  // [min(q[0], n), n), over its workgroups with the static stride (no per-frame atomics)
  const bool qjob = QUEUE && J.q != nullptr && J.qmode == 1;
  if (!QUEUE && J.q != nullptr && J.qmode == 1) return;   // (the launcher never pairs these)
  __shared__ int s_q[4];
  int f = wk - wbeg;
  if (J.q != nullptr && J.qmode == 2)
    f += (int)min(__hip_atomic_load(J.q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), (unsigned)n_frames);
  int row_f = 0, row_q1 = 0, f_q1 = 0;
  if (qjob) {
    // first two frames of this workgroup from the queue (before any setup: a workgroup that
    // finds the queue empty or stopped leaves at once)
    if (tid == 0) {
      const int g0 = ts_grab(J);
      const int g1 = g0 < n_frames ? ts_grab(J) : n_frames;
      s_q[0] = g0;
      s_q[1] = g1;
      s_q[2] = g0 < n_frames ? (J.rows ? J.rows[g0] : g0) : 0;
      s_q[3] = g1 < n_frames ? (J.rows ? J.rows[g1] : g1) : 0;
    }
    __syncthreads();
    f = __builtin_amdgcn_readfirstlane(s_q[0]);
    f_q1 = __builtin_amdgcn_readfirstlane(s_q[1]);
    row_f = __builtin_amdgcn_readfirstlane(s_q[2]);
    row_q1 = __builtin_amdgcn_readfirstlane(s_q[3]);
  }
  if (f >= n_frames) return;
  const bool conv3_wave = wave == 2, conv2_wave = wave < 3, pf_wave = wave >= 3;
  const int t5 = tid - 192;   // prefetch thread index (waves 3..7)
  const int t7 = tid < 128 ? tid : tid - 64;   // int8 path: prefetch thread index (waves != 2)

  // ---- once: W2 hi / lo -> LDS; W1 (conv1 waves) or W3 (wave 2) fragments -> registers; biases;
  //      the first frame -> LDS
  for (int i = tid; i < 32 * 64; i += NT) {
    const int r = i >> 6, c = i & 63;
    *(bf16x8*)(w2h + r * 520 + c * 8) = *(const bf16x8*)(J.w2 + r * 512 + c * 8);
    *(bf16x8*)(w2l + r * 520 + c * 8) = *(const bf16x8*)(J.w2l + r * 512 + c * 8);
  }
  bf16x8 wfh[16], wfl[16];
  float c1_scale = 0.f;
  {   // int8 digits of W1 -> LDS (act1 region) -> conv1 lanes' fragments
    c1_scale = c1_digits(J.w1, J.w1l, tid, a1h, (int*)(lds + OFF_SC), (float*)(a1h + 3 * 8192));
    c1_scale = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(c1_scale)));   // SGPR
    __syncthreads();
    if (!conv3_wave) c1_frags(a1h, lane, wfh, wfl);
  }
  if (conv3_wave) {
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const bf16* ph = conv3_wave ? J.w3 + l32 * 288 + s * 16 + half * 8 : J.w1 + l32 * 256 + s * 16 + half * 8;
      const bf16* pl = conv3_wave ? J.w3l + l32 * 288 + s * 16 + half * 8 : J.w1l + l32 * 256 + s * 16 + half * 8;
      wfh[s] = *(const bf16x8*)ph;
      wfl[s] = *(const bf16x8*)pl;
    }
  }
  if (tid < 96) lb[tid] = tid < 32 ? J.b2[tid] : tid < 64 ? J.b3[tid - 32] : J.b1[tid - 64];
  if (tid < 256) {   // W3 K columns 256..287, hi then lo: [32 rows][32] bf16 each
    const int pl = tid >> 7, r = (tid >> 2) & 31, c = tid & 3;
    *(bf16x8*)(w3t + pl * 2048 + (r * 32 + c * 8) * 2) = *(const bf16x8*)((pl ? J.w3l : J.w3) + r * 288 + 256 + c * 8);
  }
  {
    const size_t row = qjob ? (size_t)row_f : J.rows ? (size_t)ld_uniform_i32(J.rows, f) : (size_t)f;
    const u32x4* src = (const u32x4*)(args.frames + row * IN_BYTES);
    // int8 conv1 reads the frame as (byte - 128): the shift is applied once here / at the
    // phase-B store, not per conv1 lane per K step (16 XORs per 16-pixel half tile)
    const uint32_t sh = 0x80808080u;
    for (int c = tid; c < IN_CHUNKS2; c += NT) ((u32x4*)fr)[c] = src[c] ^ sh;
  }
  const int t1b = c_s2_begin[wave], t1n = c_s2_count[wave];
  int row_nx = qjob ? row_q1
               : f + stride < n_frames ? (J.rows ? ld_uniform_i32(J.rows, f + stride) : f + stride) : 0;
  // queue jobs: the next frame (fn) is known one iteration ahead; the one after (fnn) is grabbed
  // during phase B by wave 3's first lane (it only stores its share of the prefetched frame there)
  int f_nx = qjob ? f_q1 : f + stride;
  __syncthreads();

  int fprev = -1;
  int it_dbg = 0;
  unsigned q_g = 0u, q_st = 0u, q_stop = 0u;   // queue job, thread 192 only
  long long* tr = (args.trace && blockIdx.x == 0 && lane == 0) ? args.trace + wave * 16 * 5 : nullptr;
#define TS2_STAMP(k) \
  if (tr && it_dbg < 16) tr[it_dbg * 5 + (k)] = (long long)__builtin_readcyclecounter();
  for (;;) {
    TS2_STAMP(0);
    const bool have = f < n_frames;
    const int fn = f_nx;
    int fnn = fn + stride;
    int row_nn = (!qjob && fnn < n_frames) ? (J.rows ? ld_uniform_i32(J.rows, fnn) : fnn) : 0;
    // a per-iteration zero: keeps the lane-constant LDS offsets of the MFMA loops from being
    // hoisted out of the frame loop (32+ VGPRs held across every phase otherwise)
    int oz;
    asm volatile("v_mov_b32 %0, 0" : "=v"(oz));
    // queue job: wave 3's first lane takes fnn here and hands it over at the end of phase A; its
    // row is loaded in phase B (both round trips hidden under the phases' work)
    if (qjob && tid == 192 && fn < n_frames && !q_stop) {
      q_st = __hip_atomic_load(J.q + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      q_g = __hip_atomic_fetch_add(J.q, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // =================== phase A: conv1(f) || conv3(f-1) on wave 2; frame f+1 -> registers
    // (nothing in phase A waits on vmcnt: conv1 / conv3 operands come from LDS / registers)
    if (have && fn < n_frames && !(args.dbg & 16)) {
      const u32x4* src = (const u32x4*)(args.frames + (size_t)row_nx * IN_BYTES);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int c = t7 + 448 * q;
        if (c < IN_CHUNKS2 && !conv3_wave) {
          // int8 path: the 7 conv1 waves prefetch (4 chunks per thread) and park the chunks in
          // wfl[8..11], which only the conv3 wave uses (W3 K steps 8..11 lo); the conv1 digits
          // fill slots 0..23
          wfl[8 + q] = __builtin_bit_cast(bf16x8, src[c]);
        }
      }
    }
    if (have && !(args.dbg & 1)) {
      // conv1(f) on the int8 matrix cores (c1_digits): per 16-pixel half tile, the 4 K blocks'
      // frame bytes (4 rows x 4 bytes per lane, -128 by XOR), 3 digits x 2 channel halves of
      // v_mfma_i32_16x16x64_i8, exact int32 sums
      const int l16 = lane & 15, gq = lane >> 4;
      const int* sct = (const int*)(lds + OFF_SC);
      for (int i = 0; i < t1n; ++i) {
        // both 16-pixel halves of the tile: half 1's frame bytes load under half 0's MFMAs
        i32x4_t bx[1][4];
        // pixel of this lane in half tile q (c1_pix with the half tile's uniform part hoisted):
        // a row segment (y uniform, x = l16) or a 4 x 4 piece of the x >= 16 strip
        auto pix = [&](int q, int& oy, int& ox) {
          const int nb = (t1b + i) * 32 + 16 * q;
          if (nb < 320) {
            oy = nb >> 4;
            ox = l16;
          } else if (nb < P1) {
            oy = 4 * ((nb - 320) >> 4) + (l16 >> 2);
            ox = 16 + (l16 & 3);
          } else {
            oy = 19;
            ox = 19;
          }
        };
        // frame bytes of K blocks [kb0, kb0 + 2): issued in two halves, the second after the first
        // half's MFMAs of channel half 0 (the reads of K blocks 2, 3 overlap those MFMAs)
        auto ldb = [&](const uint8_t* fb, int kb0, i32x4_t (&x)[4]) {
#pragma unroll
          for (int kb = kb0; kb < kb0 + 2; ++kb)
#pragma unroll
            for (int dy = 0; dy < 4; ++dy)
              x[kb][dy] = (int)*(const uint32_t*)(fb + (kb >> 1) * 336 + (kb & 1) * 4 + dy * 84);
        };
#pragma unroll 1
        for (int q = 0; q < 2; ++q) {
          // frame bytes and the pixel's act1 byte offset with chunk 0 (a1_off2(y, x, 0)); row
          // segments (uniform y, x = l16) split a1_off2 into uniform and per-lane parts
          const int nb = (t1b + i) * 32 + 16 * q;
          const uint8_t* fb;
          int sbase;
          if (nb < 320) {
            const int y = nb >> 4, by = y >> 1, bx = l16 >> 1;
            fb = fr + gq * 7056 + 4 * l16 + oz + 336 * y;
            const int m = (((bx + (by >> 2)) & 3) << 2) | ((2 * bx + (bx >> 2) + by + 2 * (by >> 2)) & 3);
            sbase = ((by * 10 + bx) << 8) + (((m ^ (4 * (l16 & 1))) ^ (8 * (y & 1))) << 4) + 8 * (gq & 1);
          } else {
            int py, px;
            pix(q, py, px);
            fb = fr + gq * 7056 + 4 * py * 84 + 4 * px + oz;
            sbase = a1_off2(py, px, 0) + 8 * (gq & 1);
          }
          ldb(fb, 0, bx[0]);
          const bool pst = nb < P1;   // uniform: padding half tiles store nothing
#pragma unroll
          for (int c = 0; c < 2; ++c) {   // channel halves one after the other (12 acc VGPRs)
            // rows (channels) 16c + 4 gq + e; the -128 shift's row corrections (digit row sums x
            // 128: sum d (v - 128) + 128 sum d = sum d v) start in the accumulators of digits 0
            // and 2, so the epilogue merges digits 1, 2 with one shift-add
            const int ch0 = 16 * c + 4 * gq;
            i32x4_t acc[3];
            acc[0] = *(const i32x4_t*)(sct + ch0);
            acc[1] = i32x4_t{0, 0, 0, 0};
            acc[2] = *(const i32x4_t*)(sct + 32 + ch0);
#pragma unroll
            for (int kb = 0; kb < 4; ++kb) {
              if (c == 0 && kb == 2) {
                __builtin_amdgcn_sched_barrier(0);
                ldb(fb, 2, bx[0]);
                __builtin_amdgcn_sched_barrier(0);
              }
#pragma unroll
              for (int d = 0; d < 3; ++d) {
                const int slot = 12 * c + 3 * kb + d;
                const i32x4_t a = __builtin_bit_cast(i32x4_t, slot < 16 ? wfh[slot & 15] : wfl[(slot - 16) & 15]);
                acc[d] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, bx[0][kb], acc[d], 0, 0, 0);
              }
            }
            if (pst) {
              // digits 1, 2 merge exactly in int32 (|128 i1 + i2| < 2^30)
              bf16x4 vh, vl;
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                const int i0 = acc[0][e];
                const int i12 = acc[1][e] * 128 + acc[2][e];
                const float t = fmaf((float)i12, 1.f / 16384.f, (float)i0);
                const float v = fmaxf(fmaf(t, c1_scale, lb[64 + ch0 + e]), 0.f);
                vh[e] = (bf16)v;
                vl[e] = sp_lo(v);
              }
              const int o = sbase ^ ((2 * c + (gq >> 1)) << 4);
              *(bf16x4*)(a1h + o) = vh;
              *(bf16x4*)(a1l + o) = vl;
            }
          }
        }
      }
    }
    if (fprev >= 0 && conv3_wave && !(args.dbg & 4)) {
      // conv3(f-1), both pixel tiles one after the other; K = 288 = (kh 3, kw 3, ci 32); A = W3
      // (registers; steps 16-17 from the LDS tail image); B = act2 hi / lo
#pragma unroll 1
      for (int t = 0; t < 2; ++t) {
        const int p = t * 32 + l32, pc = p < P3 ? p : P3 - 1;
        const int bo = ((pc / 7) * 9 + pc % 7) * 40 + half * 8 + oz;
        f32x16 acc = {};
        constexpr int D = 4;
        bf16x8 rbh[D], rbl[D];
        auto ldb = [&](int s, bf16x8& xh, bf16x8& xl) {
          const int khkw = s >> 1, kh = khkw / 3, kw = khkw % 3;
          const int o = bo + (kh * 9 + kw) * 40 + (s & 1) * 16;
          xh = *(const bf16x8*)(a2h + o);
          xl = *(const bf16x8*)(a2l + o);
        };
#pragma unroll
        for (int s = 0; s < D; ++s) ldb(s, rbh[s], rbl[s]);
#pragma unroll
        for (int s = 0; s < 18; ++s) {
          const bf16x8 xh = rbh[s % D], xl = rbl[s % D];
          if (s + D < 18) ldb(s + D, rbh[s % D], rbl[s % D]);
          bf16x8 ah, al;
          if (s < 16) {
            ah = wfh[s < 16 ? s : 0];
            al = wfl[s < 16 ? s : 0];
          } else {
            const int o = (l32 * 32 + (s - 16) * 16 + half * 8) * 2;
            ah = *(const bf16x8*)(w3t + o);
            al = *(const bf16x8*)(w3t + 2048 + o);
          }
          __builtin_amdgcn_sched_barrier(0);
          acc = mfma32_x3(ah, al, xh, xl, acc);
        }
        if (p < P3) {
          // one base per plane (+oz: not hoisted), the channel offsets as store immediates
          bf16* oh = J.out + (size_t)fprev * 1568 + p + 4 * half * 49 + oz;
          bf16* ol = J.out_l + (size_t)fprev * 1568 + p + 4 * half * 49 + oz;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int c0 = (r & 3) + 8 * (r >> 2);
            const float v = fmaxf(acc[r] + lb[32 + c0 + 4 * half], 0.f);
            oh[c0 * 49] = (bf16)v;
            ol[c0 * 49] = sp_lo(v);
          }
        }
      }
    }
    if (qjob && tid == 192) {
      s_q[0] = (fn < n_frames && !q_stop) ? (int)min(q_g, (unsigned)n_frames) : n_frames;
      q_stop |= q_st;     // the stop word seen: this frame is the workgroup's last grab
      q_st = 0u;
    }
    TS2_STAMP(1);
    lds_sync();
    TS2_STAMP(2);
    if (!have) break;

    // =================== phase B: frame f+1 -> LDS (conv1(f) finished reading the image before the
    // barrier above); conv2(f) on waves 0..2 || act1 save on waves 3..7
    if (fn < n_frames && !(args.dbg & 16)) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int c = t7 + 448 * q;
        if (c < IN_CHUNKS2 && !conv3_wave)
          ((u32x4*)fr)[c] = __builtin_bit_cast(u32x4, wfl[8 + q]) ^ 0x80808080u;
      }
    }
    if (qjob && tid == 192) {   // fnn's row (fnn taken in phase A), read after the barrier below
      const int g = s_q[0];
      s_q[1] = g < n_frames ? (J.rows ? J.rows[g] : g) : 0;
    }
    if (conv2_wave) {
      if (!(args.dbg & 2)) {
        int oy, ox;
        bool dup;
        c2_pixel(wave, l32, oy, ox, dup);
        const int p = oy * 9 + ox;
        const bf16* ah = w2h + l32 * 520 + half * 8;
        const bf16* al = w2l + l32 * 520 + half * 8;
        // per (kh >> 1, kw >> 1): the block's byte base | (a1_m ^ half) << 4; a K step XORs in its
        // (sub-pixel, chunk pair) slot -- one VALU per step
        int vb[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int by = oy + (q >> 1), bx = ox + (q & 1);
          vb[q] = (((by * 10 + bx) << 8) | ((a1_m(by, bx) ^ half) << 4)) + oz;
        }
        constexpr int D = 2;
        bf16x8 rah[D], ral[D], rbh[D], rbl[D];
        auto ld = [&](int s, bf16x8& xah, bf16x8& xal, bf16x8& xbh, bf16x8& xbl) {
          const int khkw = s >> 1, kh = khkw >> 2, kw = khkw & 3;
          const int q = 2 * (kh >> 1) + (kw >> 1), sub = 2 * (kh & 1) + (kw & 1);
          int ob;   // computed at the step (not hoisted: 32 live offsets otherwise)
          asm volatile("v_xor_b32 %0, %1, %2" : "=v"(ob) : "i"(((sub << 2) | ((s & 1) << 1)) << 4), "v"(vb[q]));
          xah = *(const bf16x8*)(ah + s * 16);
          xal = *(const bf16x8*)(al + s * 16);
          xbh = *(const bf16x8*)(a1h + ob);
          xbl = *(const bf16x8*)(a1l + ob);
        };
#pragma unroll
        for (int s = 0; s < D; ++s) ld(s, rah[s], ral[s], rbh[s], rbl[s]);
        f32x16 acc = {};
        // the conv2 K loop (its LDS reads cost ~25 us of the launch against MFMAs alone, measured
        // with probe instances that are gone now: profiles/r05_torso_act1_s2d.txt)
#pragma unroll
        for (int s = 0; s < 32; ++s) {
          const bf16x8 xah = rah[s % D], xal = ral[s % D], xbh = rbh[s % D], xbl = rbl[s % D];
          if (s + D < 32) ld(s + D, rah[s % D], ral[s % D], rbh[s % D], rbl[s % D]);
          __builtin_amdgcn_sched_barrier(0);
          acc = mfma32_x3(xah, xal, xbh, xbl, acc);
        }
        if (!dup) {
          bf16* d2 = J.s2 ? J.s2 + ((size_t)f * P2 + p) * 32 : nullptr;
          bf16* d2l = J.s2 ? J.s2l + ((size_t)f * P2 + p) * 32 : nullptr;
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            bf16x4 vh, vl;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int co = 4 * half + 8 * g + e;
              const float v = fmaxf(acc[4 * g + e] + lb[co], 0.f);
              vh[e] = (bf16)v;
              vl[e] = sp_lo(v);
            }
            *(bf16x4*)(a2h + p * 40 + 8 * g + 4 * half) = vh;
            *(bf16x4*)(a2l + p * 40 + 8 * g + 4 * half) = vl;
            if (d2) {
              *(bf16x4*)(d2 + 8 * g + 4 * half) = vh;
              *(bf16x4*)(d2l + 8 * g + 4 * half) = vl;
            }
          }
        }
      }
    } else {
      if (J.s1 != nullptr && !(args.dbg & 64)) {
        // act1(f) -> channels-last (400, 32) hi / lo: linear LDS chunks, scattered 16-B stores
        bf16* d1 = J.s1 + (size_t)f * P1 * 32;
        bf16* d1l = J.s1l + (size_t)f * P1 * 32;
        for (int i = tid - 192; i < P1 * 4; i += 320) {
          const int blk = i >> 4, by = blk / 10, bx = blk - 10 * by;
          const int v = (i & 15) ^ a1_m(by, bx), sub = v >> 2, c = v & 3;
          const int P = (2 * by + (sub >> 1)) * 20 + 2 * bx + (sub & 1);
          *(bf16x8*)(d1 + P * 32 + c * 8) = *(const bf16x8*)(a1h + i * 16);
          *(bf16x8*)(d1l + P * 32 + c * 8) = *(const bf16x8*)(a1l + i * 16);
        }
      }
    }
    TS2_STAMP(3);
    lds_sync();
    TS2_STAMP(4);
    ++it_dbg;
    if (qjob) {
      fnn = __builtin_amdgcn_readfirstlane(s_q[0]);
      row_nn = __builtin_amdgcn_readfirstlane(s_q[1]);
    }
    fprev = f;
    f = fn;
    f_nx = fnn;
    row_nx = row_nn;
  }
}

static int g_tsp_dbg = 0;
static long long* g_tsp_trace = nullptr;
// v2 phase clock stamps of workgroup 0: [wave][frame < 16][5] (loop top, phase A done, barrier,
// phase B done, barrier), s_memrealtime-free cycle counter
extern "C" int r2_torso_sp_trace(long long* p) { g_tsp_trace = p; return 0; }
// timing probes only (tools/sp_micro.py): bit 0 skips conv1, bit 1 conv2, bit 2 conv3, bit 4 the
// next-frame staging, bit 6 the act1 save
extern "C" int r2_torso_sp_debug(int bits) { g_tsp_dbg = bits; return 0; }

extern "C" int r2_torso_fwd_sp_multi(const uint8_t* frames, const int64_t* jobs, int njobs,
                                     int grid, void* stream) {
  if (njobs < 1 || njobs > TS_MAX_JOBS) return -1;
  TSArgs a{};
  a.frames = frames;
  a.dbg = g_tsp_dbg;
  a.trace = g_tsp_trace;
  // workgroups dealt in proportion to the frames (weighting the frames with activation saves
  // 1.15x / 1.3x measured slower, round 6)
  auto wt = [&](const int64_t* p) -> int64_t { return p[1] > 0 ? p[1] : 0; };
  int64_t total = 0;
  for (int i = 0; i < njobs; ++i) total += wt(jobs + TS_JOB_WORDS * i);
  if (total <= 0) return 0;
  if (grid <= 0) grid = 256;
  const int nw = grid;
  int wb = 0;
  int64_t seen = 0;
  for (int i = 0; i < njobs; ++i) {
    const int64_t* p = jobs + TS_JOB_WORDS * i;
    if (p[1] <= 0) continue;
    seen += wt(p);
    int end = (int)((seen * nw + total - 1) / total);
    if (end > nw) end = nw;
    int cnt = end - wb;
    if (cnt < 1) cnt = 1;
    if (cnt > p[1]) cnt = (int)p[1];
    TSJob& J = a.job[a.njobs++];
    J.rows = (const int*)p[0]; J.n = (int)p[1];
    J.w1 = (const bf16*)p[2]; J.w1l = (const bf16*)p[3]; J.b1 = (const float*)p[4];
    J.w2 = (const bf16*)p[5]; J.w2l = (const bf16*)p[6]; J.b2 = (const float*)p[7];
    J.w3 = (const bf16*)p[8]; J.w3l = (const bf16*)p[9]; J.b3 = (const float*)p[10];
    J.out = (bf16*)p[11]; J.out_l = (bf16*)p[12];
    J.s1 = (bf16*)p[13]; J.s1l = (bf16*)p[14]; J.s2 = (bf16*)p[15]; J.s2l = (bf16*)p[16];
    J.q = (unsigned*)p[17];
    J.qmode = J.q ? (int)p[18] : 0;
    if (!J.w1l || !J.w2l || !J.w3l || !J.out_l || (J.s1 && !J.s1l) || (J.s2 && !J.s2l)) return -4;
    // queue jobs: no activation saves (the saved frames are indexed by launch order), mode 1 / 2
    if (J.q && (J.s1 || J.s2 || (J.qmode != 1 && J.qmode != 2))) return -5;
    if (J.qmode == 2) a.dyn = 1;
    J.wbegin = wb; J.wcount = cnt;
    wb += cnt;
  }
  if (wb > nw) return -3;
  // the device-side deal (dyn) may give every workgroup of the grid a job: keep the whole grid
  if (grid > wb && !a.dyn) grid = wb;
  if (a.dyn && grid < a.njobs) return -3;
  bool queue = false;
  for (int i = 0; i < a.njobs; ++i) queue = queue || a.job[i].qmode == 1;
  static bool attr2 = false;
  if (!attr2) {
    hipFuncSetAttribute((const void*)torso_fwd_sp2_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                        tsp2::LDS_BYTES_I8);
    hipFuncSetAttribute((const void*)torso_fwd_sp2_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                        tsp2::LDS_BYTES_I8);
    attr2 = true;
  }
  if (queue)
    hipLaunchKernelGGL(torso_fwd_sp2_kernel<true>, dim3(grid), dim3(tsp::NT), tsp2::LDS_BYTES_I8,
                       (hipStream_t)stream, a);
  else
    hipLaunchKernelGGL(torso_fwd_sp2_kernel<false>, dim3(grid), dim3(tsp::NT), tsp2::LDS_BYTES_I8,
                       (hipStream_t)stream, a);
  R2_CHECK_LAUNCH();
  return 0;
}

// ============================================================================================
// Backward, fp32-accurate.  Per learning frame, in LDS (145.7 KB), the stages of torso_bwd.hip
// with hi / lo images:
//   S0  act1 hi / lo + act2 hi (mask) -> region R; g3 = dX3 * (out3 > 0) hi / lo (bordered HWC);
//       W3 hi / lo -> the g1 region by LDS-DMA (g1 is not live until S2)
//   S1  g2 = convT(g3, W3) * (act2 > 0)   (waves 0-5, one 16-pixel tile each, 16x16x32 MFMAs;
//       transposed product: lane = pixel, 8-byte channel-quad stores; 3 passes)
//   S2  dW2 += g2 . im2col(act1)          (3 passes; both operands by transposed reads)
//       g1 = convT_s2(g2, W2) * (act1 > 0) (4 output phases; W2 phase slices from L2; transposed
//       product, g1 rows with an 8-byte chunk swizzle that S3's transposed reads undo)
//   Every [rows][32] image (act1, act2, g3, g2) keeps a 16-byte chunk XOR swizzle (tb_sw).
//   S2b the frame -> region R as exact bf16 (act1 / act2 are dead by now: R is shared)
//   S3  dW1 += g1 . im2col(frame)         (2 passes: the frame is exact in bf16)
// dW3 / db3: torso_dw3_sp_kernel.  Slabs and their reduction are shared with the bf16 path.
namespace tbs {
constexpr int NT = 512;
constexpr int P1 = 400, P2 = 81, P3 = 49;
constexpr int IN_BYTES = 4 * 84 * 84;
constexpr int IN_CHUNKS = IN_BYTES / 16;                  // 1764
constexpr int R = 0;                                      // act1 hi | act1 lo | act2 hi, then the frame
constexpr int R_A1L = P1 * 32 * 2;                        // 25600
constexpr int R_A2 = 2 * P1 * 32 * 2;                     // 51200
constexpr int R_BYTES = IN_BYTES * 2;                     // 56448 (frame bf16 CHW)
constexpr int G3P = R + R_BYTES;                          // g3 hi, lo: [121][32] each
constexpr int G3PL = G3P + 121 * 32 * 2;
constexpr int G2P = G3PL + 121 * 32 * 2;                  // g2 hi, lo: [122][32] each
constexpr int G2PL = G2P + 122 * 32 * 2;
constexpr int G1H = G2PL + 122 * 32 * 2;                  // g1 hi, lo: [406][32] each
constexpr int G1L = G1H + 406 * 32 * 2;
// S2: all four W2 phase slices hi / lo (2 planes x 4 x 32 x 128 bf16 = 64 KB) staged by LDS-DMA
// from G1H (g1 is not written until the dact1 epilogue); the gather table sits above them
constexpr int W2ST = G1H, W2PL = 4 * 32 * 128 * 2;        // 32 KB per plane
constexpr int TBL2 = W2ST + 2 * W2PL;                     // dW2 gather offsets int2 [12][64]
constexpr int LDS = TBL2 + 12 * 64 * 8;                   // 159232
// S0 / S1: W3 hi / lo staged in the g1 region (free until S2), rows of W3S bf16
constexpr int W3S = 296, W3PL = 19 * 1024;                // 32 x 592 B per plane, padded to 19 KB
constexpr int G2_TRASH = 121, G1_TRASH = 400;
constexpr int PF1 = (P1 * 4 + NT - 1) / NT;               // act1 chunks per thread per plane (4)
constexpr int PFF = (IN_CHUNKS + NT - 1) / NT;            // frame chunks per thread (4)
constexpr int SLAB = 32 * 256 + 32 * 512 + 32 * 288 + 96;
constexpr int OFF_W2 = 32 * 256, OFF_W3 = OFF_W2 + 32 * 512, OFF_B = OFF_W3 + 32 * 288;
static_assert(R_A2 + P2 * 32 * 2 <= R_BYTES, "R");
static_assert(LDS <= 160 * 1024 && G1L + 406 * 32 * 2 <= TBL2, "LDS");
}  // namespace tbs

struct TBSArgs {
  const uint8_t* frames;
  const int* rows;
  const bf16* act1; const bf16* act1l;   // (N, 400, 32) hi / lo
  const bf16* act2; const bf16* act2l;   // (N, 81, 32)
  const bf16* dx3; const bf16* dx3l;     // (N, 1568) dL/d(torso output) hi / lo
  const bf16* out3;                      // (N, 1568) torso output hi plane (ReLU mask)
  const bf16* w3dg; const bf16* w3dgl;   // (32 ci, 288 = (kh,kw,co)) hi / lo
  const bf16* w2dg; const bf16* w2dgl;   // (4 phases, 32 ci, 128 = (khi,kwi,co)) hi / lo
  float* slab;
  int n, pad_;
  long long* trace;   // optional stage clock stamps of workgroup 0 (r2_torso_bwd_sp_trace)
};

typedef short ts_i16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) ts_i16x4 ts_lds_i16x4;
__device__ __forceinline__ bf16x8 ts_ld8(const bf16* p) { return *(const bf16x8*)p; }
__device__ __forceinline__ bf16x8 ts_tr8(const bf16* p0, const bf16* p1) {
  const ts_i16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((ts_lds_i16x4*)p0);
  const ts_i16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((ts_lds_i16x4*)p1);
  return __builtin_bit_cast(bf16x8, __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7));
}
__device__ __forceinline__ bf16x8 ts_bl(const __amdgpu_buffer_rsrc_t r, int v, int s) {
  return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(r, v, s, 0));
}

// Every [rows][32] bf16 image of the backward (act1, act2, g3, g2) keeps its 16-byte channel chunk
// c of row r at chunk c ^ ((r >> 2) & 3): 16 lanes on 16 consecutive rows at one chunk (the b128 /
// b64 reads and stores of the transposed products, the pixel-row gathers) hit 16 distinct bank
// groups instead of 4 (64-byte rows).  Element offset of (row r, channel e):
// sum over each 16-lane row on DPP (VALU; __shfl_xor goes through ds_bpermute at LDS latency):
// rotate by 8 and 4 within the row, then the two quad swaps -- every lane holds its row's sum
__device__ __forceinline__ float tb_rowsum16(float v) {
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xf, 0xf, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x124, 0xf, 0xf, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4e, 0xf, 0xf, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xb1, 0xf, 0xf, false));
  return v;
}

__device__ __forceinline__ int tb_sw(int r, int e) {
  return r * 32 + ((((e >> 3) ^ (r >> 2)) & 3) << 3) + (e & 7);
}

__global__ __launch_bounds__(512) void torso_bwd_sp_kernel(const TBSArgs a) {
  using namespace tbs;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;

  // ---- once: zero the bordered gradient images, the dW2 gather table (as torso_bwd.hip)
  for (int i = tid; i < (G1H - G3P) / 16; i += NT) ((u32x4*)(lds + G3P))[i] = u32x4{0, 0, 0, 0};
  for (int i = tid; i < 12 * 64; i += NT) {
    const int sr = i >> 6, l = i & 63, sS = sr >> 1, r = sr & 1;
    const int h = l >> 5, qq = (l >> 2) & 3, cb = 16 * ((l >> 4) & 1) + 4 * (l & 3);
    const int P = 16 * sS + 8 * h + 4 * r + qq, Pc = P < P2 ? P : P2 - 1;
    const int arow = P < P2 ? (Pc / 9 + 1) * 11 + Pc % 9 + 1 : 0;
    ((int2*)(lds + TBL2))[i] = make_int2(tb_sw(arow, cb), (2 * (Pc / 9)) * 20 + 2 * (Pc % 9));
  }

  f32x16 acc1 = {}, acc2a = {}, acc2b = {};
  float db1v[16] = {};   // db1 partials: this lane's channel quads (dact1 epilogue layout)
  float db2p = 0.f;

  u32x4 pfr[PFF], pa1[PF1], pa1l[PF1], pa2, pdx, pdxl, po3;
  // buffer loads off kernel-argument bases (SGPR descriptors, 32-bit lane offsets): 64-bit VGPR
  // addresses of these streams were spilled and their reloads waited (vmcnt(0)) on the whole
  // next-frame prefetch
  const uint32_t na = (uint32_t)a.n;
  const __amdgpu_buffer_rsrc_t r_a1 = ts_rsrc(a.act1, na * P1 * 64), r_a1l = ts_rsrc(a.act1l, na * P1 * 64);
  const __amdgpu_buffer_rsrc_t r_a2 = ts_rsrc(a.act2, na * P2 * 64);
  const __amdgpu_buffer_rsrc_t r_dx = ts_rsrc(a.dx3, na * 3136), r_dxl = ts_rsrc(a.dx3l, na * 3136);
  const __amdgpu_buffer_rsrc_t r_o3 = ts_rsrc(a.out3, na * 3136);
  auto prefetch_acts = [&](int f) {
    const uint32_t o1 = (uint32_t)f * (P1 * 64), o2 = (uint32_t)f * (P2 * 64), o3 = (uint32_t)f * 3136;
#pragma unroll
    for (int k = 0; k < PF1; ++k) {
      const int c = tid + k * NT;
      if (c < P1 * 4) {
        pa1[k] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r_a1, c * 16, o1, 0));
        pa1l[k] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r_a1l, c * 16, o1, 0));
      }
    }
    if (tid < P2 * 4) pa2 = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r_a2, tid * 16, o2, 0));
    if (tid < 196) {
      pdx = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r_dx, tid * 16, o3, 0));
      pdxl = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r_dxl, tid * 16, o3, 0));
      po3 = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r_o3, tid * 16, o3, 0));
    }
  };
  // frame bytes of frame f: loaded one stage ahead (S3 of the previous frame) so the W3 / W2
  // operand waits of S1 / S2 (in-order vmcnt) never wait on the frame's HBM fetch
  auto load_frame = [&](int f) {
    const __amdgpu_buffer_rsrc_t r_fr = ts_rsrc(a.frames + (size_t)ld_uniform_i32(a.rows, f) * IN_BYTES, IN_BYTES);
#pragma unroll
    for (int k = 0; k < PFF; ++k) {
      const int c = tid + k * NT;
      if (c < IN_CHUNKS) pfr[k] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r_fr, c * 16, 0, 0));
    }
  };
  if (blockIdx.x < a.n) {
    load_frame(blockIdx.x);
    prefetch_acts(blockIdx.x);
  }
  __syncthreads();

  int it_dbg = 0;
  long long* tr = (a.trace && blockIdx.x == 0 && lane == 0) ? a.trace + wave * 16 * 11 : nullptr;
#define TBS_STAMP(k) \
  if (tr && it_dbg < 16) tr[it_dbg * 11 + (k)] = (long long)__builtin_readcyclecounter();
  for (int f = blockIdx.x; f < a.n; f += gridDim.x) {
    TBS_STAMP(0);
    int oz;
    asm volatile("s_mov_b32 %0, 0" : "=s"(oz));
    bf16* frb = (bf16*)(lds + R + oz);
    bf16* a1 = (bf16*)(lds + R + oz);
    bf16* a1lo = (bf16*)(lds + R + R_A1L + oz);
    bf16* a2 = (bf16*)(lds + R + R_A2 + oz);
    bf16* g3p = (bf16*)(lds + G3P + oz);
    bf16* g3pl = (bf16*)(lds + G3PL + oz);
    bf16* g2p = (bf16*)(lds + G2P + oz);
    bf16* g2pl = (bf16*)(lds + G2PL + oz);
    bf16* g1h = (bf16*)(lds + G1H + oz);
    bf16* g1l = (bf16*)(lds + G1L + oz);
    const int2* tbl2 = (const int2*)(lds + TBL2 + oz);
    const int lane_f = lane + oz;
    const int l32 = lane_f & 31, half = lane_f >> 5;
    const int grp = lane_f >> 4, q = (lane_f >> 2) & 3, pp = lane_f & 3;
    const int colb = 16 * (grp & 1) + 4 * pp;
    const int kh1 = 4 * (wave & 1) + 2 * (grp & 1) + (pp >> 1);
    const bf16* fb0 = frb + (wave >> 1) * 7056 + kh1 * 84 + 4 * (pp & 1) + (4 * (2 * half)) * 84 + 4 * q;
    const bf16* fb1 = fb0 + 4 * 84;

    // ======== S0: prefetched activations / gradients -> LDS; W3 hi / lo -> the g1 region by
    // LDS-DMA (1 KB per wave-instruction, 38 of them: chunk j of a plane = row j / 37, 16-byte
    // column min(j % 37, 35); the 37th column is the row pad)
    for (int i = wave; i < 38; i += 8) {
      const int pl = i >= 19, blk = i - 19 * pl, j = blk * 64 + lane;
      const int r = j / 37, c = min(j - 37 * r, 35);
      const bf16* src = (pl ? a.w3dgl : a.w3dg) + (j < 32 * 37 ? r * 288 + c * 8 : 0);
      __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(lds + G1H + pl * W3PL + blk * 1024),
                                       16, 0, 0);
    }
#pragma unroll
    for (int k = 0; k < PF1; ++k) {
      const int c = tid + k * NT;
      const int cs = (c & ~3) | ((c ^ (c >> 4)) & 3);   // tb_sw at chunk granularity
      if (c < P1 * 4) { ((u32x4*)a1)[cs] = pa1[k]; ((u32x4*)a1lo)[cs] = pa1l[k]; }
    }
    if (tid < P2 * 4) ((u32x4*)a2)[(tid & ~3) | ((tid ^ (tid >> 4)) & 3)] = pa2;
    if (tid < 196) {
      const bf16x8 dx = __builtin_bit_cast(bf16x8, pdx), dxl = __builtin_bit_cast(bf16x8, pdxl);
      const bf16x8 o3 = __builtin_bit_cast(bf16x8, po3);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int i = tid * 8 + e, co = i / P3, p = i % P3;
        const bool on = (float)o3[e] > 0.f;
        const int o = tb_sw((p / 7 + 2) * 11 + p % 7 + 2, co);
        g3p[o] = on ? dx[e] : (bf16)0.f;
        g3pl[o] = on ? dxl[e] : (bf16)0.f;
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the W3 DMA (and older loads) landed
    lds_sync();
    TBS_STAMP(1);

    // ======== S1: g2 = convT(g3, W3) * (act2 > 0): waves 0-5, one 16-pixel tile each, both
    // 16-channel halves (v_mfma_f32_16x16x32_bf16, K step = one 3x3 tap x 32 channels), A = W3
    // from LDS, B = g3; transposed output (lane = pixel, 4 consecutive channels per accumulator):
    // one 8-byte mask read and hi / lo store per channel quad
    if (wave < 6) {
      const int l16 = lane_f & 15, kg = lane_f >> 4;
      const int qv = wave * 16 + l16, qc = qv < P2 ? qv : P2 - 1;
      const int gr = (qc / 9 + 2) * 11 + qc % 9 + 2;
      const bf16* w3h = (const bf16*)(lds + G1H + oz) + l16 * W3S + 8 * kg;
      const bf16* w3l = w3h + W3PL / 2;
      f32x4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int o = tb_sw(gr - ((t / 3) * 11 + t % 3), 8 * kg);
        const bf16x8 bh = ts_ld8(g3p + o), bl = ts_ld8(g3pl + o);
#pragma unroll
        for (int ch = 0; ch < 2; ++ch)
          acc[ch] = mfma16_x3(ts_ld8(w3h + ch * 16 * W3S + 32 * t), ts_ld8(w3l + ch * 16 * W3S + 32 * t),
                              bh, bl, acc[ch]);
      }
      TBS_STAMP(9);
      const int row = qv < P2 ? (qc / 9 + 1) * 11 + qc % 9 + 1 : G2_TRASH;
      float db[8];
#pragma unroll
      for (int ch = 0; ch < 2; ++ch) {
        const int c0 = 16 * ch + 4 * kg;
        const bf16x4 mk = *(const bf16x4*)(a2 + tb_sw(qc, c0));
        bf16x4 vh, vl;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float v = (float)mk[e] > 0.f ? acc[ch][e] : 0.f;
          vh[e] = (bf16)v;
          vl[e] = sp_lo(v);
          db[4 * ch + e] = qv < P2 ? v : 0.f;
        }
        *(bf16x4*)(g2p + tb_sw(row, c0)) = vh;
        *(bf16x4*)(g2pl + tb_sw(row, c0)) = vl;
      }
      // db2: sum over the tile's 16 pixel lanes; lane l16 = i < 8 keeps channel quad value i
      // row sums with every lane active (DPP reads of EXEC-masked lanes return 0), then the select
#pragma unroll
      for (int i = 0; i < 8; ++i) db[i] = tb_rowsum16(db[i]);
#pragma unroll
      for (int i = 0; i < 8; ++i) db2p += l16 == i ? db[i] : 0.f;
    }
    TBS_STAMP(10);
    lds_sync();
    TBS_STAMP(2);
    // W2 slices -> LDS (64 wave-instructions of 1 KB, 8 per wave); landed + visible before the
    // dact1 K loop (the dW2 products below run meanwhile).  Chunk j of a plane: phase j / 512,
    // row (j / 16) % 32, 16-byte column (j % 16) ^ (row & 15): the K loop's 32 rows x one column
    // per read hit 16 distinct bank groups
    for (int i = wave; i < 64; i += 8) {
      const int pl = i >> 5, j = (i & 31) * 64 + lane;
      const int ph = j >> 9, r = (j >> 4) & 31, c = (j & 15) ^ (r & 15);
      const bf16* src = (pl ? a.w2dgl : a.w2dg) + (ph * 32 + r) * 128 + c * 8;
      __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(lds + W2ST + pl * W2PL + (i & 31) * 1024),
                                       16, 0, 0);
    }

    // ======== S2: dW2 (tiles wave, wave+8) and dact1 -> g1 (jobs 2w, 2w+1)
    {
      const int nt = wave;
      const int pb = (nt >> 2) * 20 + (nt & 3);   // act1 pixel of this tile's (kh, kw)
      const int cbl = 16 * ((lane_f >> 4) & 1) + 4 * (lane_f & 3);
      const int2* tl = tbl2 + lane_f;
#pragma unroll
      for (int s = 0; s < 6; ++s) {
        const int x0 = tl[(2 * s) * 64].x, x1 = tl[(2 * s + 1) * 64].x;
        const int y0 = tl[(2 * s) * 64].y, y1 = tl[(2 * s + 1) * 64].y;
        const bf16x8 ah = ts_tr8(g2p + x0, g2p + x1), al = ts_tr8(g2pl + x0, g2pl + x1);
        const int u0 = tb_sw(pb + y0, cbl), u1 = tb_sw(pb + y1, cbl);
        const int v0 = tb_sw(pb + 40 + y0, cbl), v1 = tb_sw(pb + 40 + y1, cbl);
        const bf16x8 b0h = ts_tr8(a1 + u0, a1 + u1), b0l = ts_tr8(a1lo + u0, a1lo + u1);
        const bf16x8 b1h = ts_tr8(a1 + v0, a1 + v1);
        const bf16x8 b1l = ts_tr8(a1lo + v0, a1lo + v1);
        acc2a = mfma32_x3(ah, al, b0h, b0l, acc2a);
        acc2b = mfma32_x3(ah, al, b1h, b1l, acc2b);
      }
    }
    TBS_STAMP(6);
    {
      // dact1 -> g1: both of this wave's 32-pixel jobs (phase = wave >> 1) in one pass over K, so
      // every W2 phase fragment (L2, hi / lo) is fetched once per frame, not once per job.
      // Transposed product (A = W2 phase slice, B = g2 pixels): lane l32 owns one act1 pixel and
      // each accumulator quad 4 consecutive channels, so the epilogue is one pixel's mask row read
      // and one 8-byte hi / lo store per quad (vs 16 scattered 2-byte stores and mask reads per
      // lane with the pixel-row layout: ~16k cycles per frame against 1.5k of MFMA).  g1 rows keep
      // S3's 4x4-block order; the 8-byte channel chunk c of row R sits at c ^ ((R >> 1) & 7).
      const int phase = wave >> 1, py = phase >> 1, px = phase & 1;
      int ab[2];
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const int mt = (wave & 1) * 2 + jj;
        const int m = mt * 32 + l32, mc = m < 100 ? m : 99;
        ab[jj] = (mc / 10 + 1) * 11 + mc % 10 + 1;   // g2 bordered row of tap (0, 0)
      }
      // the epilogue's act1 mask rows (act1 stays put until S2b), read ahead of the K loop so
      // their latency is not exposed one quad at a time after it
      bf16x4 mk[2][4];
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const int m = ((wave & 1) * 2 + jj) * 32 + l32, mc = m < 100 ? m : 99;
        const int P = (2 * (mc / 10) + py) * 20 + 2 * (mc % 10) + px;   // act1 pixel
#pragma unroll
        for (int g = 0; g < 4; ++g) mk[jj][g] = *(const bf16x4*)(a1 + tb_sw(P, 8 * g + 4 * half));
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's W2 DMAs landed
      __syncthreads();                                     // ... and every other wave's
      const bf16* w2row = (const bf16*)(lds + W2ST + oz) + (phase * 32 + l32) * 128;
      const int wsw = l32 & 15;
      f32x16 accj[2] = {{}, {}};
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        const int wo = (((2 * s + half) ^ wsw) << 3);
        const bf16x8 bh = ts_ld8(w2row + wo), bl = ts_ld8(w2row + W2PL / 2 + wo);
        const int tap = s >> 1;
        const int dr = (tap >> 1) * 11 + (tap & 1), e0 = (s & 1) * 16 + half * 8;
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
          const int o = tb_sw(ab[jj] - dr, e0);
          accj[jj] = mfma32_x3(bh, bl, ts_ld8(g2p + o), ts_ld8(g2pl + o), accj[jj]);
        }
      }
      lds_sync();   // every wave's W2 reads done before g1 (same region) is written
      TBS_STAMP(7);
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const int mt = (wave & 1) * 2 + jj;
        const int m = mt * 32 + l32, mc = m < 100 ? m : 99;
        const int ay = mc / 10, bx = mc % 10;
        const int row = m < 100 ? 16 * (5 * (ay >> 1) + (bx >> 1)) + 8 * (ay & 1) + 2 * (bx & 1) +
                                  4 * py + px : G1_TRASH;
        const int sw = (row >> 1) & 7;
        const float keep = m < 100 ? 1.f : 0.f;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          bf16x4 vh, vl;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float v = (float)mk[jj][g][e] > 0.f ? accj[jj][4 * g + e] : 0.f;
            vh[e] = (bf16)v;
            vl[e] = sp_lo(v);
            db1v[4 * g + e] = fmaf(v, keep, db1v[4 * g + e]);
          }
          const int o = row * 32 + (((2 * g + half) ^ sw) << 2);
          *(bf16x4*)(g1h + o) = vh;
          *(bf16x4*)(g1l + o) = vl;
        }
      }
    }
    if (f + (int)gridDim.x < a.n) prefetch_acts(f + gridDim.x);
    TBS_STAMP(8);
    lds_sync();
    TBS_STAMP(3);

    // ======== S2b: frame -> R (act1 / act2 no longer read)
#pragma unroll
    for (int k = 0; k < PFF; ++k) {
      const int c = tid + k * NT;
      if (c < IN_CHUNKS) {
        ((bf16x8*)(frb + c * 16))[0] = u8x8_to_bf16(pfr[k][0], pfr[k][1]);
        ((bf16x8*)(frb + c * 16))[1] = u8x8_to_bf16(pfr[k][2], pfr[k][3]);
      }
    }
    lds_sync();
    TBS_STAMP(4);

    // ======== S3: dW1 += g1 . im2col(frame), 25 K steps of one 4x4 pixel block each (2 passes)
    if (f + (int)gridDim.x < a.n) load_frame(f + gridDim.x);
    {
      constexpr int D = 2;
      bf16x8 rah[D], ral[D], rb[D];
      // g1 rows 16 s + 8 half + q and + 4: their chunk swizzles ((R >> 1) & 7) do not depend on s
      const int c4 = colb >> 2;
      const int g0 = (8 * half + q) * 32 + ((c4 ^ ((4 * half + (q >> 1)) & 7)) << 2);
      const int g4 = (8 * half + q + 4) * 32 + ((c4 ^ ((4 * half + 2 + (q >> 1)) & 7)) << 2);
      auto ld = [&](int s, bf16x8& xah, bf16x8& xal, bf16x8& xb) {
        const int blk = (16 * (s / 5)) * 84 + 16 * (s % 5);
        xah = ts_tr8(g1h + 512 * s + g0, g1h + 512 * s + g4);
        xal = ts_tr8(g1l + 512 * s + g0, g1l + 512 * s + g4);
        xb = ts_tr8(fb0 + blk, fb1 + blk);
      };
#pragma unroll
      for (int s = 0; s < D; ++s) ld(s, rah[s], ral[s], rb[s]);
#pragma unroll
      for (int s = 0; s < 25; ++s) {
        const bf16x8 xah = rah[s % D], xal = ral[s % D], xb = rb[s % D];
        if (s + D < 25) ld(s + D, rah[s % D], ral[s % D], rb[s % D]);
        __builtin_amdgcn_sched_barrier(0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xal, xb, acc1, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xah, xb, acc1, 0, 0, 0);
      }
    }
    lds_sync();
    TBS_STAMP(5);
    ++it_dbg;
  }

  // ---- epilogue: this workgroup's partial gradients -> slab (dW3 / db3: torso_dw3_sp_kernel)
  const int l32 = lane & 31, half = lane >> 5;
  float* sl = a.slab + (size_t)blockIdx.x * SLAB;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int co = (r & 3) + 8 * (r >> 2) + 4 * half;
    sl[co * 256 + wave * 32 + l32] = acc1[r];
    sl[OFF_W2 + co * 512 + wave * 32 + l32] = acc2a[r];
    sl[OFF_W2 + co * 512 + (wave + 8) * 32 + l32] = acc2b[r];
  }
  float* red = (float*)(lds + G1H);
  // db1: lane partials of channels 8 (r >> 2) + 4 half + (r & 3), summed over the 32 pixel lanes
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    float v = db1v[r];
#pragma unroll
    for (int o = 1; o < 32; o <<= 1) v += __shfl_xor(v, o, 64);
    if (l32 == 0) red[wave * 32 + 8 * (r >> 2) + 4 * half + (r & 3)] = v;
  }
  red[512 + tid] = wave < 6 ? db2p : 0.f;
  __syncthreads();
  if (tid < 64) {
    const int part = tid >> 5, c = tid & 31;
    float v = 0.f;
    if (part == 0) {
#pragma unroll
      for (int w = 0; w < 8; ++w) v += red[w * 32 + c];
    } else {   // channel c = 16 ch + 4 kg + e at lane 16 kg + 4 ch + e
      const int ln = 16 * ((c >> 2) & 3) + 4 * (c >> 4) + (c & 3);
#pragma unroll
      for (int w = 0; w < 6; ++w) v += red[512 + w * 64 + ln];
    }
    sl[OFF_B + tid] = v;
  }
}

// dW3 += g3 . im2col(act2) and db3 (3 passes), straight from global dX3 / out3 / act2.  Two
// frames in flight per workgroup (1024 threads: half fs of the workgroup takes frames
// 2 blockIdx + fs + 2 k gridDim): per frame the work is ~12 MFMAs per wave against a global
// prefetch, an LDS scatter and two barriers, so a second frame's waves hide the first's waits.
// The halves' accumulators are summed through LDS before the slab store (slab of blockIdx.x).
__global__ __launch_bounds__(1024) void torso_dw3_sp_kernel(const TBSArgs a) {
  using namespace tbs;
  constexpr int G3C_S = 72;
  __shared__ __attribute__((aligned(16))) bf16 g3c[2][2][32 * G3C_S];
  __shared__ __attribute__((aligned(16))) bf16 a2s[2][2][P2 * 32];
  const int fs = threadIdx.x >> 9, tid = threadIdx.x & 511, wave = tid >> 6, lane = tid & 63;
  const int l32 = lane & 31, half = lane >> 5;
  const int grp = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
  const int colb = 16 * (grp & 1) + 4 * pp;
  bf16 (&g3)[2][32 * G3C_S] = g3c[fs];
  bf16 (&a2)[2][P2 * 32] = a2s[fs];
  for (int i = threadIdx.x; i < 2 * 2 * 32 * G3C_S * 2 / 16; i += 1024) ((u32x4*)g3c)[i] = u32x4{0, 0, 0, 0};
  f32x16 acc = {}, acc8 = {};
  float db3p = 0.f;
  u32x4 pa2, pa2l, pdx, pdxl, po3;
  auto prefetch = [&](int f) {
    if (tid < P2 * 4) {
      pa2 = ((const u32x4*)(a.act2 + (size_t)f * P2 * 32))[tid];
      pa2l = ((const u32x4*)(a.act2l + (size_t)f * P2 * 32))[tid];
    }
    if (tid < 196) {
      pdx = ((const u32x4*)(a.dx3 + (size_t)f * 1568))[tid];
      pdxl = ((const u32x4*)(a.dx3l + (size_t)f * 1568))[tid];
      po3 = ((const u32x4*)(a.out3 + (size_t)f * 1568))[tid];
    }
  };
  const int fstride = 2 * gridDim.x;
  int f = 2 * blockIdx.x + fs;
  if (f < a.n) prefetch(f);
  __syncthreads();
  auto im2col_off3 = [&](int s, int r) {
    int P = 16 * s + 8 * half + 4 * r + q;
    P = P < P3 ? P : P3 - 1;
    return ((P / 7) * 9 + P % 7) * 32 + colb;
  };
  const int b0 = ((wave / 3) * 9 + wave % 3) * 32;
  const int b8 = (2 * 9 + 2) * 32;
  // both halves run the same number of iterations (barriers); a half past the end idles
  const int iters = (a.n - 2 * (int)blockIdx.x + fstride - 1) / fstride;
  for (int it = 0; it < iters; ++it, f += fstride) {
    const bool have = f < a.n;
    if (have) {
      if (tid < P2 * 4) { ((u32x4*)a2[0])[tid] = pa2; ((u32x4*)a2[1])[tid] = pa2l; }
      if (tid < 196) {
        const bf16x8 dx = __builtin_bit_cast(bf16x8, pdx), dxl = __builtin_bit_cast(bf16x8, pdxl);
        const bf16x8 o3 = __builtin_bit_cast(bf16x8, po3);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int i = tid * 8 + e, co = i / P3, p = i % P3;
          const bool on = (float)o3[e] > 0.f;
          g3[0][co * G3C_S + p] = on ? dx[e] : (bf16)0.f;
          g3[1][co * G3C_S + p] = on ? dxl[e] : (bf16)0.f;
        }
      }
      if (f + fstride < a.n) prefetch(f + fstride);
    }
    lds_sync();
    if (have) {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int ao = l32 * G3C_S + s * 16 + half * 8;
        const bf16x8 ah = ts_ld8(g3[0] + ao), al = ts_ld8(g3[1] + ao);
        const int o0 = im2col_off3(s, 0), o1 = im2col_off3(s, 1);
        acc = mfma32_x3(ah, al, ts_tr8(a2[0] + b0 + o0, a2[0] + b0 + o1), ts_tr8(a2[1] + b0 + o0, a2[1] + b0 + o1), acc);
        if (wave == 0)
          acc8 = mfma32_x3(ah, al, ts_tr8(a2[0] + b8 + o0, a2[0] + b8 + o1), ts_tr8(a2[1] + b8 + o0, a2[1] + b8 + o1), acc8);
      }
      if (wave == 7) {
        float sum = 0.f;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const bf16x8 v = ts_ld8(g3[0] + l32 * G3C_S + half * 32 + c * 8);
          const bf16x8 vl = ts_ld8(g3[1] + l32 * G3C_S + half * 32 + c * 8);
#pragma unroll
          for (int e = 0; e < 8; ++e) sum += (float)v[e] + (float)vl[e];
        }
        sum += __shfl_xor(sum, 32, 64);
        db3p += sum;
      }
    }
    lds_sync();
  }
  // half 1's accumulators -> LDS (the g3 images are dead: 18 KB), half 0 adds them; every
  // thread takes every barrier
  float* xa = (float*)g3c;
#pragma unroll
  for (int pass = 0; pass < 3; ++pass) {
    // pass 0 / 1: acc rows 8 pass .. +7 of the 8 waves (16 KB); pass 2: wave 0's acc8 + db3
    if (fs == 1) {
      if (pass < 2) {
#pragma unroll
        for (int r = 0; r < 8; ++r) xa[(wave * 8 + r) * 64 + lane] = acc[pass * 8 + r];
      } else {
        if (wave == 0) {
#pragma unroll
          for (int r = 0; r < 16; ++r) xa[r * 64 + lane] = acc8[r];
        }
        if (wave == 7) xa[16 * 64 + lane] = db3p;
      }
    }
    __syncthreads();
    if (fs == 0) {
      if (pass < 2) {
#pragma unroll
        for (int r = 0; r < 8; ++r) acc[pass * 8 + r] += xa[(wave * 8 + r) * 64 + lane];
      } else {
        if (wave == 0) {
#pragma unroll
          for (int r = 0; r < 16; ++r) acc8[r] += xa[r * 64 + lane];
        }
        if (wave == 7) db3p += xa[16 * 64 + lane];
      }
    }
    __syncthreads();
  }
  if (fs == 1) return;
  float* sl = a.slab + (size_t)blockIdx.x * SLAB;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int co = (r & 3) + 8 * (r >> 2) + 4 * half;
    sl[OFF_W3 + co * 288 + wave * 32 + l32] = acc[r];
    if (wave == 0) sl[OFF_W3 + co * 288 + 8 * 32 + l32] = acc8[r];
  }
  if (wave == 7 && lane < 32) sl[OFF_B + 64 + lane] = db3p;
}

extern "C" int r2_torso_grad_reduce(const float* slab, int grid, const int* dst, const float* scale,
                                    float* grad, void* stream);

static long long* g_tbs_trace = nullptr;
static int g_tbs_dbg = 0;   // timing probes: bit 0 W2 fragments not re-fetched, bit 1 no g1 stores
extern "C" int r2_torso_bwd_sp_debug(int bits) { g_tbs_dbg = bits; return 0; }
// stage clock stamps of workgroup 0: [wave][frame < 16][11] (loop top, after S0, S1, S2, S2b, S3,
// S2 dW2 part done, S2 dact1 MFMA loop done, S2 epilogue + prefetch issued, S1 tap loop done,
// S1 epilogue done)
extern "C" int r2_torso_bwd_sp_trace(long long* p) { g_tbs_trace = p; return 0; }

// Split-precision torso backward: every activation / gradient operand as hi / lo planes (out3:
// the torso output's hi plane, a ReLU mask only).  slab: grid x r2_torso_bwd_slab_floats().
// grad == nullptr: the slabs are left for the optimizer launch (optim.hip r2_rmsprop_pack_slab).
extern "C" int r2_torso_bwd_sp(const uint8_t* frames, const int* rows, int n, const bf16* act1,
                               const bf16* act1l, const bf16* act2, const bf16* act2l,
                               const bf16* dx3, const bf16* dx3l, const bf16* out3,
                               const bf16* w3dg, const bf16* w3dgl, const bf16* w2dg,
                               const bf16* w2dgl, float* slab, int grid, const int* dst,
                               const float* scale, float* grad, void* stream) {
  if (n <= 0) return 0;
  if (!rows || !act1l || !act2l || !dx3l || !w3dgl || !w2dgl) return -1;
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)torso_bwd_sp_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                        tbs::LDS);
    attr = true;
  }
  if (grid <= 0 || grid > n) grid = n < 256 ? n : 256;
  TBSArgs a{frames, rows, act1, act1l, act2, act2l, dx3, dx3l, out3, w3dg, w3dgl, w2dg, w2dgl,
            slab, n, g_tbs_dbg, g_tbs_trace};
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(torso_bwd_sp_kernel, dim3(grid), dim3(tbs::NT), tbs::LDS, s, a);
  hipLaunchKernelGGL(torso_dw3_sp_kernel, dim3(grid), dim3(1024), 0, s, a);
  R2_CHECK_LAUNCH();
  if (!grad) return 0;
  return r2_torso_grad_reduce(slab, grid, dst, scale, grad, stream);
}
