// Dueling Q head epilogues for gfx950.
//
// Reference: model.py:26-36,62-64:  val = Linear(256,1)(relu(Linear(256,256)(h))),
// adv = Linear(256,A)(relu(Linear(256,256)(h))),  q = val + adv - mean(adv).
//
// The two 256->256 hidden layers are ONE concatenated GEMM  z = h . [Wv1;Wa1]^T  (N x 512)
// done by the library GEMM.  These kernels fuse everything after it: bias + ReLU, the tiny
// block-diagonal 512 -> (1 + A) projection, the dueling combine (forward), and its exact
// backward (dz for the GEMM backward plus the per-row dv/da used for the small weight grads).
// One wave per row; each lane owns 4 of the 256 value-branch and 4 of the 256 advantage-branch
// features (HD = 256).
#include "../common.h"
#include "../split.h"

#define HEAD_MAXA 32

// z: (N, 2*HD) bf16 pre-activation of [val.0 ; adv.0] WITHOUT bias; b1: (2*HD) fp32
// w2: (1 + A, HD) fp32 rows [val.2.weight ; adv.2.weight]; b2: (1 + A)
// q: (N, A) fp32 out.  zr (optional): (N, 2*HD) bf16 relu(z + b1) out (for weight grads)
// Up to 3 heads (online / target / online-on-next) per launch: wave w takes row w - row0[j] of
// the head j whose row range holds it.
#define HEAD_MAXJ 3
// ZT = bf16 (bf16 mode) or float (split-precision mode: z from an fp32-output GEMM, zr fp32)
struct DuelJob {
  const void* z; const float* b1; const float* w2; const float* b2; float* q; void* zr;
  int N, row0;
};
struct DuelArgs {
  DuelJob j[HEAD_MAXJ];
  int nj, A;
};

template <int HD, typename ZT>
__global__ __launch_bounds__(256) void dueling_fwd_kernel(const DuelArgs args) {
  constexpr int PER = HD / 64;
  const int lane = threadIdx.x & 63;
  const int w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  int ji = 0;
#pragma unroll
  for (int i = 1; i < HEAD_MAXJ; ++i)
    if (i < args.nj && w >= args.j[i].row0) ji = i;
  const DuelJob& J = args.j[ji];
  const int row = w - J.row0, N = J.N, A = args.A;
  if (row >= N) return;
  const ZT* __restrict__ z = (const ZT*)J.z;
  const float* __restrict__ b1 = J.b1;
  const float* __restrict__ w2 = J.w2;
  const float* __restrict__ b2 = J.b2;
  float* __restrict__ q = J.q;
  ZT* __restrict__ zr = (ZT*)J.zr;
  const ZT* zrow = z + (size_t)row * 2 * HD;
  float hv[PER], ha[PER];
#pragma unroll
  for (int e = 0; e < PER; ++e) {
    const int c = lane * PER + e;
    hv[e] = fmaxf((float)zrow[c] + b1[c], 0.f);
    ha[e] = fmaxf((float)zrow[HD + c] + b1[HD + c], 0.f);
  }
  if (zr) {
    ZT* o = zr + (size_t)row * 2 * HD;
#pragma unroll
    for (int e = 0; e < PER; ++e) {
      o[lane * PER + e] = (ZT)hv[e];
      o[HD + lane * PER + e] = (ZT)ha[e];
    }
  }
  float v = 0.f;
#pragma unroll
  for (int e = 0; e < PER; ++e) v += hv[e] * w2[lane * PER + e];
  v = wave_sum_x(v) + b2[0];
  float amean = 0.f, mine = 0.f;
  for (int a = 0; a < A; ++a) {
    float s = 0.f;
#pragma unroll
    for (int e = 0; e < PER; ++e) s += ha[e] * w2[(size_t)(1 + a) * HD + lane * PER + e];
    s = wave_sum_x(s) + b2[1 + a];
    mine = (a == lane) ? s : mine;
    amean += s;
  }
  amean /= (float)A;
  if (lane < A) q[(size_t)row * A + lane] = v + mine - amean;
}

// Backward.  dq: (N, A) fp32.  zr: (N, 2*HD) bf16 relu'd hidden (from forward).
// dz: (N, 2*HD) bf16 out = dL/d(z) (through relu), dva: (N, 1 + A) fp32 out = [dv, da_0..].
template <int HD>
__global__ __launch_bounds__(256) void dueling_bwd_kernel(
    const float* __restrict__ dq, const bf16* __restrict__ zr, const float* __restrict__ w2,
    bf16* __restrict__ dz, float* __restrict__ dva, int N, int A) {
  constexpr int PER = HD / 64;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (row >= N) return;
  const float* dqr = dq + (size_t)row * A;
  float dv = 0.f;
  for (int a = 0; a < A; ++a) dv += dqr[a];
  const float dmean = dv / (float)A;
  if (lane == 0) dva[(size_t)row * (1 + A)] = dv;
  if (lane < A) dva[(size_t)row * (1 + A) + 1 + lane] = dqr[lane] - dmean;
  const bf16* zrow = zr + (size_t)row * 2 * HD;
  bf16* dzrow = dz + (size_t)row * 2 * HD;
#pragma unroll
  for (int e = 0; e < PER; ++e) {
    const int c = lane * PER + e;
    const float gv = dv * w2[c];
    float ga = 0.f;
    for (int a = 0; a < A; ++a) ga += (dqr[a] - dmean) * w2[(size_t)(1 + a) * HD + c];
    dzrow[c] = (bf16)(((float)zrow[c] > 0.f) ? gv : 0.f);
    dzrow[HD + c] = (bf16)(((float)zrow[HD + c] > 0.f) ? ga : 0.f);
  }
}

template <typename ZT>
static int dueling_fwd_launch(const int64_t* jobs, int nj, int A, int HD, void* stream) {
  if (nj < 1 || nj > HEAD_MAXJ) return -3;
  if (A < 1 || A > HEAD_MAXA) return -1;
  DuelArgs a{};
  a.nj = nj;
  a.A = A;
  int rows = 0;
  for (int i = 0; i < nj; ++i) {
    const int64_t* p = jobs + 7 * i;
    DuelJob& J = a.j[i];
    J.z = (const void*)p[0]; J.b1 = (const float*)p[1]; J.w2 = (const float*)p[2];
    J.b2 = (const float*)p[3]; J.q = (float*)p[4]; J.zr = (void*)p[5];
    J.N = (int)(p[6] > 0 ? p[6] : 0); J.row0 = rows;
    rows += J.N;
  }
  for (int i = nj; i < HEAD_MAXJ; ++i) a.j[i].row0 = 1 << 30;
  if (rows <= 0) return 0;
  dim3 grid((rows + 3) / 4), block(256);
  hipStream_t s = (hipStream_t)stream;
  switch (HD) {
    case 64: hipLaunchKernelGGL((dueling_fwd_kernel<64, ZT>), grid, block, 0, s, a); break;
    case 128: hipLaunchKernelGGL((dueling_fwd_kernel<128, ZT>), grid, block, 0, s, a); break;
    case 256: hipLaunchKernelGGL((dueling_fwd_kernel<256, ZT>), grid, block, 0, s, a); break;
    case 512: hipLaunchKernelGGL((dueling_fwd_kernel<512, ZT>), grid, block, 0, s, a); break;
    default: return -2;
  }
  R2_CHECK_LAUNCH();
  return 0;
}

// jobs: nj x 7 int64 {z, b1, w2, b2, q, zr, N}; z / zr bf16
extern "C" int r2_dueling_fwd_multi(const int64_t* jobs, int nj, int A, int HD, void* stream) {
  return dueling_fwd_launch<bf16>(jobs, nj, A, HD, stream);
}
// split precision: z / zr fp32
extern "C" int r2_dueling_fwd_multi_f32(const int64_t* jobs, int nj, int A, int HD, void* stream) {
  return dueling_fwd_launch<float>(jobs, nj, A, HD, stream);
}

extern "C" int r2_dueling_fwd(const bf16* z, const float* b1, const float* w2, const float* b2,
                              float* q, bf16* zr, int N, int A, int HD, void* stream) {
  const int64_t job[7] = {(int64_t)z, (int64_t)b1, (int64_t)w2, (int64_t)b2, (int64_t)q,
                          (int64_t)zr, N};
  return r2_dueling_fwd_multi(job, 1, A, HD, stream);
}

extern "C" int r2_dueling_bwd(const float* dq, const bf16* zr, const float* w2, bf16* dz,
                              float* dva, int N, int A, int HD, void* stream) {
  if (N <= 0) return 0;
  if (A < 1 || A > HEAD_MAXA) return -1;
  dim3 grid((N + 3) / 4), block(256);
  hipStream_t s = (hipStream_t)stream;
  switch (HD) {
    case 64: hipLaunchKernelGGL(dueling_bwd_kernel<64>, grid, block, 0, s, dq, zr, w2, dz, dva, N, A); break;
    case 128: hipLaunchKernelGGL(dueling_bwd_kernel<128>, grid, block, 0, s, dq, zr, w2, dz, dva, N, A); break;
    case 256: hipLaunchKernelGGL(dueling_bwd_kernel<256>, grid, block, 0, s, dq, zr, w2, dz, dva, N, A); break;
    case 512: hipLaunchKernelGGL(dueling_bwd_kernel<512>, grid, block, 0, s, dq, zr, w2, dz, dva, N, A); break;
    default: return -2;
  }
  R2_CHECK_LAUNCH();
  return 0;
}
