// LSTM recurrence kernels for gfx950 (MI355X).
//
// Replaces the reference's Python time loop of nn.LSTMCell calls (model.py:54-57), which on
// ROCm is 2 GEMMs + a fused pointwise kernel + torch.cat per step per chain.  Design:
//
//  * The input projection x_t . W_ih^T + b_ih + b_hh is hoisted out of the recurrence and done
//    as ONE library GEMM over all T*B rows before these kernels run ("xproj").
//  * The hidden dimension is split across workgroups: workgroup j owns hidden units
//    [16j, 16j+16) and therefore the 64 gate rows {g*H + 16j + u}.  Its slice of W_hh
//    (64 x H bf16 = 32 KB at H=256) is re-read from L2 each step; the gate pre-activations of
//    its 16 units never leave the workgroup, so the pointwise cell is fused into the GEMM
//    epilogue and c/h are produced in place.
//  * Weights and xproj use a *packed* gate-column order: packed column j*64 + g*16 + u holds
//    original gate row g*H + 16j + u (PyTorch order i,f,g,o).  The packing is done once per
//    optimizer step by the pack kernel (optim.hip), so these kernels read contiguous 64-column
//    slices.
//  * Several independent chains (online / target / online-on-next) advance in the same launch
//    (grid.y = chain), so their latencies overlap instead of adding.
//  * The recurrent GEMM runs on MFMA (v_mfma_f32_32x32x16_bf16): M = batch (32-row tiles),
//    N = 64 gate columns (two 32-col tiles), K = H.  One wave per (M-tile, N-tile).
//
// Backward (BPTT) uses the same unit split.  Workgroup j turns dh/dc of its units into the 64
// packed pre-activation gate gradients (pointwise, local) and multiplies them by its W_hh slice
// to get a partial dh_{t-1} over ALL H units (B x H fp32 slab).  The next step's kernel sums the
// 16 slabs for its own units (a reduce-scatter through L2; kernel boundaries order it).
#include "../common.h"

#define LSTM_UNITS 16          // hidden units per workgroup
#define LSTM_GCOLS 64          // gate columns per workgroup (4 gates x 16 units)
#define LSTM_MAX_CHAINS 4

struct LstmChain {
  const float* xproj;  // (T, B, G) packed gate pre-activations incl. biases, chain-local t
  const bf16* whh;     // packed (NWG, 64, H) bf16
  const bf16* h0;      // (B, H) bf16
  const float* c0;     // (B, H)
  bf16* h_seq;         // (T, B, H) bf16 out
  float* c_seq;        // (T, B, H) fp32 out
  float* h32;          // optional (T, B, H) fp32 out
  float* gates;        // optional (T - save_from, B, G) packed post-activation gates
  int save_from;
  int pad_;
};

struct LstmFwdArgs {
  LstmChain ch[LSTM_MAX_CHAINS];
  int B;
  int t;
};

template <int H>
__global__ __launch_bounds__(512) void lstm_fwd_step_kernel(const LstmFwdArgs a) {
  constexpr int G = 4 * H;
  constexpr int LDSW = LSTM_GCOLS + 4;
  __shared__ float gl[128 * LDSW];
  const LstmChain& cd = a.ch[blockIdx.y];
  const int j = blockIdx.x;
  const int B = a.B, t = a.t;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int mt = wave >> 1, nt = wave & 1;
  const bf16* hp = (t == 0) ? cd.h0 : cd.h_seq + (size_t)(t - 1) * B * H;
  const float* cp = (t == 0) ? cd.c0 : cd.c_seq + (size_t)(t - 1) * B * H;

  // ---- recurrent GEMM on MFMA: gates[b][n] = sum_k h[b][k] * Whh_pk[j][n][k]
  {
    const int m = mt * 32 + (lane & 31);
    const int kh = (lane >> 5) * 8;
    const bf16* arow = hp + (size_t)(m < B ? m : B - 1) * H + kh;
    const bf16* brow = cd.whh + ((size_t)j * LSTM_GCOLS + nt * 32 + (lane & 31)) * H + kh;
    f32x16 acc = {};
#pragma unroll 8
    for (int s = 0; s < H / 16; ++s) {
      bf16x8 av = *(const bf16x8*)(arow + s * 16);
      bf16x8 bv = *(const bf16x8*)(brow + s * 16);
      acc = mfma32(av, bv, acc);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      gl[row * LDSW + nt * 32 + (lane & 31)] = acc[r];
    }
  }
  __syncthreads();

  // ---- fused LSTM cell for this workgroup's 16 units
  const bool save = cd.gates != nullptr && t >= cd.save_from;
  for (int idx = threadIdx.x; idx < B * LSTM_UNITS; idx += blockDim.x) {
    const int b = idx >> 4, u = idx & 15;
    const float* xr = cd.xproj + ((size_t)t * B + b) * G + j * LSTM_GCOLS;
    const float* gr = gl + b * LDSW;
    const float gi = sigmoidf_(gr[u] + xr[u]);
    const float gf = sigmoidf_(gr[16 + u] + xr[16 + u]);
    const float gg = tanhf_(gr[32 + u] + xr[32 + u]);
    const float go = sigmoidf_(gr[48 + u] + xr[48 + u]);
    const size_t hidx = (size_t)b * H + j * LSTM_UNITS + u;
    const float c = gf * cp[hidx] + gi * gg;
    const float h = go * tanhf_(c);
    const size_t o = (size_t)t * B * H + hidx;
    cd.c_seq[o] = c;
    cd.h_seq[o] = (bf16)h;
    if (cd.h32) cd.h32[o] = h;
    if (save) {
      float* gp = cd.gates + ((size_t)(t - cd.save_from) * B + b) * G + j * LSTM_GCOLS;
      gp[u] = gi;
      gp[16 + u] = gf;
      gp[32 + u] = gg;
      gp[48 + u] = go;
    }
  }
}

struct LstmBwdArgs {
  const float* dh_ext;  // (Tl, B, H) dL/dh from the head at each learning step (may be null)
  const float* gates;   // (Tl, B, G) packed post-activation gates saved by forward
  const float* c_seq;   // (T, B, H) chain cell states (chain-local time)
  const float* c0;      // (B, H) initial cell state
  const bf16* whhT;     // packed transposed (NWG, H, 64) bf16
  const float* p_in;    // (NWG, B, H) partial dh from step t+1 (null on first bwd step)
  float* p_out;         // (NWG, B, H) partial dh for step t-1 (null on last bwd step)
  float* dc;            // (B, H) dc carry, in/out (zeroed by caller before first step)
  bf16* dgates;         // (Tl, B, G) packed pre-activation gate grads
  int B, t, t0, nwg;    // t chain-local step, t0 = first learning step (save_from)
};

template <int H>
__global__ __launch_bounds__(512) void lstm_bwd_step_kernel(const LstmBwdArgs a) {
  constexpr int G = 4 * H;
  constexpr int LDSW = LSTM_GCOLS + 8;  // bf16 row stride 144 B: conflict-free ds_read_b128
  __shared__ __attribute__((aligned(16))) bf16 dg_lds[128 * LDSW];
  const int j = blockIdx.x;
  const int B = a.B, t = a.t, tl = a.t - a.t0;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;

  // ---- phase A: pointwise BPTT for this workgroup's 16 units
  for (int idx = threadIdx.x; idx < 128 * LSTM_UNITS; idx += blockDim.x) {
    const int b = idx >> 4, u = idx & 15;
    bf16* lrow = dg_lds + b * LDSW;
    if (b >= B) {  // zero padding rows so the MFMA below reads finite values
      lrow[u] = (bf16)0.f; lrow[16 + u] = (bf16)0.f; lrow[32 + u] = (bf16)0.f; lrow[48 + u] = (bf16)0.f;
      continue;
    }
    const size_t hidx = (size_t)b * H + j * LSTM_UNITS + u;
    float dh = a.dh_ext ? a.dh_ext[(size_t)tl * B * H + hidx] : 0.f;
    if (a.p_in) {
      for (int i = 0; i < a.nwg; ++i) dh += a.p_in[(size_t)i * B * H + hidx];
    }
    const float* gp = a.gates + ((size_t)tl * B + b) * G + j * LSTM_GCOLS;
    const float gi = gp[u], gf = gp[16 + u], gg = gp[32 + u], go = gp[48 + u];
    const float ct = a.c_seq[(size_t)t * B * H + hidx];
    const float cprev = (t == 0) ? a.c0[hidx] : a.c_seq[(size_t)(t - 1) * B * H + hidx];
    const float tc = tanhf_(ct);
    const float dc = a.dc[hidx] + dh * go * (1.f - tc * tc);
    const float d_o = dh * tc;
    const float d_i = dc * gg, d_g = dc * gi, d_f = dc * cprev;
    a.dc[hidx] = dc * gf;
    const float pi = d_i * gi * (1.f - gi);
    const float pf = d_f * gf * (1.f - gf);
    const float pg = d_g * (1.f - gg * gg);
    const float po = d_o * go * (1.f - go);
    bf16* dgo = a.dgates + ((size_t)tl * B + b) * G + j * LSTM_GCOLS;
    const bf16 bi = (bf16)pi, bfv = (bf16)pf, bg = (bf16)pg, bo = (bf16)po;
    dgo[u] = bi; dgo[16 + u] = bfv; dgo[32 + u] = bg; dgo[48 + u] = bo;
    lrow[u] = bi; lrow[16 + u] = bfv; lrow[32 + u] = bg; lrow[48 + u] = bo;
  }
  if (a.p_out == nullptr) return;
  __syncthreads();

  // ---- phase B: partial dh_{t-1}[b][n] = sum_k dg[b][k] * Whh_pk[j][k][n]  (K = 64)
  const int mtiles = (B + 31) >> 5;
  const int nwaves = blockDim.x >> 6;
  const int ntiles = mtiles * (H / 32);
  float* pout = a.p_out + (size_t)j * B * H;
  for (int tile = wave; tile < ntiles; tile += nwaves) {
    const int mt = tile / (H / 32), nt = tile % (H / 32);
    const int m = mt * 32 + (lane & 31);
    const int kh = (lane >> 5) * 8;
    const bf16* arow = dg_lds + m * LDSW + kh;
    const bf16* brow = a.whhT + ((size_t)j * H + nt * 32 + (lane & 31)) * LSTM_GCOLS + kh;
    f32x16 acc = {};
#pragma unroll
    for (int s = 0; s < LSTM_GCOLS / 16; ++s) {
      bf16x8 av = *(const bf16x8*)(arow + s * 16);
      bf16x8 bv = *(const bf16x8*)(brow + s * 16);
      acc = mfma32(av, bv, acc);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      if (row < B) pout[(size_t)row * H + nt * 32 + (lane & 31)] = acc[r];
    }
  }
}

// ------------------------------------------------------------------------------------------
// launchers

static inline int lstm_block(int B) {
  const int mtiles = (B + 31) / 32;
  return 128 * mtiles;  // 2 waves (N tiles) per M tile
}

// chain_ptrs: n_chains x 9 int64 values:
//   xproj, whh, h0, c0, h_seq, c_seq, h32, gates, save_from
extern "C" int r2_lstm_fwd(const int64_t* chain_ptrs, int n_chains, int B, int T, int H,
                           int t_begin, void* stream) {
  if (n_chains < 1 || n_chains > LSTM_MAX_CHAINS || B < 1 || B > 128) return -1;
  if (H != 256 && H != 512 && H != 128 && H != 64) return -2;
  LstmFwdArgs args;
  for (int c = 0; c < n_chains; ++c) {
    const int64_t* p = chain_ptrs + 9 * c;
    LstmChain& ch = args.ch[c];
    ch.xproj = (const float*)p[0];
    ch.whh = (const bf16*)p[1];
    ch.h0 = (const bf16*)p[2];
    ch.c0 = (const float*)p[3];
    ch.h_seq = (bf16*)p[4];
    ch.c_seq = (float*)p[5];
    ch.h32 = (float*)p[6];
    ch.gates = (float*)p[7];
    ch.save_from = (int)p[8];
    ch.pad_ = 0;
  }
  args.B = B;
  dim3 grid(H / LSTM_UNITS, n_chains);
  dim3 block(lstm_block(B));
  hipStream_t s = (hipStream_t)stream;
  for (int t = t_begin; t < T; ++t) {
    args.t = t;
    switch (H) {
      case 64: hipLaunchKernelGGL(lstm_fwd_step_kernel<64>, grid, block, 0, s, args); break;
      case 128: hipLaunchKernelGGL(lstm_fwd_step_kernel<128>, grid, block, 0, s, args); break;
      case 256: hipLaunchKernelGGL(lstm_fwd_step_kernel<256>, grid, block, 0, s, args); break;
      default: hipLaunchKernelGGL(lstm_fwd_step_kernel<512>, grid, block, 0, s, args); break;
    }
  }
  R2_CHECK_LAUNCH();
  return 0;
}

// BPTT over chain-local steps t in [t0, T) (descending).  slab0/slab1: two (NWG,B,H) fp32
// ping-pong buffers.  dc must be zeroed by the caller.
extern "C" int r2_lstm_bwd(const float* dh_ext, const float* gates, const float* c_seq,
                           const float* c0, const bf16* whhT, float* slab0, float* slab1,
                           float* dc, bf16* dgates, int B, int T, int t0, int H, void* stream) {
  if (B < 1 || B > 128) return -1;
  if (H != 256 && H != 512 && H != 128 && H != 64) return -2;
  const int nwg = H / LSTM_UNITS;
  LstmBwdArgs a;
  a.dh_ext = dh_ext; a.gates = gates; a.c_seq = c_seq; a.c0 = c0; a.whhT = whhT;
  a.dc = dc; a.dgates = dgates; a.B = B; a.t0 = t0; a.nwg = nwg;
  hipStream_t s = (hipStream_t)stream;
  dim3 grid(nwg), block(lstm_block(B) < 256 ? 256 : lstm_block(B));
  float* slabs[2] = {slab0, slab1};
  for (int t = T - 1, k = 0; t >= t0; --t, ++k) {
    a.t = t;
    a.p_in = (t == T - 1) ? nullptr : slabs[(k + 1) & 1];
    a.p_out = (t == t0) ? nullptr : slabs[k & 1];
    switch (H) {
      case 64: hipLaunchKernelGGL(lstm_bwd_step_kernel<64>, grid, block, 0, s, a); break;
      case 128: hipLaunchKernelGGL(lstm_bwd_step_kernel<128>, grid, block, 0, s, a); break;
      case 256: hipLaunchKernelGGL(lstm_bwd_step_kernel<256>, grid, block, 0, s, a); break;
      default: hipLaunchKernelGGL(lstm_bwd_step_kernel<512>, grid, block, 0, s, a); break;
    }
  }
  R2_CHECK_LAUNCH();
  return 0;
}
