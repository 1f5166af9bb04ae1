// Deterministic column reductions of the learner's backward pass (gfx950).
//
// Reference math: the dueling head's last-layer weight / bias gradients and the LSTM / head
// first-layer bias gradients of learner.py:99 (autograd of model.py:26-36,62-66 and the LSTMCell
// bias).  All of them are sums over the N = learn_len x B rows of one step:
//
//   head_grads:  d val.2.weight = dva[:,0]^T zr[:, :HD]      d adv.2.weight = dva[:,1:]^T zr[:, HD:]
//                d {val,adv}.2.bias = colsum(dva)            d {val,adv}.0.bias = colsum(dz)
//   colsum:      d lstm.bias_ih = d lstm.bias_hh = colsum(dgates), packed gate order -> torch order
//
// Before: four library GEMVs against a ones row, a bf16->fp32 copy, slicing copies and an
// index_select (9 launches).  Here one launch each: (64 columns) x (row split) workgroups,
// per-workgroup partials stored write-through (sc1) and drained, an agent-scope ticket per column
// block, and the last arriving workgroup of a column block sums the partials in row-split order
// (fixed order => bit-reproducible) and writes the gradients in place in the flat buffer.
#include "../common.h"

#include "../gradsum.h"

__global__ __launch_bounds__(256) void head_grads_kernel(const HeadGradArgs a) {
  head_grads_body(a, blockIdx.x, blockIdx.y % a.RS, blockIdx.y / a.RS);
}

struct ColsumArgs {
  const bf16* X;      // (N, C) bf16
  const int* perm;    // output index of column c (or null)
  float* out;
  float* out2;        // optional second copy
  float* ws;          // (CB, RS, 64, NV)
  unsigned* ticket;   // (CB)
  int N, C, RS;
};

__global__ __launch_bounds__(256) void colsum_kernel(const ColsumArgs a) {
  __shared__ float red[4][64];
  __shared__ int flag;
  const int cb = blockIdx.x, rs = blockIdx.y;
  const int tid = threadIdx.x, c = tid & 63, rg = tid >> 6;
  const int col = cb * 64 + c;
  const int r0 = (int)((long)a.N * rs / a.RS), r1 = (int)((long)a.N * (rs + 1) / a.RS);
  float s = 0.f;
  constexpr int U = 10;
  if (col < a.C)
    for (int rb = r0 + rg; rb < r1; rb += 4 * U) {
      float x[U];
#pragma unroll
      for (int u = 0; u < U; ++u) x[u] = (float)a.X[(size_t)min(rb + 4 * u, r1 - 1) * a.C + col];
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (rb + 4 * u < r1) s += x[u];
    }
  red[rg][c] = s;
  __syncthreads();
  float v[gs::NV] = {};
  if (tid < 64) v[0] = (red[0][c] + red[1][c]) + (red[2][c] + red[3][c]);
  float* blk = a.ws + ((size_t)cb * a.RS + rs) * 64 * gs::NV;
  if (!gs_publish(blk, v, a.ticket + cb, a.RS, &flag)) return;
  if (tid >= 64) return;
  float tv[gs::NV];
  gs_gather(a.ws + (size_t)cb * a.RS * 64 * gs::NV, a.RS, c, tv);
  const float t = tv[0];
  if (col < a.C) {
    const int o = a.perm ? a.perm[col] : col;
    a.out[o] = t;
    if (a.out2) a.out2[o] = t;
  }
  if (c == 0) __hip_atomic_store(a.ticket + cb, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ws: >= r2_gradsum_ws_floats() floats; ticket: >= 64 unsigned, zero at first use.
extern "C" int r2_gradsum_ws_floats() { return 64 * 32 * 64 * gs::NV; }

static int head_grads_launch(HeadGradArgs a, void* stream) {
  if (a.HD % 64 != 0 || a.N < 1 || a.A < 1 || a.A > 63) return -1;
  const int CB = (2 * a.HD + 63) / 64;
  a.RS = 32;
  a.NP = (a.A + 6) / 7;
  if (CB * a.NP > 32 || CB * a.RS * a.NP > 64 * 32) return -2;   // tickets / workspace
  hipLaunchKernelGGL(head_grads_kernel, dim3(CB, a.RS * a.NP), dim3(gs::NT), 0, (hipStream_t)stream, a);
  R2_CHECK_LAUNCH();
  return 0;
}

// tickets: >= 32 unsigned, zero at first use (the engine's colsum uses the next 32)
extern "C" int r2_head_grads(const float* dva, const bf16* zr, const bf16* dz, float* gw2,
                             float* gb2, float* gb1, int N, int A, int HD, float* ws,
                             unsigned* ticket, void* stream) {
  HeadGradArgs a{dva, zr, dz, gw2, gb2, gb1, ws, ticket, N, A, HD, 32, 1, nullptr, nullptr};
  return head_grads_launch(a, stream);
}

// split precision: zr fp32, dz as hi / lo planes
extern "C" int r2_head_grads_sp(const float* dva, const float* zr32, const bf16* dz,
                                const bf16* dz_lo, float* gw2, float* gb2, float* gb1, int N, int A,
                                int HD, float* ws, unsigned* ticket, void* stream) {
  HeadGradArgs a{dva, nullptr, dz, gw2, gb2, gb1, ws, ticket, N, A, HD, 32, 1, zr32, dz_lo};
  return head_grads_launch(a, stream);
}

extern "C" int r2_colsum_bf16(const bf16* X, int N, int C, const int* perm, float* out,
                              float* out2, float* ws, unsigned* ticket, void* stream) {
  const int CB = (C + 63) / 64, RS = 32;
  if (CB > 64 || N < 1) return -1;
  ColsumArgs a{X, perm, out, out2, ws, ticket, N, C, RS};
  hipLaunchKernelGGL(colsum_kernel, dim3(CB, RS), dim3(gs::NT), 0, (hipStream_t)stream, a);
  R2_CHECK_LAUNCH();
  return 0;
}
