// Device code of the dueling head's last-layer / bias gradient reduction (gradsum.hip), shared
// with the BPTT kernel, whose otherwise idle workgroups run it beside the recurrence
// (lstm_persist.hip, lstm_bwd_tag_kernel helper blocks).
#pragma once
#include "common.h"

namespace gs {
constexpr int NT = 256;     // 64 columns x 4 row groups
constexpr int MAXW = 8;     // weight columns (1 + n_actions) handled per launch
constexpr int NV = 12;      // per column: sum, dva-sum, 8 weighted sums, 2 pad (3 x 16 B)
constexpr int QB = 8;       // partials in flight per reduction batch
}  // namespace gs

struct HeadGradArgs {
  const float* dva;   // (N, 1+A) fp32
  const bf16* zr;     // (N, 2HD) bf16, relu'd layer-1 activations [value | advantage]
  const bf16* dz;     // (N, 2HD) bf16, layer-1 pre-activation gradient
  float* gw2;         // (1+A, HD): row 0 = val.2.weight, rows 1.. = adv.2.weight
  float* gb2;         // (1+A): val.2.bias, adv.2.bias
  float* gb1;         // (2HD): val.0.bias, adv.0.bias
  float* ws;          // partials: (NP, CB, RS, 64, NV)
  unsigned* ticket;   // (NP, CB), 0 between launches
  int N, A, HD, RS;
  int NP;             // passes over the advantage rows (7 per pass: A <= 7 -> 1, Seaquest 18 -> 3)
  const float* zr32;  // split precision: zr fp32 (replaces zr)
  const bf16* dz_lo;  // split precision: lo plane of dz
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t gs_rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, 0, 0x7fffffff, 0x00020000);
}

// Publish this workgroup's 64 x NV partials (write-through sc1 b128 stores, drained), take the
// column block's ticket; true in the last arriver (every thread).
__device__ __forceinline__ bool gs_publish(float* ws_blk, const float (&v)[gs::NV],
                                           unsigned* ticket, int RS, int* flag) {
  const int tid = threadIdx.x;
  if (tid < 64) {
    const __amdgpu_buffer_rsrc_t r = gs_rsrc(ws_blk);
#pragma unroll
    for (int i = 0; i < gs::NV / 4; ++i) {
      u32x4 w;
#pragma unroll
      for (int e = 0; e < 4; ++e) w[e] = __builtin_bit_cast(uint32_t, v[4 * i + e]);
      __builtin_amdgcn_raw_buffer_store_b128(w, r, (tid * gs::NV + 4 * i) * 4, 0, 16);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const unsigned t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = t == (unsigned)RS - 1;
  }
  __syncthreads();
  return *flag != 0;
}

// Last arriver, thread c < 64: t = sum over the RS partials of column c, in row-split order.
// sc1 b128 loads (every load of cross-workgroup bytes: MI355X_MICROARCH.md hand-off table),
// QB partials in flight per batch.
__device__ __forceinline__ void gs_gather(const float* ws_cb, int RS, int c, float (&t)[gs::NV]) {
  const __amdgpu_buffer_rsrc_t r = gs_rsrc(ws_cb);
#pragma unroll
  for (int i = 0; i < gs::NV; ++i) t[i] = 0.f;
  for (int q0 = 0; q0 < RS; q0 += gs::QB) {
    u32x4 w[gs::QB][gs::NV / 4];
#pragma unroll
    for (int q = 0; q < gs::QB; ++q) {
      const int qq = q0 + q < RS ? q0 + q : RS - 1;
#pragma unroll
      for (int i = 0; i < gs::NV / 4; ++i)
        w[q][i] = __builtin_amdgcn_raw_buffer_load_b128(r, ((qq * 64 + c) * gs::NV + 4 * i) * 4, 0, 16);
    }
#pragma unroll
    for (int q = 0; q < gs::QB; ++q) {
      if (q0 + q >= RS) break;
#pragma unroll
      for (int i = 0; i < gs::NV / 4; ++i) {
        // whole-vector bit_cast: per-element bit_casts of the loaded u32x4 let the compiler
        // shrink the b128 load to one dword and reuse it for all four elements (observed)
        const f32x4 f = __builtin_bit_cast(f32x4, w[q][i]);
#pragma unroll
        for (int e = 0; e < 4; ++e) t[4 * i + e] += f[e];
      }
    }
  }
}

// One (column block cb, row split rs, advantage pass p) work item, run by a whole workgroup of
// >= 256 threads: threads >= 256 only take part in the barriers (the BPTT kernel's helper
// workgroups have 320).  Pass p covers advantage rows [7p, 7p + 7); the value row, the bias sums
// and the dva column sums belong to pass 0.
__device__ __forceinline__ void head_grads_body(const HeadGradArgs& a, int cb, int rs, int p = 0) {
  __shared__ float red[4][64][gs::NV];
  __shared__ int flag;
  const int tid = threadIdx.x, c = tid & 63, rg = min(tid >> 6, 3);
  const bool act = tid < 256;
  const int C = 2 * a.HD, col = cb * 64 + c;
  const bool vcol = col < C;
  const bool adv = col >= a.HD;            // uniform per column block (HD % 64 == 0)
  const int W = 1 + a.A;
  const int r0 = (int)((long)a.N * rs / a.RS), r1 = (int)((long)a.N * (rs + 1) / a.RS);
  float s = 0.f, dvs = 0.f, w[gs::MAXW];
#pragma unroll
  for (int i = 0; i < gs::MAXW; ++i) w[i] = 0.f;
  // rows r0+rg, +4, ...: loads of U rows issued together, then accumulated in row order
  constexpr int U = 5;
  for (int rb = r0 + rg; act && rb < r1; rb += 4 * U) {
    float z[U], d[U], dvv[U][gs::MAXW], dsl[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int r = min(rb + 4 * u, r1 - 1);
      const float* dv = a.dva + (size_t)r * W;
      const size_t o = (size_t)r * C + col;
      z[u] = vcol ? (a.zr32 ? a.zr32[o] : (float)a.zr[o]) : 0.f;
      d[u] = vcol ? (float)a.dz[o] + (a.dz_lo ? (float)a.dz_lo[o] : 0.f) : 0.f;
      dvv[u][0] = dv[0];
#pragma unroll
      for (int i = 1; i < gs::MAXW; ++i) dvv[u][i] = 7 * p + i < W ? dv[7 * p + i] : 0.f;
      dsl[u] = (cb == 0 && p == 0 && c < W) ? dv[c] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (rb + 4 * u >= r1) break;
      s += d[u];
      if (!adv) {
        w[0] += dvv[u][0] * z[u];
      } else {
#pragma unroll
        for (int i = 0; i < gs::MAXW - 1; ++i) w[i] += dvv[u][1 + i] * z[u];
      }
      dvs += dsl[u];
    }
  }
  if (act) {
    red[rg][c][0] = s;
    red[rg][c][1] = dvs;
#pragma unroll
    for (int i = 0; i < gs::MAXW; ++i) red[rg][c][2 + i] = w[i];
    red[rg][c][10] = red[rg][c][11] = 0.f;
  }
  __syncthreads();
  float v[gs::NV];
#pragma unroll
  for (int i = 0; i < gs::NV; ++i)
    v[i] = tid < 64 ? ((red[0][c][i] + red[1][c][i]) + (red[2][c][i] + red[3][c][i])) : 0.f;
  const int CB = (2 * a.HD + 63) / 64, pcb = p * CB + cb;
  float* blk = a.ws + ((size_t)pcb * a.RS + rs) * 64 * gs::NV;
  if (!gs_publish(blk, v, a.ticket + pcb, a.RS, &flag)) return;
  if (tid >= 64) return;
  float t[gs::NV];
  gs_gather(a.ws + (size_t)pcb * a.RS * 64 * gs::NV, a.RS, c, t);
  if (vcol) {
    if (p == 0) a.gb1[col] = t[0];
    if (!adv) {
      if (p == 0) a.gw2[col] = t[2];
    } else {
      for (int i = 0; i < 7 && 7 * p + i < a.A; ++i)
        a.gw2[(size_t)(1 + 7 * p + i) * a.HD + (col - a.HD)] = t[2 + i];
    }
  }
  if (p == 0 && cb == 0 && c < W) a.gb2[c] = t[1];
  if (c == 0) __hip_atomic_store(a.ticket + pcb, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
