// Column sums of the torso backward's per-workgroup fp32 gradient slabs (G slabs of SL floats):
// one 256-thread block covers 64 columns x 4 row-groups (coalesced 256-B row segments, 16
// independent loads in flight per thread), the 4 partials combined through LDS in a fixed order.
// Shared by torso_bwd.hip's torso_grad_reduce_kernel and optim.hip's folded update (rms_pack.h
// torso section) so both produce the same bits.
#pragma once
#include "common.h"

// column blockIdx-relative: e = blk * 64 + (tid & 63); returns the full sum on threads tid < 64
// (valid when e < SL), after a __syncthreads every thread of the block reaches
__device__ __forceinline__ float slab_column_sum(const float* __restrict__ slab, int G, int SL,
                                                 int blk, float (*part)[64]) {
  const int c = threadIdx.x & 63, gq = threadIdx.x >> 6;
  const int e = blk * 64 + c;
  float s = 0.f;
  if (e < SL) {
    const float* p = slab + e;
    int g = gq;
    for (; g + 60 < G; g += 64) {
      float v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = p[(size_t)(g + 4 * u) * SL];
#pragma unroll
      for (int u = 0; u < 16; ++u) s += v[u];
    }
    for (; g < G; g += 4) s += p[(size_t)g * SL];
  }
  part[gq][c] = s;
  __syncthreads();
  return part[0][c] + part[1][c] + part[2][c] + part[3][c];
}
