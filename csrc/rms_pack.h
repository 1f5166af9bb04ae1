// The centered-RMSprop update + row packs (optim.hip rmsprop_pack_kernel) as a device function.
// (Round 5 ran it on extra workgroups of the priority tail's launch: correct, but the update's
// ~67 MB of HBM traffic slowed the tail's latency-bound barrier phases -- 35.6 us for the pair vs
// 22.9 + 14.9 apart, step +4 us -- and was removed.)
//   sq = a*sq + (1-a)*g^2 ; ga = a*ga + (1-a)*g ; p -= lr * g / (sqrt(sq - ga^2) + eps)
// (torch.optim.RMSprop(centered=True), learner.py:51,97-100).  Master float4 q also lands, as bf16
// hi (and split-precision lo) planes, at packed position dst4[q] (-1: packed by pack_step's
// gather); when the target sync is due ((step + 1) % interval == 0, learner.py:107-108) the
// target master and target packs are written too.
#pragma once
#include "common.h"

struct RmsPackArgs {
  float* p;
  const float* g;
  float* sq;
  float* ga;
  int64_t n;
  float lr, alpha, eps, gscale;
  const float* clip_sumsq;
  float max_norm;
  const int* dst4;
  bf16* bf;
  bf16* bf_t;
  int64_t lo_off;
  float* target;
  const int64_t* step;
  int64_t interval;
};

__device__ __forceinline__ void rmsprop_pack_items(const RmsPackArgs& a, int64_t first, int64_t stride) {
  float scale = a.gscale;
  if (a.clip_sumsq != nullptr && a.max_norm > 0.f) {
    const float norm = sqrtf(*a.clip_sumsq) * a.gscale;
    if (norm > a.max_norm) scale *= a.max_norm / (norm + 1e-6f);
  }
  const float lr = a.lr, alpha = a.alpha, eps = a.eps;
  float* __restrict__ p = a.p;
  const float* __restrict__ g = a.g;
  float* __restrict__ sq = a.sq;
  float* __restrict__ ga = a.ga;
  const bool due = a.interval <= 1 || ((*a.step) + 1) % a.interval == 0;
  const int64_t n = a.n, n4 = n >> 2;
  for (int64_t i = first; i < n4; i += stride) {
    f32x4 pv = ((f32x4*)p)[i], gv = ((const f32x4*)g)[i];
    f32x4 sv = ((f32x4*)sq)[i], av = ((f32x4*)ga)[i];
    const int d = a.dst4[i];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float gr = gv[e] * scale;
      sv[e] = alpha * sv[e] + (1.f - alpha) * gr * gr;
      av[e] = alpha * av[e] + (1.f - alpha) * gr;
      pv[e] -= lr * gr / (sqrtf(sv[e] - av[e] * av[e]) + eps);
    }
    ((f32x4*)p)[i] = pv;
    ((f32x4*)sq)[i] = sv;
    ((f32x4*)ga)[i] = av;
    if (due) ((f32x4*)a.target)[i] = pv;
    if (d >= 0) {
      bf16x4 h, l;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        h[e] = (bf16)pv[e];
        l[e] = (bf16)(pv[e] - (float)h[e]);
      }
      *(bf16x4*)(a.bf + d) = h;
      if (a.lo_off) *(bf16x4*)(a.bf + a.lo_off + d) = l;
      if (due) {
        *(bf16x4*)(a.bf_t + d) = h;
        if (a.lo_off) *(bf16x4*)(a.bf_t + a.lo_off + d) = l;
      }
    }
  }
  for (int64_t i = (n4 << 2) + first; i < n; i += stride) {
    const float gr = g[i] * scale;
    sq[i] = alpha * sq[i] + (1.f - alpha) * gr * gr;
    ga[i] = alpha * ga[i] + (1.f - alpha) * gr;
    p[i] -= lr * gr / (sqrtf(sq[i] - ga[i] * ga[i]) + eps);
    if (due) a.target[i] = p[i];
  }
}

// host-side argument checks: 16-B master / grad / state / target, 8-B packs
inline bool rms_pack_args_ok(const RmsPackArgs& a) {
  return !((((uintptr_t)a.p | (uintptr_t)a.g | (uintptr_t)a.sq | (uintptr_t)a.ga | (uintptr_t)a.target) & 15) ||
           (((uintptr_t)a.bf | (uintptr_t)a.bf_t) & 7) || (a.lo_off & 3) || !a.dst4 || !a.step);
}
