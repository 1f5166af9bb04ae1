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
#include "slab_reduce.h"

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
  // optional torso section (r2_rmsprop_pack_slab, world 1): the first tblocks workgroups sum the
  // torso backward's slabs (slab_reduce.h, tG slabs of tSL floats) and update master elements
  // tdst[e] with gradient tscale[e] * sum (written to gw too) -- the torso_grad_reduce launch
  // folded in; the quad loop then ends at quad tq (every master element from 4 * tq on is a
  // torso element or zero padding: the torso bucket is the master's tail, layout.py)
  const float* slab;
  const int* tdst;
  const float* tscale;
  float* gw;
  int tG, tSL, tblocks, pad_;
  int64_t tq;
};

// one element of the centered update (every path below: the same expression, the same bits)
__device__ __forceinline__ float rms_elem(float& sq, float& ga, float p, float gr, float lr,
                                          float alpha, float eps) {
  sq = alpha * sq + (1.f - alpha) * gr * gr;
  ga = alpha * ga + (1.f - alpha) * gr;
  return p - lr * gr / (sqrtf(sq - ga * ga) + eps);
}

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
  // quad q: update, row pack (dst4)
  auto quad = [&](int64_t q) {
    f32x4 pv = ((f32x4*)p)[q], gv = ((const f32x4*)g)[q];
    f32x4 sv = ((f32x4*)sq)[q], av = ((f32x4*)ga)[q];
    const int d = a.dst4[q];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float s = sv[e], m = av[e];
      pv[e] = rms_elem(s, m, pv[e], gv[e] * scale, lr, alpha, eps);
      sv[e] = s;
      av[e] = m;
    }
    ((f32x4*)p)[q] = pv;
    ((f32x4*)sq)[q] = sv;
    ((f32x4*)ga)[q] = av;
    if (due) ((f32x4*)a.target)[q] = pv;
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
  };
  const int64_t qend = a.tblocks ? a.tq : n4;
  for (int64_t i = first; i < qend; i += stride) quad(i);
  for (int64_t i = (n4 << 2) + first; i < n && !a.tblocks; i += stride) {
    float sv = sq[i], av = ga[i];
    p[i] = rms_elem(sv, av, p[i], g[i] * scale, lr, alpha, eps);
    sq[i] = sv;
    ga[i] = av;
    if (due) a.target[i] = p[i];
  }
}

// torso section block blk: column sums of 64 slab columns, then the element update at tdst[e]
// (the same per-element arithmetic as the quad path; gscale 1 at world 1, no clipping)
__device__ __forceinline__ void rmsprop_torso_items(const RmsPackArgs& a, int blk) {
  __shared__ float part[4][64];
  const float s = slab_column_sum(a.slab, a.tG, a.tSL, blk, part);
  const int e = blk * 64 + (int)threadIdx.x;
  if (threadIdx.x >= 64 || e >= a.tSL) return;
  const int m = a.tdst[e];
  const float gv = s * a.tscale[e];
  a.gw[m] = gv;
  float sv = a.sq[m], av = a.ga[m];
  const float pv = rms_elem(sv, av, a.p[m], gv * a.gscale, a.lr, a.alpha, a.eps);
  a.sq[m] = sv;
  a.ga[m] = av;
  a.p[m] = pv;
  if (a.interval <= 1 || ((*a.step) + 1) % a.interval == 0) a.target[m] = pv;
}

// host-side argument checks: 16-B master / grad / state / target, 8-B packs
inline bool rms_pack_args_ok(const RmsPackArgs& a) {
  return !((((uintptr_t)a.p | (uintptr_t)a.g | (uintptr_t)a.sq | (uintptr_t)a.ga | (uintptr_t)a.target) & 15) ||
           (((uintptr_t)a.bf | (uintptr_t)a.bf_t) & 7) || (a.lo_off & 3) || !a.dst4 || !a.step);
}
