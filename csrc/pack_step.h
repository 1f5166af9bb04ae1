// The per-step weight repack (optim.hip pack_step_kernel) as a device function, shared with the
// fused priority tail (replay.hip prio_tail_kernel's pack workgroups).
//
// Work items (grid-stride): [target copy, 4 floats each (due only)] [bf pack, 4 elements each:
// one 16-B index load, 4 gathers, one 8-B store] [bf tail] [f32 gather] [lstm bias]
//   * online: bf16 kernel-layout pack (+ split-precision lo plane), fp32 small-vector gather,
//     packed b_ih + b_hh
//   * target, only when (step + 1) % interval == 0 (learner.py:107-108 target sync): target =
//     master, and its packs are the online packs of the same master values (no read of the copy)
#pragma once
#include "common.h"

struct PackStepArgs {
  const float* master;
  float* target;
  int64_t n_master;      // 0: the target master is written by the optimizer (rmsprop_pack)
  const int* bf_idx;
  bf16* bf;
  bf16* bf_t;
  int64_t n_bf;
  const int* f_idx;
  float* f32;
  float* f32_t;
  int64_t n_f, o_bih, o_bhh;
  float* lstm_b;
  float* lstm_b_t;
  int64_t G;
  const int64_t* step;
  int64_t interval, lo_off;
};

__device__ __forceinline__ void pack_step_items(const PackStepArgs& a, int64_t first, int64_t stride) {
  const bool due = a.interval <= 1 || ((*a.step) + 1) % a.interval == 0;
  const int64_t nm4 = due ? a.n_master >> 2 : 0, nb4 = a.n_bf >> 2, nbt = a.n_bf & 3;
  const int64_t total = nm4 + nb4 + nbt + a.n_f + a.G;
  const float* __restrict__ master = a.master;
  for (int64_t i = first; i < total; i += stride) {
    int64_t j = i;
    if (j < nm4) {
      ((f32x4*)a.target)[j] = ((const f32x4*)master)[j];
      continue;
    }
    j -= nm4;
    if (j < nb4) {
      const int4 ix = ((const int4*)a.bf_idx)[j];
      bf16x4 v;
      v[0] = (bf16)master[ix.x];
      v[1] = (bf16)master[ix.y];
      v[2] = (bf16)master[ix.z];
      v[3] = (bf16)master[ix.w];
      ((bf16x4*)a.bf)[j] = v;
      if (due) ((bf16x4*)a.bf_t)[j] = v;
      if (a.lo_off) {   // split precision: lo plane (split.h)
        bf16x4 l;
        l[0] = (bf16)(master[ix.x] - (float)v[0]);
        l[1] = (bf16)(master[ix.y] - (float)v[1]);
        l[2] = (bf16)(master[ix.z] - (float)v[2]);
        l[3] = (bf16)(master[ix.w] - (float)v[3]);
        ((bf16x4*)(a.bf + a.lo_off))[j] = l;
        if (due) ((bf16x4*)(a.bf_t + a.lo_off))[j] = l;
      }
      continue;
    }
    j -= nb4;
    if (j < nbt) {
      j += nb4 << 2;
      const float x = master[a.bf_idx[j]];
      const bf16 v = (bf16)x;
      a.bf[j] = v;
      if (due) a.bf_t[j] = v;
      if (a.lo_off) {
        const bf16 l = (bf16)(x - (float)v);
        a.bf[j + a.lo_off] = l;
        if (due) a.bf_t[j + a.lo_off] = l;
      }
      continue;
    }
    j -= nbt;
    if (j < a.n_f) {
      const float v = master[a.f_idx[j]];
      a.f32[j] = v;
      if (due) a.f32_t[j] = v;
      continue;
    }
    j -= a.n_f;
    const float b = master[a.f_idx[a.o_bih + j]] + master[a.f_idx[a.o_bhh + j]];
    a.lstm_b[j] = b;
    if (due) a.lstm_b_t[j] = b;
  }
}

// host-side argument checks shared by the launchers: 16-B master / target / index rows, 8-B packs
inline bool pack_step_args_ok(const PackStepArgs& a) {
  return !((a.n_master & 3) || (((uintptr_t)a.master | (uintptr_t)a.target | (uintptr_t)a.bf_idx) & 15) ||
           (((uintptr_t)a.bf | (uintptr_t)a.bf_t) & 7) || (a.lo_off & 3));
}
