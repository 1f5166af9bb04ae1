// Fused multi-tensor optimizer + weight packing kernels (gfx950).
//
// Reference: learner.py:51,97-100 uses torch.optim.RMSprop(centered=True), a per-tensor
// foreach loop over 18 parameter tensors.  Here all parameters live in ONE flat fp32 master
// buffer (the same buffer layout is the gradient all-reduce bucket), so the whole update is
// one grid-stride launch with float4 accesses.  Numerics follow torch.optim.RMSprop exactly:
//   sq = a*sq + (1-a)*g^2 ; ga = a*ga + (1-a)*g ; p -= lr * g / (sqrt(sq - ga^2) + eps)
// Adam (paper preset) follows torch.optim.Adam (bias-corrected, eps outside the sqrt), with
// the step count read from device memory so HIP-graph replays advance it.
// Gradient scale (1/world for DP averaging) and optional global-norm clipping are fused.
#include "../common.h"
#include "../pack_step.h"
#include "../rms_pack.h"

__global__ void rmsprop_centered_kernel(float* __restrict__ p, const float* __restrict__ g,
                                        float* __restrict__ sq, float* __restrict__ ga, int64_t n,
                                        float lr, float alpha, float eps, float gscale,
                                        const float* __restrict__ clip_sumsq, float max_norm) {
  float scale = gscale;
  if (clip_sumsq != nullptr && max_norm > 0.f) {
    const float norm = sqrtf(*clip_sumsq) * gscale;
    if (norm > max_norm) scale *= max_norm / (norm + 1e-6f);
  }
  const int64_t n4 = n >> 2;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += stride) {
    f32x4 pv = ((f32x4*)p)[i], gv = ((const f32x4*)g)[i];
    f32x4 sv = ((f32x4*)sq)[i], av = ((f32x4*)ga)[i];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float s = sv[e], m = av[e];
      pv[e] = rms_elem(s, m, pv[e], gv[e] * scale, lr, alpha, eps);
      sv[e] = s;
      av[e] = m;
    }
    ((f32x4*)p)[i] = pv;
    ((f32x4*)sq)[i] = sv;
    ((f32x4*)ga)[i] = av;
  }
  for (int64_t i = (n4 << 2) + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += stride) {
    float sv = sq[i], av = ga[i];
    p[i] = rms_elem(sv, av, p[i], g[i] * scale, lr, alpha, eps);
    sq[i] = sv;
    ga[i] = av;
  }
}

// rmsprop_centered_kernel + the row packs (rms_pack.h rmsprop_pack_items): same arithmetic
// (bit-identical master), one HBM pass fewer over the big LSTM / head weights than
// update-then-gather.
// With a torso section (r2_rmsprop_pack_slab) the first tblocks workgroups reduce + update the
// torso elements and the rest run the quad loop up to quad tq.
__global__ __launch_bounds__(256) void rmsprop_pack_kernel(const RmsPackArgs a) {
  const int b = (int)blockIdx.x - a.tblocks;
  if (b < 0) {
    rmsprop_torso_items(a, blockIdx.x);
    return;
  }
  rmsprop_pack_items(a, b * (int64_t)blockDim.x + threadIdx.x, (int64_t)(gridDim.x - a.tblocks) * blockDim.x);
}

__global__ void adam_kernel(float* __restrict__ p, const float* __restrict__ g,
                            float* __restrict__ m, float* __restrict__ v, int64_t n, float lr,
                            float b1, float b2, float eps, float gscale,
                            const int64_t* __restrict__ step, const float* __restrict__ clip_sumsq,
                            float max_norm) {
  float scale = gscale;
  if (clip_sumsq != nullptr && max_norm > 0.f) {
    const float norm = sqrtf(*clip_sumsq) * gscale;
    if (norm > max_norm) scale *= max_norm / (norm + 1e-6f);
  }
  const float t = (float)(*step + 1);
  const float bc1 = 1.f - powf(b1, t), bc2 = 1.f - powf(b2, t);
  const float step_size = lr / bc1;
  const float bc2s = sqrtf(bc2);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += stride) {
    const float gr = g[i] * scale;
    const float mi = b1 * m[i] + (1.f - b1) * gr;
    const float vi = b2 * v[i] + (1.f - b2) * gr * gr;
    m[i] = mi;
    v[i] = vi;
    p[i] -= step_size * mi / (sqrtf(vi) / bc2s + eps);
  }
}

__global__ void sumsq_kernel(const float* __restrict__ g, int64_t n, float* __restrict__ out) {
  float s = 0.f;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += stride) s += g[i] * g[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) atomicAdd(out, s);
}

// out[i] = bf16(src[idx[i]]) : one launch re-packs every weight into the kernel layouts
// (conv channels-last k order, LSTM packed gate columns, W_hh^T slices, head concat).
__global__ void pack_bf16_kernel(const float* __restrict__ src, const int* __restrict__ idx,
                                 bf16* __restrict__ out, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += stride)
    out[i] = (bf16)src[idx[i]];
}

// split precision (split.h): hi = bf16(x) at out[i], lo = bf16(x - hi) at out[i + lo_off]
__global__ void pack_split_kernel(const float* __restrict__ src, const int* __restrict__ idx,
                                  bf16* __restrict__ out, int64_t n, int64_t lo_off) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += stride) {
    const float x = src[idx[i]];
    const bf16 h = (bf16)x;
    out[i] = h;
    out[i + lo_off] = (bf16)(x - (float)h);
  }
}

__global__ void gather_f32_kernel(const float* __restrict__ src, const int* __restrict__ idx,
                                  float* __restrict__ out, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += stride)
    out[i] = src[idx[i]];
}

// target sync inside a captured graph: copy when (step + 1) % interval == 0
__global__ void copy_if_due_kernel(float* __restrict__ dst, const float* __restrict__ src,
                                   int64_t n, const int64_t* __restrict__ step, int64_t interval) {
  if (((*step) + 1) % interval != 0) return;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += stride) dst[i] = src[i];
}

static inline int grid_for(int64_t n, int per_thread) {
  int64_t b = (n / per_thread + 255) / 256;
  if (b > 2048) b = 2048;
  if (b < 1) b = 1;
  return (int)b;
}

extern "C" int r2_rmsprop_centered(float* p, const float* g, float* sq, float* ga, int64_t n,
                                   float lr, float alpha, float eps, float gscale,
                                   const float* clip_sumsq, float max_norm, void* stream) {
  if (((uintptr_t)p | (uintptr_t)g | (uintptr_t)sq | (uintptr_t)ga) & 15) return -1;
  hipLaunchKernelGGL(rmsprop_centered_kernel, dim3(grid_for(n, 4)), dim3(256), 0,
                     (hipStream_t)stream, p, g, sq, ga, n, lr, alpha, eps, gscale, clip_sumsq,
                     max_norm);
  R2_CHECK_LAUNCH();
  return 0;
}

// n: the master length (float4 rows: dst4 has n / 4 entries); the pack launch after it then
// gathers only the packs before bf_rows_begin and skips the target master copy
extern "C" int r2_rmsprop_pack(float* p, const float* g, float* sq, float* ga, int64_t n, float lr,
                               float alpha, float eps, float gscale, const float* clip_sumsq,
                               float max_norm, const int* dst4, bf16* bf, bf16* bf_t, int64_t lo_off,
                               float* target, const int64_t* step, int64_t interval, void* stream) {
  RmsPackArgs a{p, g, sq, ga, n, lr, alpha, eps, gscale, clip_sumsq, max_norm, dst4, bf, bf_t,
                lo_off, target, step, interval};
  if (!rms_pack_args_ok(a)) return -1;
  hipLaunchKernelGGL(rmsprop_pack_kernel, dim3(grid_for(n, 4)), dim3(256), 0, (hipStream_t)stream, a);
  R2_CHECK_LAUNCH();
  return 0;
}

// r2_rmsprop_pack with the torso slab reduction folded in (world 1, no clipping): the torso
// backward's slabs (grid x SL floats, torso_bwd.hip) are summed by the first ceil(SL / 64)
// workgroups, which update master element dst[e] with gradient scale[e] * sum (and write it to g
// like torso_grad_reduce); the quad loop stops at quad tq (the caller guarantees every master
// element from 4 * tq on is a torso element or zero padding, with no row pack there).
extern "C" int r2_rmsprop_pack_slab(float* p, float* g, float* sq, float* ga, int64_t n, float lr,
                                    float alpha, float eps, float gscale, const int* dst4, bf16* bf,
                                    bf16* bf_t, int64_t lo_off, float* target, const int64_t* step,
                                    int64_t interval, const float* slab, int grid, int SL,
                                    const int* dst, const float* scale, int64_t tq, void* stream) {
  RmsPackArgs a{p, g, sq, ga, n, lr, alpha, eps, gscale, nullptr, 0.f, dst4, bf, bf_t,
                lo_off, target, step, interval};
  a.slab = slab; a.tdst = dst; a.tscale = scale; a.gw = g;
  a.tG = grid; a.tSL = SL; a.tblocks = (SL + 63) / 64; a.tq = tq;
  if (!rms_pack_args_ok(a) || !slab || !dst || !scale || grid <= 0 || SL <= 0 || tq < 0 ||
      4 * tq > n)
    return -1;
  hipLaunchKernelGGL(rmsprop_pack_kernel, dim3(a.tblocks + grid_for(4 * tq, 4)), dim3(256), 0,
                     (hipStream_t)stream, a);
  R2_CHECK_LAUNCH();
  return 0;
}

extern "C" int r2_adam(float* p, const float* g, float* m, float* v, int64_t n, float lr, float b1,
                       float b2, float eps, float gscale, const int64_t* step,
                       const float* clip_sumsq, float max_norm, void* stream) {
  hipLaunchKernelGGL(adam_kernel, dim3(grid_for(n, 1)), dim3(256), 0, (hipStream_t)stream, p, g, m,
                     v, n, lr, b1, b2, eps, gscale, step, clip_sumsq, max_norm);
  R2_CHECK_LAUNCH();
  return 0;
}

extern "C" int r2_sumsq(const float* g, int64_t n, float* out, void* stream) {
  hipMemsetAsync(out, 0, sizeof(float), (hipStream_t)stream);
  hipLaunchKernelGGL(sumsq_kernel, dim3(grid_for(n, 4)), dim3(256), 0, (hipStream_t)stream, g, n,
                     out);
  R2_CHECK_LAUNCH();
  return 0;
}

extern "C" int r2_pack_bf16(const float* src, const int* idx, bf16* out, int64_t n, void* stream) {
  hipLaunchKernelGGL(pack_bf16_kernel, dim3(grid_for(n, 2)), dim3(256), 0, (hipStream_t)stream, src,
                     idx, out, n);
  R2_CHECK_LAUNCH();
  return 0;
}

extern "C" int r2_pack_split(const float* src, const int* idx, bf16* out, int64_t n,
                             int64_t lo_off, void* stream) {
  hipLaunchKernelGGL(pack_split_kernel, dim3(grid_for(n, 2)), dim3(256), 0, (hipStream_t)stream,
                     src, idx, out, n, lo_off);
  R2_CHECK_LAUNCH();
  return 0;
}

extern "C" int r2_gather_f32(const float* src, const int* idx, float* out, int64_t n, void* stream) {
  hipLaunchKernelGGL(gather_f32_kernel, dim3(grid_for(n, 2)), dim3(256), 0, (hipStream_t)stream,
                     src, idx, out, n);
  R2_CHECK_LAUNCH();
  return 0;
}

extern "C" int r2_copy_if_due(float* dst, const float* src, int64_t n, const int64_t* step,
                              int64_t interval, void* stream) {
  hipLaunchKernelGGL(copy_if_due_kernel, dim3(grid_for(n, 4)), dim3(256), 0, (hipStream_t)stream,
                     dst, src, n, step, interval);
  R2_CHECK_LAUNCH();
  return 0;
}

// One launch for everything between the optimizer and the next step's kernels (replaces
// copy_if_due + 2 x {bf16 pack, fp32 gather, LSTM bias add}): pack_step.h pack_step_items.  The
// learner's single-rank step runs the same items on extra workgroups of the priority-tail launch
// instead (replay.hip r2_prio_tail_pack).
__global__ void pack_step_kernel(const PackStepArgs a) {
  pack_step_items(a, blockIdx.x * (int64_t)blockDim.x + threadIdx.x, (int64_t)gridDim.x * blockDim.x);
}

extern "C" int r2_pack_step(const float* master, float* target, int64_t n_master, const int* bf_idx,
                            bf16* bf, bf16* bf_t, int64_t n_bf, const int* f_idx, float* f32,
                            float* f32_t, int64_t n_f, int64_t o_bih, int64_t o_bhh, float* lstm_b,
                            float* lstm_b_t, int64_t G, const int64_t* step, int64_t interval,
                            int64_t lo_off, void* stream) {
  const PackStepArgs a{master, target, n_master, bf_idx, bf, bf_t, n_bf, f_idx, f32, f32_t, n_f,
                       o_bih, o_bhh, lstm_b, lstm_b_t, G, step, interval, lo_off};
  if (!pack_step_args_ok(a)) return -1;
  hipLaunchKernelGGL(pack_step_kernel, dim3(1024), dim3(256), 0, (hipStream_t)stream, a);
  R2_CHECK_LAUNCH();
  return 0;
}

extern "C" int r2_abi_version() { return 1; }
