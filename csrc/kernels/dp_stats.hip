// Data-parallel global prioritized sampling: the step's per-rank scalars on the device
// (parallel/sharded_replay.py local_stats / global_is_params are the torch references).
//
// As torch ops they were ~16 tiny launches per step, twelve of them on the critical path between
// the gathered stats and the TD launch (~90 us of a 1.1 ms step, profiles/r03_force_dp_trace.txt);
// here one single-wave launch on each side of the 12-byte all-gather.
#include "../common.h"

// out = [S_k, N_k, min_b q_k(b)] of this shard
__global__ __launch_bounds__(64) void dp_local_stats_kernel(const float* root, const int* n_valid,
                                                            const float* probs, int B, float* out) {
  const int lane = threadIdx.x;
  float m = 3.402823466e38f;
  for (int i = lane; i < B; i += 64) m = fminf(m, probs[i]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fminf(m, __shfl_xor(m, o, 64));
  if (lane == 0) {
    out[0] = *root;
    out[1] = (float)*n_valid;
    out[2] = m;
  }
}

// stats: (W, 3) gathered [S_k, N_k, min q_k]; out = [W S_r / S, S_r / S, N, max_k w_max(k)] with
// w_max(k) = W s_k (N min_k s_k)^-beta (beta > 0) or W s_k, s_k = S_k / S
__global__ __launch_bounds__(64) void dp_is_params_kernel(const float* stats, int W, int rank,
                                                          float beta, float* out) {
  const int lane = threadIdx.x;
  float S = 0.f, N = 0.f;
  for (int k = lane; k < W; k += 64) {
    S += stats[3 * k];
    N += stats[3 * k + 1];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    S += __shfl_xor(S, o, 64);
    N += __shfl_xor(N, o, 64);
  }
  S = fmaxf(S, 1e-30f);
  float wmax = -3.402823466e38f;
  for (int k = lane; k < W; k += 64) {
    const float s = stats[3 * k] / S, f = (float)W * s;
    const float w = beta > 0.f ? f * powf(fmaxf(N * stats[3 * k + 2] * s, 1e-30f), -beta) : f;
    wmax = fmaxf(wmax, w);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) wmax = fmaxf(wmax, __shfl_xor(wmax, o, 64));
  if (lane == 0) {
    const float s = stats[3 * rank] / S;
    out[0] = (float)W * s;
    out[1] = s;
    out[2] = N;
    out[3] = wmax;
  }
}

extern "C" int r2_dp_local_stats(const float* root, const int* n_valid, const float* probs, int B,
                                 float* out, void* stream) {
  if (!root || !n_valid || !probs || !out || B < 1) return -1;
  hipLaunchKernelGGL(dp_local_stats_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, root,
                     n_valid, probs, B, out);
  R2_CHECK_LAUNCH();
  return 0;
}

extern "C" int r2_dp_is_params(const float* stats, int W, int rank, float beta, float* out,
                               void* stream) {
  if (!stats || !out || W < 1 || rank < 0 || rank >= W) return -1;
  hipLaunchKernelGGL(dp_is_params_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, stats, W,
                     rank, beta, out);
  R2_CHECK_LAUNCH();
  return 0;
}
