// Synthetic Atari-shaped environments, one launch per env step for all E envs.
//
// Replaces the ~12 torch ops (and ~150 us of an actor step at E = 256, profiles/
// r02_native_concurrent.txt) of envs/synthetic.py VecSyntheticAtari.step: the cue-and-act
// dynamics (reward 1 when the action equals the current target, the target redrawn every
// `switch` agent steps, episodes of `episode_len` steps, auto-reset) plus the render of the next
// observation (uniform noise 0..47 on every stacked plane, the target's column band painted 220,
// on every step or -- cue_only_first -- only on the first step after a switch).
//
// One workgroup per env: thread 0 advances the env's scalars (read by the rest through LDS), all
// 256 threads write the env's C*H*W observation bytes as 16-byte vectors.  Random numbers are a
// counter-based hash of (seed, the env's own step counter k[e], byte index), so the launch is
// graph-capturable and needs no torch generator; k[e] is owned by the env's workgroup.
#include "../common.h"

struct EnvArgs {
  const long long* action;   // (E) actions of this step
  long long* t;              // (E) step within the episode
  long long* target;         // (E) rewarded action
  long long* k;              // (E) per-env RNG step counter
  float* ep_return;          // (E)
  float* reward;             // (E) out
  bool* done;                // (E) out
  float* finished;           // (E) out: the episode return where done, else NaN
  uint8_t* frames;           // (E, C*H*W) out: the next observation
  unsigned long long seed;
  int E, A, C, H, W, episode_len, sw, cue_only_first;
};

__device__ __forceinline__ uint32_t env_hash(uint64_t seed, uint64_t a, uint64_t b) {
  return (uint32_t)(r2_mix64(seed ^ r2_mix64(a * 0x9E3779B97F4A7C15ull + b)) >> 32);
}

__global__ __launch_bounds__(256) void synth_env_step_kernel(const EnvArgs a) {
  const int e = blockIdx.x, tid = threadIdx.x;
  __shared__ int s_target, s_show;
  __shared__ long long s_k;
  if (tid == 0) {
    const long long k = a.k[e];
    const long long tgt = a.target[e];
    const float r = (a.action[e] == tgt) ? 1.f : 0.f;
    const float ret = a.ep_return[e] + r;
    long long t = a.t[e] + 1;
    long long nt = tgt;
    if (t % a.sw == 0) nt = (long long)(env_hash(a.seed, (uint64_t)k, 0xFFFFFFFFull + e) % (uint32_t)a.A);
    const bool d = t >= a.episode_len;
    a.reward[e] = r;
    a.done[e] = d;
    a.finished[e] = d ? ret : __builtin_nanf("");
    if (d) t = 0;
    a.t[e] = t;
    a.target[e] = nt;
    a.ep_return[e] = d ? 0.f : ret;
    a.k[e] = k + 1;
    s_target = (int)nt;
    s_show = (!a.cue_only_first) || (t % a.sw == 0);
    s_k = k;
  }
  __syncthreads();
  const int band = a.W / a.A;
  const int lo = s_target * band, hi = lo + band;
  const bool show = s_show;
  const uint64_t kk = (uint64_t)s_k * 0x100000001B3ull + (uint64_t)e;
  const int FB = a.C * a.H * a.W;
  uint8_t* dst = a.frames + (size_t)e * FB;
  // 16 bytes per thread per iteration; every W (84 / 96) is a multiple of 4, so a 4-byte word
  // never straddles a row, and FB is a multiple of 16
  for (int v = tid; v < FB / 16; v += blockDim.x) {
    uint32_t w[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int byte0 = v * 16 + q * 4;
      const uint32_t h = env_hash(a.seed, kk, (uint64_t)byte0);
      const int col0 = byte0 % a.W;
      uint32_t word = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        uint32_t b = (((h >> (8 * j)) & 0xffu) * 48u) >> 8;   // uniform-ish 0..47
        const int col = col0 + j;
        if (show && col >= lo && col < hi) b = 220u;
        word |= b << (8 * j);
      }
      w[q] = word;
    }
    reinterpret_cast<u32x4*>(dst)[v] = u32x4{w[0], w[1], w[2], w[3]};
  }
}

extern "C" int r2_env_args_bytes() { return (int)sizeof(EnvArgs); }

extern "C" int r2_synth_env_step(const EnvArgs* a, void* stream) {
  if (a->E <= 0 || a->A <= 0 || a->sw <= 0 || a->W % 4 != 0 || (a->C * a->H * a->W) % 16 != 0)
    return -1;
  hipLaunchKernelGGL(synth_env_step_kernel, dim3(a->E), dim3(256), 0, (hipStream_t)stream, *a);
  R2_CHECK_LAUNCH();
  return 0;
}
