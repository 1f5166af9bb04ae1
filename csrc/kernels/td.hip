// Fused n-step double-Q TD target / loss / gradient / priority kernel (gfx950).
//
// Reference: learner.py:82-104 computes, over 6 separate PyTorch ops plus a D2H copy and a
// numpy scatter:
//   q      = Q_online(s_t).gather(a_t)                         (learner.py:86)
//   a*     = argmax_a Q_online(s_{t+n})                         (learner.py:90-91)
//   y      = R_t + gamma^n * Q_target(s_{t+n})[a*] * (1 - d_t)  (learner.py:92-94)
//   loss   = mean(0.5 (q - y)^2)                                (learner.py:98)
//   p_row  = (|q - y| + 1e-6)^0.6  -> replay priority[index]    (learner.py:102-103)
// Here it is ONE kernel (one thread per transition, ceil(Tl*B/256) workgroups) that also gathers
// a_t / R_t / d_t from the HBM replay by ring row, applies optional R2D2 value rescaling h / h^-1
// and IS weights, writes dL/dQ (the only gradient the head backward needs) and scatters the new
// row priorities.  The loss is reduced deterministically: every workgroup publishes its partial
// (sc1 store, drained), takes a ticket with an agent-scope atomic, and the last arriver sums the
// partials in workgroup order with sc1 loads (MI355X_MICROARCH.md hand-off table, row 1).
#include "../common.h"

__device__ __forceinline__ float vr_h(float x, float eps) {
  return copysignf(sqrtf(fabsf(x) + 1.f) - 1.f, x) + eps * x;
}
__device__ __forceinline__ float vr_hinv(float x, float eps) {
  const float s = (sqrtf(1.f + 4.f * eps * (fabsf(x) + 1.f + eps)) - 1.f) / (2.f * eps);
  return copysignf(s * s - 1.f, x);
}

__device__ __forceinline__ int ring_row(int start, int t, int cap_e) {
  const int base = start - start % cap_e;
  return base + (start - base + t) % cap_e;
}

struct TdArgs {
  const float* q_sa;    // (Tl, B, A)
  const float* q_arg;   // (Tl, B, A)  online Q at s_{t+n} (argmax)
  const float* q_tgt;   // (Tl, B, A)  target Q at s_{t+n}
  const int* starts;    // (B) sequence start rows
  const float* probs;   // (B) sampling probability of each sequence (IS weights) or null
  const uint8_t* action;  // (cap)
  const float* reward;  // (cap)
  const uint8_t* done;  // (cap)
  float* dq;            // (Tl, B, A) out
  float* loss;          // (1) out
  float* td_abs;        // (Tl, B) out, may be null
  float* priority;      // (cap) row priorities, scatter out (may be null)
  float* is_w;          // (B) normalised IS weights out, may be null
  const int* n_valid;   // number of sampleable sequences (device), for IS weights
  float* part;          // (gridDim.x) loss partials
  unsigned* ticket;     // arrival counter, 0 between launches (reset by the last arriver)
  int Tl, B, A, burn_in, cap_e;
  float gamma_n, vr_eps, alpha, prio_eps, beta;
  int value_rescale;
};

__global__ __launch_bounds__(256) void td_kernel(const TdArgs a) {
  __shared__ float red[8];
  __shared__ float wsh[256];
  __shared__ int last;
  const int tid = threadIdx.x;
  // ---- IS weights w_b = (N * P_b)^-beta / max_b  (B <= 256; recomputed per workgroup)
  float w = 1.f;
  if (tid < a.B && a.probs != nullptr && a.beta > 0.f) {
    const float nv = a.n_valid ? (float)max(*a.n_valid, 1) : 1.f;
    w = powf(fmaxf(nv * a.probs[tid], 1e-30f), -a.beta);
  }
  float m = wave_max(tid < a.B ? w : 0.f);
  if ((tid & 63) == 0) red[tid >> 6] = m;
  __syncthreads();
  const float wmax = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  if (tid < a.B) {
    wsh[tid] = w / wmax;
    if (a.is_w && blockIdx.x == 0) a.is_w[tid] = w / wmax;
  }
  __syncthreads();

  const int n = a.Tl * a.B;
  const float inv_n = 1.f / (float)n;
  float lsum = 0.f;
  const int i = blockIdx.x * 256 + tid;
  if (i < n) {
    const int b = i % a.B, tl = i / a.B;
    const int row = ring_row(a.starts[b], a.burn_in + tl, a.cap_e);
    const int act = (int)a.action[row];
    const float* qs = a.q_sa + (size_t)i * a.A;
    const float* qa = a.q_arg + (size_t)i * a.A;
    const float* qt = a.q_tgt + (size_t)i * a.A;
    int best = 0;
    float bv = qa[0];
    for (int k = 1; k < a.A; ++k) {
      if (qa[k] > bv) { bv = qa[k]; best = k; }
    }
    float boot = qt[best];
    if (a.value_rescale) boot = vr_hinv(boot, a.vr_eps);
    float y = a.reward[row] + (a.done[row] ? 0.f : a.gamma_n * boot);
    if (a.value_rescale) y = vr_h(y, a.vr_eps);
    const float delta = qs[act] - y;
    const float wb = wsh[b];
    lsum = wb * 0.5f * delta * delta;
    float* d = a.dq + (size_t)i * a.A;
    for (int k = 0; k < a.A; ++k) d[k] = (k == act) ? wb * delta * inv_n : 0.f;
    const float ad = fabsf(delta);
    if (a.td_abs) a.td_abs[i] = ad;
    if (a.priority) a.priority[row] = powf(ad + a.prio_eps, a.alpha);
  }
  lsum = wave_sum(lsum);
  __syncthreads();
  if ((tid & 63) == 0) red[tid >> 6] = lsum;
  __syncthreads();
  if (tid == 0) {
    const float v = red[0] + red[1] + red[2] + red[3];
    __hip_atomic_store(a.part + blockIdx.x, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // sc1
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned t = __hip_atomic_fetch_add(a.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = t == gridDim.x - 1;
  }
  __syncthreads();
  if (last && tid == 0) {
    float tot = 0.f;
    for (unsigned g = 0; g < gridDim.x; ++g)
      tot += __hip_atomic_load(a.part + g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *a.loss = tot * inv_n;
    __hip_atomic_store(a.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

extern "C" int r2_td_loss(const float* q_sa, const float* q_arg, const float* q_tgt,
                          const int* starts, const float* probs, const uint8_t* action,
                          const float* reward, const uint8_t* done, float* dq, float* loss,
                          float* td_abs, float* priority, float* is_w, const int* n_valid,
                          int Tl, int B, int A, int burn_in, int cap_e, float gamma_n,
                          int value_rescale, float vr_eps, float alpha, float prio_eps,
                          float beta, float* part, unsigned* ticket, void* stream) {
  if (B > 256) return -1;
  const int grid = (Tl * B + 255) / 256;
  if (grid > 4096) return -2;   // part[] holds one float per workgroup (engine: 4096)
  TdArgs a{q_sa, q_arg, q_tgt, starts, probs, action, reward, done, dq, loss, td_abs, priority,
           is_w, n_valid, part, ticket, Tl, B, A, burn_in, cap_e, gamma_n, vr_eps, alpha, prio_eps,
           beta, value_rescale};
  hipLaunchKernelGGL(td_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, a);
  R2_CHECK_LAUNCH();
  return 0;
}
