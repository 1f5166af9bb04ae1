// Fused n-step double-Q TD target / loss / gradient / priority kernel (gfx950).
#define HEAD_FWD_MAXA 32
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
#include <type_traits>
#include "../common.h"
#include "../split.h"

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
  // data-parallel global prioritized sampling (parallel/sharded_replay.py), or null:
  // {W*S_k/S, S_k/S, N_global, global max of the weights}; the weight of sample b is
  // (W*S_k/S) * (N_global * P_global(b))^-beta / gmax with P_global = probs[b] * S_k/S
  const float* dp;
};

// Deterministic row-priority scatter.  Two sampled sequences can share learning rows (overlapping
// starts, or one start sampled twice); the reference resolves the duplicate indices of
// `update_priority(index[burn_in:].reshape(-1), ...)` (learner.py:101-103) as numpy does: the
// LAST element in (t, b) row-major order wins.  Transition (tl, b) therefore writes only if no
// (tl', b') with tl' * B + b' > tl * B + b maps to the same ring row.  `st`: the B starts.
__device__ __forceinline__ bool prio_owner(const int* st, int B, int Tl, int burn_in, int cap_e,
                                           int tl, int b, int lane0, int lanes) {
  const int sb = st[b];
  const int base = sb - sb % cap_e, ob = sb - base;
  bool own = true;
  for (int c = lane0; c < B; c += lanes) {
    const int sc = st[c];
    if (sc - sc % cap_e != base) continue;                 // another sub-ring
    // tl' with start_c + burn_in + tl' == start_b + burn_in + tl (mod cap_e)
    int d = (ob - (sc - base) + tl) % cap_e;
    if (d < 0) d += cap_e;
    if (d < Tl && d * B + c > tl * B + b) own = false;
  }
  return own;
}

// un-normalised IS weight of sample b (b < B); *global_norm: already normalised across ranks
__device__ __forceinline__ float is_weight(const TdArgs& a, int b, bool* global_norm) {
  *global_norm = a.dp != nullptr;
  if (a.dp != nullptr) {
    const float f = a.dp[0];
    const float w = (a.beta > 0.f && a.probs != nullptr)
                        ? powf(fmaxf(a.dp[2] * a.probs[b] * a.dp[1], 1e-30f), -a.beta) : 1.f;
    return f * w / a.dp[3];
  }
  if (a.probs != nullptr && a.beta > 0.f) {
    const float nv = a.n_valid ? (float)max(*a.n_valid, 1) : 1.f;
    return powf(fmaxf(nv * a.probs[b], 1e-30f), -a.beta);
  }
  return 1.f;
}

__global__ __launch_bounds__(256) void td_kernel(const TdArgs a) {
  __shared__ float red[8];
  __shared__ float wsh[256];
  __shared__ int sst[256];
  __shared__ int last;
  const int tid = threadIdx.x;
  if (tid < a.B) sst[tid] = a.starts[tid];
  // ---- IS weights w_b = (N * P_b)^-beta / max_b  (B <= 256; recomputed per workgroup)
  bool gn = false;
  const float w = tid < a.B ? is_weight(a, tid, &gn) : 1.f;
  float m = wave_max(tid < a.B ? w : 0.f);
  if ((tid & 63) == 0) red[tid >> 6] = m;
  __syncthreads();
  const float wmax = gn ? 1.f : fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
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
    if (a.priority && prio_owner(sst, a.B, a.Tl, a.burn_in, a.cap_e, tl, b, 0, 1))
      a.priority[row] = powf(ad + a.prio_eps, a.alpha);
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
                          float beta, float* part, unsigned* ticket, const float* dp,
                          void* stream) {
  if (B > 256) return -1;
  const int grid = (Tl * B + 255) / 256;
  if (grid > 4096) return -2;   // part[] holds one float per workgroup (engine: 4096)
  TdArgs a{q_sa, q_arg, q_tgt, starts, probs, action, reward, done, dq, loss, td_abs, priority,
           is_w, n_valid, part, ticket, Tl, B, A, burn_in, cap_e, gamma_n, vr_eps, alpha, prio_eps,
           beta, value_rescale, dp};
  hipLaunchKernelGGL(td_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, a);
  R2_CHECK_LAUNCH();
  return 0;
}

// ============================================================================================
// TD loss fused with the dueling-head backward (head.hip dueling_bwd_kernel): one WAVE per
// transition.  dL/dQ of a row is nonzero only at the taken action, so right where the TD error is
// known the wave also writes dva = [dV, dA_0..] and dz = relu'(z) * (dva . W2) for its row --
// the same arithmetic, in the same order, as dueling_bwd_kernel (bit-identical dz / dva), one
// launch instead of two (each ~9 us, most of it the launch floor of a graph node).
// The loss is reduced deterministically: per-workgroup partials (sc1), arrival ticket, the last
// workgroup sums the partials in a fixed order.
struct TdDuelArgs {
  TdArgs td;
  const void* zr;       // (Tl*B, 2*HD) relu'd hidden of the online head's learning rows (ZT)
  const float* w2;      // (1 + A, HD) second-layer weights [value row; advantage rows]
  bf16* dz;             // (Tl*B, 2*HD) out (hi plane in split precision)
  float* dva;           // (Tl*B, 1 + A) out
  bf16* dz_lo;          // split precision: lo plane of dz
  // optional fused head backward to the LSTM output: dh = dz @ W1 for the workgroup's 16 rows
  const bf16* w1t;      // (256, 2*HD) = W1^T (k contiguous); null = not fused
  const bf16* w1t_lo;   // split precision: lo plane of W1^T
  float* dh;            // (Tl*B, 256) out
  // optional fused head FORWARD (fixed / reference target modes, where the three Q rows of
  // transition i are row i of each head): zh = pre-bias layer-1 outputs (ZT) of the online,
  // online-on-next and target heads; the kernel forms relu(z + b1), the dueling Q rows (the
  // arithmetic of head.hip dueling_fwd_kernel, bit-identical), writes them to qo[] (optional) and
  // the online relu'd rows to zr (then an OUTPUT) -- one launch instead of dueling_fwd + td
  const void* zh[3];
  const float* b1[2];   // online, target
  const float* w2t;     // target second layer (1 + A, HD)
  const float* b2[2];   // online, target
  float* qo[3];
  int fuse_fwd;
  // optional stage stamps (r2_td_duel_set_trace): [workgroup][wave][12] s_memrealtime (100 MHz)
  long long* trace;
  // optional (r2_td_duel_set_done, the hoisted step's early fork): the row priorities go out
  // write-through and drained before the arrival ticket, and the last arriver stores 1 here --
  // the priority tail launched beside this kernel waits for it (replay.hip prio_tail_kernel)
  unsigned* done;
};

// head.hip dueling_fwd_kernel for one row on one wave (same order of operations, same
// wave_sum_x, so the Q rows agree bit for bit): returns the lane's Q (lane < A); hv / ha =
// relu(z + b1) of the lane's features.  z: the row's pre-bias layer-1 outputs (already in
// registers), b1 / w2 / b2: the net's head parameters staged in LDS -- second-layer rows up to
// MAXA there, further rows (many-action heads) from w2g in memory.  The 1 + A lane partials are
// formed first (their LDS / memory reads issued together), then reduced; amean accumulates in
// action order as in dueling_fwd_kernel.
template <int HD, typename ZT, int MAXA>
__device__ __forceinline__ float td_duel_row(const ZT (&z)[2 * (HD / 64)], const float* b1,
                                             const float* w2, const float* w2g, const float* b2,
                                             int A, int lane, float (&hv)[HD / 64],
                                             float (&ha)[HD / 64]) {
  constexpr int PER = HD / 64;
#pragma unroll
  for (int e = 0; e < PER; ++e) {
    const int c = lane * PER + e;
    hv[e] = fmaxf((float)z[e] + b1[c], 0.f);
    ha[e] = fmaxf((float)z[PER + e] + b1[HD + c], 0.f);
  }
  float part[1 + MAXA];
  part[0] = 0.f;
#pragma unroll
  for (int e = 0; e < PER; ++e) part[0] += hv[e] * w2[lane * PER + e];
#pragma unroll
  for (int a = 0; a < MAXA; ++a) {
    float s = 0.f;
    if (a < A) {
#pragma unroll
      for (int e = 0; e < PER; ++e) s += ha[e] * w2[(1 + a) * HD + lane * PER + e];
    }
    part[1 + a] = s;
  }
  float red[1 + MAXA];
#pragma unroll
  for (int a = 0; a <= MAXA; ++a) red[a] = (a <= A) ? wave_sum_x(part[a]) : 0.f;
  const float v = red[0] + b2[0];
  float amean = 0.f, mine = 0.f;
#pragma unroll
  for (int a = 0; a < MAXA; ++a) {
    if (a < A) {
      const float s = red[1 + a] + b2[1 + a];
      mine = (a == lane) ? s : mine;
      amean += s;
    }
  }
  for (int a = MAXA; a < A; ++a) {
    float s = 0.f;
#pragma unroll
    for (int e = 0; e < PER; ++e) s += ha[e] * w2g[(size_t)(1 + a) * HD + lane * PER + e];
    s = wave_sum_x(s) + b2[1 + a];
    mine = (a == lane) ? s : mine;
    amean += s;
  }
  amean /= (float)A;
  return v + mine - amean;
}

// SP: zr fp32, dz written as hi / lo planes (split.h).  Actions beyond the MAXA LDS-staged
// second-layer rows are read from memory inside the same loops (same order, same bits).
//
// Latency layout (one wave per transition, 16 per workgroup; the kernel is a chain of dependent
// round trips, not bandwidth): every independent load is issued at the top -- the wave's z rows of
// all three heads, the start -> row -> action / reward / done chain, the workgroup's cooperative
// staging of both nets' head parameters into LDS, the IS-weight maximum -- before ONE barrier;
// the wave re-derives its own sample's IS weight instead of a second barrier; the loss ticket is
// taken before the dh product so its round trip hides under the MFMAs; 8 W1^T fragments in flight.
template <int HD, bool SP>
__global__ __launch_bounds__(1024) void td_duel_kernel(const TdDuelArgs args) {
  constexpr int PER = HD / 64, MAXA = 8, NW = 16;
  constexpr int WROWS = (1 + MAXA) * HD;     // staged second-layer rows of one net
  const TdArgs& a = args.td;
  __shared__ int sst[256];
  __shared__ float wst[256];    // un-normalised IS weight of every sample (this launch's staging)
  __shared__ float red[NW];
  __shared__ float lred[NW];
  __shared__ float tot_sh[NW];
  __shared__ int last;
  __shared__ __attribute__((aligned(16))) float w2s[2][WROWS];
  __shared__ __attribute__((aligned(16))) float b1s[2][2 * HD];
  __shared__ float b2s[2][1 + HEAD_FWD_MAXA];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  long long* tr = (args.trace && lane == 0) ? args.trace + ((size_t)blockIdx.x * NW + wave) * 12 : nullptr;
#define TD_STAMP(k) if (tr) tr[k] = (long long)__builtin_amdgcn_s_memrealtime();
  TD_STAMP(0);
  const int n = a.Tl * a.B;
  const int i = blockIdx.x * NW + wave;      // this wave's transition
  const bool valid = i < n;
  const int b = valid ? i % a.B : 0, tl = valid ? i / a.B : 0;
  const int start = valid ? a.starts[b] : 0;
  const float NEG = -3.0e38f;
  typedef typename std::conditional<SP, float, bf16>::type ZT;
  const bool fwd = args.fuse_fwd != 0;
  // ---- the wave's rows: z of the three heads (fused forward) or the online relu'd row
  ZT zq[3][2 * PER];
#pragma unroll
  for (int h = 0; h < 3; ++h)
#pragma unroll
    for (int e = 0; e < 2 * PER; ++e) zq[h][e] = (ZT)0.f;
  float qa = NEG, qt = 0.f, qs = 0.f;
  if (valid) {
    if (fwd) {
#pragma unroll
      for (int h = 0; h < 3; ++h) {
        const ZT* zrow = (const ZT*)args.zh[h] + (size_t)i * 2 * HD;
#pragma unroll
        for (int e = 0; e < PER; ++e) {
          zq[h][e] = zrow[lane * PER + e];
          zq[h][PER + e] = zrow[HD + lane * PER + e];
        }
      }
    } else {
      const ZT* zrow = (const ZT*)args.zr + (size_t)i * 2 * HD;
#pragma unroll
      for (int e = 0; e < PER; ++e) {
        zq[0][e] = zrow[lane * PER + e];
        zq[0][PER + e] = zrow[HD + lane * PER + e];
      }
      if (lane < a.A) {
        qa = a.q_arg[(size_t)i * a.A + lane];
        qt = a.q_tgt[(size_t)i * a.A + lane];
        qs = a.q_sa[(size_t)i * a.A + lane];
      }
    }
  }
  const int row = valid ? ring_row(start, a.burn_in + tl, a.cap_e) : 0;
  const int act = valid ? (int)a.action[row] : 0;
  const float rew = valid ? a.reward[row] : 0.f;
  const bool dn = valid ? a.done[row] != 0 : true;
  // ---- workgroup staging: second-layer rows 0..min(A, MAXA) of the online (and target) head,
  // b1 / b2 of both nets (forward fusion), the B starts; IS-weight maxima per wave
  {
    const int rows = 1 + min(a.A, MAXA);
    const int nets = fwd ? 2 : 1;
    for (int q = tid; q < nets * rows * (HD / 4); q += NW * 64) {
      const int net = q / (rows * (HD / 4)), r = q - net * rows * (HD / 4);
      const float* src = net ? args.w2t : args.w2;
      *(f32x4*)&w2s[net][4 * r] = *(const f32x4*)(src + 4 * r);
    }
    if (fwd) {
      for (int q = tid; q < 2 * (2 * HD / 4); q += NW * 64) {
        const int net = q / (2 * HD / 4), r = q - net * (2 * HD / 4);
        *(f32x4*)&b1s[net][4 * r] = *(const f32x4*)(args.b1[net] + 4 * r);
      }
      if (tid < 2 * (1 + a.A)) {
        const int net = tid / (1 + a.A), r = tid - net * (1 + a.A);
        b2s[net][r] = args.b2[net][r];
      }
    }
  }
  if (tid < a.B) sst[tid] = a.starts[tid];
  bool gn = false;
  const float w_t = tid < a.B ? is_weight(a, tid, &gn) : 1.f;
  if (tid < a.B) wst[tid] = w_t;
  const float m = wave_max(tid < a.B ? w_t : 0.f);
  if (lane == 0) red[wave] = m;
  TD_STAMP(1);
  __syncthreads();
  float wmax = red[0];
#pragma unroll
  for (int q = 1; q < NW; ++q) wmax = fmaxf(wmax, red[q]);
  if (gn) wmax = 1.f;
  if (tid < a.B && a.is_w && blockIdx.x == 0) a.is_w[tid] = w_t / wmax;
  TD_STAMP(2);

  // ---- the three heads' dueling forward for row i (online, online-on-next, target)
  ZT zv[PER], za[PER];
#pragma unroll
  for (int e = 0; e < PER; ++e) { zv[e] = zq[0][e]; za[e] = zq[0][PER + e]; }
  if (fwd) {
    float hv[PER], ha[PER];
    qs = qa = qt = 0.f;
    if (valid) {
#pragma unroll
      for (int h = 0; h < 3; ++h) {
        const int net = h == 2;
        const float q = td_duel_row<HD, ZT, MAXA>(zq[h], b1s[net], w2s[net], net ? args.w2t : args.w2,
                                                  b2s[net], a.A, lane, hv, ha);
        if (args.qo[h] && lane < a.A) args.qo[h][(size_t)i * a.A + lane] = q;
        if (h == 0) {
          qs = q;
          ZT* zo = (ZT*)args.zr + (size_t)i * 2 * HD;
#pragma unroll
          for (int e = 0; e < PER; ++e) {
            zv[e] = (ZT)hv[e];
            za[e] = (ZT)ha[e];
            zo[lane * PER + e] = zv[e];
            zo[HD + lane * PER + e] = za[e];
          }
        } else if (h == 1) {
          qa = q;
        } else {
          qt = q;
        }
      }
    }
    if (!(valid && lane < a.A)) { qa = NEG; qt = 0.f; qs = 0.f; }
  }
  TD_STAMP(8);

  const float inv_n = 1.f / (float)n;
  float lsum = 0.f;
  float dz_v[PER], dz_a[PER];   // pre-mask dz of this row (value / advantage halves) for the fused dh
#pragma unroll
  for (int e = 0; e < PER; ++e) { dz_v[e] = 0.f; dz_a[e] = 0.f; }
  if (valid) {
    // argmax_a Q_online(s_{t+n}): first maximum, as td_kernel's sequential scan -- the wave max
    // (DPP), then the lowest lane holding it (ballot); best / act are wave-uniform, so the lane
    // reads are v_readlane, not LDS permutes
    const float bv = wave_max_x(qa);
    const unsigned long long hit = __ballot(lane < a.A && qa == bv);
    const int best = hit ? __ffsll((long long)hit) - 1 : 0;
    float boot = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(qt), best));
    if (a.value_rescale) boot = vr_hinv(boot, a.vr_eps);
    float y = rew + (dn ? 0.f : a.gamma_n * boot);
    if (a.value_rescale) y = vr_h(y, a.vr_eps);
    const float delta = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(qs), act)) - y;
    const float wb = wst[b] / wmax;          // == td_kernel's staged w / wmax of sample b
    const float g = wb * delta * inv_n;      // dL/dQ[act]; every other action 0
    // the wave checks the B starts 64 at a time for a later duplicate of this row
    const bool own = a.priority ? __all(prio_owner(sst, a.B, a.Tl, a.burn_in, a.cap_e, tl, b, lane, 64))
                                : false;
    if (lane == 0) {
      lsum = wb * 0.5f * delta * delta;
      const float ad = fabsf(delta);
      if (a.td_abs) a.td_abs[i] = ad;
      if (own) {
        const float pv = powf(ad + a.prio_eps, a.alpha);
        if (args.done) __hip_atomic_store(a.priority + row, pv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else a.priority[row] = pv;
      }
    }
    if (lane < a.A) a.dq[(size_t)i * a.A + lane] = lane == act ? g : 0.f;
    TD_STAMP(9);
    // dueling backward of row i (dueling_bwd_kernel's arithmetic on dq = g e_act)
    float dv = 0.f;
    for (int k = 0; k < a.A; ++k) dv += (k == act) ? g : 0.f;
    const float dmean = dv / (float)a.A;
    float* dvr = args.dva + (size_t)i * (1 + a.A);
    if (lane == 0) dvr[0] = dv;
    if (lane < a.A) dvr[1 + lane] = ((lane == act) ? g : 0.f) - dmean;
    bf16* dzrow = args.dz + (size_t)i * 2 * HD;
    float ov[PER], oa[PER];
#pragma unroll
    for (int e = 0; e < PER; ++e) {
      const float gv = dv * w2s[0][lane * PER + e];
      float ga = 0.f;
#pragma unroll
      for (int k = 0; k < MAXA; ++k)
        if (k < a.A) ga += (((k == act) ? g : 0.f) - dmean) * w2s[0][(1 + k) * HD + lane * PER + e];
      for (int k = MAXA; k < a.A; ++k)     // many-action heads (Seaquest 18, DMLab 15)
        ga += (((k == act) ? g : 0.f) - dmean) * args.w2[(size_t)(1 + k) * HD + lane * PER + e];
      ov[e] = ((float)zv[e] > 0.f) ? gv : 0.f;
      oa[e] = ((float)za[e] > 0.f) ? ga : 0.f;
      dz_v[e] = gv;
      dz_a[e] = ga;
    }
#pragma unroll
    for (int e = 0; e < PER; ++e) {
      dzrow[lane * PER + e] = (bf16)ov[e];
      dzrow[HD + lane * PER + e] = (bf16)oa[e];
      if constexpr (SP) {
        bf16* dzl = args.dz_lo + (size_t)i * 2 * HD;
        dzl[lane * PER + e] = sp_lo(ov[e]);
        dzl[HD + lane * PER + e] = sp_lo(oa[e]);
      }
    }
  }
  TD_STAMP(3);
  // ---- fused dh = dz @ W1 of the 16 rows (dz staged in LDS; wave w owns dh columns 16w..16w+15,
  // K = 2HD on v_mfma_f32_16x16x32_bf16, W1^T fragments from L2; 3 passes in split precision).
  // K order: step s covers k = 32 s + 8 kq + [0, 8) for lane group kq -- the dh GEMM's own order,
  // so dh is bit-identical to the separate launch (tests/test_engine_gpu.py)
  constexpr int KD = 2 * HD, DZS = KD + 8;             // padded LDS rows
  constexpr int KS = KD / 32, D = SP ? 8 : 4;         // W1^T fragments in flight
  __shared__ __attribute__((aligned(16))) bf16 dzs[SP ? 2 : 1][NW * DZS];
  const int r16 = lane & 15, kq = lane >> 4;
  auto koff = [&](int s) { return 32 * s + 8 * kq; };
  bf16x8 rb[D], rbl[D];
  const bf16* bt = args.w1t ? args.w1t + (size_t)(wave * 16 + r16) * KD : nullptr;
  const bf16* btl = (SP && args.w1t) ? args.w1t_lo + (size_t)(wave * 16 + r16) * KD : nullptr;
  if (args.w1t) {
    // the first W1^T fragments are independent of this launch's results: in flight across the
    // staging barrier
#pragma unroll
    for (int s = 0; s < D; ++s) {
      rb[s] = *(const bf16x8*)(bt + koff(s));
      if constexpr (SP) rbl[s] = *(const bf16x8*)(btl + koff(s));
    }
#pragma unroll
    for (int e = 0; e < PER; ++e) {
      const float v0 = valid ? ((float)zv[e] > 0.f ? dz_v[e] : 0.f) : 0.f;
      const float v1 = valid ? ((float)za[e] > 0.f ? dz_a[e] : 0.f) : 0.f;
      dzs[0][wave * DZS + lane * PER + e] = (bf16)v0;
      dzs[0][wave * DZS + HD + lane * PER + e] = (bf16)v1;
      if constexpr (SP) {
        dzs[SP ? 1 : 0][wave * DZS + lane * PER + e] = sp_lo(v0);
        dzs[SP ? 1 : 0][wave * DZS + HD + lane * PER + e] = sp_lo(v1);
      }
    }
  }
  // ---- loss: wave partial (lane 0) -> workgroup partial -> arrival ticket (before dh: the
  // atomic's round trip overlaps the product) -> the last arriver sums in workgroup order
  if (lane == 0) lred[wave] = lsum;
  if (args.done) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // priorities performed
  __syncthreads();
  TD_STAMP(4);
  unsigned tk = 0;
  if (tid == 0) {
    float v = 0.f;
#pragma unroll
    for (int q = 0; q < NW; ++q) v += lred[q];
    __hip_atomic_store(a.part + blockIdx.x, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // sc1
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    tk = __hip_atomic_fetch_add(a.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (args.w1t) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const bf16x8 b0 = rb[s % D];
      bf16x8 b1;
      if constexpr (SP) b1 = rbl[s % D];
      if (s + D < KS) {
        rb[s % D] = *(const bf16x8*)(bt + koff(s + D));
        if constexpr (SP) rbl[s % D] = *(const bf16x8*)(btl + koff(s + D));
      }
      const bf16x8 a0 = *(const bf16x8*)(&dzs[0][r16 * DZS + koff(s)]);
      if constexpr (SP) {
        const bf16x8 a1 = *(const bf16x8*)(&dzs[SP ? 1 : 0][r16 * DZS + koff(s)]);
        acc = mfma16_x3(a0, a1, b0, b1, acc);
      } else {
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b0, acc, 0, 0, 0);
      }
    }
    // acc[e] = dh[row 4 kq + e of the workgroup][column 16 wave + r16]
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int ri = blockIdx.x * NW + 4 * kq + e;
      if (ri < n) args.dh[(size_t)ri * 256 + wave * 16 + r16] = acc[e];
    }
  }
  TD_STAMP(5);
  if (tid == 0) last = tk == gridDim.x - 1;
  __syncthreads();
  TD_STAMP(6);
  if (!last) return;
  if (args.done && tid == 0) __hip_atomic_store(args.done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  float s = 0.f;
  for (unsigned g = tid; g < gridDim.x; g += NW * 64)
    s += __hip_atomic_load(a.part + g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  s = wave_sum(s);
  if (lane == 0) tot_sh[wave] = s;
  __syncthreads();
  if (tid == 0) {
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < NW; ++q) t += tot_sh[q];
    *a.loss = t * inv_n;
    __hip_atomic_store(a.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  TD_STAMP(7);
#undef TD_STAMP
}

template <bool SP>
static int td_duel_launch(const TdDuelArgs& d, int HD, int grid, hipStream_t s) {
  switch (HD) {
    case 64: hipLaunchKernelGGL((td_duel_kernel<64, SP>), dim3(grid), dim3(1024), 0, s, d); break;
    case 128: hipLaunchKernelGGL((td_duel_kernel<128, SP>), dim3(grid), dim3(1024), 0, s, d); break;
    case 256: hipLaunchKernelGGL((td_duel_kernel<256, SP>), dim3(grid), dim3(1024), 0, s, d); break;
    case 512: hipLaunchKernelGGL((td_duel_kernel<512, SP>), dim3(grid), dim3(1024), 0, s, d); break;
    default: return -4;
  }
  R2_CHECK_LAUNCH();
  return 0;
}

extern "C" int r2_td_duel_dh(const float*, const float*, const float*, const int*, const float*,
                             const uint8_t*, const float*, const uint8_t*, float*, float*, float*,
                             float*, float*, const int*, int, int, int, int, int, float, int, float,
                             float, float, float, float*, unsigned*, const void*, const float*,
                             bf16*, float*, int, bf16*, const float*, const bf16*, const bf16*,
                             float*, int, void*);

// Head-forward operands of the fused launch (r2_td_duel_fwd_set, consumed by the next
// r2_td_duel_dh call on this host thread): 12 int64 {z_on, z_nx, z_tg, b1_on, b1_tg, w2_tg,
// b2_on, b2_tg, q_on, q_nx, q_tg (q outs may be 0)} -- zr of r2_td_duel_dh becomes an output.
static thread_local int64_t g_td_fwd[12];
static thread_local bool g_td_fwd_on = false;
// Stage-stamp buffer of the next eager launches on this host thread (tools/td_micro.py).  A
// launch being captured into a graph never takes it (r2_td_duel_dh): the graph would keep
// writing stamps into the buffer after it is cleared or freed.
static thread_local long long* g_td_trace = nullptr;
extern "C" int r2_td_duel_set_trace(long long* tr) {
  g_td_trace = tr;
  return 0;
}
// done flag of the NEXT r2_td_duel_dh launch on this host thread (consumed by it; TdDuelArgs::done)
static thread_local unsigned* g_td_done = nullptr;
extern "C" int r2_td_duel_set_done(unsigned* done) {
  g_td_done = done;
  return 0;
}
extern "C" int r2_td_duel_fwd_set(const int64_t* fwd) {
  g_td_fwd_on = fwd != nullptr;
  if (fwd)
    for (int k = 0; k < 11; ++k) g_td_fwd[k] = fwd[k];
  return 0;
}

// zr: bf16 (dz_lo null) or fp32 (split precision: dz_lo = the lo plane of dz)
extern "C" int r2_td_duel(const float* q_sa, const float* q_arg, const float* q_tgt,
                          const int* starts, const float* probs, const uint8_t* action,
                          const float* reward, const uint8_t* done, float* dq, float* loss,
                          float* td_abs, float* priority, float* is_w, const int* n_valid,
                          int Tl, int B, int A, int burn_in, int cap_e, float gamma_n,
                          int value_rescale, float vr_eps, float alpha, float prio_eps,
                          float beta, float* part, unsigned* ticket, const void* zr,
                          const float* w2, bf16* dz, float* dva, int HD, bf16* dz_lo,
                          const float* dp, void* stream) {
  return r2_td_duel_dh(q_sa, q_arg, q_tgt, starts, probs, action, reward, done, dq, loss, td_abs,
                       priority, is_w, n_valid, Tl, B, A, burn_in, cap_e, gamma_n, value_rescale,
                       vr_eps, alpha, prio_eps, beta, part, ticket, zr, w2, dz, dva, HD, dz_lo, dp,
                       nullptr, nullptr, nullptr, 0, stream);
}

// + the fused head backward to the LSTM output: dh (Tl*B, H) = dz @ W1 from W1^T (H, 2HD) (and its
// lo plane in split precision).  H must be 256 (16 waves x 16 columns); w1t = null: not fused.
extern "C" int r2_td_duel_dh(const float* q_sa, const float* q_arg, const float* q_tgt,
                             const int* starts, const float* probs, const uint8_t* action,
                             const float* reward, const uint8_t* done, float* dq, float* loss,
                             float* td_abs, float* priority, float* is_w, const int* n_valid,
                             int Tl, int B, int A, int burn_in, int cap_e, float gamma_n,
                             int value_rescale, float vr_eps, float alpha, float prio_eps,
                             float beta, float* part, unsigned* ticket, const void* zr,
                             const float* w2, bf16* dz, float* dva, int HD, bf16* dz_lo,
                             const float* dp, const bf16* w1t, const bf16* w1t_lo, float* dh, int H,
                             void* stream) {
  unsigned* const td_done = g_td_done;
  g_td_done = nullptr;
  if (B > 256) return -1;
  if (A < 1 || A > 64) return -3;             // one lane per action
  const int grid = (Tl * B + 15) / 16;
  if (grid > 4096) return -2;   // part[] holds one float per workgroup (engine: 4096)
  if (w1t && (H != 256 || !dh || (dz_lo && !w1t_lo) || (2 * HD) % 32)) return -5;
  TdDuelArgs d{{q_sa, q_arg, q_tgt, starts, probs, action, reward, done, dq, loss, td_abs, priority,
                is_w, n_valid, part, ticket, Tl, B, A, burn_in, cap_e, gamma_n, vr_eps, alpha,
                prio_eps, beta, value_rescale, dp},
               zr, w2, dz, dva, dz_lo, w1t, w1t_lo, dh};
  d.fuse_fwd = 0;
  d.done = td_done;
  if (td_done && !priority) return -8;
  {   // never bake a stamp buffer into a captured launch
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    const bool cap = hipStreamIsCapturing((hipStream_t)stream, &st) == hipSuccess &&
                     st != hipStreamCaptureStatusNone;
    d.trace = cap ? nullptr : g_td_trace;
  }
  if (g_td_fwd_on) {
    g_td_fwd_on = false;   // one launch per set
    if (A > HEAD_FWD_MAXA) return -6;
    for (int k = 0; k < 3; ++k) d.zh[k] = (const void*)g_td_fwd[k];
    d.b1[0] = (const float*)g_td_fwd[3]; d.b1[1] = (const float*)g_td_fwd[4];
    d.w2t = (const float*)g_td_fwd[5];
    d.b2[0] = (const float*)g_td_fwd[6]; d.b2[1] = (const float*)g_td_fwd[7];
    for (int k = 0; k < 3; ++k) d.qo[k] = (float*)g_td_fwd[8 + k];
    if (!d.zh[0] || !d.zh[1] || !d.zh[2] || !d.b1[0] || !d.b1[1] || !d.w2t || !d.b2[0] || !d.b2[1])
      return -7;
    d.fuse_fwd = 1;
  }
  hipStream_t s = (hipStream_t)stream;
  return dz_lo ? td_duel_launch<true>(d, HD, grid, s) : td_duel_launch<false>(d, HD, grid, s);
}
