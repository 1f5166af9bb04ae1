// Batched GPU actor: the per-env-step bookkeeping of an actor group fused into three launches
// around the environment step (pytorch_r2d2_amd/actor_batched.py).
//
// Replaces, for E envs at once, what the reference does per actor process on the host with
// numpy and Python deques: replay row writes (replay_memory.py:93-123 `add`), the n-step return
// builder (replay_memory.py:12-55 NStepMemory), the double-Q initial priority
// (actor.py:144-157 calc_priority), epsilon-greedy action selection (actor.py:96-106), episode
// end flush + sequence segmentation (actor.py:108-135, :159-167) and the LSTM state reset.
// Earlier this was ~450 small PyTorch kernels per env step (1.2 ms at E = 256, launch-bound);
// here every env is one workgroup and the whole step is a handful of launches.
//
//   actor_pre_kernel   (grid E): invalidate the rows about to be overwritten (and, on a sub-ring
//                      wrap, the old windows reaching into them), copy the observation into
//                      the replay row, store both nets' recurrent state, finalise the
//                      transition of step t-n (n-step return, bootstrap Q_tgt(s_t, argmax Q)),
//                      pick the epsilon-greedy action (counter-based hash RNG).
//   <environment step on the device>
//   actor_post_kernel  (grid E): push this step into the n-step history, mark the start whose
//                      window just completed, on episode end flush every pending transition
//                      (truncated return, done = 1) and mark the final starts, write the
//                      finished return into the return ring, reset / advance the LSTM state.
//   mark_starts_kernel + tree update (replay.hip), then
//   actor_tail_kernel  (1 thread): t += 1, head = (head + 1) % cap_e, return count, dirty reset.
//
// Deferred mode (defer_D > 0; the concurrent actor / learner topology, engine/concurrent.py): the
// actor never touches the sequence-start flags, the sum tree, n_valid or the dirty list -- the
// learner reads those while it runs on other CUs.  Instead every start it would clear or mark is
// appended to a pending list (mark: row >= 0; clear: -2 - row) that the learner's stream applies
// between its steps (replay.hip apply_pending_kernel).  Rows are invalidated defer_D steps AHEAD
// of the write head, so by the time a row is overwritten every learner step that could have
// sampled a sequence through it has finished.
#include "../common.h"

struct ActArgs {
  // replay (HBMReplay)
  uint8_t* frames;            // (cap, FB)
  const uint8_t* obs;         // (E, FB) current observations
  float* hs_cs;               // (cap, 2H) online stored state
  float* ths_cs;              // (cap, 2H) target stored state
  uint8_t* action;            // (cap)
  float* reward;              // (cap)
  uint8_t* done;              // (cap)
  float* priority;            // (cap)
  uint8_t* is_start;          // (cap)
  float* leaves;              // (cap) sum-tree leaves
  int* n_valid;
  int* dirty;
  int* dcount;
  // actor state
  const float* q_on;          // (E, A)
  const float* q_tg;          // (E, A)
  const float* st_h[2];       // (E, H) fp32 state stored with this step's row (pre or post)
  const float* st_c[2];
  const float* h_new[2];      // (E, H) next state from the LSTM step
  const float* c_new[2];
  float* h32[2];              // (E, H) carried state (reset on done)
  float* c[2];
  bf16* h_bf[2];
  int64_t* h_row;             // (n, E) n-step history
  float* h_q;                 // (n, E, A)
  int64_t* h_a;               // (n, E)
  float* h_r;                 // (n, E)
  int64_t* h_step;            // (n, E)
  uint8_t* h_valid;           // (n, E)
  int64_t* ep_start;          // (E)
  int64_t* t;                 // (1) actor step
  int64_t* head;              // (1) common sub-ring write position
  const float* eps;           // (E) epsilon ladder
  int64_t* act;               // (E) chosen actions (env input)
  const float* env_reward;    // (E)
  const uint8_t* env_done;    // (E) bool
  const float* env_finished;  // (E)
  float* ret_ring;            // (R)
  int64_t* ret_cnt;           // (1)
  int* ret_env;               // (R) env of each ring return (per-epsilon return statistics)
  int* marks;                 // (E * (n + 2)) start rows to mark, -1 = none
  int* pend;                  // deferred mode: pending start edits (mark row | clear -2-row)
  int* pend_cnt;              // (1) entries appended (reset by the learner's apply)
  long long FB;
  unsigned long long seed;
  int E, A, H, n, T, stride, cap_e, W, wrap, max_dirty, R, value_rescale;
  int pend_cap, defer_D;      // defer_D > 0: deferred mode, invalidate defer_D rows ahead
  float gamma, gamma_n, prio_eps, alpha, vr_eps;
};

__device__ __forceinline__ long long pymod(long long a, long long m) {
  long long r = a % m;
  return r < 0 ? r + m : r;
}

__device__ __forceinline__ float vr_h(float x, float e) {
  return copysignf(sqrtf(fabsf(x) + 1.f) - 1.f, x) * (x != 0.f) + e * x;
}
__device__ __forceinline__ float vr_hinv(float x, float e) {
  const float s = (sqrtf(1.f + 4.f * e * (fabsf(x) + 1.f + e)) - 1.f) / (2.f * e);
  return ((x > 0.f) - (x < 0.f)) * (s * s - 1.f);
}

__device__ __forceinline__ float init_prio(const ActArgs& a, float q_sel, float y) {
  return powf(fabsf(q_sel - y) + a.prio_eps, a.alpha);
}

// sum_k gamma^(s_k - from) r_k over the buffered steps s_k in [from, upto] of env e
__device__ __forceinline__ float returns_from(const ActArgs& a, int e, long long from, long long upto) {
  float R = 0.f;
  for (int j = 0; j < a.n; ++j) {
    const long long st = a.h_step[(size_t)j * a.E + e];
    if (st >= from && st <= upto && st >= 0) R += a.h_r[(size_t)j * a.E + e] * powf(a.gamma, (float)(st - from));
  }
  return R;
}

__device__ __forceinline__ int argmax_row(const float* q, int A) {
  int best = 0;
  float bv = q[0];
  for (int i = 1; i < A; ++i)
    if (q[i] > bv) { bv = q[i]; best = i; }
  return best;
}

__device__ __forceinline__ void clear_row(const ActArgs& a, long long r) {
  if (a.is_start[r] || a.leaves[r] != 0.f) {
    if (a.is_start[r]) atomicSub(a.n_valid, 1);
    a.is_start[r] = 0;
    a.leaves[r] = 0.f;
    const int slot = atomicAdd(a.dcount, 1);
    if (slot < a.max_dirty) a.dirty[slot] = (int)r;
  }
}

__device__ __forceinline__ void pend_push(const ActArgs& a, int v) {
  const int slot = atomicAdd(a.pend_cnt, 1);
  if (slot < a.pend_cap) a.pend[slot] = v;      // overflow is detected by the apply kernel
}

__global__ __launch_bounds__(256) void actor_pre_kernel(const ActArgs a) {
  const int e = blockIdx.x, tid = threadIdx.x;
  const long long t = *a.t, head = *a.head;
  const long long base = (long long)e * a.cap_e, row = base + head;
  // 1. rows about to be overwritten stop being sequence starts (deferred: defer_D rows ahead)
  if (a.defer_D > 0) {
    // no wrap clears here: the D-ahead clears already invalidated rows cap_e-W+1 .. cap_e-1
    // before this step, and a clear queued now would share the pending list with this step's
    // start mark at head-W+1 (the apply kernel runs its entries in no fixed order)
    if (tid == 0) pend_push(a, -2 - (int)(base + (head + a.defer_D) % a.cap_e));
  } else {
    if (tid == 0) clear_row(a, row);
    if (a.wrap)
      for (int i = tid; i < a.W - 1; i += blockDim.x) clear_row(a, base + a.cap_e - a.W + 1 + i);
  }
  // 2. observation -> replay row (16-byte vectors when aligned)
  {
    const uint8_t* src = a.obs + (size_t)e * a.FB;
    uint8_t* dst = a.frames + (size_t)row * a.FB;
    if ((a.FB & 15) == 0) {
      const long long nv = a.FB >> 4;
      for (long long i = tid; i < nv; i += blockDim.x)
        reinterpret_cast<u32x4*>(dst)[i] = reinterpret_cast<const u32x4*>(src)[i];
    } else {
      for (long long i = tid; i < a.FB; i += blockDim.x) dst[i] = src[i];
    }
  }
  // 3. stored recurrent state of both nets: [h | c]
  for (int k = 0; k < 2; ++k) {
    float* dst = (k ? a.ths_cs : a.hs_cs) + (size_t)row * 2 * a.H;
    for (int i = tid; i < a.H; i += blockDim.x) {
      dst[i] = a.st_h[k][(size_t)e * a.H + i];
      dst[a.H + i] = a.st_c[k][(size_t)e * a.H + i];
    }
  }
  if (tid != 0) return;
  // 4. finalise the transition of step t-n: its n rewards are known, bootstrap from Q(s_t)
  const int slot = (int)pymod(t, a.n);
  const size_t hs = (size_t)slot * a.E + e;
  const float* qo = a.q_on + (size_t)e * a.A;
  const int greedy = argmax_row(qo, a.A);
  if (a.h_valid[hs]) {
    const float boot = a.q_tg[(size_t)e * a.A + greedy];
    const float R = returns_from(a, e, a.h_step[hs], t - 1);
    const float y = a.value_rescale ? vr_h(R + a.gamma_n * vr_hinv(boot, a.vr_eps), a.vr_eps)
                                    : R + a.gamma_n * boot;
    const float q_sel = a.h_q[hs * a.A + a.h_a[hs]];
    const long long r = a.h_row[hs];
    a.reward[r] = R;
    a.done[r] = 0;
    a.priority[r] = init_prio(a, q_sel, y);
  }
  a.h_valid[hs] = 0;
  // 5. epsilon-greedy over the per-env ladder (counter-based RNG: seed, step, env)
  const float u = r2_uniform(a.seed, (uint64_t)t, 2 * (uint64_t)e);
  const int ra = min((int)(r2_uniform(a.seed, (uint64_t)t, 2 * (uint64_t)e + 1) * a.A), a.A - 1);
  const int act = u < a.eps[e] ? ra : greedy;
  a.act[e] = act;
  a.action[row] = (uint8_t)act;
}

__global__ __launch_bounds__(256) void actor_post_kernel(const ActArgs a) {
  const int e = blockIdx.x, tid = threadIdx.x, E = a.E, n = a.n;
  const long long t = *a.t, head = *a.head;
  const long long base = (long long)e * a.cap_e, row = base + head;
  const bool dn = a.env_done[e] != 0;
  const long long ep0 = a.ep_start[e];
  // recurrent state advances; an episode that ended restarts from zero state
  for (int k = 0; k < 2; ++k)
    for (int i = tid; i < a.H; i += blockDim.x) {
      const size_t o = (size_t)e * a.H + i;
      const float h = dn ? 0.f : a.h_new[k][o];
      a.h32[k][o] = h;
      a.c[k][o] = dn ? 0.f : a.c_new[k][o];
      a.h_bf[k][o] = (bf16)h;
    }
  // finished return -> ring slot (count of done envs before e: deterministic order)
  if (dn) {
    int before = 0;
    for (int j = tid; j < e; j += blockDim.x) before += a.env_done[j] != 0;
    before = (int)wave_sum((float)before);   // blockDim == 64
    if (tid == 0) {
      const long long slot = pymod(*a.ret_cnt + before, a.R);
      a.ret_ring[slot] = a.env_finished[e];
      a.ret_env[slot] = e;
    }
  }
  if (tid != 0) return;
  // this step enters the n-step history
  const int slot = (int)pymod(t, n);
  const size_t hs = (size_t)slot * E + e;
  a.h_row[hs] = row;
  for (int i = 0; i < a.A; ++i) a.h_q[hs * a.A + i] = a.q_on[(size_t)e * a.A + i];
  a.h_a[hs] = a.act[e];
  a.h_r[hs] = a.env_reward[e];
  a.h_step[hs] = t;
  a.h_valid[hs] = 1;
  // the start whose window became complete (rows finalised through t-n)
  {
    const long long o = (t - n) - ep0 - a.T + 1;
    const bool ok = o >= 0 && o % a.stride == 0;
    const int m = ok ? (int)(base + pymod(head - (t - ep0) + o, a.cap_e)) : -1;
    if (a.defer_D > 0) {
      if (m >= 0) pend_push(a, m);
    } else {
      a.marks[e] = m;
    }
  }
  // episode end: every pending transition gets its truncated return, done = 1 (no bootstrap);
  // starts whose windows end inside the just-finalised tail, plus the final start L - T
  for (int j = 0; j < n; ++j) {
    const size_t hj = (size_t)j * E + e;
    if (dn && a.h_valid[hj]) {
      const float R = returns_from(a, e, a.h_step[hj], t);
      const float y = a.value_rescale ? vr_h(R, a.vr_eps) : R;
      const long long r = a.h_row[hj];
      a.reward[r] = R;
      a.done[r] = 1;
      a.priority[r] = init_prio(a, a.h_q[hj * a.A + a.h_a[hj]], y);
      a.h_valid[hj] = 0;
    }
  }
  const long long L = (t - ep0) + 1, prev_newest = (t - n) - ep0;
  for (int jj = 0; jj <= n; ++jj) {
    const long long o = L - a.T - jj;
    const bool ok = dn && o >= 0 && o > prev_newest - a.T + 1 && (o % a.stride == 0 || jj == 0);
    const int m = ok ? (int)(base + pymod(head - (t - ep0) + o, a.cap_e)) : -1;
    if (a.defer_D > 0) {
      if (m >= 0) pend_push(a, m);
    } else {
      a.marks[(size_t)(1 + jj) * E + e] = m;
    }
  }
  if (dn) a.ep_start[e] = t + 1;
}

__global__ void actor_tail_kernel(int64_t* t, int64_t* head, int cap_e, const uint8_t* env_done,
                                  int E, int64_t* ret_cnt, int* dcount) {
  if (threadIdx.x != 0) return;
  int nd = 0;
  for (int e = 0; e < E; ++e) nd += env_done[e] != 0;
  *ret_cnt += nd;
  *t += 1;
  *head = (*head + 1) % cap_e;
  if (dcount) *dcount = 0;
}

static bool act_args_ok(const ActArgs& a) {
  return a.E > 0 && a.A > 0 && a.A <= 64 && a.H > 0 && a.n > 0 && a.T > 0 && a.stride > 0 &&
         a.cap_e > a.W && a.R > 0 && a.FB >= 0 &&
         (a.defer_D <= 0 || (a.pend && a.pend_cnt && a.pend_cap > 0 && a.cap_e > a.defer_D + a.W));
}

extern "C" int r2_actor_pre(const ActArgs* a, void* stream) {
  if (!act_args_ok(*a)) return -1;
  hipLaunchKernelGGL(actor_pre_kernel, dim3(a->E), dim3(256), 0, (hipStream_t)stream, *a);
  R2_CHECK_LAUNCH();
  return 0;
}

extern "C" int r2_actor_post(const ActArgs* a, void* stream) {
  if (!act_args_ok(*a)) return -1;
  hipLaunchKernelGGL(actor_post_kernel, dim3(a->E), dim3(64), 0, (hipStream_t)stream, *a);
  R2_CHECK_LAUNCH();
  return 0;
}

extern "C" int r2_actor_tail(const ActArgs* a, void* stream) {
  hipLaunchKernelGGL(actor_tail_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, a->t, a->head,
                     a->cap_e, a->env_done, a->E, a->ret_cnt, a->defer_D > 0 ? nullptr : a->dcount);
  R2_CHECK_LAUNCH();
  return 0;
}

extern "C" int r2_actor_args_bytes() { return (int)sizeof(ActArgs); }
