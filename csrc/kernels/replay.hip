// HBM-resident prioritized sequence replay kernels (gfx950).
//
// Reference: replay_memory.py:58-262 keeps the replay in host numpy, samples with
// WeightedRandomSampler -> torch.multinomial on CPU after an O(capacity) scan of is_seq_start
// (replay_memory.py:225-232), builds batches with 2*T*B Python get_stacked_state calls and
// ships ~36 MB H2D per step (replay_memory.py:236-260).  Here:
//
//  * the ring lives in HBM and is split into `n_sub` contiguous sub-rings (one per actor env)
//    so every episode is contiguous; row(start, t) wraps inside the start's sub-ring;
//  * sequence sampling weights sit in a 64-ary sum tree whose leaf level IS the per-row
//    `sequence_priority` array (0 where no sequence starts).  A 64-ary tree is 4 levels for
//    16M rows: one wave per sample reads 64 children with one coalesced load per level and
//    finds the child with a wave prefix-scan -- O(B log64 N), no host involvement;
//  * priority refresh after a train step recomputes the eta-mix of EVERY sequence whose
//    window overlaps an updated row (fixes Q8/Q9: replay_memory.py:204-213 refreshes idx-i
//    instead of idx+i and ignores ring wraparound at :186-188), appends the changed leaves to
//    a dirty list, and the tree is repaired bottom-up one level per launch (parents are
//    recomputed from children -- deterministic, no float drift, duplicates are benign).
#include "../common.h"
#include "../pack_step.h"

#define TREE_MAX_LEVELS 8

struct TreeGeom {
  int64_t off[TREE_MAX_LEVELS];
  int64_t size[TREE_MAX_LEVELS];
  int levels;
};

__device__ __forceinline__ int ring_row_s(int start, int t, int cap_e) {
  const int base = start - start % cap_e;
  int r = (start - base + t) % cap_e;
  if (r < 0) r += cap_e;
  return base + r;
}

// inclusive wave scan on the VALU (DPP): Hillis-Steele inside each 16-lane row (row_shr 1, 2, 4,
// 8; lanes shifted in from outside the row read 0), then the row totals carried across rows
// with row_bcast:15 (rows 1, 3) and row_bcast:31 (rows 2, 3) -- instead of six ds_bpermute round
// trips on the tree descent's per-level critical path
__device__ __forceinline__ float wave_incl_scan(float v, int lane) {
  (void)lane;
  v += dpp_mov<0x111>(v);   // row_shr:1
  v += dpp_mov<0x112>(v);   // row_shr:2
  v += dpp_mov<0x114>(v);   // row_shr:4
  v += dpp_mov<0x118>(v);   // row_shr:8
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x142, 0xA, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x143, 0xC, 0xF, false));
  return v;
}

// ---- sampling: one wave per sample, stratified over [0, total).  Returns the leaf (row) and
// sets *prob = leaf / total (lane 0's value is the one to use).
// COH: the tree (and the step counter) were written earlier in the SAME launch by workgroups on
// other XCDs (prio_tail_kernel's fused sample): agent-scope loads, never a stale L2 line.
template <bool COH = false>
__device__ __forceinline__ int tree_descend(const float* __restrict__ tree, const TreeGeom& g,
                                            int B, int b, uint64_t seed,
                                            const int64_t* __restrict__ step, int lane,
                                            float* prob) {
  auto ld = [&](int64_t i) -> float {
    if constexpr (COH) return __hip_atomic_load(tree + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else return tree[i];
  };
  const float total = ld(g.off[g.levels - 1]);
  uint64_t ctr = 0ull;
  if (step) {
    if constexpr (COH) ctr = (uint64_t)__hip_atomic_load(step, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else ctr = (uint64_t)(*step);
  }
  float u = ((float)b + r2_uniform(seed, ctr, (uint64_t)b)) / (float)B * total;
  int64_t node = 0;
  float leaf = 0.f;   // the picked leaf's value, already in hand at the last level
  for (int lvl = g.levels - 1; lvl >= 1; --lvl) {
    const int64_t c = node * 64 + lane;
    const float v = (c < g.size[lvl - 1]) ? ld(g.off[lvl - 1] + c) : 0.f;
    const float incl = wave_incl_scan(v, lane);
    const float excl = incl - v;
    const unsigned long long hit = __ballot(incl > u && v > 0.f);
    int pick;
    if (hit) {
      pick = __ffsll((long long)hit) - 1;
    } else {  // float round-off past the end: take the last non-empty child
      const unsigned long long nz = __ballot(v > 0.f);
      pick = nz ? 63 - __clzll((long long)nz) : 0;
    }
    const float ex = __shfl(excl, pick, 64);
    const float pv = __shfl(v, pick, 64);
    u = fminf(fmaxf(u - ex, 0.f), pv * 0.99999f);
    node = node * 64 + pick;
    leaf = pv;
  }
  // leaf == tree[g.off[0] + node] (the level-1 pass loaded it): no dependent re-load of the leaf
  // on the batch head's critical path
  if (g.levels == 1) leaf = ld(g.off[0]);
  *prob = total > 0.f ? leaf / total : 0.f;
  return (int)node;
}

__global__ void tree_sample_kernel(const float* __restrict__ tree, TreeGeom g, int B,
                                   uint64_t seed, const int64_t* __restrict__ step,
                                   int* __restrict__ out_idx, float* __restrict__ out_prob) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (b >= B) return;
  float prob;
  const int node = tree_descend(tree, g, B, b, seed, step, lane, &prob);
  if (lane == 0) {
    out_idx[b] = node;
    if (out_prob) out_prob[b] = prob;
  }
}

// ---- the learner's batch head in one launch, one workgroup per sampled sequence b: tree
// descent (wave 0) -> time-major row list rows[t*B + b] = row(s_b, t) for t < Tn -> stored
// recurrent states of up to 3 chains (row(s_b, off_j): h as bf16, c fp32).  Replaces
// tree_sample + make_rows + one gather_state per chain (4-5 dependent launches).
struct SampleBatchArgs {
  const float* tree;
  TreeGeom g;
  uint64_t seed;
  const int64_t* step;
  int* starts;
  float* probs;
  int* rows;
  const float* hs[3];
  bf16* h[3];
  float* c[3];
  int off[3];
  int B, Tn, cap_e, H, nstate;
  int h_f32;      // split-precision learner: h out as fp32 (the h pointers are float*)
  // optional: the hoisted torso's frame-queue words (torso_sp.hip TSJob::q [0], [1]) zeroed for
  // the launches of the step this sample feeds
  unsigned* qreset;
};

// sequence b of the batch, one 256-thread workgroup (sample_batch_kernel, and prio_tail_kernel's
// fused sample with COH)
template <bool COH>
__device__ __forceinline__ void sample_one(const SampleBatchArgs& a, int b) {
  __shared__ int s_start;
  const int tid = threadIdx.x;
  if (a.qreset && b == 0 && tid == 0) {
    __hip_atomic_store(a.qreset, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(a.qreset + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (tid < 64) {
    float prob;
    const int node = tree_descend<COH>(a.tree, a.g, a.B, b, a.seed, a.step, tid, &prob);
    if (tid == 0) {
      a.starts[b] = node;
      a.probs[b] = prob;
      s_start = node;
    }
  }
  __syncthreads();
  const int s = s_start;
  for (int t = tid; t < a.Tn; t += blockDim.x) a.rows[t * a.B + b] = ring_row_s(s, t, a.cap_e);
  for (int j = 0; j < a.nstate; ++j) {
    const float* src = a.hs[j] + (size_t)ring_row_s(s, a.off[j], a.cap_e) * 2 * a.H;
    for (int k = tid; k < a.H; k += blockDim.x) {
      if (a.h_f32) ((float*)a.h[j])[(size_t)b * a.H + k] = src[k];
      else a.h[j][(size_t)b * a.H + k] = (bf16)src[k];
      a.c[j][(size_t)b * a.H + k] = src[a.H + k];
    }
  }
  __syncthreads();   // s_start is reused by the next sequence of this workgroup
}

__global__ __launch_bounds__(256) void sample_batch_kernel(const SampleBatchArgs a) {
  sample_one<false>(a, blockIdx.x);
}

// ---- rebuild one level from its children (full pass; used after bulk fills)
__global__ void tree_rebuild_level_kernel(float* __restrict__ tree, TreeGeom g, int lvl) {
  const int lane = threadIdx.x & 63;
  const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x >> 6);
  const float* child = tree + g.off[lvl];
  float* parent = tree + g.off[lvl + 1];
  for (int64_t p = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); p < g.size[lvl + 1];
       p += nwaves) {
    const int64_t c = p * 64 + lane;
    float v = c < g.size[lvl] ? child[c] : 0.f;
    v = wave_sum_x(v);
    if (lane == 0) parent[p] = v;
  }
}

// ---- repair ancestors of dirty leaves at level lvl+1
__global__ void tree_update_level_kernel(float* __restrict__ tree, TreeGeom g, int lvl,
                                         const int* __restrict__ dirty,
                                         const int* __restrict__ count, int max_dirty) {
  const int lane = threadIdx.x & 63;
  const int n = min(*count, max_dirty);
  const int nwaves = gridDim.x * (blockDim.x >> 6);
  const float* child = tree + g.off[lvl];
  float* parent = tree + g.off[lvl + 1];
  for (int e = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); e < n; e += nwaves) {
    const int64_t node = ((int64_t)dirty[e]) >> (6 * lvl);
    const int64_t p = node >> 6;
    const int64_t c = p * 64 + lane;
    float v = c < g.size[lvl] ? child[c] : 0.f;
    v = wave_sum_x(v);
    if (lane == 0) parent[p] = v;
  }
}

// ---- the same repair at level 1 (-> level 2) with the small upper levels folded into the
// launch: every workgroup publishes its level-2 sums write-through (sc1 stores, drained), one
// lane per workgroup adds to an arrival ticket, and the workgroup whose add comes last
// recomputes every node of levels 3.. from the level below (sc1 loads; the same wave_sum_x order,
// so the values are bit-identical to the per-level launches) and, with end_step, also does
// step_end_kernel's work.  Replaces levels - 2 launches (+ step_end) of ~4.5 us each in a graph
// (MI355X_MICROARCH.md hand-off table: last-arriver row).  Needs every level >= 3 to have
// at most 64 * 64 nodes below it (host checks).
__global__ void tree_update_tail_kernel(float* __restrict__ tree, TreeGeom g,
                                        const int* __restrict__ dirty, int* __restrict__ count,
                                        int max_dirty, unsigned* __restrict__ ticket,
                                        int64_t* __restrict__ step, int reset_count) {
  __shared__ int last;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int n = min(*count, max_dirty);
  const int nwaves = gridDim.x * nw;
  {
    const float* child = tree + g.off[1];
    float* parent = tree + g.off[2];
    for (int e = blockIdx.x * nw + wave; e < n; e += nwaves) {
      const int64_t p = (((int64_t)dirty[e]) >> 6) >> 6;
      const int64_t c = p * 64 + lane;
      float v = c < g.size[1] ? child[c] : 0.f;
      v = wave_sum_x(v);
      if (lane == 0) __hip_atomic_store(parent + p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    last = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
           gridDim.x - 1;
  __syncthreads();
  if (!last) return;
  for (int l = 2; l + 1 < g.levels; ++l) {
    const float* child = tree + g.off[l];
    float* parent = tree + g.off[l + 1];
    for (int64_t p = wave; p < g.size[l + 1]; p += nw) {
      const int64_t c = p * 64 + lane;
      float v = c < g.size[l] ? __hip_atomic_load(child + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.f;
      v = wave_sum_x(v);
      if (lane == 0) __hip_atomic_store(parent + p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    *ticket = 0u;
    if (step) *step += 1;
    if (reset_count) *count = 0;
  }
}

// one workgroup per sampled start: the waves scan 64-offset chunks of the candidate range into
// an LDS list, then take the listed starts round-robin (a wave per start, not a start loop).
// SC1: leaves / dirty entries stored write-through at agent scope (prio_tail_kernel reads them
// from other CUs after its grid barrier).
template <bool SC1>
__device__ __forceinline__ void seqprio_refresh_wg(const int* __restrict__ starts,
                                                   const uint8_t* __restrict__ is_start,
                                                   const float* __restrict__ priority,
                                                   float* __restrict__ leaves, int T, int upd_lo,
                                                   int upd_hi, int cap_e, float eta,
                                                   int* __restrict__ dirty, int* __restrict__ count,
                                                   int max_dirty, const int b) {
  constexpr int MAXC = 2048;     // host checks the candidate range fits
  __shared__ int list[MAXC];
  __shared__ int n_list;
  __shared__ int dbase;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if (threadIdx.x == 0) n_list = 0;
  __syncthreads();
  const int sb = starts[b];
  const int lo = upd_lo - T + 1, hi = upd_hi - 1;  // candidate offsets, inclusive
  for (int k0 = lo + 64 * wave; k0 <= hi; k0 += 64 * nw) {
    const int k = k0 + lane;
    const bool cand = (k <= hi) && is_start[ring_row_s(sb, k, cap_e)];
    const unsigned long long m = __ballot(cand);
    int base = 0;
    if (lane == 0 && m) base = atomicAdd(&n_list, __popcll(m));
    base = __shfl(base, 0, 64);
    const int pos = base + __popcll(m & ((1ull << lane) - 1));
    if (cand && pos < MAXC) list[pos] = ring_row_s(sb, k, cap_e);
  }
  __syncthreads();
  const int nl = min(n_list, MAXC);
  // one dirty-list reservation per workgroup (a per-start atomicAdd on the shared counter
  // serialised ~4 x B agent-scope atomics on one address)
  if (threadIdx.x == 0) dbase = nl > 0 ? atomicAdd(count, nl) : 0;
  __syncthreads();
  for (int i = wave; i < nl; i += nw) {
    const int s = list[i];
    float mx = 0.f, sm = 0.f;
    for (int t = lane; t < T; t += 64) {
      const float p = priority[ring_row_s(s, t, cap_e)];
      mx = fmaxf(mx, p);
      sm += p;
    }
    mx = wave_max_x(mx);
    sm = wave_sum_x(sm);
    if (lane == 0) {
      // one explicit fma: the two kernels that inline this must round identically
      const float leaf = __builtin_fmaf(eta, mx, (1.f - eta) * (sm / (float)T));
      const int slot = dbase + i;
      if constexpr (SC1) {
        __hip_atomic_store(leaves + s, leaf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (slot < max_dirty) __hip_atomic_store(dirty + slot, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        leaves[s] = leaf;
        if (slot < max_dirty) dirty[slot] = s;
      }
    }
  }
}

// ---- eta-mixed sequence priority of every marked start overlapping the updated window
// For sampled start s_b the learner rewrote rows [s_b + upd_lo, s_b + upd_hi).  Sequence s
// (rows [s, s+T)) overlaps iff s in (s_b + upd_lo - T, s_b + upd_hi).
__global__ void seqprio_refresh_kernel(const int* __restrict__ starts, int B,
                                       const uint8_t* __restrict__ is_start,
                                       const float* __restrict__ priority,
                                       float* __restrict__ leaves, int T, int upd_lo,
                                       int upd_hi, int cap_e, float eta,
                                       int* __restrict__ dirty, int* __restrict__ count,
                                       int max_dirty) {
  (void)B;
  seqprio_refresh_wg<false>(starts, is_start, priority, leaves, T, upd_lo, upd_hi, cap_e, eta,
                            dirty, count, max_dirty, blockIdx.x);
}

// pack workgroups of r2_prio_tail_pack (grid-stride over ~115k items of the fp32 paper config)
#define PRIO_PACK_BLOCKS 192

// grid barrier of a launch whose workgroups are all resident (r2_prio_tail checks B against the
// occupancy-derived resident capacity): every thread drains its stores, one arrival add per
// workgroup, thread 0 polls the counter (agent-scope loads).  Bounded: 2^22 polls with
// s_sleep 2 (~128 cycles each) plus the load round trip, i.e. a few seconds, then it sets *err
// and goes on (a wrong tree rather than a hung GPU; LearnerEngine.check_errors reads the word).
__device__ __forceinline__ void prio_grid_barrier(unsigned* ctr, unsigned target, unsigned* err) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned it = 0;
    while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(2);
      if (++it > (1u << 22)) {
        __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  __syncthreads();
}

// prio_tail_kernel's fused sample (below): wait for the tree, sample this workgroup's sequences,
// the last sampler clears the flag words
__device__ __forceinline__ void prio_tail_sample(const SampleBatchArgs& sb, unsigned* sync, int nprio,
                                                 int role) {
  __shared__ int last_s;
  if (threadIdx.x == 0) {
    unsigned spins = 0;
    while (__hip_atomic_load(sync + 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) {
      __builtin_amdgcn_s_sleep(2);
      if (++spins > (1u << 22)) {
        __hip_atomic_fetch_or(sync + 3, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  __syncthreads();
  for (int b = role; b < sb.B; b += nprio) sample_one<true>(sb, b);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    last_s = __hip_atomic_fetch_add(sync + 5, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
             (unsigned)nprio - 1;
  __syncthreads();
  if (last_s && threadIdx.x == 0) {
    __hip_atomic_store(sync + 4, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(sync + 5, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// ---- the learner's whole priority tail in ONE launch (seqprio_refresh + tree_update_level(0)
// + tree_update_tail): refresh of the sampled windows' sequence priorities (leaves), grid
// barrier, level-0 repair of the dirty list, grid barrier, level-1 repair, arrival ticket, and
// the last arriver recomputes levels 3.. and (with step) ends the learner step.  Same leaves, the
// same wave_sum_x sums over the same children: bit-identical to the three launches.
// sync[0..2]: barrier counters + ticket (zero between launches, reset by the last arriver);
// sync[3]: error word (barrier timeout).
//
// Optional pack workgroups (r2_prio_tail_pack, the single-rank step): blocks nprio.. of the grid
// run the weight repack of the step that just updated the master (pack_step.h, the former
// pack_step_kernel launch) beside the tail; they take no part in the two grid barriers (target
// nprio) and arrive on the final ticket like the tail's workgroups, so the step counter -- which
// their target-sync test reads -- advances only after every one of them has read it.
//
// Optional fused sample (r2_prio_tail_sample, the hoisted learner step: the NEXT step's batch from
// the repaired tree, the former sample_batch_kernel launch): the last arriver publishes the step
// counter and the top levels write-through, then raises sync[4]; the nprio tail workgroups wait
// for it and sample sequences b = blockIdx.x, +nprio, ... with agent-scope tree loads (the levels
// were written by workgroups on other XCDs in this launch); the last of them (ticket sync[5])
// clears sync[4..5].  sync[3] bit 1: that wait timed out.
__global__ __launch_bounds__(256) void prio_tail_kernel(
    const int* __restrict__ starts, const uint8_t* __restrict__ is_start,
    const float* __restrict__ priority, float* __restrict__ tree, TreeGeom g, int T, int upd_lo,
    int upd_hi, int cap_e, float eta, int* __restrict__ dirty, int* __restrict__ count,
    int max_dirty, unsigned* __restrict__ sync, int64_t* __restrict__ step, int reset_count,
    int nprio, int npart, int skip, const PackStepArgs pk, const SampleBatchArgs sb,
    unsigned* __restrict__ wait) {
  __shared__ int last;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  // role of this block among the npart participants.  skip > 0 (the hoisted step): blocks b with
  // b % 8 < skip -- placed on the XCDs that hold the BPTT recurrence beside this launch -- sit it
  // out, so no tail workgroup shares a CU with a recurrence workgroup (the placement only moves
  // work; the roles, and so the results, do not depend on it)
  int role = blockIdx.x;
  if (skip) {
    const int x = blockIdx.x & 7;
    if (x < skip) return;
    role = (blockIdx.x >> 3) * (8 - skip) + x - skip;
  }
  if (role >= npart) return;
  if (wait && role < nprio) {
    // the hoisted step's early fork: launched beside the TD kernel, the tail workgroups wait for
    // its done flag (the priorities it wrote are performed write-through), then acquire; bounded
    // (sync[3] bit 2 on a timeout); the last arriver below clears the flag
    if (threadIdx.x == 0) {
      unsigned spins = 0;
      while (__hip_atomic_load(wait, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > (1u << 22)) {
          __hip_atomic_fetch_or(sync + 3, 4u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
  }
  if (role >= nprio) {
    const int64_t pb = role - nprio, npb = npart - nprio;
    pack_step_items(pk, pb * blockDim.x + threadIdx.x, npb * blockDim.x);
  } else {
    const int nwaves = nprio * nw;
    seqprio_refresh_wg<true>(starts, is_start, priority, tree, T, upd_lo, upd_hi, cap_e, eta, dirty,
                             count, max_dirty, role);
    prio_grid_barrier(sync + 0, nprio, sync + 3);
    const int n = min(__hip_atomic_load(count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), max_dirty);
    for (int lvl = 0; lvl < 2; ++lvl) {
      const float* child = tree + g.off[lvl];
      float* parent = tree + g.off[lvl + 1];
      for (int e = role * nw + wave; e < n; e += nwaves) {
        const int64_t p = ((int64_t)__hip_atomic_load(dirty + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                          >> (6 * (lvl + 1));
        const int64_t c = p * 64 + lane;
        float v = c < g.size[lvl]
                      ? __hip_atomic_load(child + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.f;
        v = wave_sum_x(v);
        if (lane == 0) __hip_atomic_store(parent + p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (lvl == 0) prio_grid_barrier(sync + 1, nprio, sync + 3);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    last = __hip_atomic_fetch_add(sync + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
           (unsigned)npart - 1;
  __syncthreads();
  const bool sampler = sb.B > 0 && role < nprio;
  if (!last) {
    if (sampler) prio_tail_sample(sb, sync, nprio, role);
    return;
  }
  // levels 3.. recomputed by this workgroup alone: level 2 comes from memory (the other
  // workgroups' sc1 stores), every level above from the LDS copy of the one below it -- one
  // memory round trip for the whole top of the tree instead of one per level (the stores still
  // go out write-through for the next step's sampling)
  __shared__ float lvl_buf[2][64];       // levels >= 3 hold <= 64 nodes (r2_prio_tail checks)
  int cur = 0;
  for (int l = 2; l + 1 < g.levels; ++l) {
    const float* child = tree + g.off[l];
    float* parent = tree + g.off[l + 1];
    for (int64_t p = wave; p < g.size[l + 1]; p += nw) {
      const int64_t c = p * 64 + lane;
      float v = 0.f;
      if (c < g.size[l])
        v = l == 2 ? __hip_atomic_load(child + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                   : lvl_buf[cur ^ 1][c];
      v = wave_sum_x(v);
      if (lane == 0) {
        __hip_atomic_store(parent + p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        lvl_buf[cur][p] = v;
      }
    }
    __syncthreads();
    cur ^= 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (threadIdx.x == 0) {
    sync[0] = 0u;
    sync[1] = 0u;
    sync[2] = 0u;
    if (step) {
      if (sb.B > 0)   // read by the fused sample's workgroups on other XCDs: write-through
        __hip_atomic_store(step, *step + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else
        *step += 1;
    }
    if (reset_count) *count = 0;
    if (wait) __hip_atomic_store(wait, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (sb.B > 0) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(sync + 4, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (sampler) prio_tail_sample(sb, sync, nprio, role);
}

// ---- mark new sequence starts (actor side): set flag, compute eta-mix, append dirty
__global__ void mark_starts_kernel(const int* __restrict__ rows, const int* __restrict__ n_rows,
                                   int max_rows, uint8_t* __restrict__ is_start,
                                   const float* __restrict__ priority,
                                   float* __restrict__ leaves, int T, int cap_e, float eta,
                                   int* __restrict__ n_valid, int* __restrict__ dirty,
                                   int* __restrict__ count, int max_dirty) {
  const int lane = threadIdx.x & 63;
  const int n = n_rows ? min(*n_rows, max_rows) : max_rows;
  const int w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (w >= n) return;
  const int s = rows[w];
  if (s < 0) return;
  float mx = 0.f, sm = 0.f;
  for (int t = lane; t < T; t += 64) {
    const float p = priority[ring_row_s(s, t, cap_e)];
    mx = fmaxf(mx, p);
    sm += p;
  }
  mx = wave_max_x(mx);
  sm = wave_sum_x(sm);
  if (lane == 0) {
    if (!is_start[s]) atomicAdd(n_valid, 1);
    is_start[s] = 1;
    leaves[s] = eta * mx + (1.f - eta) * (sm / (float)T);
    const int slot = atomicAdd(count, 1);
    if (slot < max_dirty) dirty[slot] = s;
  }
}

// ---- deferred start edits of a concurrent actor group (actor.hip deferred mode), applied on the
// learner's stream between its steps: entry >= 0 marks a start (flag, eta-mix leaf, n_valid),
// entry <= -2 clears row -2 - entry (flag, leaf, n_valid).  One wave per entry; the flag byte is
// flipped with a word atomic so duplicate entries never double-count n_valid.  Changed leaves go to
// the dirty list.  err bit 2: the pending list overflowed (entries were lost).
__device__ __forceinline__ int flag_exchange(uint8_t* flags, int row, int v) {
  unsigned* w = reinterpret_cast<unsigned*>(flags) + (row >> 2);
  const int sh = (row & 3) * 8;
  const unsigned old = v ? atomicOr(w, 1u << sh) : atomicAnd(w, ~(0xFFu << sh));
  return (int)((old >> sh) & 0xFF);
}

__global__ void apply_pending_kernel(const int* __restrict__ pend, const int* __restrict__ pend_cnt,
                                     int pend_cap, uint8_t* __restrict__ is_start,
                                     const float* __restrict__ priority, float* __restrict__ leaves,
                                     int T, int cap_e, float eta, int* __restrict__ n_valid,
                                     int* __restrict__ dirty, int* __restrict__ count, int max_dirty,
                                     unsigned* __restrict__ err) {
  const int lane = threadIdx.x & 63;
  const int cnt = *pend_cnt;
  if (blockIdx.x == 0 && threadIdx.x == 0 && cnt > pend_cap) atomicOr(err, 2u);
  const int n = min(cnt, pend_cap);
  const int nwv = gridDim.x * (blockDim.x >> 6);
  for (int w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); w < n; w += nwv) {
    const int v = pend[w];
    if (v >= 0) {
      float mx = 0.f, sm = 0.f;
      for (int t = lane; t < T; t += 64) {
        const float p = priority[ring_row_s(v, t, cap_e)];
        mx = fmaxf(mx, p);
        sm += p;
      }
      mx = wave_max_x(mx);
      sm = wave_sum_x(sm);
      if (lane == 0) {
        if (!flag_exchange(is_start, v, 1)) atomicAdd(n_valid, 1);
        leaves[v] = eta * mx + (1.f - eta) * (sm / (float)T);
        const int slot = atomicAdd(count, 1);
        if (slot < max_dirty) dirty[slot] = v;
      }
    } else if (lane == 0) {
      const int r = -2 - v;
      const int was = flag_exchange(is_start, r, 0);
      if (was) atomicSub(n_valid, 1);
      if (was || leaves[r] != 0.f) {
        leaves[r] = 0.f;
        const int slot = atomicAdd(count, 1);
        if (slot < max_dirty) dirty[slot] = r;
      }
    }
  }
}

// ---- time-major row list for (T x B) frames of sampled sequences: rows[t*B+b] = row(s_b, off+t)
__global__ void make_rows_kernel(const int* __restrict__ starts, int B, int Tn, int off,
                                 int cap_e, int* __restrict__ rows) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * Tn) return;
  const int t = i / B, b = i % B;
  rows[i] = ring_row_s(starts[b], off + t, cap_e);
}

// ---- stored recurrent state gather: hs_cs (cap, 2H) fp32 -> h (B,H) bf16, c (B,H) fp32
__global__ void gather_state_kernel(const float* __restrict__ hs_cs, const int* __restrict__ starts,
                                    int B, int off, int cap_e, int H, bf16* __restrict__ h,
                                    float* __restrict__ c, float* __restrict__ h32) {
  const int b = blockIdx.x;
  const int row = ring_row_s(starts[b], off, cap_e);
  const float* src = hs_cs + (size_t)row * 2 * H;
  for (int k = threadIdx.x; k < H; k += blockDim.x) {
    const float hv = src[k];
    h[(size_t)b * H + k] = (bf16)hv;
    if (h32) h32[(size_t)b * H + k] = hv;
    c[(size_t)b * H + k] = src[H + k];
  }
}

// ---- end of learner step: bump the device step counter, reset the dirty list
__global__ void step_end_kernel(int64_t* step, int* count) {
  if (threadIdx.x == 0) {
    if (step) *step += 1;
    if (count) *count = 0;
  }
}

static TreeGeom make_geom(const int64_t* offs, const int64_t* sizes, int levels) {
  TreeGeom g;
  g.levels = levels;
  for (int i = 0; i < TREE_MAX_LEVELS; ++i) {
    g.off[i] = i < levels ? offs[i] : 0;
    g.size[i] = i < levels ? sizes[i] : 0;
  }
  return g;
}

extern "C" int r2_tree_sample(const float* tree, const int64_t* offs, const int64_t* sizes,
                              int levels, int B, uint64_t seed, const int64_t* step, int* out_idx,
                              float* out_prob, void* stream) {
  if (levels < 2 || levels > TREE_MAX_LEVELS) return -1;
  TreeGeom g = make_geom(offs, sizes, levels);
  hipLaunchKernelGGL(tree_sample_kernel, dim3((B + 3) / 4), dim3(256), 0, (hipStream_t)stream,
                     tree, g, B, seed, step, out_idx, out_prob);
  R2_CHECK_LAUNCH();
  return 0;
}

static SampleBatchArgs make_sample_args(const float* tree, const int64_t* offs, const int64_t* sizes,
                                        int levels, int B, uint64_t seed, const int64_t* step,
                                        int* starts, float* probs, int* rows, int Tn, int cap_e, int H,
                                        int nstate, const int64_t* hs, const int* off,
                                        const int64_t* h, const int64_t* c, int h_f32,
                                        unsigned* qreset) {
  SampleBatchArgs a;
  a.qreset = qreset;
  a.tree = tree; a.g = make_geom(offs, sizes, levels); a.seed = seed; a.step = step;
  a.starts = starts; a.probs = probs; a.rows = rows;
  for (int j = 0; j < 3; ++j) {
    a.hs[j] = j < nstate ? (const float*)hs[j] : nullptr;
    a.h[j] = j < nstate ? (bf16*)h[j] : nullptr;
    a.c[j] = j < nstate ? (float*)c[j] : nullptr;
    a.off[j] = j < nstate ? off[j] : 0;
  }
  a.B = B; a.Tn = Tn; a.cap_e = cap_e; a.H = H; a.nstate = nstate; a.h_f32 = h_f32;
  return a;
}

static int sample_batch_launch(const float* tree, const int64_t* offs, const int64_t* sizes,
                               int levels, int B, uint64_t seed, const int64_t* step, int* starts,
                               float* probs, int* rows, int Tn, int cap_e, int H, int nstate,
                               const int64_t* hs, const int* off, const int64_t* h,
                               const int64_t* c, int h_f32, void* stream,
                               unsigned* qreset = nullptr) {
  if (levels < 2 || levels > TREE_MAX_LEVELS || nstate < 0 || nstate > 3 || B < 1) return -1;
  const SampleBatchArgs a = make_sample_args(tree, offs, sizes, levels, B, seed, step, starts, probs,
                                             rows, Tn, cap_e, H, nstate, hs, off, h, c, h_f32, qreset);
  hipLaunchKernelGGL(sample_batch_kernel, dim3(B), dim3(256), 0, (hipStream_t)stream, a);
  R2_CHECK_LAUNCH();
  return 0;
}

// hs/h/c: nstate pointers each (host arrays, int64); off: nstate row offsets; h bf16
extern "C" int r2_sample_batch(const float* tree, const int64_t* offs, const int64_t* sizes,
                               int levels, int B, uint64_t seed, const int64_t* step, int* starts,
                               float* probs, int* rows, int Tn, int cap_e, int H, int nstate,
                               const int64_t* hs, const int* off, const int64_t* h,
                               const int64_t* c, void* stream) {
  return sample_batch_launch(tree, offs, sizes, levels, B, seed, step, starts, probs, rows, Tn,
                             cap_e, H, nstate, hs, off, h, c, 0, stream);
}

// the same with h written fp32 (split-precision learner)
extern "C" int r2_sample_batch_f32h(const float* tree, const int64_t* offs, const int64_t* sizes,
                                    int levels, int B, uint64_t seed, const int64_t* step,
                                    int* starts, float* probs, int* rows, int Tn, int cap_e, int H,
                                    int nstate, const int64_t* hs, const int* off,
                                    const int64_t* h, const int64_t* c, void* stream) {
  return sample_batch_launch(tree, offs, sizes, levels, B, seed, step, starts, probs, rows, Tn,
                             cap_e, H, nstate, hs, off, h, c, 1, stream);
}

// r2_sample_batch(_f32h) that also zeroes the hoisted torso's frame-queue words qreset[0..1]
extern "C" int r2_sample_batch_q(const float* tree, const int64_t* offs, const int64_t* sizes,
                                 int levels, int B, uint64_t seed, const int64_t* step, int* starts,
                                 float* probs, int* rows, int Tn, int cap_e, int H, int nstate,
                                 const int64_t* hs, const int* off, const int64_t* h,
                                 const int64_t* c, int h_f32, unsigned* qreset, void* stream) {
  return sample_batch_launch(tree, offs, sizes, levels, B, seed, step, starts, probs, rows, Tn,
                             cap_e, H, nstate, hs, off, h, c, h_f32, stream, qreset);
}

extern "C" int r2_tree_rebuild(float* tree, const int64_t* offs, const int64_t* sizes, int levels,
                               void* stream) {
  if (levels < 2 || levels > TREE_MAX_LEVELS) return -1;
  TreeGeom g = make_geom(offs, sizes, levels);
  for (int l = 0; l + 1 < levels; ++l) {
    int64_t nb = (g.size[l + 1] + 3) / 4;
    if (nb > 4096) nb = 4096;
    if (nb < 1) nb = 1;
    hipLaunchKernelGGL(tree_rebuild_level_kernel, dim3((unsigned)nb), dim3(256), 0,
                       (hipStream_t)stream, tree, g, l);
  }
  R2_CHECK_LAUNCH();
  return 0;
}

extern "C" int r2_tree_update(float* tree, const int64_t* offs, const int64_t* sizes, int levels,
                              const int* dirty, const int* count, int max_dirty, void* stream) {
  if (levels < 2 || levels > TREE_MAX_LEVELS) return -1;
  TreeGeom g = make_geom(offs, sizes, levels);
  int nb = (max_dirty + 3) / 4;
  if (nb > 256) nb = 256;
  if (nb < 1) nb = 1;
  for (int l = 0; l + 1 < levels; ++l)
    hipLaunchKernelGGL(tree_update_level_kernel, dim3(nb), dim3(256), 0, (hipStream_t)stream,
                       tree, g, l, dirty, count, max_dirty);
  R2_CHECK_LAUNCH();
  return 0;
}

// Level 0 as its own launch, then level 1 with every upper level (and, given `step`, the step
// counter + dirty-list reset) folded into one launch (tree_update_tail_kernel).  ticket: one
// zeroed uint, reset by the kernel.  -3: the tree is too shallow or too wide for the fold.
static int tree_update_fused(float* tree, const int64_t* offs, const int64_t* sizes, int levels,
                             const int* dirty, int* count, int max_dirty, unsigned* ticket,
                             int64_t* step, int reset_count, void* stream) {
  if (levels < 4 || levels > TREE_MAX_LEVELS) return -3;
  for (int l = 3; l < levels; ++l)
    if (sizes[l - 1] > 64 * 64) return -3;
  TreeGeom g = make_geom(offs, sizes, levels);
  int nb = (max_dirty + 3) / 4;
  if (nb > 256) nb = 256;
  if (nb < 1) nb = 1;
  hipLaunchKernelGGL(tree_update_level_kernel, dim3(nb), dim3(256), 0, (hipStream_t)stream,
                     tree, g, 0, dirty, count, max_dirty);
  // fewer workgroups than level 0: each one adds to the single arrival ticket (agent-scope
  // atomics on one address serialise); 64 x 4 waves cover a learner step's dirty list in a pass
  const int nbt = nb < 64 ? nb : 64;
  hipLaunchKernelGGL(tree_update_tail_kernel, dim3(nbt), dim3(256), 0, (hipStream_t)stream,
                     tree, g, dirty, count, max_dirty, ticket, step, reset_count);
  R2_CHECK_LAUNCH();
  return 0;
}

// step: non-null = the learner step's end (step counter + 1 and the dirty-list reset)
extern "C" int r2_tree_update_fused(float* tree, const int64_t* offs, const int64_t* sizes,
                                    int levels, const int* dirty, int* count, int max_dirty,
                                    unsigned* ticket, int64_t* step, void* stream) {
  return tree_update_fused(tree, offs, sizes, levels, dirty, count, max_dirty, ticket, step,
                           step != nullptr, stream);
}

// the dirty-list reset without the step counter (the priority tail on a side stream: the
// counter is advanced on the main stream after the optimizer's target-sync read, r2_step_inc)
extern "C" int r2_tree_update_fused_reset(float* tree, const int64_t* offs, const int64_t* sizes,
                                          int levels, const int* dirty, int* count, int max_dirty,
                                          unsigned* ticket, void* stream) {
  return tree_update_fused(tree, offs, sizes, levels, dirty, count, max_dirty, ticket, nullptr, 1,
                           stream);
}

extern "C" int r2_seqprio_refresh(const int* starts, int B, const uint8_t* is_start,
                                  const float* priority, float* leaves, int T, int upd_lo,
                                  int upd_hi, int cap_e, float eta, int* dirty, int* count,
                                  int max_dirty, void* stream) {
  if (upd_hi - upd_lo + T - 1 > 2048) return -2;   // candidate list (seqprio_refresh_kernel MAXC)
  if (B <= 0) return 0;
  hipLaunchKernelGGL(seqprio_refresh_kernel, dim3(B), dim3(256), 0, (hipStream_t)stream,
                     starts, B, is_start, priority, leaves, T, upd_lo, upd_hi, cap_e, eta, dirty,
                     count, max_dirty);
  R2_CHECK_LAUNCH();
  return 0;
}

// the fused priority tail (prio_tail_kernel); sync: 4 zeroed uints.  -3: the tree shape does not
// allow the fold (tree_update_fused's conditions) or B > 256 (all workgroups must be resident)
extern "C" int r2_get_num_cus();   // lstm_persist.hip: CUs of the learner's stream

// TD done flag the NEXT r2_prio_tail_sample launch on this host thread waits for (consumed by it):
// the hoisted step forks its side branch before the TD launch (td.hip TdDuelArgs::done)
static thread_local unsigned* g_prio_wait = nullptr;
extern "C" int r2_prio_tail_set_wait(unsigned* wait) {
  g_prio_wait = wait;
  return 0;
}

static int prio_tail_launch(const int* starts, int B, const uint8_t* is_start, const float* priority,
                            float* tree, const int64_t* offs, const int64_t* sizes, int levels,
                            int T, int upd_lo, int upd_hi, int cap_e, float eta, int* dirty,
                            int* count, int max_dirty, unsigned* sync, int64_t* step,
                            int reset_count, const PackStepArgs* pk, void* stream,
                            const SampleBatchArgs* sb = nullptr, int skip = 0,
                            unsigned* wait = nullptr) {
  if (upd_hi - upd_lo + T - 1 > 2048) return -2;
  if (B <= 0 || B > 256) return -3;
  {   // every workgroup must be resident at once (grid barriers): B <= CUs x blocks per CU
    static int per_cu = 0;
    if (!per_cu && hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)prio_tail_kernel,
                                                                256, 0) != hipSuccess)
      per_cu = 1;
    if (B > r2_get_num_cus() * (per_cu > 0 ? per_cu : 1)) return -4;   // caller: 3-launch path
  }
  if (levels < 4 || levels > TREE_MAX_LEVELS) return -3;
  for (int l = 3; l < levels; ++l)
    if (sizes[l - 1] > 64 * 64) return -3;
  TreeGeom g = make_geom(offs, sizes, levels);
  PackStepArgs none{};
  SampleBatchArgs no_sample{};
  no_sample.B = 0;
  int grid = B;
  if (pk) {
    if (!pack_step_args_ok(*pk) || !step) return -5;
    grid += PRIO_PACK_BLOCKS;
  }
  // the fused sample: its own tree (the same), every tail workgroup resident (checked above), no
  // pack workgroups (their late arrival would hold the samplers' wait)
  if (sb && (pk || sb->tree != tree)) return -5;
  if (skip < 0 || skip > 4) return -1;
  const int npart = grid;
  if (skip) grid = (npart + 8 - skip - 1) / (8 - skip) * 8;
  hipLaunchKernelGGL(prio_tail_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, starts, is_start,
                     priority, tree, g, T, upd_lo, upd_hi, cap_e, eta, dirty, count, max_dirty, sync,
                     step, reset_count, B, npart, skip, pk ? *pk : none, sb ? *sb : no_sample, wait);
  R2_CHECK_LAUNCH();
  return 0;
}

extern "C" int r2_prio_tail(const int* starts, int B, const uint8_t* is_start, const float* priority,
                            float* tree, const int64_t* offs, const int64_t* sizes, int levels,
                            int T, int upd_lo, int upd_hi, int cap_e, float eta, int* dirty,
                            int* count, int max_dirty, unsigned* sync, int64_t* step,
                            int reset_count, void* stream) {
  return prio_tail_launch(starts, B, is_start, priority, tree, offs, sizes, levels, T, upd_lo, upd_hi,
                          cap_e, eta, dirty, count, max_dirty, sync, step, reset_count, nullptr, stream);
}

// r2_prio_tail + the step's weight repack (the r2_pack_step arguments) on PRIO_PACK_BLOCKS extra
// workgroups of the same launch: one launch fewer between the optimizer and the next step.  The
// tail must end the step (step != null): the counter advances after the pack workgroups read it.
extern "C" int r2_prio_tail_pack(const int* starts, int B, const uint8_t* is_start,
                                 const float* priority, float* tree, const int64_t* offs,
                                 const int64_t* sizes, int levels, int T, int upd_lo, int upd_hi,
                                 int cap_e, float eta, int* dirty, int* count, int max_dirty,
                                 unsigned* sync, int64_t* step, int reset_count,
                                 const float* master, float* target, int64_t n_master,
                                 const int* bf_idx, bf16* bf, bf16* bf_t, int64_t n_bf,
                                 const int* f_idx, float* f32, float* f32_t, int64_t n_f,
                                 int64_t o_bih, int64_t o_bhh, float* lstm_b, float* lstm_b_t,
                                 int64_t G, int64_t interval, int64_t lo_off, void* stream) {
  const PackStepArgs pk{master, target, n_master, bf_idx, bf, bf_t, n_bf, f_idx, f32, f32_t, n_f,
                        o_bih, o_bhh, lstm_b, lstm_b_t, G, step, interval, lo_off};
  return prio_tail_launch(starts, B, is_start, priority, tree, offs, sizes, levels, T, upd_lo, upd_hi,
                          cap_e, eta, dirty, count, max_dirty, sync, step, reset_count, &pk, stream);
}

extern "C" int r2_mark_starts(const int* rows, const int* n_rows, int max_rows, uint8_t* is_start,
                              const float* priority, float* leaves, int T, int cap_e, float eta,
                              int* n_valid, int* dirty, int* count, int max_dirty, void* stream) {
  if (max_rows <= 0) return 0;
  hipLaunchKernelGGL(mark_starts_kernel, dim3((max_rows + 3) / 4), dim3(256), 0,
                     (hipStream_t)stream, rows, n_rows, max_rows, is_start, priority, leaves, T,
                     cap_e, eta, n_valid, dirty, count, max_dirty);
  R2_CHECK_LAUNCH();
  return 0;
}

// grid-stride over the pending list (fixed grid: capture-safe for any count)
extern "C" int r2_apply_pending(const int* pend, const int* pend_cnt, int pend_cap, uint8_t* is_start,
                                const float* priority, float* leaves, int T, int cap_e, float eta,
                                int* n_valid, int* dirty, int* count, int max_dirty, unsigned* err,
                                void* stream) {
  if (pend_cap <= 0) return -1;
  int nb = (pend_cap + 3) / 4;
  if (nb > 512) nb = 512;
  hipLaunchKernelGGL(apply_pending_kernel, dim3(nb), dim3(256), 0, (hipStream_t)stream, pend,
                     pend_cnt, pend_cap, is_start, priority, leaves, T, cap_e, eta, n_valid, dirty,
                     count, max_dirty, err);
  R2_CHECK_LAUNCH();
  return 0;
}

extern "C" int r2_make_rows(const int* starts, int B, int Tn, int off, int cap_e, int* rows,
                            void* stream) {
  const int n = B * Tn;
  hipLaunchKernelGGL(make_rows_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                     starts, B, Tn, off, cap_e, rows);
  R2_CHECK_LAUNCH();
  return 0;
}

extern "C" int r2_gather_state(const float* hs_cs, const int* starts, int B, int off, int cap_e,
                               int H, bf16* h, float* c, float* h32, void* stream) {
  hipLaunchKernelGGL(gather_state_kernel, dim3(B), dim3(256), 0, (hipStream_t)stream, hs_cs,
                     starts, B, off, cap_e, H, h, c, h32);
  R2_CHECK_LAUNCH();
  return 0;
}

extern "C" int r2_step_end(int64_t* step, int* count, void* stream) {
  hipLaunchKernelGGL(step_end_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, step, count);
  R2_CHECK_LAUNCH();
  return 0;
}

// r2_prio_tail (ending the step: step counter + 1) + the NEXT step's sample (r2_sample_batch_q
// arguments, the same tree and step counter) in one launch: the hoisted learner step's side
// branch (engine/learner_engine.py).  sync: 6 zeroed uints.
extern "C" int r2_prio_tail_sample(const int* starts, int B, const uint8_t* is_start,
                                   const float* priority, float* tree, const int64_t* offs,
                                   const int64_t* sizes, int levels, int T, int upd_lo, int upd_hi,
                                   int cap_e, float eta, int* dirty, int* count, int max_dirty,
                                   unsigned* sync, int64_t* step, uint64_t seed, int* s_starts,
                                   float* s_probs, int* s_rows, int Tn, int H, int nstate,
                                   const int64_t* hs, const int* off, const int64_t* h,
                                   const int64_t* c, int h_f32, unsigned* qreset, int skip_xcds,
                                   void* stream) {
  unsigned* const wait = g_prio_wait;   // consumed by this call whatever it returns
  g_prio_wait = nullptr;
  if (!step || nstate < 0 || nstate > 3) return -1;
  const SampleBatchArgs sb = make_sample_args(tree, offs, sizes, levels, B, seed, step, s_starts,
                                              s_probs, s_rows, Tn, cap_e, H, nstate, hs, off, h, c,
                                              h_f32, qreset);
  return prio_tail_launch(starts, B, is_start, priority, tree, offs, sizes, levels, T, upd_lo, upd_hi,
                          cap_e, eta, dirty, count, max_dirty, sync, step, 1, nullptr, stream, &sb,
                          skip_xcds, wait);
}
