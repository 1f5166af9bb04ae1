// Shared pieces of the persistent LSTM kernels (csrc/kernels/lstm_persist.hip: forward kernels,
// placement / counter protocol; csrc/kernels/lstm_bptt.hip: the tagged BPTT): counter-word layout,
// workgroup -> (group, slice) decoding, the XCD placement check and the launch-epoch finish, plus
// the host-side device facts both launch paths read (one definition each, C++17 inline variables).
#pragma once
#include "common.h"

#define PL_UNITS 16
#define PL_GCOLS 64
#define PL_MAX_CHAINS 4
#define PL_SPIN_LIMIT (1u << 22)
// Dynamic LDS reserved (unused) so that at most ONE workgroup fits per CU: each workgroup
// streams its h / slab hand-off through its own CU's load path (per-CU bandwidth, not latency,
// bounds a step once two workgroups share a CU: measured 3.6 -> 5.1 us/step at B=64).
#define PL_LDS_RESERVE (84 * 1024)
// Each (chain, batch-tile) arrival counter sits on its own 128-byte line: several groups
// polling / atomically adding on one line serialise at the memory-side atomic unit.
#define PL_CTR_STRIDE 32
#define PL_MAX_GROUPS 32
// [0, 1024): per-group step counters; [1024, 2048): per-group XCC bitmask; [2048, 3072): arrivals
#define PL_CTR_WORDS (3 * PL_MAX_GROUPS * PL_CTR_STRIDE)
#define PL_OFF_XMASK (PL_MAX_GROUPS * PL_CTR_STRIDE)
#define PL_OFF_ARRIVE (2 * PL_MAX_GROUPS * PL_CTR_STRIDE)
// tagged-hand-off kernels (below): finished-workgroup counter (zeroed with the counters) and the
// launch epoch (never zeroed; advanced by the last workgroup of every launch)
#define PT_DONE_OFF PL_CTR_WORDS
#define PT_MEMSET_WORDS (PL_CTR_WORDS + 32)
#define PT_EPOCH_FWD (PL_CTR_WORDS + 32)
#define PT_EPOCH_BWD (PL_CTR_WORDS + 64)
#define PT_CTR_WORDS (PL_CTR_WORDS + 96)

struct PChain {
  const float* xproj;  // (T, B, G) packed, chain-local time
  const bf16* whh;     // packed (NWG, 64, H)
  const bf16* h0;      // (B, H)
  const float* c0;     // (B, H)
  bf16* h_seq;         // (T, B, H)
  float* c_seq;        // (T, B, H)
  float* h32;          // optional (T, B, H)
  float* gates;        // optional (T - save_from, B, G)
  int save_from;
  int pad_;
  // split precision (split.h; the *_sp launchers): lo planes of W_hh and of h_seq; h0 is fp32
  const bf16* whh_lo;
  bf16* h_seq_lo;
};

struct PFwdArgs {
  PChain ch[PL_MAX_CHAINS];
  int B, T;
  unsigned* ctr;  // (n_chains, MB) arrival counters, zeroed before launch
  unsigned* err;  // error word (nonzero = a spin timed out)
  long long* dbg; // optional per-step phase clock trace of group 0, slice 0 (tools/lstm_probe.py)
  int MB, groups, xcd_map, force_slow;
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t pl_rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, 0, bytes, 0x00020000);
}

// Workgroup (g = recurrence group, j = unit slice) of this block; false for idle blocks.
// xcd_map: block b -> (g = b % 8, j = b / 8), so a group's blocks share b % 8 (one XCD under the
// dispatcher's round-robin placement); otherwise linear (g = b / nwg, j = b % nwg).
__device__ __forceinline__ bool pl_decode(int xcd_map, int groups, int nwg, int& g, int& j) {
  const int b = blockIdx.x;
  if (xcd_map == 2) {   // two groups per XCD: blocks b = 8 l + x, group x + 8 (l / nwg)
    const int l = b >> 3;
    g = (b & 7) + 8 * (l / nwg);
    j = l % nwg;
  } else if (xcd_map == 3) {   // packed pairs: groups 2x, 2x+1 on XCD x (x < groups / 2), so
    // whole XCDs stay free (the hoisted target torso beside the BPTT); blocks b = 8 l + x
    const int l = b >> 3, slot = l / nwg;
    g = slot < 2 ? 2 * (b & 7) + slot : groups;
    j = l % nwg;
  } else if (xcd_map) { g = b & 7; j = b >> 3; }
  else { g = b / nwg; j = b % nwg; }
  return g < groups && j < nwg;
}

// One-time exchange: does every workgroup of group g run on the same XCD?  Each member ORs its
// XCC bit into the group mask (returned atomic: completes before the arrival add), then arrives;
// once all nwg have arrived the mask is final.  Bounded spin; on timeout reports err and says no.
__device__ __forceinline__ int pl_same_xcd(unsigned* ctr, int g, int nwg, int force_slow,
                                           unsigned* err, int* flag_lds) {
  if (threadIdx.x == 0) {
    unsigned x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    unsigned* mask = ctr + PL_OFF_XMASK + g * PL_CTR_STRIDE;
    unsigned* arrive = ctr + PL_OFF_ARRIVE + g * PL_CTR_STRIDE;
    __hip_atomic_fetch_or(mask, 1u << (x & 15), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // the OR must be performed before this member counts as arrived: a returning atomic
    // decrements vmcnt only once performed
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_fetch_add(arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned spins = 0;
    int ok = 1;
    while (__hip_atomic_load(arrive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)nwg) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > PL_SPIN_LIMIT) {
        __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = 0;
        break;
      }
    }
    const unsigned m = __hip_atomic_load(mask, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag_lds = (ok && !force_slow && __builtin_popcount(m) == 1) ? 1 : (ok ? 0 : -1);
  }
  __syncthreads();
  return *flag_lds;
}

// one lane waits until *ctr >= target; result broadcast through LDS; bounded.  The barrier is
// LDS-only (lds_sync): loads/stores this wave issued earlier stay in flight across it.
__device__ __forceinline__ bool pl_wait(unsigned* ctr, unsigned target, unsigned* err,
                                        int* flag_lds) {
  if (threadIdx.x == 0) {
    unsigned spins = 0;
    int ok = 1;
    while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > PL_SPIN_LIMIT) {
        __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = 0;
        break;
      }
    }
    *flag_lds = ok;
  }
  lds_sync();
  return *flag_lds != 0;
}

// CUs of the device (set by the engine from hipDeviceProp_t::multiProcessorCount): every
// persistent grid must be co-resident at one workgroup per CU
inline int g_num_cus = 256;
// CUs of each XCD the engine's stream may use (a CU-masked learner stream beside an actor group,
// parallel/placement.py): the XCD-placed grids below (block b -> XCD b % 8) need their groups'
// blocks co-resident on their own XCD
inline int g_xcd_cus[8] = {32, 32, 32, 32, 32, 32, 32, 32};
// do the recurrence groups of an XCD-mapped grid fit their XCDs?  map 1: group x on XCD x;
// map 2: groups x and x + 8 on XCD x; ``full``: the whole XCD must be free (a group's XCD also
// hosts helper workgroups that take part in the launch)
inline bool pl_xcd_fit(int xcd_map, int groups, int nwg, bool full = false) {
  for (int x = 0; x < 8; ++x) {
    const int n = xcd_map == 3 ? min(max(groups - 2 * x, 0), 2)
                               : (x < groups ? 1 : 0) + (xcd_map == 2 && x + 8 < groups ? 1 : 0);
    if (n == 0) continue;
    if (n * nwg > g_xcd_cus[x] || (full && g_xcd_cus[x] < 32)) return false;
  }
  return true;
}


// probes only (r2_lstm_persist_set_debug / r2_lstm_persist_force_slow, lstm_persist.hip)
inline long long* g_pl_dbg = nullptr;
// The kernels' clock-stamp hooks (per-step traces, per-workgroup startup / per-role stamps for
// tools/lstm_startup_probe.py, tools/bptt_roles_probe.py) are compiled in only with
// -DR2_LSTM_PROBES=1 (R2D2_PROBES=1 python -m pytorch_r2d2_amd._build); the production kernels
// carry none of their code
#ifndef R2_LSTM_PROBES
#define R2_LSTM_PROBES 0
#endif
#define PL_PROBE(p) (R2_LSTM_PROBES ? (p) : nullptr)
inline int g_pl_slow = 0;

#define PT_ROWS 16

// Run by ONE lane of every workgroup at its very end: the last workgroup to finish (done ticket)
// advances the launch epoch and returns the counter words (XCD masks / arrivals of `groups`
// groups, the done ticket) to zero, so the next launch needs no memset node.  Returns true in the
// last workgroup.
__device__ __forceinline__ bool pt_finish(unsigned* ctr, int groups, int total_wgs, int epoch_off) {
  const unsigned done = __hip_atomic_fetch_add(ctr + PT_DONE_OFF, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (done != (unsigned)total_wgs - 1) return false;
  for (int g = 0; g < groups; ++g) {
    __hip_atomic_store(ctr + PL_OFF_XMASK + g * PL_CTR_STRIDE, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(ctr + PL_OFF_ARRIVE + g * PL_CTR_STRIDE, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __hip_atomic_store(ctr + PT_DONE_OFF, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_fetch_add(ctr + epoch_off, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return true;
}

__device__ __forceinline__ uint32_t pt_pack_bf16x2(float a, float b) {
  bf16x2 v;
  v[0] = (bf16)a;
  v[1] = (bf16)b;
  return __builtin_bit_cast(uint32_t, v);
}

// Staged per-step rows filled by LDS-DMA (16 rows of the x-projection / saved gates, 64 floats;
// c / dh rows, 16 floats): the DMA writes LDS slots in lane order, so the swizzle is applied
// through the SOURCE address of each lane -- LDS chunk c of row r holds global chunk c ^ f(r).
// Without it the pointwise's 4-byte reads (row = lane >> 2, 4 units per wave) hit 4 banks (64-float
// rows) or 16 (16-float rows).
__device__ __forceinline__ int pt_swz64(int r, int col) {      // 64-float rows, f(r) = r
  return r * 64 + ((((col >> 2) ^ r) & 15) << 2) + (col & 3);
}
__device__ __forceinline__ int pt_swz16(int r, int col) {      // 16-float rows, f(r) = r >> 2
  return r * 16 + ((((col >> 2) ^ (r >> 2)) & 3) << 2) + (col & 3);
}

