// Persistent LSTM recurrence kernels (gfx950, MI355X).
//
// Why: a per-step kernel pays the dependent-launch floor (1.6 us measured under HIP-graph
// replay) plus a full re-load of its W_hh slice, h_{t-1}, x-projection and c_{t-1} every step;
// at B=64 that is ~100 KB per workgroup per step and the per-CU load path makes a step ~7 us.
// Here ONE launch runs the whole sequence:
//
//  * grid = (H/16 unit slices) x (ceil(B/32) batch tiles) x (chains); workgroup (j, mb, c) owns
//    hidden units [16j,16j+16) of batch rows [32mb, 32mb+32) of chain c for ALL steps.
//  * its W_hh slice (64 gate rows x H, bf16) is loaded ONCE into VGPRs (MFMA B fragments);
//    the cell state c (fwd) / dc carry (bwd) lives in registers; x-projection rows for step
//    t+1 are loaded while step t computes.
//  * per step only h_{t-1} (32 x H bf16 = 16 KB at H=256) moves between workgroups.
//
// Inter-workgroup hand-off (the MI355X recipe, cdna_hip_programming.md Guideline 16, table row
// "ONE lane of each storing workgroup ... agent-scope atomic add / sc1 poll"): the producer
// stores its payload write-through (sc1), drains it (s_waitcnt vmcnt(0)), then ONE lane does a
// relaxed agent-scope atomic add on the (chain, batch-tile) counter; the consumer polls that
// counter with relaxed agent loads + s_sleep and reads every handed-off byte with sc1 loads.
// No placement / dispatch-order assumption for correctness; counters are zeroed by a memset
// node before every launch; every spin is bounded and reports through an error word.
//
// Same-XCD fast path (speed only): the grid deals the workgroups of one recurrence group
// (chain, batch tile) to blocks b with equal b % 8, which the dispatcher places on one XCD.  At
// launch every workgroup reports its HW_REG_XCC_ID; only if all members of its group really share
// one XCD does the group publish h / dh partials with PLAIN stores, which keep the lines in that
// XCD's L2 (sc1 stores drop them, so every consumer read would go to the memory side).  Consumers
// always load with sc1 (L1 bypass, served by the shared L2).  Any other placement falls back to
// sc1 write-through stores -- the placement-independent protocol above.
// All (H/16)*ceil(B/32)*chains workgroups (<= 256 for the supported shapes) must be
// co-resident: 256 threads, <= 40 KB LDS, one per CU is enough.
#include "../common.h"
#include "../split.h"
#include "../gradsum.h"

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

template <int H>
__global__ __launch_bounds__(256) void lstm_fwd_persist_kernel(const PFwdArgs a) {
  constexpr int G = 4 * H;
  constexpr int NWG = H / PL_UNITS;
  constexpr int KS = H / 16;
  constexpr int KH = KS / 2;           // k-steps per wave (K split across wave pairs)
  constexpr int PW = PL_GCOLS + 4;     // fp32 row stride of the partial-gate tiles
  constexpr int HS = H + 8;            // bf16 row stride of the staged h_{t-1} tile
  __shared__ float part[2][32 * PW];
  __shared__ __attribute__((aligned(16))) bf16 hst[32 * PL_UNITS];
  __shared__ __attribute__((aligned(16))) bf16 hin[32 * HS];
  __shared__ int flag;
  int g, j;
  if (!pl_decode(a.xcd_map, a.groups, NWG, g, j)) return;
  const int MB = a.MB, mb = g % MB;
  const PChain& cd = a.ch[g / MB];
  const int B = a.B, T = a.T;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int nt = wave & 1, kq = wave >> 1;
  unsigned* ctr = a.ctr + g * PL_CTR_STRIDE;
  const uint32_t hbytes = (uint32_t)((size_t)T * B * H * sizeof(bf16));
  const __amdgpu_buffer_rsrc_t hrs = pl_rsrc(cd.h_seq, hbytes);
  const int fast = pl_same_xcd(a.ctr, g, NWG, a.force_slow, a.err, &flag);
  if (fast < 0) return;
  if (a.dbg && tid == 0) {
    unsigned x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    a.dbg[256 + blockIdx.x] = (long long)(1000 + g * 100 + (x & 15) * 10 + fast);
  }

  // ---- resident W_hh fragments: B[k][n] = Whh_pk[j][nt*32 + n][k], k-steps kq*KH .. +KH
  bf16x8 wf[KH];
  {
    const bf16* brow = cd.whh + ((size_t)j * PL_GCOLS + nt * 32 + (lane & 31)) * H +
                       kq * KH * 16 + (lane >> 5) * 8;
#pragma unroll
    for (int s = 0; s < KH; ++s) wf[s] = *(const bf16x8*)(brow + s * 16);
  }
  // ---- pointwise ownership: row prl, units pu0 and pu0+1 (8-byte LDS / global accesses);
  // c lives in registers
  const int prl = tid >> 3, pu0 = 2 * (tid & 7);
  const int pb = mb * 32 + prl;
  const bool pv = pb < B;
  const int pbc = pv ? pb : B - 1;
  float2 creg = *(const float2*)(cd.c0 + (size_t)pbc * H + j * PL_UNITS + pu0);
  const int acol = kq * KH * 16 + (lane >> 5) * 8;

  const bool trace = a.dbg && g == 0 && j == 0 && tid == 0;
#define PL_TRACE(k) \
  if (trace && t < 32) a.dbg[t * 8 + (k)] = clock64();
  // x-projection rows (plain loads: written by an earlier kernel), one step ahead.  Issue order
  // matters: vmcnt retires in order, so next step's rows are issued AFTER this step's h loads --
  // waiting for h never waits for an HBM x-projection fetch.
  float2 xv[4], xn[4];
  auto load_x = [&](int t, float2 (&d)[4]) {
    const float* xr = cd.xproj + ((size_t)t * B + pbc) * G + j * PL_GCOLS + pu0;
#pragma unroll
    for (int gi = 0; gi < 4; ++gi) d[gi] = *(const float2*)(xr + 16 * gi);
  };
  load_x(0, xv);
  for (int t = 0; t < T; ++t) {
    PL_TRACE(0);
    // h_{t-1} tile (32 rows x H) staged ONCE per workgroup in LDS: each thread moves HL 16-B
    // chunks (the MFMA fragments of the two N halves would otherwise fetch it twice)
    constexpr int HC = H / 8;              // 16-B chunks per row
    constexpr int HL = 32 * HC / 256;      // chunks per thread
    u32x4 hv4[HL];
    if (t == 0) {
#pragma unroll
      for (int i = 0; i < HL; ++i) {
        const int c = tid + i * 256, r = c / HC, col = (c % HC) * 8;
        hv4[i] = *(const u32x4*)(cd.h0 + (size_t)min(mb * 32 + r, B - 1) * H + col);
      }
    } else {
      if (!pl_wait(ctr, (unsigned)NWG * (unsigned)t, a.err, &flag)) return;
      PL_TRACE(1);
#pragma unroll
      for (int i = 0; i < HL; ++i) {
        const int c = tid + i * 256, r = c / HC, col = (c % HC) * 8;
        const uint32_t off = (uint32_t)((((size_t)(t - 1) * B + min(mb * 32 + r, B - 1)) * H + col) * sizeof(bf16));
        hv4[i] = __builtin_amdgcn_raw_buffer_load_b128(hrs, off, 0, 16);  // sc1
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    // unconditional (clamped): a conditional issue would make the compiler's vmcnt for the MFMA
    // operands count these loads as possibly absent and wait for them
    load_x(t + 1 < T ? t + 1 : t, xn);
#pragma unroll
    for (int i = 0; i < HL; ++i) {
      const int c = tid + i * 256, r = c / HC, col = (c % HC) * 8;
      *(u32x4*)(hin + r * HS + col) = hv4[i];
    }
    lds_sync();
    bf16x8 av[KH];
#pragma unroll
    for (int s = 0; s < KH; ++s) av[s] = *(const bf16x8*)(hin + (lane & 31) * HS + acol + s * 16);
    __builtin_amdgcn_sched_barrier(0);
    f32x16 acc = {};
#pragma unroll
    for (int s = 0; s < KH; ++s) acc = mfma32(av[s], wf[s], acc);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      part[kq][row * PW + nt * 32 + (lane & 31)] = acc[r];
    }
    lds_sync();
    PL_TRACE(2);
    float2 hv, gsv[4];
    {
      float2 pre[4];
#pragma unroll
      for (int gi = 0; gi < 4; ++gi) {
        const float2 a0 = *(const float2*)(part[0] + prl * PW + 16 * gi + pu0);
        const float2 a1 = *(const float2*)(part[1] + prl * PW + 16 * gi + pu0);
        pre[gi] = make_float2(a0.x + a1.x + xv[gi].x, a0.y + a1.y + xv[gi].y);
      }
      gsv[0] = make_float2(sigmoidf_(pre[0].x), sigmoidf_(pre[0].y));
      gsv[1] = make_float2(sigmoidf_(pre[1].x), sigmoidf_(pre[1].y));
      gsv[2] = make_float2(tanhf_(pre[2].x), tanhf_(pre[2].y));
      gsv[3] = make_float2(sigmoidf_(pre[3].x), sigmoidf_(pre[3].y));
      creg.x = gsv[1].x * creg.x + gsv[0].x * gsv[2].x;
      creg.y = gsv[1].y * creg.y + gsv[0].y * gsv[2].y;
      hv = make_float2(gsv[3].x * tanhf_(creg.x), gsv[3].y * tanhf_(creg.y));
      bf16x2 hb;
      hb[0] = (bf16)hv.x;
      hb[1] = (bf16)hv.y;
      *(bf16x2*)(hst + prl * PL_UNITS + pu0) = hb;
    }
    lds_sync();
    PL_TRACE(3);
    // ---- publish h_t slice: wave 0 stores 32 rows x 32 B, drains, signals.  Bookkeeping
    // stores (c, h32, gates) are issued after the signal, off the recurrence's critical path.
    if (wave == 0) {
      const int rl = lane >> 1, hf = lane & 1;
      const int b = mb * 32 + rl;
      if (b < B) {
        const u32x4 v = *(const u32x4*)(hst + rl * PL_UNITS + hf * 8);
        const uint32_t off = (uint32_t)((((size_t)t * B + b) * H + j * PL_UNITS + hf * 8) * sizeof(bf16));
        if (fast) __builtin_amdgcn_raw_buffer_store_b128(v, hrs, off, 0, 0);   // stays in this XCD's L2
        else __builtin_amdgcn_raw_buffer_store_b128(v, hrs, off, 0, 16);       // sc1 write-through
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    PL_TRACE(4);
    const bool save = cd.gates != nullptr && t >= cd.save_from;
    if (pv) {
      const size_t o = ((size_t)t * B + pb) * H + j * PL_UNITS + pu0;
      *(float2*)(cd.c_seq + o) = creg;
      if (cd.h32) *(float2*)(cd.h32 + o) = hv;
      if (save) {
        float* gp = cd.gates + ((size_t)(t - cd.save_from) * B + pb) * G + j * PL_GCOLS + pu0;
#pragma unroll
        for (int gi = 0; gi < 4; ++gi) *(float2*)(gp + 16 * gi) = gsv[gi];
      }
    }
#pragma unroll
    for (int gi = 0; gi < 4; ++gi) xv[gi] = xn[gi];
  }
}

struct PBwdArgs {
  const float* dh_ext;  // (Tl, B, H) or null
  const float* gates;   // (Tl, B, G) packed post-activation
  const float* c_seq;   // (T, B, H)
  const float* c0;      // (B, H)
  const bf16* whhT;     // packed (NWG, H, 64)
  float* slab;          // (2, NWG, B, H) partial dh ping-pong
  bf16* dgates;         // (Tl, B, G)
  int B, T, t0;
  unsigned* ctr;        // PL_CTR_WORDS, zeroed before launch
  unsigned* err;
  int groups, xcd_map, force_slow;
};

template <int H>
__global__ __launch_bounds__(256) void lstm_bwd_persist_kernel(const PBwdArgs a) {
  constexpr int G = 4 * H;
  constexpr int NWG = H / PL_UNITS;
  constexpr int NT32 = H / 32;
  constexpr int TPW = (NT32 + 3) / 4;  // output N tiles per wave in phase B
  constexpr int DW = PL_GCOLS + 8;     // bf16 stride of the dgates tile (144 B)
  constexpr int PS = H + 4;            // fp32 stride of the partial-dh staging tile
  __shared__ __attribute__((aligned(16))) bf16 dg[32 * DW];
  __shared__ __attribute__((aligned(16))) float pst[32 * PS];
  __shared__ float red[2][32 * PL_UNITS];
  __shared__ int flag;
  int mb, j;
  if (!pl_decode(a.xcd_map, a.groups, NWG, mb, j)) return;
  const int B = a.B, T = a.T, t0 = a.t0;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  unsigned* ctr = a.ctr + mb * PL_CTR_STRIDE;
  const uint32_t sbytes = (uint32_t)((size_t)2 * NWG * B * H * sizeof(float));
  const __amdgpu_buffer_rsrc_t srs = pl_rsrc(a.slab, sbytes);
  const int fast = pl_same_xcd(a.ctr, mb, NWG, a.force_slow, a.err, &flag);
  if (fast < 0) return;

  // ---- resident W_hh^T fragments for phase B: B[k][n] = Whh_pk[j][k][n] = whhT[j][n][k]
  bf16x8 wt[TPW][4];
#pragma unroll
  for (int q = 0; q < TPW; ++q) {
    const int ntl = min(wave + q * 4, NT32 - 1);
    const bf16* brow = a.whhT + ((size_t)j * H + ntl * 32 + (lane & 31)) * PL_GCOLS + (lane >> 5) * 8;
#pragma unroll
    for (int s = 0; s < 4; ++s) wt[q][s] = *(const bf16x8*)(brow + s * 16);
  }
  // pointwise ownership: row prl, units pu0 and pu0+1 (8-byte accesses); dc carry in registers
  const int prl = tid >> 3, pu0 = 2 * (tid & 7);
  const int pb = mb * 32 + prl;
  const bool pv = pb < B;
  const int pbc = pv ? pb : B - 1;
  float2 dcr = make_float2(0.f, 0.f);
  // slab-reduction ownership: (row, float4 group) pairs, two threads per pair split producers
  const int rr = (tid & 127) >> 2, u4 = tid & 3, hh = tid >> 7;
  const int rb = min(mb * 32 + rr, B - 1);

  // per-step operands (plain loads of earlier kernels' outputs), one step ahead and issued after
  // the step's slab loads: vmcnt retires in order, so waiting for the partials never waits for an
  // HBM operand fetch
  float2 dhv, gv[4], ctv, cpv, dhn, gn[4], ctn, cpn;
  auto load_ops = [&](int t, float2& dh, float2 (&gq)[4], float2& ct, float2& cp) {
    const int tl = t - t0;
    const size_t hidx = (size_t)pbc * H + j * PL_UNITS + pu0;
    dh = a.dh_ext ? *(const float2*)(a.dh_ext + (size_t)tl * B * H + hidx) : make_float2(0.f, 0.f);
    const float* gp = a.gates + ((size_t)tl * B + pbc) * G + j * PL_GCOLS + pu0;
#pragma unroll
    for (int gi = 0; gi < 4; ++gi) gq[gi] = *(const float2*)(gp + 16 * gi);
    ct = *(const float2*)(a.c_seq + (size_t)t * B * H + hidx);
    cp = *(const float2*)((t == 0) ? a.c0 + hidx : a.c_seq + (size_t)(t - 1) * B * H + hidx);
  };
  load_ops(T - 1, dhv, gv, ctv, cpv);
  for (int t = T - 1, k = 0; t >= t0; --t, ++k) {
    const int tl = t - t0;
    // recurrent partials from step t+1 (written by the NWG workgroups of this batch tile)
    if (k > 0) {
      if (!pl_wait(ctr, (unsigned)NWG * (unsigned)k, a.err, &flag)) return;
      const int slot = (k - 1) & 1;
      // all NWG/2 partial loads in flight at once (compile-time trip count), then the sum
      u32x4 pv4[NWG / 2];
#pragma unroll
      for (int ii = 0; ii < NWG / 2; ++ii) {
        const int i = hh + 2 * ii;
        const uint32_t off = (uint32_t)((((size_t)(slot * NWG + i) * B + rb) * H + j * PL_UNITS + u4 * 4) * sizeof(float));
        pv4[ii] = __builtin_amdgcn_raw_buffer_load_b128(srs, off, 0, 16);  // sc1
      }
      f32x4 sum = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ii = 0; ii < NWG / 2; ++ii) sum += __builtin_bit_cast(f32x4, pv4[ii]);
#pragma unroll
      for (int e = 0; e < 4; ++e) red[hh][rr * PL_UNITS + u4 * 4 + e] = sum[e];
    }
    __builtin_amdgcn_sched_barrier(0);
    load_ops(t > t0 ? t - 1 : t, dhn, gn, ctn, cpn);  // unconditional: see the forward kernel
    lds_sync();
    bf16x2 dgv[4];
    {
      float2 dh = dhv;
      if (k > 0) {
        const float2 r0 = *(const float2*)(red[0] + prl * PL_UNITS + pu0);
        const float2 r1 = *(const float2*)(red[1] + prl * PL_UNITS + pu0);
        dh.x += r0.x + r1.x;
        dh.y += r0.y + r1.y;
      }
      float dgf[4][2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const float gi = e ? gv[0].y : gv[0].x, gf = e ? gv[1].y : gv[1].x;
        const float gg = e ? gv[2].y : gv[2].x, go = e ? gv[3].y : gv[3].x;
        const float dhe = e ? dh.y : dh.x, cte = e ? ctv.y : ctv.x, cpe = e ? cpv.y : cpv.x;
        const float tc = tanhf_(cte);
        const float dc = (e ? dcr.y : dcr.x) + dhe * go * (1.f - tc * tc);
        const float d_o = dhe * tc;
        const float d_i = dc * gg, d_g = dc * gi, d_f = dc * cpe;
        if (e) dcr.y = dc * gf; else dcr.x = dc * gf;
        dgf[0][e] = d_i * gi * (1.f - gi);
        dgf[1][e] = d_f * gf * (1.f - gf);
        dgf[2][e] = d_g * (1.f - gg * gg);
        dgf[3][e] = d_o * go * (1.f - go);
      }
      bf16* lrow = dg + prl * DW + pu0;
#pragma unroll
      for (int gi = 0; gi < 4; ++gi) {
        dgv[gi][0] = (bf16)dgf[gi][0];
        dgv[gi][1] = (bf16)dgf[gi][1];
        bf16x2 z;
        z[0] = pv ? dgv[gi][0] : (bf16)0.f;
        z[1] = pv ? dgv[gi][1] : (bf16)0.f;
        *(bf16x2*)(lrow + 16 * gi) = z;
      }
    }
    if (t > t0) {
      lds_sync();
      // ---- phase B: partial dh_{t-1}[r][n] = sum_k dg[r][k] * Whh_pk[j][k][n]  (K = 64)
      const bf16* arow = dg + (lane & 31) * DW + (lane >> 5) * 8;
      bf16x8 afr[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) afr[s] = *(const bf16x8*)(arow + s * 16);
#pragma unroll
      for (int q = 0; q < TPW; ++q) {
        const int ntl = wave + q * 4;
        if (ntl < NT32) {
          f32x16 acc = {};
#pragma unroll
          for (int s = 0; s < 4; ++s) acc = mfma32(afr[s], wt[q][s], acc);
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
            pst[row * PS + ntl * 32 + (lane & 31)] = acc[r];
          }
        }
      }
      lds_sync();
      // store the 32 x H fp32 partial slab (rows < B), 16 B per lane, drain, then signal
      const int slot = k & 1;
      constexpr int C4 = H / 4;  // float4 per row
      for (int c = tid; c < 32 * C4; c += 256) {
        const int r = c / C4, col = (c % C4) * 4;
        const int b = mb * 32 + r;
        if (b < B) {
          const u32x4 v = *(const u32x4*)(pst + r * PS + col);
          const uint32_t off = (uint32_t)((((size_t)(slot * NWG + j) * B + b) * H + col) * sizeof(float));
          if (fast) __builtin_amdgcn_raw_buffer_store_b128(v, srs, off, 0, 0);   // stays in L2
          else __builtin_amdgcn_raw_buffer_store_b128(v, srs, off, 0, 16);       // sc1
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      lds_sync();
      if (tid == 0) __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // dgates output for the weight-gradient GEMMs, off the recurrence's critical path
    if (pv) {
      bf16* dgo = a.dgates + ((size_t)tl * B + pb) * G + j * PL_GCOLS + pu0;
#pragma unroll
      for (int gi = 0; gi < 4; ++gi) *(bf16x2*)(dgo + 16 * gi) = dgv[gi];
    }
    dhv = dhn; ctv = ctn; cpv = cpn;
#pragma unroll
    for (int gi = 0; gi < 4; ++gi) gv[gi] = gn[gi];
  }
}

// CUs of the device (set by the engine from hipDeviceProp_t::multiProcessorCount): every
// persistent grid must be co-resident at one workgroup per CU
static int g_num_cus = 256;
// CUs of each XCD the engine's stream may use (a CU-masked learner stream beside an actor group,
// parallel/placement.py): the XCD-placed grids below (block b -> XCD b % 8) need their groups'
// blocks co-resident on their own XCD
static int g_xcd_cus[8] = {32, 32, 32, 32, 32, 32, 32, 32};
extern "C" int r2_set_num_cus(int n) {
  if (n > 0) {
    g_num_cus = n;
    for (int x = 0; x < 8; ++x) g_xcd_cus[x] = n / 8;     // an even split unless told otherwise
  }
  return 0;
}
extern "C" int r2_set_xcd_cus(const int* c) {
  int n = 0;
  for (int x = 0; x < 8; ++x) n += c[x];
  if (n <= 0) return -1;
  for (int x = 0; x < 8; ++x) g_xcd_cus[x] = c[x];
  g_num_cus = n;
  return 0;
}
extern "C" int r2_get_num_cus() { return g_num_cus; }

// do the recurrence groups of an XCD-mapped grid fit their XCDs?  map 1: group x on XCD x;
// map 2: groups x and x + 8 on XCD x; ``full``: the whole XCD must be free (a group's XCD also
// hosts helper workgroups that take part in the launch)
static bool pl_xcd_fit(int xcd_map, int groups, int nwg, bool full = false) {
  for (int x = 0; x < 8; ++x) {
    const int n = xcd_map == 3 ? min(max(groups - 2 * x, 0), 2)
                               : (x < groups ? 1 : 0) + (xcd_map == 2 && x + 8 < groups ? 1 : 0);
    if (n == 0) continue;
    if (n * nwg > g_xcd_cus[x] || (full && g_xcd_cus[x] < 32)) return false;
  }
  return true;
}

static long long* g_pl_dbg = nullptr;
static long long* g_pl_fwd_stamps = nullptr;   // tagged forward: >= 4 x grid words
extern "C" int r2_lstm_fwd_set_stamps(long long* p) { g_pl_fwd_stamps = p; return 0; }
static int g_pl_slow = 0;
extern "C" int r2_lstm_persist_set_debug(long long* p) { g_pl_dbg = p; return 0; }
static int g_pl_nomap2 = 0;
// testing / diagnostics: bit 0 = always use the placement-independent sc1 protocol; bit 1 = no
// two-groups-per-XCD placement in the tagged forward (groups 9..16 spread over every XCD)
extern "C" int r2_lstm_persist_force_slow(int v) {
  g_pl_slow = v & 1;
  g_pl_nomap2 = (v >> 1) & 1;
  return 0;
}

// chain_ptrs: n_chains x 9 int64 (same layout as r2_lstm_fwd).  ctr: >= PL_CTR_WORDS (1024) unsigned,
// err: 1 unsigned.  Both are zeroed here with memset nodes (graph-capturable).
extern "C" int r2_lstm_fwd_persist(const int64_t* chain_ptrs, int n_chains, int B, int T, int H,
                                   unsigned* ctr, unsigned* err, void* stream) {
  if (n_chains < 1 || n_chains > PL_MAX_CHAINS || B < 1 || B > 256) return -1;
  if (H != 64 && H != 128 && H != 256 && H != 512) return -2;
  const int MB = (B + 31) / 32;
  if ((H / PL_UNITS) * MB * n_chains > g_num_cus || MB > 8) return -3;  // co-resident, 1 WG per CU
  if ((size_t)T * B * H * 2 >= (1ull << 32)) return -4;
  PFwdArgs args;
  for (int c = 0; c < n_chains; ++c) {
    const int64_t* p = chain_ptrs + 9 * c;
    PChain& ch = args.ch[c];
    ch.xproj = (const float*)p[0]; ch.whh = (const bf16*)p[1]; ch.h0 = (const bf16*)p[2];
    ch.c0 = (const float*)p[3]; ch.h_seq = (bf16*)p[4]; ch.c_seq = (float*)p[5];
    ch.h32 = (float*)p[6]; ch.gates = (float*)p[7]; ch.save_from = (int)p[8]; ch.pad_ = 0;
  }
  const int groups = n_chains * MB, nwg = H / PL_UNITS;
  args.B = B; args.T = T; args.ctr = ctr; args.err = err; args.dbg = g_pl_dbg;
  args.MB = MB; args.groups = groups; args.xcd_map = groups <= 8 && nwg <= 32 && pl_xcd_fit(1, groups, nwg);
  args.force_slow = g_pl_slow;
  hipStream_t s = (hipStream_t)stream;
  hipMemsetAsync(ctr, 0, PL_CTR_WORDS * sizeof(unsigned), s);
  dim3 grid(args.xcd_map ? 8 * nwg : groups * nwg), block(256);
  const void* fn = H == 64 ? (const void*)lstm_fwd_persist_kernel<64>
                 : H == 128 ? (const void*)lstm_fwd_persist_kernel<128>
                 : H == 256 ? (const void*)lstm_fwd_persist_kernel<256>
                            : (const void*)lstm_fwd_persist_kernel<512>;
  hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, PL_LDS_RESERVE);
  switch (H) {
    case 64: hipLaunchKernelGGL(lstm_fwd_persist_kernel<64>, grid, block, PL_LDS_RESERVE, s, args); break;
    case 128: hipLaunchKernelGGL(lstm_fwd_persist_kernel<128>, grid, block, PL_LDS_RESERVE, s, args); break;
    case 256: hipLaunchKernelGGL(lstm_fwd_persist_kernel<256>, grid, block, PL_LDS_RESERVE, s, args); break;
    default: hipLaunchKernelGGL(lstm_fwd_persist_kernel<512>, grid, block, PL_LDS_RESERVE, s, args); break;
  }
  R2_CHECK_LAUNCH();
  return 0;
}

// slab: (2, H/16, B, H) fp32.  ctr: >= MB unsigned.
extern "C" int r2_lstm_bwd_persist(const float* dh_ext, const float* gates, const float* c_seq,
                                   const float* c0, const bf16* whhT, float* slab, bf16* dgates,
                                   int B, int T, int t0, int H, unsigned* ctr, unsigned* err,
                                   void* stream) {
  if (B < 1 || B > 256) return -1;
  if (H != 64 && H != 128 && H != 256 && H != 512) return -2;
  const int MB = (B + 31) / 32;
  if ((H / PL_UNITS) * MB > g_num_cus || MB > 8) return -3;
  if ((size_t)2 * (H / PL_UNITS) * B * H * 4 >= (1ull << 32)) return -4;
  const int nwg = H / PL_UNITS;
  const int xmap = MB <= 8 && nwg <= 32 && pl_xcd_fit(1, MB, nwg);
  PBwdArgs a{dh_ext, gates, c_seq, c0, whhT, slab, dgates, B, T, t0, ctr, err, MB, xmap, g_pl_slow};
  hipStream_t s = (hipStream_t)stream;
  hipMemsetAsync(ctr, 0, PL_CTR_WORDS * sizeof(unsigned), s);
  dim3 grid(xmap ? 8 * nwg : MB * nwg), block(256);
  const void* fn = H == 64 ? (const void*)lstm_bwd_persist_kernel<64>
                 : H == 128 ? (const void*)lstm_bwd_persist_kernel<128>
                 : H == 256 ? (const void*)lstm_bwd_persist_kernel<256>
                            : (const void*)lstm_bwd_persist_kernel<512>;
  hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, PL_LDS_RESERVE);
  switch (H) {
    case 64: hipLaunchKernelGGL(lstm_bwd_persist_kernel<64>, grid, block, PL_LDS_RESERVE, s, a); break;
    case 128: hipLaunchKernelGGL(lstm_bwd_persist_kernel<128>, grid, block, PL_LDS_RESERVE, s, a); break;
    case 256: hipLaunchKernelGGL(lstm_bwd_persist_kernel<256>, grid, block, PL_LDS_RESERVE, s, a); break;
    default: hipLaunchKernelGGL(lstm_bwd_persist_kernel<512>, grid, block, PL_LDS_RESERVE, s, a); break;
  }
  R2_CHECK_LAUNCH();
  return 0;
}

// ============================================================================================
// Forward v3: data-tagged granule hand-off (cdna_hip_programming / MI355X_MICROARCH price list,
// "handoff-1to1": ~half the latency of a payload + flag / counter hand-off), 16-row batch tiles,
// wave-owned gate columns.
//
//  * group = (chain, 16-row batch tile); its H/16 workgroups own 16 hidden units each; wave w of a
//    workgroup owns units 4w..4w+3 of that slice, all four gates (16 MFMA columns), over the FULL
//    K = H: no cross-wave K reduction, the gate exchange for the pointwise is wave-private LDS.
//  * h_t is published as 8-byte granules {bf16 h[u], bf16 h[u+1], tag} (one store per granule,
//    tag = epoch << 16 | t + 1) into a 2-slot ring; consumers poll the granules themselves with
//    sc1 loads -- no counter, no drain, no ordering between granules.  Slot reuse is safe: a
//    workgroup writes h_{t+1} only after every workgroup of its group has published h_t, i.e.
//    finished loading h_{t-1} from that slot.  The epoch (advanced by the last workgroup of each
//    launch) makes granules of earlier launches unmatchable, so the ring is never cleared.
//  * same-XCD fast path as v2 (plain granule stores stay in the XCD's L2); sc1 stores otherwise.
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

struct PTArgs {
  PChain ch[PL_MAX_CHAINS];
  int B, T;
  unsigned* ctr;
  unsigned* err;
  long long* dbg;
  long long* stamps;   // optional per-workgroup startup stamps (4 per block of the grid)
  void* ring;     // (chains, 2, MB*16, H/2) granules
  int MB, groups, xcd_map, force_slow;
};

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

// SP (split precision, split.h): W_hh hi / lo fragments stay in VGPRs and every product is 3
// MFMA passes; h_seq is written as hi / lo planes.  h_t travels one of two ways:
//  * T4 (default): ONE 4-byte word per unit -- fp32 h rounded to 19 explicit mantissa bits with a
//    4-bit tag in the low nibble, {epoch parity, (t + 1) mod 8}.  Every word is its own granule
//    (a 4-byte store is single-copy atomic), so the consumer polls 16-B chunks of 4 units and
//    checks 4 nibbles.  Half the bytes of the 8-byte form (16 KB per workgroup per step, what the
//    bf16 kernel moves), and no accuracy lost: the consumer splits the rounded value into hi / lo
//    exactly as before (hi + lo of the full fp32 value is itself only ~2^-17 accurate; the 2^-20
//    rounding sits below it).  Why 4 bits suffice: a slot read at step t holds either step t-1
//    (wanted), step t-3 of this launch ((t + 1) mod 8 differs by 2), or -- for t <= 2 only --
//    the previous launch's step of the same parity, whose epoch parity differs because every
//    launch of one launch SITE (fixed chain set, one ring, one ctr) advances the epoch by one.
//    Requirement (the engine keeps it): a ring + ctr pair serves one launch site.
//  * !T4 (the bf16 kernel): {bf16 h pair, 32-bit tag} 8-byte granules.  (The split-precision
//    8-byte form lost the round-2 A/B, profiles/archive/bench_r02_tag_words_ab.log; removed.)
template <int H, bool SP, bool T4 = false>
__global__ __launch_bounds__(320) void lstm_fwd_tag_kernel(const PTArgs a) {
  static_assert(!T4 || SP, "T4 is a split-precision hand-off");
  constexpr int G = 4 * H;
  constexpr int NWG = H / PL_UNITS;
  constexpr int KS = H / 32;                  // 16x16x32 k-steps
  // bf16 stride of a staged h row: H + 16 puts consecutive rows 2 bank quads apart (2 mod 16),
  // the stride at which every ds_read_b128 lane group of the A-fragment reads (rows 0-15 x two
  // 16-B k halves) hits 16 distinct quads; H + 8 (1 quad) collided in every group (PMC bank
  // conflict / LDS active 0.56)
  constexpr int HS = H + 16;
  constexpr int UG = SP ? 1 : 2;              // hidden units per granule
  constexpr int GR = H / UG;                  // granules per row
  constexpr int CPR = T4 ? H / 4 : GR / 2;    // 16-B chunks per row (4 units / 2 granules)
  constexpr int CH = PT_ROWS * CPR / 256;     // chunks per compute thread
  constexpr int XS = 20;                      // fp32 stride of a gate-exchange row
  static_assert(CH >= 1 && PT_ROWS * CPR % 256 == 0, "H");
  // LDS: staged h (2 slots), wave-private gate exchange, x-projection ring (3 slots, filled by
  // the I/O wave), per-step outputs (2 slots, drained by the I/O wave)
  __shared__ __attribute__((aligned(16))) bf16 hin[2][PT_ROWS * HS];
  __shared__ __attribute__((aligned(16))) bf16 hinl[2][SP ? PT_ROWS * HS : 8];   // lo image (SP)
  __shared__ __attribute__((aligned(16))) float xch[4][PT_ROWS * XS];
  __shared__ __attribute__((aligned(1024))) float xl[3][PT_ROWS * PL_GCOLS];
  __shared__ __attribute__((aligned(16))) float oc[2][PT_ROWS * PL_UNITS];
  __shared__ __attribute__((aligned(16))) float oh32[2][PT_ROWS * PL_UNITS];
  __shared__ __attribute__((aligned(16))) bf16 ohs[2][PT_ROWS * PL_UNITS];
  __shared__ __attribute__((aligned(16))) bf16 ohsl[2][SP ? PT_ROWS * PL_UNITS : 8];
  __shared__ __attribute__((aligned(16))) float og[2][PT_ROWS * PL_GCOLS];
  __shared__ int flag;
  int g, j;
  if (!pl_decode(a.xcd_map, a.groups, NWG, g, j)) return;
  // per-workgroup clock stamps (r2_lstm_fwd_set_stamps, tools/lstm_startup_probe.py): stamps[4 b +
  // {0 start, 1 rendezvous done, 2 compute loop entry, 3 end}] (s_memrealtime, 100 MHz)
  long long* const wst = a.stamps ? a.stamps + 4 * blockIdx.x : nullptr;
  if (wst && threadIdx.x == 0) wst[0] = (long long)__builtin_amdgcn_s_memrealtime();
  const int MB = a.MB, mb = g % MB, chn = g / MB;
  const PChain& cd = a.ch[chn];
  const int B = a.B, T = a.T;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int rows_all = MB * PT_ROWS;
  const uint32_t ring_bytes = (uint32_t)((size_t)a.groups / MB * 2 * rows_all * GR * 8);
  const __amdgpu_buffer_rsrc_t rrs = pl_rsrc(a.ring, ring_bytes);
  const unsigned ep = __hip_atomic_load(a.ctr + PT_EPOCH_FWD, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // I/O wave: x-projection rows of step t -> ring slot t % 3 (LDS-DMA)
  auto io_load_x = [&](int t) {
    float* dst = xl[t % 3];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      // LDS chunk (lane & 15) of row r holds global chunk (lane & 15) ^ r (pt_swz64): the
      // pointwise reads of 16 rows x 4 units then cover 64 distinct banks
      const int r = 4 * q + (lane >> 4);
      const int b = min(mb * PT_ROWS + r, B - 1);
      const float* src = cd.xproj + ((size_t)t * B + b) * G + j * PL_GCOLS + 4 * ((lane & 15) ^ r);
      __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(dst + q * 256),
                                       16, 0, 0);
    }
  };
  // the first two steps' x rows load under the XCD rendezvous below (its barrier waits for them)
  if (wave == 4) {
    io_load_x(0);
    if (T > 1) io_load_x(1);
  }
  // compute waves: resident W_hh fragments (loaded under the rendezvous too): wave column c
  // (0..15) = gate c>>2 of unit 4*wave + (c&3), i.e. packed row 16*(c>>2) + 4*wave + (c&3) of
  // this workgroup's 64
  bf16x8 wf[KS], wfl[SP ? KS : 1];
  if (wave < 4) {
    const int c = lane & 15;
    const int n = 16 * (c >> 2) + 4 * wave + (c & 3);
    const size_t o = ((size_t)j * PL_GCOLS + n) * H + 8 * (lane >> 4);
#pragma unroll
    for (int s = 0; s < KS; ++s) wf[s] = *(const bf16x8*)(cd.whh + o + 32 * s);
    if constexpr (SP) {
#pragma unroll
      for (int s = 0; s < KS; ++s) wfl[s] = *(const bf16x8*)(cd.whh_lo + o + 32 * s);
    }
  }
  const int fast = pl_same_xcd(a.ctr, g, NWG, a.force_slow, a.err, &flag);
  if (fast < 0) return;
  if (wst && tid == 0) wst[1] = (long long)__builtin_amdgcn_s_memrealtime();
  if (a.dbg && tid == 0) {
    unsigned x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    a.dbg[256 + blockIdx.x] = (long long)(1000 + g * 100 + (x & 15) * 10 + fast);
  }
  const bool save_any = cd.gates != nullptr;

  if (wave == 4) {
    // ================= I/O wave: x-projection prefetch (2 steps ahead) + output drain.  Its
    // loads and stores never sit in a compute wave's vmcnt queue in front of a granule poll.
    auto io_store = [&](int t) {
      const int s = t & 1;
      {
        const int r = lane >> 2, q = lane & 3, b = mb * PT_ROWS + r;
        if (b < B) {
          const size_t o = ((size_t)t * B + b) * H + j * PL_UNITS + 4 * q;
          *(f32x4*)(cd.c_seq + o) = *(const f32x4*)(oc[s] + r * PL_UNITS + 4 * q);
          if (cd.h32) *(f32x4*)(cd.h32 + o) = *(const f32x4*)(oh32[s] + r * PL_UNITS + 4 * q);
        }
      }
      if (lane < 32) {
        const int r = lane >> 1, hf = lane & 1, b = mb * PT_ROWS + r;
        if (b < B)
          *(u32x4*)(cd.h_seq + ((size_t)t * B + b) * H + j * PL_UNITS + 8 * hf) =
              *(const u32x4*)(ohs[s] + r * PL_UNITS + 8 * hf);
      } else if (SP) {
        const int r = (lane - 32) >> 1, hf = lane & 1, b = mb * PT_ROWS + r;
        if (b < B)
          *(u32x4*)(cd.h_seq_lo + ((size_t)t * B + b) * H + j * PL_UNITS + 8 * hf) =
              *(const u32x4*)(ohsl[s] + r * PL_UNITS + 8 * hf);
      }
      if (save_any && t >= cd.save_from) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int r = 4 * q + (lane >> 4), c4 = lane & 15, b = mb * PT_ROWS + r;
          if (b < B)   // og rows are chunk-swizzled (pt_swz64)
            *(f32x4*)(cd.gates + ((size_t)(t - cd.save_from) * B + b) * G + j * PL_GCOLS + 4 * c4) =
                *(const f32x4*)(og[s] + r * PL_GCOLS + (((c4 ^ r) & 15) << 2));
        }
      }
    };
    // x(t) must have landed by barrier t; the 4 DMA loads issued for x(t+2) in step t stay in
    // flight across barrier t+1 (counted wait: vmcnt retires in order, the stores come first).
    // x(0), x(1) were issued before the XCD rendezvous
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_sync();                                   // barrier 0
    for (int t = 0; t < T; ++t) {
      if (t >= 1) io_store(t - 1);
      if (t + 2 < T) {
        io_load_x(t + 2);
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      if (a.dbg && g == 0 && j == 0 && lane == 0 && t + 1 < 32) a.dbg[(t + 1) * 8 + 6] = clock64();
      lds_sync();                                 // barrier t + 1
    }
    io_store(T - 1);
    return;
  }

  // ================= compute waves 0..3
  auto goff = [&](int slot, int r, int p) -> uint32_t {
    return (uint32_t)((((size_t)(chn * 2 + slot) * rows_all + mb * PT_ROWS + r) * GR + p) * 8);
  };
  // T4: byte offset of unit u's word (same ring, 4 B per unit)
  auto woff = [&](int slot, int r, int u_) -> uint32_t {
    return (uint32_t)((((size_t)(chn * 2 + slot) * rows_all + mb * PT_ROWS + r) * H + u_) * 4);
  };
  // pointwise ownership: lane = (row prow, unit 4*wave + pu); c lives in a register
  const int prow = lane >> 2, pu = lane & 3;
  const int ul = 4 * wave + pu, u = j * PL_UNITS + ul;
  const int pb = mb * PT_ROWS + prow;
  const bool pv = pb < B;
  float creg = cd.c0[(size_t)(pv ? pb : B - 1) * H + u];
  // compiler-visible drain of the one-time loads (W_hh fragments, c0): otherwise the waitcnt
  // pass carries them as pending into the loop and waits on vmcnt inside every step -- behind
  // that step's granule store
  __builtin_amdgcn_s_waitcnt(0);
  const bool trace = a.dbg && g == 0 && j == 0 && tid == 0;
#define PT_TRACE(k) \
  if (trace && t < 32) a.dbg[t * 8 + (k)] = clock64();
  if (wst && tid == 0) wst[2] = (long long)__builtin_amdgcn_s_memrealtime();

  for (int t = 0; t < T; ++t) {
    PT_TRACE(0);
    bf16* hb = hin[t & 1];
    bf16* hbl = hinl[t & 1];
    if (t == 0) {
#pragma unroll
      for (int i = 0; i < CH; ++i) {
        const int c = tid + 256 * i, r = c / CPR, cc = c % CPR;
        const int b = min(mb * PT_ROWS + r, B - 1);
        if constexpr (T4) {   // fp32 h0, units 4cc .. 4cc+3 (the T4 chunk geometry)
          const f32x4 x = *(const f32x4*)((const float*)cd.h0 + (size_t)b * H + 4 * cc);
          *(u32x2*)(hb + r * HS + 4 * cc) = u32x2{pt_pack_bf16x2(x[0], x[1]), pt_pack_bf16x2(x[2], x[3])};
          *(u32x2*)(hbl + r * HS + 4 * cc) = u32x2{pt_pack_bf16x2(sp_lo(x[0]), sp_lo(x[1])),
                                                   pt_pack_bf16x2(sp_lo(x[2]), sp_lo(x[3]))};
        } else if constexpr (SP) {   // fp32 h0, units 2cc, 2cc+1
          const float2 x = *(const float2*)((const float*)cd.h0 + (size_t)b * H + 2 * cc);
          *(uint32_t*)(hb + r * HS + 2 * cc) = pt_pack_bf16x2(x.x, x.y);
          *(uint32_t*)(hbl + r * HS + 2 * cc) = pt_pack_bf16x2(sp_lo(x.x), sp_lo(x.y));
        } else {
          *(u32x2*)(hb + r * HS + 4 * cc) = *(const u32x2*)((const bf16*)cd.h0 + (size_t)b * H + 4 * cc);
        }
      }
    } else {
      // h_{t-1}: poll the granules themselves (all CH loads in flight, then re-poll stragglers)
      const unsigned want = T4 ? (((ep & 1u) << 3) | ((unsigned)t & 7u)) : ((ep << 16) | (unsigned)t);
      const int slot = (t - 1) & 1;
      auto ld = [&](int r, int cc) -> u32x4 {   // sc1 poll loads
        return T4 ? __builtin_amdgcn_raw_buffer_load_b128(rrs, woff(slot, r, 4 * cc), 0, 16)
                  : __builtin_amdgcn_raw_buffer_load_b128(rrs, goff(slot, r, 2 * cc), 0, 16);
      };
      u32x4 v[CH];
#pragma unroll
      for (int i = 0; i < CH; ++i) {
        const int c = tid + 256 * i, r = c / CPR, cc = c % CPR;
        v[i] = ld(r, cc);
      }
      // re-poll every stale chunk at once: one round trip per retry round, not one per chunk
      for (unsigned spins = 0;; ++spins) {
        bool all = true;
        bool ok[CH];
#pragma unroll
        for (int i = 0; i < CH; ++i) {
          const int r = (tid + 256 * i) / CPR;
          bool fresh;
          if constexpr (T4)
            fresh = (v[i][0] & 15u) == want && (v[i][1] & 15u) == want && (v[i][2] & 15u) == want &&
                    (v[i][3] & 15u) == want;
          else
            fresh = v[i][1] == want && v[i][3] == want;
          ok[i] = mb * PT_ROWS + r >= B || fresh;
          all = all && ok[i];
        }
        if (all) break;
        if (spins > PL_SPIN_LIMIT) {
          __hip_atomic_store(a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        asm volatile("" ::: "memory");
#pragma unroll
        for (int i = 0; i < CH; ++i) {
          const int c = tid + 256 * i, r = c / CPR, cc = c % CPR;
          if (!ok[i]) v[i] = ld(r, cc);
        }
      }
#pragma unroll
      for (int i = 0; i < CH; ++i) {
        const int c = tid + 256 * i, r = c / CPR, cc = c % CPR;
        if constexpr (T4) {   // 4 tagged words (units 4cc .. 4cc+3) -> hi / lo images
          float f[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) f[e] = __uint_as_float(v[i][e] & ~15u);
          *(u32x2*)(hb + r * HS + 4 * cc) = u32x2{pt_pack_bf16x2(f[0], f[1]), pt_pack_bf16x2(f[2], f[3])};
          *(u32x2*)(hbl + r * HS + 4 * cc) = u32x2{pt_pack_bf16x2(sp_lo(f[0]), sp_lo(f[1])),
                                                   pt_pack_bf16x2(sp_lo(f[2]), sp_lo(f[3]))};
        } else if constexpr (SP) {   // {h[2cc], tag, h[2cc+1], tag} -> hi / lo images
          const f32x4 f = __builtin_bit_cast(f32x4, v[i]);
          *(uint32_t*)(hb + r * HS + 2 * cc) = pt_pack_bf16x2(f[0], f[2]);
          *(uint32_t*)(hbl + r * HS + 2 * cc) = pt_pack_bf16x2(sp_lo(f[0]), sp_lo(f[2]));
        } else {
          *(u32x2*)(hb + r * HS + 4 * cc) = u32x2{v[i][0], v[i][2]};
        }
      }
    }
    PT_TRACE(5);
    lds_sync();                                   // barrier t (with the I/O wave)
    PT_TRACE(1);
    // gates of this wave's 16 columns for the 16 rows: acc[e] = C[4(l>>4)+e][l&15]
    bf16x8 av[KS], avl[SP ? KS : 1];
#pragma unroll
    for (int s = 0; s < KS; ++s) av[s] = *(const bf16x8*)(hb + (lane & 15) * HS + 32 * s + 8 * (lane >> 4));
    if constexpr (SP) {
#pragma unroll
      for (int s = 0; s < KS; ++s) avl[s] = *(const bf16x8*)(hbl + (lane & 15) * HS + 32 * s + 8 * (lane >> 4));
    }
    float xv[4];
    {
      const float* xr = xl[t % 3];
#pragma unroll
      for (int gi = 0; gi < 4; ++gi) xv[gi] = xr[pt_swz64(prow, ul + 16 * gi)];
    }
    // every fragment read issued before the first MFMA: the scheduler otherwise interleaves them
    // just in time and exposes the LDS latency once per k-step pair (7 waits per step)
    __builtin_amdgcn_sched_barrier(0);
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KS; s += 2) {
      if constexpr (SP) {
        acc0 = mfma16_x3(av[s], avl[s], wf[s], wfl[s], acc0);
        if (s + 1 < KS) acc1 = mfma16_x3(av[s + 1], avl[s + 1], wf[s + 1], wfl[s + 1], acc1);
      } else {
        acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[s], wf[s], acc0, 0, 0, 0);
        if (s + 1 < KS) acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[s + 1], wf[s + 1], acc1, 0, 0, 0);
      }
    }
    // wave-private exchange: column c = (gate c>>2, unit c&3) -> xch[row][unit][gate]
    {
      float* xw = xch[wave];
      const int c = lane & 15;
#pragma unroll
      for (int e = 0; e < 4; ++e) xw[(4 * (lane >> 4) + e) * XS + (c & 3) * 4 + (c >> 2)] = acc0[e] + acc1[e];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const f32x4 gp = *(const f32x4*)(xch[wave] + prow * XS + pu * 4);
    PT_TRACE(2);
    const float si = sigmoidf_(gp[0] + xv[0]);
    const float sf = sigmoidf_(gp[1] + xv[1]);
    const float tg = tanhf_(gp[2] + xv[2]);
    const float so = sigmoidf_(gp[3] + xv[3]);
    creg = sf * creg + si * tg;
    const float hv = so * tanhf_(creg);
    PT_TRACE(3);
    if constexpr (T4) {
      // publish h_t: every unit stores one word, h rounded to 19 mantissa bits | 4-bit tag
      if (pv) {
        const uint32_t w = ((__float_as_uint(hv) + 8u) & ~15u) | ((ep & 1u) << 3) | ((unsigned)(t + 1) & 7u);
        const uint32_t off = woff(t & 1, prow, u);
        if (fast) __builtin_amdgcn_raw_buffer_store_b32(w, rrs, off, 0, 0);
        else __builtin_amdgcn_raw_buffer_store_b32(w, rrs, off, 0, 16);
      }
    } else if constexpr (SP) {
      // publish h_t: every unit stores {fp32 h[u], tag}
      if (pv) {
        const u32x2 gr = {__float_as_uint(hv), (ep << 16) | (unsigned)(t + 1)};
        const uint32_t off = goff(t & 1, prow, u);
        if (fast) __builtin_amdgcn_raw_buffer_store_b64(gr, rrs, off, 0, 0);
        else __builtin_amdgcn_raw_buffer_store_b64(gr, rrs, off, 0, 16);
      }
    } else {
      const float hp = __shfl_xor(hv, 1, 64);      // partner unit of the granule
      // publish h_t: even units store {h[u], h[u+1], tag} (one 8-byte store per granule)
      const uint32_t hpair = pt_pack_bf16x2(hv, hp);
      if (pv && (pu & 1) == 0) {
        const u32x2 gr = {hpair, (ep << 16) | (unsigned)(t + 1)};
        const uint32_t off = goff(t & 1, prow, u >> 1);
        if (fast) __builtin_amdgcn_raw_buffer_store_b64(gr, rrs, off, 0, 0);   // stays in the XCD's L2
        else __builtin_amdgcn_raw_buffer_store_b64(gr, rrs, off, 0, 16);       // sc1 write-through
      }
    }
    PT_TRACE(4);
    // outputs of step t for the I/O wave (LDS; drained after barrier t + 1)
    {
      const int s = t & 1;
      oc[s][prow * PL_UNITS + ul] = creg;
      oh32[s][prow * PL_UNITS + ul] = hv;
      ohs[s][prow * PL_UNITS + ul] = (bf16)hv;
      if constexpr (SP) ohsl[s][prow * PL_UNITS + ul] = sp_lo(hv);
      if (save_any) {   // swizzled (pt_swz64): a plain 64-float row stride put a wave on one bank
        float* gq = og[s];
        gq[pt_swz64(prow, ul)] = si;
        gq[pt_swz64(prow, ul + 16)] = sf;
        gq[pt_swz64(prow, ul + 32)] = tg;
        gq[pt_swz64(prow, ul + 48)] = so;
      }
    }
  }
#undef PT_TRACE
  lds_sync();                                     // barrier T: outputs of step T-1 complete
  if (wst && tid == 0) wst[3] = (long long)__builtin_amdgcn_s_memrealtime();
  // the last workgroup to finish advances the epoch (every workgroup read it before any
  // finished) and clears the counters
  if (tid == 0) pt_finish(a.ctr, a.groups, a.groups * NWG, PT_EPOCH_FWD);
}

extern "C" int r2_lstm_tag_ring_bytes(int n_chains, int B, int H) {
  // one unit per 8-byte granule (the split-precision layout; the bf16 kernel uses half of it)
  const long long n = (long long)n_chains * 2 * ((B + PT_ROWS - 1) / PT_ROWS) * PT_ROWS * H * 8;
  return n < (1ll << 31) ? (int)n : -1;
}

// Same chain layout / ctr as r2_lstm_fwd_persist; ring: r2_lstm_tag_ring_bytes bytes.  bf16: any
// content.  Split precision (4-bit tagged words): zero- or (-1)-filled at allocation, and one
// ring + ctr pair per launch site (a fixed chain set), see lstm_fwd_tag_kernel.
// Returns -3 when the grid cannot be co-resident at one workgroup per CU (caller falls back).
template <bool SP>
static int lstm_fwd_tag_launch(const int64_t* chain_ptrs, int words, int n_chains, int B, int T,
                               int H, unsigned* ctr, unsigned* err, void* ring, void* stream) {
  if (n_chains < 1 || n_chains > PL_MAX_CHAINS || B < 1) return -1;
  if (H != 64 && H != 128 && H != 256 && H != 512) return -2;
  if (SP && H > 256) return -2;    // W_hh hi/lo + h hi/lo fragments: 4*H/8 VGPRs
  const int MB = (B + PT_ROWS - 1) / PT_ROWS, nwg = H / PL_UNITS;
  const int groups = n_chains * MB;
  if (groups * nwg > g_num_cus || groups > PL_MAX_GROUPS) return -3;
  if ((size_t)T * B * H * 4 >= (1ull << 32) || T >= 65535 ||
      r2_lstm_tag_ring_bytes(n_chains, B, H) < 0) return -4;
  PTArgs args;
  for (int c = 0; c < n_chains; ++c) {
    const int64_t* p = chain_ptrs + words * c;
    PChain& ch = args.ch[c];
    ch.xproj = (const float*)p[0]; ch.whh = (const bf16*)p[1]; ch.h0 = (const bf16*)p[2];
    ch.c0 = (const float*)p[3]; ch.h_seq = (bf16*)p[4]; ch.c_seq = (float*)p[5];
    ch.h32 = (float*)p[6]; ch.gates = (float*)p[7]; ch.save_from = (int)p[8]; ch.pad_ = 0;
    ch.whh_lo = words > 9 ? (const bf16*)p[9] : nullptr;
    ch.h_seq_lo = words > 10 ? (bf16*)p[10] : nullptr;
    if (SP && (!ch.whh_lo || !ch.h_seq_lo)) return -5;
  }
  args.B = B; args.T = T; args.ctr = ctr; args.err = err; args.dbg = g_pl_dbg; args.ring = ring;
  args.stamps = g_pl_fwd_stamps;
  // group -> XCD placement (workgroup b runs on XCD b % 8): one group per XCD up to 8 groups,
  // two per XCD up to 16 (the fixed-target step's 3 chains x 4 batch tiles = 12 groups), so a
  // group's h hand-off stays in one XCD's L2 (pl_same_xcd: plain stores, L2-hit polls) instead
  // of crossing the fabric with write-through stores
  args.MB = MB; args.groups = groups;
  args.xcd_map = groups <= 8 && nwg <= 32 ? 1 : (groups <= 16 && nwg <= 16 && !g_pl_nomap2 ? 2 : 0);
  if (args.xcd_map && !pl_xcd_fit(args.xcd_map, groups, nwg)) args.xcd_map = 0;
  args.force_slow = g_pl_slow;
  hipStream_t s = (hipStream_t)stream;   // counters are left zeroed by the previous launch
  const int nblk = args.xcd_map == 1 ? 8 * nwg : args.xcd_map == 2 ? 16 * nwg : groups * nwg;
  dim3 grid(nblk), block(320);   // 4 compute waves + 1 I/O wave
  if constexpr (SP) {   // 4-byte tagged-word hand-off (lstm_fwd_tag_kernel T4)
#define PT_T4(HH)                                                                              \
  hipFuncSetAttribute((const void*)lstm_fwd_tag_kernel<HH, true, true>,                       \
                      hipFuncAttributeMaxDynamicSharedMemorySize, PL_LDS_RESERVE);             \
  hipLaunchKernelGGL((lstm_fwd_tag_kernel<HH, true, true>), grid, block, PL_LDS_RESERVE, s, args)
    switch (H) {
      case 64: PT_T4(64); break;
      case 128: PT_T4(128); break;
      default: PT_T4(256); break;
    }
#undef PT_T4
    R2_CHECK_LAUNCH();
    return 0;
  }
  const void* fn = H == 64 ? (const void*)lstm_fwd_tag_kernel<64, false>
                 : H == 128 ? (const void*)lstm_fwd_tag_kernel<128, false>
                 : H == 256 ? (const void*)lstm_fwd_tag_kernel<256, false>
                            : (const void*)lstm_fwd_tag_kernel<512, false>;
  hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, PL_LDS_RESERVE);
  switch (H) {
    case 64: hipLaunchKernelGGL((lstm_fwd_tag_kernel<64, false>), grid, block, PL_LDS_RESERVE, s, args); break;
    case 128: hipLaunchKernelGGL((lstm_fwd_tag_kernel<128, false>), grid, block, PL_LDS_RESERVE, s, args); break;
    case 256: hipLaunchKernelGGL((lstm_fwd_tag_kernel<256, false>), grid, block, PL_LDS_RESERVE, s, args); break;
    default: hipLaunchKernelGGL((lstm_fwd_tag_kernel<512, false>), grid, block, PL_LDS_RESERVE, s, args); break;
  }
  R2_CHECK_LAUNCH();
  return 0;
}

// Same chain layout / ctr as r2_lstm_fwd_persist; ring: r2_lstm_tag_ring_bytes bytes, any content.
// Returns -3 when the grid cannot be co-resident at one workgroup per CU (caller falls back).
extern "C" int r2_lstm_fwd_tag(const int64_t* chain_ptrs, int n_chains, int B, int T, int H,
                               unsigned* ctr, unsigned* err, void* ring, void* stream) {
  return lstm_fwd_tag_launch<false>(chain_ptrs, 9, n_chains, B, T, H, ctr, err, ring, stream);
}

// Split precision: chain_ptrs n_chains x 11 int64 (the 9 above, h0 fp32, + whh_lo, h_seq_lo).
extern "C" int r2_lstm_fwd_tag_sp(const int64_t* chain_ptrs, int n_chains, int B, int T, int H,
                                  unsigned* ctr, unsigned* err, void* ring, void* stream) {
  return lstm_fwd_tag_launch<true>(chain_ptrs, 11, n_chains, B, T, H, ctr, err, ring, stream);
}

// ============================================================================================
// BPTT v3: tagged-granule reduce-scatter of the recurrent dh partials, 16-row batch tiles.
//
//  * group = 16-row batch tile; its H/16 workgroups own 16 units each (pointwise), and 64 packed
//    gate columns each (the partial product dgates_t[:, own 64] @ W_hh[own 64, :] over ALL H
//    units, 4 N tiles of 16 units per wave, K = 64, W_hh^T fragments resident in VGPRs).
//  * partials are published as 8-byte granules {fp32 partial, tag} into a 2-slot ring
//    [slot][source workgroup][row][unit]; a consumer gathers its 16 units from all sources with
//    sc1 b128 loads (2 granules each), re-polls stale ones together, and sums them in source
//    order (deterministic).  Slot reuse: a source publishes iteration k+2's partials only after
//    consuming iteration k+1's from every source, i.e. after every consumer finished iteration k.
//  * an I/O wave prefetches the per-step operands (saved gates, c_t, c_{t-1}, dh_ext) two steps
//    ahead into an LDS ring and drains the dgates tiles; compute waves keep only granule traffic.
struct PTBArgs {
  const float* dh_ext;  // (Tl, B, H) or null
  const float* gates;   // (Tl, B, G) packed post-activation
  const float* c_seq;   // (T, B, H)
  const float* c0;      // (B, H)
  const bf16* whhT;     // packed (NWG, H, 64)
  bf16* dgates;         // (Tl, B, G)
  void* ring;           // (2, NWG, MB*16, H) granules
  int B, T, t0;
  unsigned* ctr;
  unsigned* err;
  int MB, xcd_map, force_slow, pad_;
  // fused LSTM bias gradient (optional): per-tile column sums of dgates -> bias_ws (MB, G), summed
  // in tile order by the last workgroup into db1[perm[c]] (and db2[perm[c]])
  float* bias_ws;
  const int* perm;
  float* db1;
  float* db2;
  // optional side job for the idle workgroups (groups >= MB of the XCD map, i.e. XCDs the
  // recurrence does not use): the dueling head's gradient reduction, (CB x 8) work items
  HeadGradArgs hg;
  int hg_on, hg_wgs;    // hg_wgs: helpers that take head-gradient items (the rest leave at once)
  // optional stop word (r2_lstm_bwd_set_stop): workgroup (0, 0) stores 0 at iteration 0 and 1 at
  // iteration stop_at -- the hoisted target-net torso frames beside this launch (torso_sp.hip
  // qmode 1) stop taking frames then, so they end about when the recurrence does
  unsigned* stop;
  int stop_at, pad2_;
  // split precision (the _sp launcher): W_hh^T lo plane; dgates lo plane out
  const bf16* whhT_lo;
  bf16* dgates_lo;
  // split precision, optional (r2_lstm_bwd_set_dz): the dueling head's input gradient dh_ext =
  // dz . W1 computed HERE instead of read from dh_ext (the TD launch then skips its fused dh, which
  // streamed all of W1^T through every one of its 160 workgroups: 11 us, tools/td_micro.py).  dz
  // (Tl*B, 512) hi / lo planes (time-major learning rows), w1t = W1^T (H, 512) hi / lo planes.
  // dh_ext(t-1) rides on the recurrent hand-off: workgroup j already publishes, at iteration k, its
  // partial of dh_{t-1} over its 64 dgates columns for all H units; it adds dz_{t-1}[:, 32j, +32]
  // . W1[32j, +32][:] to that partial (one 16x16x32 K step, 3 passes, per N tile: W1^T fragments
  // resident, the 16 x 32 dz slice staged with iteration k's operands, 2 KB), so the consumers'
  // sum over the 16 sources is dh_{t-1} + dh_ext(t-1).  Only dh_ext(T-1) (iteration 0, no
  // hand-off) is a full-K product: each wave's K quarter for the 16 units, from 32 KB of dz rows
  // staged once before the loop.
  const bf16* dz;
  const bf16* dz_lo;
  const bf16* w1t;
  const bf16* w1t_lo;
  // per-role clock stamps (r2_lstm_persist_set_debug, probes only): s_memrealtime ticks (100 MHz,
  // one clock for every CU), 8 words per workgroup: [0] start, [1] end of its work, [2] role (1
  // recurrence, 2 helper), [3] ticks spent waiting for dgates rows (helpers), [4] dX tiles done,
  // [5] end of the weight-gradient tile / head-gradient job (helpers); from word 2048: iteration
  // start stamps of recurrence workgroup (0, 0)
  long long* dbg;
};
#define PT_DZ_K 512                                   // dz row length (2 x head hidden 256)
// chunk swizzle of the staged 16 x 32 dz slices: 16-B chunk c of row r at c ^ dzs_f(r).  The
// ds_read_b128 lane groups of the A fragment ({0-3,12-15,20-27}, ...: rows 0-3 and 12-15 at one
// chunk, rows 4-11 at the next) then hit 16 distinct 16-B slots of the 256-B bank row
__device__ __forceinline__ int dzs_f(int r) { return (0x1230 >> (4 * (r >> 2))) & 3; }
#define PT_DZ_SLOT (2 * PT_ROWS * PT_DZ_K * 2)        // 16 dz rows x 512 x hi/lo = 32 KB
#define PT_DZ_LDS PT_DZ_SLOT                          // iteration 0's rows (dynamic LDS)

// SP (split precision, split.h): W_hh^T hi / lo fragments, dgates tile kept as hi / lo images for
// the partial-dh MFMAs (3 passes) and written as hi / lo planes for the weight-gradient GEMMs.
// T4 (every launch; the 8-byte granule form was removed in round 6): each partial travels as ONE 4-byte
// word, fp32 rounded to 19 mantissa bits | 4-bit {epoch parity, (k + 1) mod 8} tag (the forward's
// T4 scheme, lstm_fwd_tag_kernel): half the ring bytes; a consumer wave gathers 4 units x 4 sources
// per 16-B load and the 4 waves split the 16 sources (sums in source order, then wave order).
template <int H, bool SP, bool T4 = false>
__global__ __launch_bounds__(320) void lstm_bwd_tag_kernel(const PTBArgs a) {
  constexpr int G = 4 * H;
  constexpr int NWG = H / PL_UNITS;
  constexpr int NTW = H / 64;                 // 16-unit N tiles per wave (4 waves x 16 x NTW = H)
  constexpr int DS = PL_GCOLS + 16;           // bf16 stride of the dgates tile rows (160 B: 10
                                              // quads = 2 mod 4, conflict-free b128 fragment reads)
  constexpr int SRCH = NWG / 2;               // sources per consumer half
  static_assert(NTW >= 1 && NWG % 2 == 0, "H");
  __shared__ __attribute__((aligned(16))) bf16 dgl[2][PT_ROWS * DS];
  __shared__ __attribute__((aligned(16))) bf16 dgll[2][SP ? PT_ROWS * DS : 8];
  __shared__ __attribute__((aligned(16))) float red[T4 ? 4 : 2][PT_ROWS * PL_UNITS];
  __shared__ __attribute__((aligned(1024))) float gl[3][PT_ROWS * PL_GCOLS];  // saved gates
  __shared__ __attribute__((aligned(1024))) float cl[3][PT_ROWS * PL_UNITS];  // c_t
  __shared__ __attribute__((aligned(1024))) float cpl[3][PT_ROWS * PL_UNITS]; // c_{t-1}
  __shared__ __attribute__((aligned(1024))) float dhl[3][PT_ROWS * PL_UNITS]; // dh_ext
  __shared__ __attribute__((aligned(1024))) bf16 dzsl[3][2][PT_ROWS * 32];    // dz K slices (a.dz)
  __shared__ int flag;
  extern __shared__ __attribute__((aligned(1024))) uint8_t pt_dyn[];   // helper GEMM LDS ring
  int mb, j;
  const int B = a.B, T = a.T, t0 = a.t0, K = T - t0;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  long long* const stamp = a.dbg ? a.dbg + 8 * blockIdx.x : nullptr;
  if (stamp && tid == 0) stamp[0] = (long long)__builtin_amdgcn_s_memrealtime();
  if (!pl_decode(a.xcd_map, a.MB, NWG, mb, j)) {
    // ================= helper workgroup (4 waves): work beside the recurrence
    if (wave == 4) return;                 // helpers run 256 threads (barriers: surviving waves)
    const int b = blockIdx.x, g = b & 7, jj = b >> 3;
    int h;   // helper ordinal: blocks before b that are not recurrence blocks
    if (a.xcd_map == 3) {
      // rows jj < NWG (slot 0) hold recurrence blocks on XCDs x < r0, rows NWG .. 2 NWG - 1
      // (slot 1) on XCDs x < r1 (one fewer when MB is odd), later rows none
      const int r0 = (a.MB + 1) / 2, r1 = a.MB / 2;
      h = jj < NWG ? jj * (8 - r0) + (g - r0)
        : jj < 2 * NWG ? NWG * (8 - r0) + (jj - NWG) * (8 - r1) + (g - r1)
                       : NWG * (16 - r0 - r1) + (jj - 2 * NWG) * 8 + g;
    } else {
      h = b - (min(jj, NWG) * a.MB + (jj < NWG ? min(g, a.MB) : 0));
    }
    const int nh = (int)gridDim.x - a.MB * NWG;
    // the dueling head's gradient reduction (independent of the BPTT) on the first a.hg_wgs
    // helpers; the others leave at once and free their CUs (the hoisted target-net torso frames
    // of the next step run there, engine/learner_engine.py).  Round 5's GEMM helpers (dX / weight
    // gradients on these workgroups) slowed the recurrence in every arm and are gone
    // (profiles/r05_bptt_helpers_roles.txt).
    if (a.hg_on && h < min(nh, a.hg_wgs)) {
      const int nx = min(nh, a.hg_wgs);
      const int cbn = (2 * a.hg.HD + 63) / 64;
      for (int it = h; it < cbn * a.hg.RS * a.hg.NP; it += nx)
        head_grads_body(a.hg, it % cbn, (it / cbn) % a.hg.RS, it / (cbn * a.hg.RS));
    }
    if (stamp && tid == 0) {
      stamp[1] = (long long)__builtin_amdgcn_s_memrealtime();
      stamp[2] = 2;
    }
    if (tid == 0) flag = pt_finish(a.ctr, a.MB, (int)gridDim.x, PT_EPOCH_BWD) ? 1 : 0;
    __syncthreads();
    if (flag && a.bias_ws) {
      for (int c = tid; c < G; c += 256) {
        float v = 0.f;
        for (int m = 0; m < a.MB; ++m)
          v += __hip_atomic_load(a.bias_ws + (size_t)m * G + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int o = a.perm[c];
        a.db1[o] = v;
        if (a.db2) a.db2[o] = v;
      }
    }
    return;
  }
  const int rows_all = a.MB * PT_ROWS;
  const uint32_t ring_bytes = (uint32_t)((size_t)2 * NWG * rows_all * H * 8);
  const __amdgpu_buffer_rsrc_t rrs = pl_rsrc(a.ring, ring_bytes);
  const unsigned ep = __hip_atomic_load(a.ctr + PT_EPOCH_BWD, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // I/O wave operand loads (LDS-DMA into the rings)
  auto io_load = [&](int k) {       // operands of iteration k (step t = T-1-k) into slot k % 3
    const int t = T - 1 - k, tl = t - t0, s = k % 3;
    typedef __attribute__((address_space(3))) void lds_t;
#pragma unroll
    for (int q = 0; q < 4; ++q) {   // gates: 16 rows x 64 fp32, swizzled (pt_swz64)
      const int r = 4 * q + (lane >> 4), b = min(mb * PT_ROWS + r, B - 1);
      __builtin_amdgcn_global_load_lds(a.gates + ((size_t)tl * B + b) * G + j * PL_GCOLS + 4 * ((lane & 15) ^ r),
                                       (lds_t*)(gl[s] + q * 256), 16, 0, 0);
    }
    const int r = lane >> 2, b = min(mb * PT_ROWS + r, B - 1);   // 16-float rows (pt_swz16)
    const size_t hidx = (size_t)b * H + j * PL_UNITS + 4 * ((lane & 3) ^ (r >> 2));
    __builtin_amdgcn_global_load_lds(a.c_seq + (size_t)t * B * H + hidx, (lds_t*)cl[s], 16, 0, 0);
    __builtin_amdgcn_global_load_lds((t == 0 ? a.c0 : a.c_seq + (size_t)(t - 1) * B * H) + hidx,
                                     (lds_t*)cpl[s], 16, 0, 0);
    if (a.dh_ext && !a.dz)
      __builtin_amdgcn_global_load_lds(a.dh_ext + (size_t)tl * B * H + hidx, (lds_t*)dhl[s], 16, 0, 0);
    if (a.dz) {
      // the dz slice of step t-1 (iteration k's publish): 16 rows x 32 K (this workgroup's
      // slice) x hi / lo; row r's 16-B chunk c holds global chunk c ^ dzs_f(r) (conflict-free
      // A-fragment reads); t = t0 has no publish: the previous row stands in
      const int rr = lane >> 2, bb = min(mb * PT_ROWS + rr, B - 1);
      const int tlp = max(tl - 1, 0);
      const size_t o = ((size_t)tlp * B + bb) * PT_DZ_K + 32 * j + 8 * ((lane & 3) ^ dzs_f(rr));
      __builtin_amdgcn_global_load_lds(a.dz + o, (lds_t*)dzsl[s][0], 16, 0, 0);
      __builtin_amdgcn_global_load_lds(a.dz_lo + o, (lds_t*)dzsl[s][1], 16, 0, 0);
    }
  };
  const bool dzon = a.dz != nullptr;
  auto io_load_dz = [&](int k) {    // dz rows of iteration k (only k = 0) -> LDS (32 DMAs)
    typedef __attribute__((address_space(3))) void lds_t;
    const int tl = T - 1 - k - t0;
    uint8_t* slot = pt_dyn;
#pragma unroll
    for (int pl = 0; pl < 2; ++pl)
#pragma unroll
      for (int r = 0; r < PT_ROWS; ++r) {
        // row r: 64 chunks of 16 B; LDS chunk i holds global chunk i ^ r (conflict-free
        // fragment reads of 16 rows at one k)
        const int b = min(mb * PT_ROWS + r, B - 1);
        const bf16* src = (pl ? a.dz_lo : a.dz) + ((size_t)tl * B + b) * PT_DZ_K + 8 * ((lane ^ r) & 63);
        __builtin_amdgcn_global_load_lds(src, (lds_t*)(slot + (pl * PT_ROWS + r) * 1024), 16, 0, 0);
      }
  };
  // the first iterations' operands load under the XCD rendezvous below (its barrier waits for them)
  if (wave == 4) {
    io_load(0);
    if (dzon) io_load_dz(0);
    if (K > 1) io_load(1);
  }
  // compute waves: W_hh^T fragments (loaded under the rendezvous): N tile q of this wave = units
  // (H/4)*wave + 16*q + (l&15); B[k][n] = Whh_pk[j][k][n]
  bf16x8 wt[NTW][2], wtl[SP ? NTW : 1][2];
  if (wave < 4) {
#pragma unroll
    for (int q = 0; q < NTW; ++q) {
      const int n = (H / 4) * wave + 16 * q + (lane & 15);
      const size_t o = ((size_t)j * H + n) * PL_GCOLS + 8 * (lane >> 4);
#pragma unroll
      for (int s = 0; s < 2; ++s) wt[q][s] = *(const bf16x8*)(a.whhT + o + 32 * s);
      if constexpr (SP) {
#pragma unroll
        for (int s = 0; s < 2; ++s) wtl[q][s] = *(const bf16x8*)(a.whhT_lo + o + 32 * s);
      }
    }
  }
  const int fast = pl_same_xcd(a.ctr, mb, NWG, a.force_slow, a.err, &flag);
  if (fast < 0) return;
  if (stamp && tid == 0) stamp[6] = (long long)__builtin_amdgcn_s_memrealtime();   // rendezvous done
  auto goff = [&](int slot, int src, int r, int unit) -> uint32_t {
    return (uint32_t)((((size_t)(slot * NWG + src) * rows_all + mb * PT_ROWS + r) * H + unit) * 8);
  };
  auto woff = [&](int slot, int src, int r, int unit) -> uint32_t {   // T4: 4 B per unit
    return (uint32_t)((((size_t)(slot * NWG + src) * rows_all + mb * PT_ROWS + r) * H + unit) * 4);
  };

  if (wave == 4) {
    // ================= I/O wave
    const int nload = (a.dh_ext && !dzon ? 7 : 6) + (dzon ? 2 : 0);    // DMA instructions per iteration
    const __amdgpu_buffer_rsrc_t drs = pl_rsrc(a.dgates, (uint32_t)((size_t)K * B * G * 2));
    const __amdgpu_buffer_rsrc_t drsl = pl_rsrc(SP ? a.dgates_lo : a.dgates, (uint32_t)((size_t)K * B * G * 2));
    auto io_store = [&](int k) {      // dgates tile of iteration k (write-through: helpers read it)
      const int tl = T - 1 - k - t0, s = k & 1;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int c = lane + 64 * q, r = c >> 3, ch = c & 7, b = mb * PT_ROWS + r;
        if (b < B) {
          const uint32_t off = (uint32_t)((((size_t)tl * B + b) * G + j * PL_GCOLS + 8 * ch) * 2);
          __builtin_amdgcn_raw_buffer_store_b128(*(const u32x4*)(dgl[s] + r * DS + 8 * ch), drs, off, 0, 16);
          if constexpr (SP)
            __builtin_amdgcn_raw_buffer_store_b128(*(const u32x4*)(dgll[s] + r * DS + 8 * ch), drsl, off, 0, 16);
        }
      }
    };
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // iterations 0, 1 (issued before the rendezvous)
    if (dzon) lds_sync();                 // barrier P: dz of iteration 0 landed (compute: dh_ext(0))
    for (int k = 0; k < K; ++k) {
      lds_sync();                         // barrier A_k: operands of k landed
      if (k >= 1) io_store(k - 1);
      const bool more = k + 2 < K;
      if (more) io_load(k + 2);
      lds_sync();                         // barrier B_k
      // operands of k+1 (issued in iteration k-1) must land before barrier A_{k+1}
      if (more) {
        if (nload == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else if (nload == 7) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
    lds_sync();                           // barrier E: dgates of the last iteration complete
    io_store(K - 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {

  // ================= compute waves 0..3
  const int prow = lane >> 2, pu = lane & 3;
  const int ul = 4 * wave + pu;
  const bool pv = mb * PT_ROWS + prow < B;
  float dcr = 0.f;
  float bsum[4] = {0.f, 0.f, 0.f, 0.f};      // this lane's dgates summed over time (bias grad)
  // consumer ownership of the partial gather: (row, unit pair) x source half
  const int cmb = tid & 127, cr = cmb >> 3, cp2 = 2 * (cmb & 7), sh = tid >> 7;
  const bool crow_ok = mb * PT_ROWS + cr < B;
  // T4 ownership: (row, unit quad) x source quarter (= wave)
  constexpr int SRC4 = NWG / 4;
  const int cr4 = lane >> 2, cq4 = 4 * (lane & 3), sq = wave;
  const bool crow4_ok = mb * PT_ROWS + cr4 < B;
  // dh_ext = dz . W1 (a.dz).  Iteration 0: this wave's K quarter [128 wave, +128) of the 16
  // units' W1^T rows (w1f); every publish: K slice [32 j, +32) of W1^T for this wave's NTW N tiles
  // (w1s, B fragments: lane l holds k = 32 j + 8 (l >> 4) .. +7 of unit n)
  const bool dzon = SP && a.dz != nullptr;
  bf16x8 w1f[4], w1fl[4], w1s[NTW], w1sl[NTW];
  if (dzon) {
    const bf16* r1 = a.w1t + (size_t)(j * PL_UNITS + (lane & 15)) * PT_DZ_K + 128 * wave + 8 * (lane >> 4);
    const bf16* r1l = a.w1t_lo + (size_t)(j * PL_UNITS + (lane & 15)) * PT_DZ_K + 128 * wave + 8 * (lane >> 4);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      w1f[s] = *(const bf16x8*)(r1 + 32 * s);
      w1fl[s] = *(const bf16x8*)(r1l + 32 * s);
    }
#pragma unroll
    for (int q = 0; q < NTW; ++q) {
      const size_t o = (size_t)((H / 4) * wave + 16 * q + (lane & 15)) * PT_DZ_K + 32 * j + 8 * (lane >> 4);
      w1s[q] = *(const bf16x8*)(a.w1t + o);
      w1sl[q] = *(const bf16x8*)(a.w1t_lo + o);
    }
  }
  // partial dh_ext of iteration 0 (this wave's K quarter) -> dxp[wave] (read at iteration 0's
  // pointwise, after barrier A_0)
  float* dxp = (float*)(pt_dyn + PT_DZ_LDS);   // [4 waves][16 rows][16 units]
  auto dz_product = [&](int kk) {
    const uint8_t* slot = pt_dyn;
    const int r = lane & 15;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int c = 16 * wave + 4 * s + (lane >> 4);     // 16-B chunk of the 1-KB row
      const int o = r * 1024 + ((c ^ r) & 63) * 16;
      const bf16x8 ah = *(const bf16x8*)(slot + o);
      const bf16x8 al = *(const bf16x8*)(slot + PT_ROWS * 1024 + o);
      acc = mfma16_x3(ah, al, w1f[s], w1fl[s], acc);
    }
    float* d = dxp + wave * (PT_ROWS * PL_UNITS);
#pragma unroll
    for (int e = 0; e < 4; ++e) d[(4 * (lane >> 4) + e) * PL_UNITS + r] = acc[e];
  };
  __builtin_amdgcn_s_waitcnt(0);          // drain the one-time loads (see the forward kernel)
  if (dzon) {
    lds_sync();                           // barrier P: dz of iteration 0 staged
    dz_product(0);
  }

  const bool itrace = a.dbg && mb == 0 && j == 0 && tid == 0;
  if (stamp && tid == 0) stamp[7] = (long long)__builtin_amdgcn_s_memrealtime();   // loop entry
  const bool stopper = a.stop && mb == 0 && j == 0 && tid == 0;
  for (int k = 0; k < K; ++k) {
    const int t = T - 1 - k;
    if (itrace && k < 512) a.dbg[2048 + k] = (long long)__builtin_amdgcn_s_memrealtime();
    if (stopper) {
      if (k == 0) __hip_atomic_store(a.stop, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (k == a.stop_at) __hip_atomic_store(a.stop, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (T4 && k > 0) {
      const unsigned want = ((ep & 1u) << 3) | ((unsigned)k & 7u);
      const int slot = (k - 1) & 1;
      u32x4 v[SRC4];
#pragma unroll
      for (int i = 0; i < SRC4; ++i)
        v[i] = __builtin_amdgcn_raw_buffer_load_b128(rrs, woff(slot, sq * SRC4 + i, cr4, j * PL_UNITS + cq4), 0, 16);
      for (unsigned spins = 0;; ++spins) {
        bool all = true;
        bool ok[SRC4];
#pragma unroll
        for (int i = 0; i < SRC4; ++i) {
          ok[i] = !crow4_ok || ((v[i][0] & 15u) == want && (v[i][1] & 15u) == want &&
                                (v[i][2] & 15u) == want && (v[i][3] & 15u) == want);
          all = all && ok[i];
        }
        if (all) break;
        if (spins > PL_SPIN_LIMIT) {
          __hip_atomic_store(a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        asm volatile("" ::: "memory");
#pragma unroll
        for (int i = 0; i < SRC4; ++i)
          if (!ok[i]) v[i] = __builtin_amdgcn_raw_buffer_load_b128(rrs, woff(slot, sq * SRC4 + i, cr4, j * PL_UNITS + cq4), 0, 16);
      }
      f32x4 sum = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < SRC4; ++i) sum += __builtin_bit_cast(f32x4, v[i] & ~15u);
      *(f32x4*)(red[T4 ? sq : 0] + pt_swz16(cr4, cq4)) = sum;   // read back at o16
    } else if (k > 0) {
      const unsigned want = (ep << 16) | (unsigned)k;
      const int slot = (k - 1) & 1;
      u32x4 v[SRCH];
#pragma unroll
      for (int i = 0; i < SRCH; ++i)
        v[i] = __builtin_amdgcn_raw_buffer_load_b128(rrs, goff(slot, sh * SRCH + i, cr, j * PL_UNITS + cp2), 0, 16);
      for (unsigned spins = 0;; ++spins) {
        bool all = true;
        bool ok[SRCH];
#pragma unroll
        for (int i = 0; i < SRCH; ++i) {
          ok[i] = !crow_ok || (v[i][1] == want && v[i][3] == want);
          all = all && ok[i];
        }
        if (all) break;
        if (spins > PL_SPIN_LIMIT) {
          __hip_atomic_store(a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        asm volatile("" ::: "memory");
#pragma unroll
        for (int i = 0; i < SRCH; ++i)
          if (!ok[i]) v[i] = __builtin_amdgcn_raw_buffer_load_b128(rrs, goff(slot, sh * SRCH + i, cr, j * PL_UNITS + cp2), 0, 16);
      }
      // NOTE: __builtin_bit_cast of single vector ELEMENTS is miscompiled here (ROCm 7.2: every
      // element read as element 0); cast whole vectors, then index
      float s0 = 0.f, s1 = 0.f;
#pragma unroll
      for (int i = 0; i < SRCH; ++i) {
        const f32x4 f = __builtin_bit_cast(f32x4, v[i]);
        s0 += f[0];
        s1 += f[2];
      }
      *(float2*)(red[sh] + cr * PL_UNITS + cp2) = make_float2(s0, s1);
    }
    lds_sync();                           // barrier A_k
    // ---- pointwise (row prow, unit ul)
    const int s3 = k % 3;
    const int o16 = pt_swz16(prow, ul);
    float dh;
    if (dzon) {   // iteration 0: the full-K product; later: inside the hand-off partials
      const float* d = dxp + prow * PL_UNITS + ul;
      dh = k == 0 ? ((d[0] + d[PT_ROWS * PL_UNITS]) + d[2 * PT_ROWS * PL_UNITS]) + d[3 * PT_ROWS * PL_UNITS]
                  : 0.f;
    } else {
      dh = a.dh_ext ? dhl[s3][o16] : 0.f;
    }
    if (k > 0) {
      if constexpr (T4)
        dh += ((red[0][o16] + red[1][o16]) + red[T4 ? 2 : 0][o16]) + red[T4 ? 3 : 0][o16];
      else
        dh += red[0][prow * PL_UNITS + ul] + red[1][prow * PL_UNITS + ul];
    }
    const float* gq = gl[s3];
    const float gi = gq[pt_swz64(prow, ul)], gf = gq[pt_swz64(prow, ul + 16)];
    const float gg = gq[pt_swz64(prow, ul + 32)], go = gq[pt_swz64(prow, ul + 48)];
    const float ct = cl[s3][o16], cpv = cpl[s3][o16];
    const float tc = tanhf_(ct);
    const float dc = dcr + dh * go * (1.f - tc * tc);
    const float d_o = dh * tc;
    dcr = dc * gf;
    const float dgi = pv ? dc * gg * gi * (1.f - gi) : 0.f;
    const float dgf = pv ? dc * cpv * gf * (1.f - gf) : 0.f;
    const float dgg = pv ? dc * gi * (1.f - gg * gg) : 0.f;
    const float dgo = pv ? d_o * go * (1.f - go) : 0.f;
    bsum[0] += dgi;
    bsum[1] += dgf;
    bsum[2] += dgg;
    bsum[3] += dgo;
    bf16* drow = dgl[k & 1] + prow * DS + ul;
    drow[0] = (bf16)dgi;
    drow[16] = (bf16)dgf;
    drow[32] = (bf16)dgg;
    drow[48] = (bf16)dgo;
    if constexpr (SP) {
      bf16* drl = dgll[k & 1] + prow * DS + ul;
      drl[0] = sp_lo(dgi);
      drl[16] = sp_lo(dgf);
      drl[32] = sp_lo(dgg);
      drl[48] = sp_lo(dgo);
    }
    lds_sync();                           // barrier B_k: dgates tile complete
    if (t > t0) {
      // ---- partial dh_{t-1}[r][n] = sum_k dg[r][k] Whh_pk[j][k][n], published as granules
      const bf16* arow = dgl[k & 1] + (lane & 15) * DS + 8 * (lane >> 4);
      const bf16x8 a0 = *(const bf16x8*)arow, a1 = *(const bf16x8*)(arow + 32);
      bf16x8 a0l, a1l;
      if constexpr (SP) {
        const bf16* arl = dgll[k & 1] + (lane & 15) * DS + 8 * (lane >> 4);
        a0l = *(const bf16x8*)arl;
        a1l = *(const bf16x8*)(arl + 32);
      }
      const unsigned tag = (ep << 16) | (unsigned)(k + 1);
      const int slot = k & 1;
      bf16x8 zf, zfl;   // dz_{t-1} slice A fragment (dzon): row l & 15, K chunk l >> 4
      if (dzon) {
        const int zr = lane & 15, zo = zr * 32 + 8 * ((lane >> 4) ^ dzs_f(zr));
        zf = *(const bf16x8*)(dzsl[s3][0] + zo);
        zfl = *(const bf16x8*)(dzsl[s3][1] + zo);
      }
#pragma unroll
      for (int q = 0; q < NTW; ++q) {
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        if constexpr (SP) {
          acc = mfma16_x3(a0, a0l, wt[q][0], wtl[q][0], acc);
          acc = mfma16_x3(a1, a1l, wt[q][1], wtl[q][1], acc);
          if (dzon) acc = mfma16_x3(zf, zfl, w1s[q], w1sl[q], acc);
        } else {
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, wt[q][0], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, wt[q][1], acc, 0, 0, 0);
        }
        const int n = (H / 4) * wave + 16 * q + (lane & 15);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int r = 4 * (lane >> 4) + e;
          if (mb * PT_ROWS + r < B) {
            if constexpr (T4) {
              const uint32_t w = ((__float_as_uint(acc[e]) + 8u) & ~15u) | ((ep & 1u) << 3) |
                                 ((unsigned)(k + 1) & 7u);
              const uint32_t off = woff(slot, j, r, n);
              if (fast) __builtin_amdgcn_raw_buffer_store_b32(w, rrs, off, 0, 0);
              else __builtin_amdgcn_raw_buffer_store_b32(w, rrs, off, 0, 16);
            } else {
              const u32x2 gr = {__float_as_uint(acc[e]), tag};
              const uint32_t off = goff(slot, j, r, n);
              if (fast) __builtin_amdgcn_raw_buffer_store_b64(gr, rrs, off, 0, 0);
              else __builtin_amdgcn_raw_buffer_store_b64(gr, rrs, off, 0, 16);
            }
          }
        }
      }
    }
  }
    if (a.bias_ws) {
      // column sums over the tile's 16 rows (lanes 4r + pu, fixed butterfly order), written
      // write-through by the row-0 lanes and drained before the done ticket
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        float v = bsum[gq];
        v += __shfl_xor(v, 4, 64);
        v += __shfl_xor(v, 8, 64);
        v += __shfl_xor(v, 16, 64);
        v += __shfl_xor(v, 32, 64);
        bsum[gq] = v;
      }
      if (prow == 0) {
#pragma unroll
        for (int gq = 0; gq < 4; ++gq)
          __hip_atomic_store(a.bias_ws + (size_t)mb * G + j * PL_GCOLS + 16 * gq + ul, bsum[gq],
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    lds_sync();                           // barrier E
    if (stamp && tid == 0) {
      stamp[1] = (long long)__builtin_amdgcn_s_memrealtime();
      stamp[2] = 1;
    }
  }
  // ---- every wave (compute and I/O): done ticket; the last workgroup sums the bias partials in
  // tile order and clears the counters
  lds_sync();                             // barrier F: the I/O wave's last stores + progress done
  if (tid == 0) flag = pt_finish(a.ctr, a.MB, (int)gridDim.x, PT_EPOCH_BWD) ? 1 : 0;
  lds_sync();                             // barrier G
  if (flag && a.bias_ws && tid < 256) {
    for (int c = tid; c < G; c += 256) {
      float v = 0.f;
      for (int m = 0; m < a.MB; ++m)
        v += __hip_atomic_load(a.bias_ws + (size_t)m * G + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int o = a.perm[c];
      a.db1[o] = v;
      if (a.db2) a.db2[o] = v;
    }
  }
}

// in-BPTT dh_ext (PTBArgs::dz): operands for the next r2_lstm_bwd_tag_sp* call on this host
// thread; dz / w1t hi / lo planes, row length PT_DZ_K.  The launcher copies and clears them on
// entry, before any check, so a refused call never leaves them armed for a later one.
static thread_local const bf16* g_bwd_dz[4] = {nullptr, nullptr, nullptr, nullptr};
extern "C" int r2_lstm_bwd_set_dz(const bf16* dz, const bf16* dz_lo, const bf16* w1t,
                                  const bf16* w1t_lo, int kd) {
  if (dz && (!dz_lo || !w1t || !w1t_lo || kd != PT_DZ_K)) return -1;
  g_bwd_dz[0] = dz; g_bwd_dz[1] = dz_lo; g_bwd_dz[2] = w1t; g_bwd_dz[3] = w1t_lo;
  return 0;
}
// stop word for the next r2_lstm_bwd_tag* call on this host thread (PTBArgs::stop), and the number
// of helpers that take head-gradient items (0 = all of them); consumed (cleared) on entry like dz
static thread_local unsigned* g_bwd_stop = nullptr;
static thread_local int g_bwd_stop_at = 0, g_bwd_hg_wgs = 0;
extern "C" int r2_lstm_bwd_set_stop(unsigned* stop, int stop_at, int hg_wgs) {
  if (stop_at < 0 || hg_wgs < 0) return -1;
  g_bwd_stop = stop;
  g_bwd_stop_at = stop_at;
  g_bwd_hg_wgs = hg_wgs;
  return 0;
}

// BPTT placement: 1 = recurrence groups packed two per XCD (PTBArgs xcd_map 3), 0 = one per XCD
static int g_bwd_pairs = 0;
extern "C" int r2_lstm_bwd_xcd_pairs(int v) { g_bwd_pairs = v; return 0; }

extern "C" int r2_lstm_bwd_tag_ring_bytes(int B, int H) {
  const long long n = 2ll * (H / PL_UNITS) * ((B + PT_ROWS - 1) / PT_ROWS) * PT_ROWS * H * 8;
  return n < (1ll << 31) ? (int)n : -1;
}

// Same operands as r2_lstm_bwd_persist minus the slab; ring: r2_lstm_bwd_tag_ring_bytes bytes,
// zero- or (-1)-filled at allocation and one ring + ctr per launch site (the 4-bit tags of the
// T4 hand-off, see lstm_fwd_tag_kernel).  -3: grid too large for one workgroup per CU (caller falls back).
// 1 when the launch's idle workgroups can take the dueling head's gradient reduction (head
// width HD): the XCD map leaves (8 - MB) * H/16 workgroups free and the job needs (2HD/64) x 8.
extern "C" int r2_lstm_bwd_tag_hg_ok(int B, int H, int HD) {
  const int MB = (B + PT_ROWS - 1) / PT_ROWS, nwg = H / PL_UNITS;
  const bool xmap = MB <= 8 && nwg <= 32 && pl_xcd_fit(1, MB, nwg, true);
  return (xmap && HD % 64 == 0 && (8 - MB) * nwg >= ((2 * HD + 63) / 64) * 8) ? 1 : 0;
}

// hg_*: optional head-gradient job (gradsum.hip r2_head_grads operands); pass dva = null for none,
// and only when r2_lstm_bwd_tag_hg_ok(B, H, HD).  Returns bit 0 = head gradients done here.
static int lstm_bwd_tag_launch(const float* dh_ext, const float* gates, const float* c_seq,
                               const float* c0, const bf16* whhT, const bf16* whhT_lo, bf16* dgates,
                               bf16* dgates_lo, int B, int T, int t0, int H, unsigned* ctr,
                               unsigned* err, void* ring, float* bias_ws, const int* perm, float* db1,
                               float* db2, const float* hg_dva, const bf16* hg_zr,
                               const float* hg_zr32, const bf16* hg_dz, const bf16* hg_dz_lo,
                               float* hg_gw2, float* hg_gb2, float* hg_gb1, int hg_N, int hg_A,
                               int hg_HD, float* hg_ws, unsigned* hg_ticket, void* stream) {
  // host-thread state of this call (set_dz / set_stop), cleared before any check
  const bf16* dz[4] = {g_bwd_dz[0], g_bwd_dz[1], g_bwd_dz[2], g_bwd_dz[3]};
  for (int i = 0; i < 4; ++i) g_bwd_dz[i] = nullptr;
  unsigned* const stop = g_bwd_stop;
  const int stop_at = g_bwd_stop_at, hg_wgs = g_bwd_hg_wgs;
  g_bwd_stop = nullptr;
  g_bwd_stop_at = g_bwd_hg_wgs = 0;
  if (B < 1 || T < 1 || t0 < 0 || t0 >= T) return -1;
  if (H != 64 && H != 128 && H != 256 && H != 512) return -2;
  const int MB = (B + PT_ROWS - 1) / PT_ROWS, nwg = H / PL_UNITS;
  if (MB * nwg > g_num_cus || MB > PL_MAX_GROUPS) return -3;
  if ((size_t)T * B * (size_t)(4 * H) * 4 >= (1ull << 32) || r2_lstm_bwd_tag_ring_bytes(B, H) < 0 ||
      T - t0 >= 65535) return -4;
  // map 3 (r2_lstm_bwd_xcd_pairs): the recurrence packed two groups per XCD, else one per XCD
  int xmap = MB <= 8 && nwg <= 32 && pl_xcd_fit(1, MB, nwg) ? 1 : 0;
  if (g_bwd_pairs && MB <= 16 && 2 * nwg <= 32 && pl_xcd_fit(3, MB, nwg, true)) xmap = 3;
  if (bias_ws && (!perm || !db1)) return -1;
  const bool sp = whhT_lo != nullptr;
  if (sp && (!dgates_lo || H > 256)) return -11;
  PTBArgs args{dh_ext, gates, c_seq, c0, whhT, dgates, ring, B, T, t0, ctr, err, MB, xmap, g_pl_slow, 0,
               bias_ws, perm, db1, db2,
               HeadGradArgs{hg_dva, hg_zr, hg_dz, hg_gw2, hg_gb2, hg_gb1, hg_ws, hg_ticket, hg_N, hg_A,
                            hg_HD, 8, (hg_A + 6) / 7, hg_zr32, hg_dz_lo},
               0, 0};
  args.stop = stop;
  args.stop_at = stop_at;
  args.dbg = g_pl_dbg;
  int taken = 0, nh = 0;
  if (hg_dva) {
    // helpers: every block of the 8 x 32 grid outside the recurrence's groups
    if (!xmap || nwg > 32 || !pl_xcd_fit(xmap, MB, nwg, true)) return -6;
    nh = 8 * 32 - MB * nwg;
    if (nh < 16) return -10;   // too few helpers
    if (hg_A > 63 || ((2 * hg_HD + 63) / 64) * ((hg_A + 6) / 7) > 32 || hg_N < 1 || hg_HD % 64)
      return -5;
    if (sp && (!hg_zr32 || !hg_dz_lo)) return -12;
    args.hg_on = 1;
    args.hg_wgs = hg_wgs > 0 ? min(hg_wgs, nh) : nh;
    // row splits: one item per head-gradient helper (8 column blocks x NP passes x RS), so the
    // helpers finish early and free their CUs (RS 8 left 64 helpers on 320-row items until ~55 us)
    const int cbn = (2 * hg_HD + 63) / 64;
    args.hg.RS = max(1, min(32, args.hg_wgs / (cbn * args.hg.NP)));
    taken |= 1;
  }
  args.whhT_lo = whhT_lo;
  args.dgates_lo = dgates_lo;
  args.dz = dz[0]; args.dz_lo = dz[1]; args.w1t = dz[2]; args.w1t_lo = dz[3];
  if (args.dz && (!sp || H != 256)) return -13;   // split-precision T4 BPTT, H 256 only
  // one workgroup per CU (the PL_LDS_RESERVE rule, comment at its definition): the dz path's
  // dynamic LDS (iteration 0's dz rows + the dh partials, 36 KB) plus the kernel's 54 KB of static
  // LDS (LDS_Block_Size in the rocprofv3 trace) is 90 KB > 80 KB, so two workgroups never share a
  // CU either way; reserving the full 84 KB there as well measured +7 us per BPTT (97 -> 104 us)
  const int dyn_lds = args.dz ? PT_DZ_LDS + 4 * PT_ROWS * PL_UNITS * 4 : PL_LDS_RESERVE;
  static_assert(PT_DZ_LDS + 4 * PT_ROWS * PL_UNITS * 4 + 48 * 1024 > 80 * 1024, "1 WG per CU");
  hipStream_t s = (hipStream_t)stream;   // counters are left zeroed by the previous launch
  dim3 grid(nh ? 256 : (xmap == 3 ? 16 * nwg : xmap ? 8 * nwg : MB * nwg)), block(320);
#define R2_BWD_LAUNCH1(HH, SPP, T4)                                                            \
  do {                                                                                         \
    hipFuncSetAttribute((const void*)lstm_bwd_tag_kernel<HH, SPP, T4>,                         \
                        hipFuncAttributeMaxDynamicSharedMemorySize, dyn_lds);                  \
    hipLaunchKernelGGL((lstm_bwd_tag_kernel<HH, SPP, T4>), grid, block, dyn_lds, s, args);     \
  } while (0)
#define R2_BWD_LAUNCH(HH, SPP) R2_BWD_LAUNCH1(HH, SPP, true)
  if (sp) {
    switch (H) {
      case 64: R2_BWD_LAUNCH(64, true); break;
      case 128: R2_BWD_LAUNCH(128, true); break;
      default: R2_BWD_LAUNCH(256, true); break;
    }
  } else {
    switch (H) {
      case 64: R2_BWD_LAUNCH(64, false); break;
      case 128: R2_BWD_LAUNCH(128, false); break;
      case 256: R2_BWD_LAUNCH(256, false); break;
      default: R2_BWD_LAUNCH(512, false); break;
    }
  }
#undef R2_BWD_LAUNCH
#undef R2_BWD_LAUNCH1
  R2_CHECK_LAUNCH();
  return taken;
}

extern "C" int r2_lstm_bwd_tag(const float* dh_ext, const float* gates, const float* c_seq,
                               const float* c0, const bf16* whhT, bf16* dgates, int B, int T,
                               int t0, int H, unsigned* ctr, unsigned* err, void* ring,
                               float* bias_ws, const int* perm, float* db1, float* db2,
                               const float* hg_dva, const bf16* hg_zr, const bf16* hg_dz,
                               float* hg_gw2, float* hg_gb2, float* hg_gb1, int hg_N, int hg_A,
                               int hg_HD, float* hg_ws, unsigned* hg_ticket, void* stream) {
  return lstm_bwd_tag_launch(dh_ext, gates, c_seq, c0, whhT, nullptr, dgates, nullptr, B, T, t0, H,
                             ctr, err, ring, bias_ws, perm, db1, db2, hg_dva, hg_zr, nullptr, hg_dz,
                             nullptr, hg_gw2, hg_gb2, hg_gb1, hg_N, hg_A, hg_HD, hg_ws, hg_ticket,
                             stream);
}

// Split precision: the same launch with W_hh^T given as hi / lo planes and dgates written as hi /
// lo planes (no side job).  Same argument list as r2_lstm_bwd_tag plus the two lo pointers.
extern "C" int r2_lstm_bwd_tag_sp(const float* dh_ext, const float* gates, const float* c_seq,
                                  const float* c0, const bf16* whhT, const bf16* whhT_lo,
                                  bf16* dgates, bf16* dgates_lo, int B, int T, int t0, int H,
                                  unsigned* ctr, unsigned* err, void* ring, float* bias_ws,
                                  const int* perm, float* db1, float* db2, void* stream) {
  if (!whhT_lo || !dgates_lo) return -5;
  return lstm_bwd_tag_launch(dh_ext, gates, c_seq, c0, whhT, whhT_lo, dgates, dgates_lo, B, T, t0, H,
                             ctr, err, ring, bias_ws, perm, db1, db2, nullptr, nullptr, nullptr,
                             nullptr, nullptr, nullptr, nullptr, nullptr, 0, 0, 0, nullptr, nullptr,
                             stream);
}

// Split precision with the dueling head's gradient reduction on the launch's idle workgroups
// (r2_head_grads_sp operands; only when r2_lstm_bwd_tag_hg_ok(B, H, HD)).  Returns the
// r2_lstm_bwd_tag bit mask: bit 0 set = the head gradients were produced here.
extern "C" int r2_lstm_bwd_tag_sp_hg(const float* dh_ext, const float* gates, const float* c_seq,
                                     const float* c0, const bf16* whhT, const bf16* whhT_lo,
                                     bf16* dgates, bf16* dgates_lo, int B, int T, int t0, int H,
                                     unsigned* ctr, unsigned* err, void* ring, float* bias_ws,
                                     const int* perm, float* db1, float* db2, const float* hg_dva,
                                     const float* hg_zr32, const bf16* hg_dz, const bf16* hg_dz_lo,
                                     float* hg_gw2, float* hg_gb2, float* hg_gb1, int hg_N, int hg_A,
                                     int hg_HD, float* hg_ws, unsigned* hg_ticket, void* stream) {
  if (!whhT_lo || !dgates_lo || !hg_zr32 || !hg_dz_lo) return -5;
  return lstm_bwd_tag_launch(dh_ext, gates, c_seq, c0, whhT, whhT_lo, dgates, dgates_lo, B, T, t0, H,
                             ctr, err, ring, bias_ws, perm, db1, db2, hg_dva, nullptr, hg_zr32, hg_dz,
                             hg_dz_lo, hg_gw2, hg_gb2, hg_gb1, hg_N, hg_A, hg_HD, hg_ws, hg_ticket,
                             stream);
}

extern "C" int r2_lstm_persist_ctr_words() { return PT_CTR_WORDS; }

// ---- placement probe (tools / tests): XCC id of every block of a launch
__global__ void xcc_probe_kernel(int* out, int spin) {
  if (threadIdx.x == 0) {
    unsigned x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    out[blockIdx.x] = (int)(x & 15);
  }
  if (spin) __builtin_amdgcn_s_sleep(100);
}

extern "C" int r2_xcc_probe(int* out, int nblocks, int threads, int lds_bytes, void* stream) {
  if (lds_bytes > 0)
    hipFuncSetAttribute((const void*)xcc_probe_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                        lds_bytes);
  hipLaunchKernelGGL(xcc_probe_kernel, dim3(nblocks), dim3(threads), lds_bytes,
                     (hipStream_t)stream, out, 1);
  R2_CHECK_LAUNCH();
  return 0;
}
