// Persistent tagged BPTT of the LSTM (gfx950, MI355X): the backward counterpart of
// lstm_persist.hip's tagged forward (shared protocol pieces: csrc/lstm_common.h).  Reference
// semantics: the LSTM of /root/reference/model.py:48-60 differentiated by learner.py:118-120.
#include "../common.h"
#include "../split.h"
#include "../gradsum.h"
#include "../lstm_common.h"

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
  long long* const stamp = PL_PROBE(a.dbg) ? PL_PROBE(a.dbg) + 8 * blockIdx.x : nullptr;
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

  const bool itrace = PL_PROBE(a.dbg) && mb == 0 && j == 0 && tid == 0;
  if (stamp && tid == 0) stamp[7] = (long long)__builtin_amdgcn_s_memrealtime();   // loop entry
  const bool stopper = a.stop && mb == 0 && j == 0 && tid == 0;
  for (int k = 0; k < K; ++k) {
    const int t = T - 1 - k;
    if (itrace && k < 512) PL_PROBE(a.dbg)[2048 + k] = (long long)__builtin_amdgcn_s_memrealtime();
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

