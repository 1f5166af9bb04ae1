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
#include "../lstm_common.h"

// (The tagged BPTT kernel lives in lstm_bptt.hip.)

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
  if (a.dbg && tid == 0) {   // placement record (tests: every group on the same-XCD path)
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

  const bool trace = PL_PROBE(a.dbg) && g == 0 && j == 0 && tid == 0;
#define PL_TRACE(k) \
  if (trace && t < 32) PL_PROBE(a.dbg)[t * 8 + (k)] = clock64();
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


static long long* g_pl_fwd_stamps = nullptr;   // tagged forward: >= 4 x grid words
extern "C" int r2_lstm_fwd_set_stamps(long long* p) { g_pl_fwd_stamps = p; return 0; }

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
  long long* const wst = PL_PROBE(a.stamps) ? a.stamps + 4 * blockIdx.x : nullptr;
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
  if (a.dbg && tid == 0) {   // placement record (tests: every group on the same-XCD path)
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
      if (PL_PROBE(a.dbg) && g == 0 && j == 0 && lane == 0 && t + 1 < 32) PL_PROBE(a.dbg)[(t + 1) * 8 + 6] = clock64();
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
  const bool trace = PL_PROBE(a.dbg) && g == 0 && j == 0 && tid == 0;
#define PT_TRACE(k) \
  if (trace && t < 32) PL_PROBE(a.dbg)[t * 8 + (k)] = clock64();
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

extern "C" int r2_lstm_persist_ctr_words() { return PT_CTR_WORDS; }
// 1 when this library was built with the clock-stamp hooks (R2D2_PROBES=1, lstm_common.h)
extern "C" int r2_lstm_probes() { return R2_LSTM_PROBES; }

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
