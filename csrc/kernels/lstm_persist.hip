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
// No placement / dispatch-order assumption; counters are zeroed by a memset node before every
// launch; every spin is bounded and reports through an error word instead of hanging.
// All (H/16)*ceil(B/32)*chains workgroups (<= 256 for the supported shapes) must be
// co-resident: 256 threads, <= 40 KB LDS, one per CU is enough.
#include "../common.h"

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
#define PL_CTR_WORDS (PL_MAX_CHAINS * 8 * PL_CTR_STRIDE)

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
};

struct PFwdArgs {
  PChain ch[PL_MAX_CHAINS];
  int B, T;
  unsigned* ctr;  // (n_chains, MB) arrival counters, zeroed before launch
  unsigned* err;  // error word (nonzero = a spin timed out)
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t pl_rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, 0, bytes, 0x00020000);
}

// one lane waits until *ctr >= target; result broadcast through LDS; bounded
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
  __syncthreads();
  return *flag_lds != 0;
}

template <int H>
__global__ __launch_bounds__(256) void lstm_fwd_persist_kernel(const PFwdArgs a) {
  constexpr int G = 4 * H;
  constexpr int KS = H / 16;
  constexpr int KH = KS / 2;           // k-steps per wave (K split across wave pairs)
  constexpr int PW = PL_GCOLS + 4;     // fp32 row stride of the partial-gate tiles
  __shared__ float part[2][32 * PW];
  __shared__ __attribute__((aligned(16))) bf16 hst[32 * PL_UNITS];
  __shared__ int flag;
  const PChain& cd = a.ch[blockIdx.z];
  const int j = blockIdx.x, mb = blockIdx.y, MB = gridDim.y;
  const int B = a.B, T = a.T;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int nt = wave & 1, kq = wave >> 1;
  unsigned* ctr = a.ctr + (blockIdx.z * MB + mb) * PL_CTR_STRIDE;
  const uint32_t hbytes = (uint32_t)((size_t)T * B * H * sizeof(bf16));
  const __amdgpu_buffer_rsrc_t hrs = pl_rsrc(cd.h_seq, hbytes);

  // ---- resident W_hh fragments: B[k][n] = Whh_pk[j][nt*32 + n][k], k-steps kq*KH .. +KH
  bf16x8 wf[KH];
  {
    const bf16* brow = cd.whh + ((size_t)j * PL_GCOLS + nt * 32 + (lane & 31)) * H +
                       kq * KH * 16 + (lane >> 5) * 8;
#pragma unroll
    for (int s = 0; s < KH; ++s) wf[s] = *(const bf16x8*)(brow + s * 16);
  }
  // ---- pointwise ownership: 2 (row, unit) items per thread; c lives in registers
  int pb[2], pu[2];
  bool pv[2];
  float creg[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int idx = tid + q * 256;
    pu[q] = idx & 15;
    pb[q] = mb * 32 + (idx >> 4);
    pv[q] = pb[q] < B;
    const int bc = pv[q] ? pb[q] : B - 1;
    creg[q] = cd.c0[(size_t)bc * H + j * PL_UNITS + pu[q]];
  }
  const int arow = min(mb * 32 + (lane & 31), B - 1);
  const int acol = kq * KH * 16 + (lane >> 5) * 8;

  for (int t = 0; t < T; ++t) {
    // x-projection of this step (plain loads: written by an earlier kernel)
    float xv[2][4];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int bc = pv[q] ? pb[q] : B - 1;
      const float* xr = cd.xproj + ((size_t)t * B + bc) * G + j * PL_GCOLS + pu[q];
      xv[q][0] = xr[0]; xv[q][1] = xr[16]; xv[q][2] = xr[32]; xv[q][3] = xr[48];
    }
    bf16x8 av[KH];
    if (t == 0) {
      const bf16* hp = cd.h0 + (size_t)arow * H + acol;
#pragma unroll
      for (int s = 0; s < KH; ++s) av[s] = *(const bf16x8*)(hp + s * 16);
    } else {
      if (!pl_wait(ctr, (unsigned)(H / PL_UNITS) * (unsigned)t, a.err, &flag)) return;
      const uint32_t off = (uint32_t)((((size_t)(t - 1) * B + arow) * H + acol) * sizeof(bf16));
#pragma unroll
      for (int s = 0; s < KH; ++s) {
        u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(hrs, off + s * 32, 0, 16);  // sc1
        av[s] = __builtin_bit_cast(bf16x8, v);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    f32x16 acc = {};
#pragma unroll
    for (int s = 0; s < KH; ++s) acc = mfma32(av[s], wf[s], acc);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      part[kq][row * PW + nt * 32 + (lane & 31)] = acc[r];
    }
    __syncthreads();
    const bool save = cd.gates != nullptr && t >= cd.save_from;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int rl = (tid + q * 256) >> 4, u = pu[q];
      const float* p0 = part[0] + rl * PW;
      const float* p1 = part[1] + rl * PW;
      const float gi = sigmoidf_(p0[u] + p1[u] + xv[q][0]);
      const float gf = sigmoidf_(p0[16 + u] + p1[16 + u] + xv[q][1]);
      const float gg = tanhf_(p0[32 + u] + p1[32 + u] + xv[q][2]);
      const float go = sigmoidf_(p0[48 + u] + p1[48 + u] + xv[q][3]);
      creg[q] = gf * creg[q] + gi * gg;
      const float h = go * tanhf_(creg[q]);
      hst[rl * PL_UNITS + u] = (bf16)h;
      if (pv[q]) {
        const size_t o = ((size_t)t * B + pb[q]) * H + j * PL_UNITS + u;
        cd.c_seq[o] = creg[q];
        if (cd.h32) cd.h32[o] = h;
        if (save) {
          float* gp = cd.gates + ((size_t)(t - cd.save_from) * B + pb[q]) * G + j * PL_GCOLS + u;
          gp[0] = gi; gp[16] = gf; gp[32] = gg; gp[48] = go;
        }
      }
    }
    __syncthreads();
    // ---- publish h_t slice: wave 0 stores 32 rows x 32 B write-through, drains, signals
    if (wave == 0) {
      const int rl = lane >> 1, hf = lane & 1;
      const int b = mb * 32 + rl;
      if (b < B) {
        const u32x4 v = *(const u32x4*)(hst + rl * PL_UNITS + hf * 8);
        const uint32_t off = (uint32_t)((((size_t)t * B + b) * H + j * PL_UNITS + hf * 8) * sizeof(bf16));
        __builtin_amdgcn_raw_buffer_store_b128(v, hrs, off, 0, 16);  // sc1
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
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
  unsigned* ctr;        // (MB) zeroed before launch
  unsigned* err;
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
  const int j = blockIdx.x, mb = blockIdx.y;
  const int B = a.B, T = a.T, t0 = a.t0;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  unsigned* ctr = a.ctr + mb * PL_CTR_STRIDE;
  const uint32_t sbytes = (uint32_t)((size_t)2 * NWG * B * H * sizeof(float));
  const __amdgpu_buffer_rsrc_t srs = pl_rsrc(a.slab, sbytes);

  // ---- resident W_hh^T fragments for phase B: B[k][n] = Whh_pk[j][k][n] = whhT[j][n][k]
  bf16x8 wt[TPW][4];
#pragma unroll
  for (int q = 0; q < TPW; ++q) {
    const int ntl = min(wave + q * 4, NT32 - 1);
    const bf16* brow = a.whhT + ((size_t)j * H + ntl * 32 + (lane & 31)) * PL_GCOLS + (lane >> 5) * 8;
#pragma unroll
    for (int s = 0; s < 4; ++s) wt[q][s] = *(const bf16x8*)(brow + s * 16);
  }
  int pb[2], pu[2];
  bool pv[2];
  float dcr[2] = {0.f, 0.f};
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int idx = tid + q * 256;
    pu[q] = idx & 15;
    pb[q] = mb * 32 + (idx >> 4);
    pv[q] = pb[q] < B;
  }
  // slab-reduction ownership: (row, float4 group) pairs, two threads per pair split producers
  const int rr = (tid & 127) >> 2, u4 = tid & 3, hh = tid >> 7;
  const int rb = min(mb * 32 + rr, B - 1);

  for (int t = T - 1, k = 0; t >= t0; --t, ++k) {
    const int tl = t - t0;
    // independent operands first
    float dhv[2], gv[2][4], ctv[2], cpv[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int bc = pv[q] ? pb[q] : B - 1;
      const size_t hidx = (size_t)bc * H + j * PL_UNITS + pu[q];
      dhv[q] = a.dh_ext ? a.dh_ext[(size_t)tl * B * H + hidx] : 0.f;
      const float* gp = a.gates + ((size_t)tl * B + bc) * G + j * PL_GCOLS + pu[q];
      gv[q][0] = gp[0]; gv[q][1] = gp[16]; gv[q][2] = gp[32]; gv[q][3] = gp[48];
      ctv[q] = a.c_seq[(size_t)t * B * H + hidx];
      cpv[q] = (t == 0) ? a.c0[hidx] : a.c_seq[(size_t)(t - 1) * B * H + hidx];
    }
    // recurrent partials from step t+1 (written by the NWG workgroups of this batch tile)
    if (k > 0) {
      if (!pl_wait(ctr, (unsigned)NWG * (unsigned)k, a.err, &flag)) return;
      const int slot = (k - 1) & 1;
      f32x4 sum = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = hh; i < NWG; i += 2) {
        const uint32_t off = (uint32_t)((((size_t)(slot * NWG + i) * B + rb) * H + j * PL_UNITS + u4 * 4) * sizeof(float));
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(srs, off, 0, 16);  // sc1
        sum += __builtin_bit_cast(f32x4, v);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) red[hh][rr * PL_UNITS + u4 * 4 + e] = sum[e];
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int rl = (tid + q * 256) >> 4, u = pu[q];
      float dh = dhv[q];
      if (k > 0) dh += red[0][rl * PL_UNITS + u] + red[1][rl * PL_UNITS + u];
      const float gi = gv[q][0], gf = gv[q][1], gg = gv[q][2], go = gv[q][3];
      const float tc = tanhf_(ctv[q]);
      const float dc = dcr[q] + dh * go * (1.f - tc * tc);
      const float d_o = dh * tc;
      const float d_i = dc * gg, d_g = dc * gi, d_f = dc * cpv[q];
      dcr[q] = dc * gf;
      const bf16 bi = (bf16)(d_i * gi * (1.f - gi));
      const bf16 bfv = (bf16)(d_f * gf * (1.f - gf));
      const bf16 bg = (bf16)(d_g * (1.f - gg * gg));
      const bf16 bo = (bf16)(d_o * go * (1.f - go));
      bf16* lrow = dg + rl * DW;
      const bool ok = pv[q];
      lrow[u] = ok ? bi : (bf16)0.f;
      lrow[16 + u] = ok ? bfv : (bf16)0.f;
      lrow[32 + u] = ok ? bg : (bf16)0.f;
      lrow[48 + u] = ok ? bo : (bf16)0.f;
      if (ok) {
        bf16* dgo = a.dgates + ((size_t)tl * B + pb[q]) * G + j * PL_GCOLS + u;
        dgo[0] = bi; dgo[16] = bfv; dgo[32] = bg; dgo[48] = bo;
      }
    }
    if (t == t0) break;  // dh into the stored initial state is not needed
    __syncthreads();
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
    __syncthreads();
    // write-through store of the 32 x H fp32 slab (rows < B), 16 B per lane, then signal
    {
      const int slot = k & 1;
      constexpr int C4 = H / 4;  // float4 per row
      for (int c = tid; c < 32 * C4; c += 256) {
        const int r = c / C4, col = (c % C4) * 4;
        const int b = mb * 32 + r;
        if (b < B) {
          const u32x4 v = *(const u32x4*)(pst + r * PS + col);
          const uint32_t off = (uint32_t)((((size_t)(slot * NWG + j) * B + b) * H + col) * sizeof(float));
          __builtin_amdgcn_raw_buffer_store_b128(v, srs, off, 0, 16);  // sc1
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// chain_ptrs: n_chains x 9 int64 (same layout as r2_lstm_fwd).  ctr: >= PL_CTR_WORDS (1024) unsigned,
// err: 1 unsigned.  Both are zeroed here with memset nodes (graph-capturable).
extern "C" int r2_lstm_fwd_persist(const int64_t* chain_ptrs, int n_chains, int B, int T, int H,
                                   unsigned* ctr, unsigned* err, void* stream) {
  if (n_chains < 1 || n_chains > PL_MAX_CHAINS || B < 1 || B > 256) return -1;
  if (H != 64 && H != 128 && H != 256 && H != 512) return -2;
  const int MB = (B + 31) / 32;
  if ((H / PL_UNITS) * MB * n_chains > 256 || MB > 8) return -3;  // co-resident, 1 WG per CU
  if ((size_t)T * B * H * 2 >= (1ull << 32)) return -4;
  PFwdArgs args;
  for (int c = 0; c < n_chains; ++c) {
    const int64_t* p = chain_ptrs + 9 * c;
    PChain& ch = args.ch[c];
    ch.xproj = (const float*)p[0]; ch.whh = (const bf16*)p[1]; ch.h0 = (const bf16*)p[2];
    ch.c0 = (const float*)p[3]; ch.h_seq = (bf16*)p[4]; ch.c_seq = (float*)p[5];
    ch.h32 = (float*)p[6]; ch.gates = (float*)p[7]; ch.save_from = (int)p[8]; ch.pad_ = 0;
  }
  args.B = B; args.T = T; args.ctr = ctr; args.err = err;
  hipStream_t s = (hipStream_t)stream;
  hipMemsetAsync(ctr, 0, PL_CTR_WORDS * sizeof(unsigned), s);
  dim3 grid(H / PL_UNITS, MB, n_chains), block(256);
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
  if ((H / PL_UNITS) * MB > 256 || MB > 8) return -3;
  if ((size_t)2 * (H / PL_UNITS) * B * H * 4 >= (1ull << 32)) return -4;
  PBwdArgs a{dh_ext, gates, c_seq, c0, whhT, slab, dgates, B, T, t0, ctr, err};
  hipStream_t s = (hipStream_t)stream;
  hipMemsetAsync(ctr, 0, PL_CTR_WORDS * sizeof(unsigned), s);
  dim3 grid(H / PL_UNITS, MB), block(256);
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

extern "C" int r2_lstm_persist_ctr_words() { return PL_CTR_WORDS; }
