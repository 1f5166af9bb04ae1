// Fused split-precision GEMM (gfx950): C = A.B with A, B given as bf16 hi / lo planes
// (split.h) and ALL THREE products taken from ONE pass over K.
//
// The round-1 split path (gemm.hip gemm4 / gemm_group) ran the products as three passes over K,
// each re-staging its operand pair through LDS: 3x the operand traffic of a bf16 GEMM and 3x the
// K loop.  Here every K tile stages A_hi, A_lo, B_hi, B_lo once (2x the bf16 traffic) and each
// fragment pair feeds three MFMAs (lo.hi, hi.lo, hi.hi, small terms first) -- the same
// arithmetic as split.h mfma16_x3 -- so the MFMA pipe, not the operand path, sets the pace.
// A plane that is null (an operand exact in bf16) is neither staged nor multiplied.
//
// Tile BM x BN x 64 (BM in {128, 192, 256}, BN in {64, 128}), 8 waves = 2 (M) x 4 (N), wave
// (BM/2) x (BN/4) as (BM/32) x (BN/64) v_mfma_f32_16x16x32_bf16 accumulators, two waves per
// SIMD.  LDS: 2 stages x {A_hi, A_lo, B_hi, B_lo} filled by global_load_lds (16 B/lane) with
// the bank swizzles of gemm.hip v4 (k-major [rows][64], chunk c of row r at c ^ ((r >> 1) & 7);
// mn-major per 128-column half [64][128], chunk c of k-row k at c ^ 2((k & 3) | ((k >> 3) & 1) << 2));
// BM = 192 needs a k-major A.  Up to 4 problems per launch, each with its own A layout and a
// K split S: a split item publishes its fp32 partial tile write-through, takes the tile's
// ticket, and the last arriver sums the S partials in split order (bit-reproducible) and runs the
// epilogue (alpha, bias, output row map, fp32 / bf16 / split-bf16 output, optional +=).
// Blocks are remapped so that consecutive items (same A rows) share an XCD and its L2.
#include "../common.h"

#include "../gemm_tile.h"

__device__ __attribute__((aligned(16))) bf16 g5_zero[8];

__device__ __forceinline__ f32x4 g5_mfma(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ int g5_mnswz(int k) { return 2 * ((k & 3) | (((k >> 3) & 1) << 2)); }
template <int BK>
__device__ __forceinline__ int g5_kswz(int r) { return BK == 64 ? ((r >> 1) & 7) : 3 * ((r >> 3) & 1); }

// Stage one R x BK operand plane: R*BK*2/1024 1-KB blocks dealt over the 8 waves (evenly when
// 8 divides the count; else wave w takes blocks w, w+8, .. -- only legal with 2 stages, whose
// wait is vmcnt(0): the deeper rings count DMAs per thread).
template <bool KMAJ, int R, int BK, int NW = 8>
__device__ __forceinline__ void g5_stage(const bf16* X, int ld, int i0, int imax, int k0, int kmax,
                                         uint8_t* tile, int wave, int lane, int oz) {
  constexpr int NBLK = R * BK * 2 / 1024, PW = (NBLK + NW - 1) / NW;
  constexpr bool EVEN = NBLK % NW == 0;
  static_assert(KMAJ || R % 128 == 0, "mn-major images are 128-column halves");
#pragma unroll
  for (int j = 0; j < PW; ++j) {
    const int blk = EVEN ? wave * PW + j : wave + NW * j;
    if (!EVEN && blk >= NBLK) break;
    int off;
    bool kin;
    if (KMAJ) {
      constexpr int CPR = BK / 8, RPB = 64 / CPR;            // chunks per row, rows per block
      const int row = blk * RPB + lane / CPR, cp = lane % CPR;
      const int c = cp ^ g5_kswz<BK>(row);
      const int k = k0 + c * 8;
      kin = k < kmax;
      off = min(i0 + row, imax - 1) * ld + k;
    } else {
      constexpr int BPH = BK / 4;                            // blocks per 128-column half
      const int h = blk / BPH, kr = (blk % BPH) * 4 + (lane >> 4), cp = lane & 15;
      const int c = cp ^ g5_mnswz(kr);
      const int col = i0 + h * 128 + c * 8;
      kin = k0 + kr < kmax;
      off = (k0 + kr) * ld + (col < imax ? col : imax - 8);
    }
    const bf16* src = kin ? X + (off + oz) : g5_zero;
    __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(tile + blk * 1024),
                                     16, 0, 0);
  }
}

// 16x16x32 fragment (k-step ks of the tile): lane l holds X[i0 + (l & 15)][32 ks + 8 (l >> 4) .. +7]
template <bool KMAJ, int BK>
__device__ __forceinline__ bf16x8 g5_frag(const uint8_t* tile, int i0, int ks, int lane) {
  const int l16 = lane & 15, g = lane >> 4;
  if (KMAJ) {
    const int r = i0 + l16, c = 4 * ks + g;
    return *(const bf16x8*)(tile + r * (BK * 2) + ((c ^ g5_kswz<BK>(r)) * 16));
  }
  const int q = (lane >> 2) & 3, p = lane & 3;
  const uint8_t* half = tile + (i0 >> 7) * (BK * 256);
  const int kr = 32 * ks + 8 * g + q;
  const int c = ((i0 & 127) >> 3) + (p >> 1);
  const uint8_t* b0 = half + kr * 256 + ((c ^ g5_mnswz(kr)) * 16) + 8 * (p & 1);
  return gm_tr8((const bf16*)b0, (const bf16*)(b0 + 4 * 256));
}

struct G5Args {
  GemmProb p[gm::MAXP];
  int split[gm::MAXP];
  int item_base[gm::MAXP];
  long long slab_base[gm::MAXP];   // first partial slab (BM x BN fp32) of each problem
  int ticket_base[gm::MAXP];
  int tiles_m[gm::MAXP];
  int np, total;
  int order; // item order of K-split problems (g5_coords)
  float* ws;
  unsigned* tickets;
};

// item -> (tm, tn, ksp).  Blocks take contiguous item ranges per XCD (the remap in the kernels), so
// the order decides which operand slices one XCD's L2 serves.  Tile-major (tn fastest, then the K
// split): an XCD's items share A row blocks and stream every B column slice -- right for an
// unsplit problem whose B is small (dX: W_ih).  order 1, K-split problems: K split slowest, then
// tn, tm fastest: an XCD's items cover a few (B column slice, K range) pairs against every A row
// block of that K range, so the big B of a weight gradient (X, h rows: K = B x T) is read by about
// one XCD instead of by every XCD whose items span its columns
__device__ __forceinline__ void g5_coords(const G5Args& a, int pi, int S, int item, int& tm,
                                          int& tn, int& ksp) {
  const GemmProb& P = a.p[pi];
  if (a.order && S > 1) {
    const int tms = a.tiles_m[pi];
    tm = item % tms;
    const int r = item / tms;
    tn = r % P.tiles_n;
    ksp = r / P.tiles_n;
  } else {
    const int tile = item / S;
    ksp = item % S;
    tm = tile / P.tiles_n;
    tn = tile % P.tiles_n;
  }
}

// C epilogue of 4 consecutive columns (row already mapped)
__device__ __forceinline__ void g5_emit(const GemmProb& P, int row, int col, f32x4 a, bool vec) {
  const int orow = P.crow ? P.crow[row] : row;
  const size_t o = (size_t)orow * P.ldc + col;
  float v[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) v[e] = P.alpha * a[e] + (P.bias && col + e < P.N ? P.bias[col + e] : 0.f);
  if (vec && col + 4 <= P.N) {
    if (P.c_f32) {
      f32x4* c = (f32x4*)((float*)P.C + o);
      f32x4 w = {v[0], v[1], v[2], v[3]};
      if (P.accumulate) w += *c;
      *c = w;
    } else if (P.C_lo) {
      bf16x4 hi, lo;
#pragma unroll
      for (int e = 0; e < 4; ++e) { hi[e] = (bf16)v[e]; lo[e] = sp_lo(v[e]); }
      *(bf16x4*)((bf16*)P.C + o) = hi;
      *(bf16x4*)(P.C_lo + o) = lo;
    } else {
      bf16x4* c = (bf16x4*)((bf16*)P.C + o);
      if (P.accumulate) {
        const bf16x4 old = *c;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] += (float)old[e];
      }
      bf16x4 w;
#pragma unroll
      for (int e = 0; e < 4; ++e) w[e] = (bf16)v[e];
      *c = w;
    }
    return;
  }
  for (int e = 0; e < 4 && col + e < P.N; ++e) {
    if (P.c_f32) {
      float* c = (float*)P.C + o + e;
      *c = P.accumulate ? *c + v[e] : v[e];
    } else if (P.C_lo) {
      sp_split(v[e], ((bf16*)P.C)[o + e], P.C_lo[o + e]);
    } else {
      bf16* c = (bf16*)P.C + o + e;
      *c = (bf16)(P.accumulate ? (float)*c + v[e] : v[e]);
    }
  }
}

// Epilogue of gemm6's 8-wave (2 x 4) tile: the BM x BN accumulators pass
// through LDS 64 rows at a time (row-contiguous, 4 columns per thread); with a K split, the
// partial tile goes write-through to the workspace and the tile's last arriver sums the splits
// in split order (bit-reproducible) and runs the epilogue.
template <int BM, int BN>
__device__ __forceinline__ void g5_epilogue(const G5Args& a, const GemmProb& P, int pi, int tile,
                                            int ksp, int S, int m0, int n0,
                                            const f32x4 (&acc)[BM / 32][BN / 64], uint8_t* lds5,
                                            int tid, int wave, int lane) {
  constexpr int FM = BM / 32, FN = BN / 64;
  const int wr = wave >> 2, wc = wave & 3;
  int& last = *(int*)(lds5 + 64 * (BN + 16) * 4);
  // acc[i][j][e] = tile[wr*(BM/2) + 16i + 4(l>>4) + e][wc*(BN/4) + 16j + (l&15)]
  constexpr int LS = BN + 16;
  constexpr int NP = FM / 2;                // 32 rows per wave row per pass -> 64 rows per pass
  float* L = (float*)lds5;
  const int l16 = lane & 15, g = lane >> 4;
  const bool vec = ((uintptr_t)P.C % 16 == 0) && (P.ldc % 4 == 0);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(a.ws, 0, 0x7fffffff, 0x00020000);
  const long long slab0 = a.slab_base[pi] + (long long)tile * S;
  // slab layout: [split][BM][BN] fp32; element (r, c) of split s at ((slab0 + s) * BM + r) * BN + c
  auto soff = [&](int s, int r, int c) {
    return (uint32_t)((((slab0 + s) * BM + r) * BN + c) * 4);
  };
  if (S > 1) {
    // publish this item's partial tile write-through (sc1), drain, take the tile's ticket
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      __builtin_amdgcn_s_barrier();
#pragma unroll
      for (int ii = 0; ii < 2; ++ii)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            L[(wr * 32 + ii * 16 + 4 * g + e) * LS + wc * (BN / 4) + 16 * j + l16] = acc[2 * p + ii][j][e];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      for (int q = tid; q < 64 * (BN / 4); q += 512) {
        const int lr = q / (BN / 4), cc = (q % (BN / 4)) * 4;
        const int r = (lr >> 5) * (BM / 2) + 32 * p + (lr & 31);
        const f32x4 v = *(const f32x4*)(L + lr * LS + cc);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rs, soff(ksp, r, cc), 0, 16);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    unsigned* tk = a.tickets + a.ticket_base[pi] + tile;
    if (tid == 0)
      last = __hip_atomic_fetch_add(tk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)(S - 1);
    __syncthreads();
    if (!last) return;
    for (int q = tid; q < BM * (BN / 4); q += 512) {
      const int r = q / (BN / 4), cc = (q % (BN / 4)) * 4;
      const int row = m0 + r, col = n0 + cc;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      for (int s = 0; s < S; ++s)
        v += __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, soff(s, r, cc), 0, 16));
      if (row < P.M && col < P.N) g5_emit(P, row, col, v, vec);
    }
    if (tid == 0) __hip_atomic_store(tk, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          L[(wr * 32 + ii * 16 + 4 * g + e) * LS + wc * (BN / 4) + 16 * j + l16] = acc[2 * p + ii][j][e];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
#pragma unroll 2
    for (int q = tid; q < 64 * (BN / 4); q += 512) {
      const int lr = q / (BN / 4), cc = (q % (BN / 4)) * 4;
      const int row = m0 + (lr >> 5) * (BM / 2) + 32 * p + (lr & 31);
      const int col = n0 + cc;
      if (row >= P.M || col >= P.N) continue;
      g5_emit(P, row, col, *(const f32x4*)(L + lr * LS + cc), vec);
    }
  }
}

// ============================================================================================
// gemm6: the split GEMM mainloop with the fragment registers refilled between the three product
// passes.  (Its predecessor gemm5 read all of a K step's fragments and then issued its MFMAs; with
// two waves per SIMD released together by the per-tile barrier both read LDS at the same moment
// and the MFMA pipe idled through the read burst -- PMC ~42 % busy, profiles/r03_pmc_gemm6.txt,
// r03_gemm6_ab.txt; gemm5 was deleted in round 6.)
// Here every K step runs its products as three passes over all FM x FN accumulators in the order
// A hi.B lo, A hi.B hi, A lo.B hi -- the only order whose last pass frees the operands the next
// step's first pass does not need -- and each plane's registers take the next step's fragments
// in the pass after their last use (B lo during pass 2, A hi during pass 3, A lo and B hi during
// the next step's pass 1), so fragment reads always overlap MFMAs without a second register set.
// The one barrier per LDS tile follows pass 1 of its last K step (the tile's last LDS reads): the
// next tile has landed, and the DMA of the tile after it refills this buffer with a whole tile
// of MFMAs to land.  8 waves in a 2 x 4 layout; split-K partials through g5_epilogue.
__device__ __forceinline__ void g6_dma(const bf16* src, uint8_t* dst) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
}

// interleave N fragment reads (issued first in program order) with the pass's M MFMAs
template <int N, int M>
__device__ __forceinline__ void g6_mix() {
  if constexpr (N > 0) {
#pragma unroll
    for (int q = 0; q < N; ++q) {
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, M / N, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, M - N * (M / N), 0);
  }
  __builtin_amdgcn_sched_barrier(0);
}

// PM (decomposition probe, r2_gemm5_set_mode bits 8-9; the 192 x 256 fast tile only): 1 =
// operand staging alone (no fragment reads, no MFMAs), 2 = the compute loop alone (no staging);
// tools/xproj_decomp.py, profiles/r06_xproj_decomposition.txt
template <bool AK, bool BKM, int BM, int BN, int BK, bool FOK, int PM = 0>
__device__ __forceinline__ void g6_mainloop(const GemmProb& P, int m0, int n0, int kt0, int kt1,
                                            uint8_t* lds6, int wave, int lane,
                                            f32x4 (&acc)[BM / 32][BN / 64]) {
  constexpr int NW = 8, KS = BK / 32;
  constexpr int FM = BM / 32, FN = BN / 64;
  constexpr int OPA = BM * BK * 2, OPB = BN * BK * 2, STB = 2 * (OPA + OPB);
  const int wr = wave >> 2, wc = wave & 3;
  // both operands k-major, no K tail (FOK: K % 32 == 0 in every problem of the launch; the
  // x-projection): each thread's 1-KB staging blocks as element offsets fixed for the whole K
  // loop (a tile adds k0); else the generic staging (g5_stage, K tail zero-filled)
  constexpr bool FAST = FOK && AK && BKM && BK == 32;
  constexpr int NBA = BM * BK * 2 / 1024, NBB = BN * BK * 2 / 1024;
  constexpr int PA = (NBA + NW - 1) / NW, PB = (NBB + NW - 1) / NW;
  uint32_t offa[FAST ? PA : 1], offb[FAST ? PB : 1];
  if constexpr (FAST) {
    const int rr = lane >> 2, cp = lane & 3;
#pragma unroll
    for (int j = 0; j < PA; ++j) {
      const int row = (wave + NW * j) * 16 + rr;
      offa[j] = (uint32_t)(min(m0 + row, P.M - 1) * P.lda + (cp ^ g5_kswz<BK>(row)) * 8);
    }
#pragma unroll
    for (int j = 0; j < PB; ++j) {
      const int row = (wave + NW * j) * 16 + rr;
      offb[j] = (uint32_t)(min(n0 + row, P.N - 1) * P.ldb + (cp ^ g5_kswz<BK>(row)) * 8);
    }
  }
  auto stage = [&](int kt) {
    uint8_t* st = lds6 + ((kt - kt0) & 1) * STB;
    if constexpr (PM == 2) {
      return;
    } else if constexpr (FAST) {
      const uint32_t k0 = (uint32_t)(kt * BK);
#pragma unroll
      for (int j = 0; j < PA; ++j) {
        if (NBA % NW == 0 || wave + NW * j < NBA) {
          uint8_t* d = st + (wave + NW * j) * 1024;
          g6_dma(P.A + (offa[j] + k0), d);
          g6_dma(P.A_lo + (offa[j] + k0), d + OPA);
        }
      }
#pragma unroll
      for (int j = 0; j < PB; ++j) {
        if (NBB % NW == 0 || wave + NW * j < NBB) {
          uint8_t* d = st + 2 * OPA + (wave + NW * j) * 1024;
          g6_dma(P.B + (offb[j] + k0), d);
          g6_dma(P.B_lo + (offb[j] + k0), d + OPB);
        }
      }
    } else {
      int oz;
      asm volatile("v_mov_b32 %0, 0" : "=v"(oz));
      const int k0 = kt * BK;
      g5_stage<AK, BM, BK>(P.A, P.lda, m0, P.M, k0, P.K, st, wave, lane, oz);
      g5_stage<AK, BM, BK>(P.A_lo, P.lda, m0, P.M, k0, P.K, st + OPA, wave, lane, oz);
      g5_stage<BKM, BN, BK>(P.B, P.ldb, n0, P.N, k0, P.K, st + 2 * OPA, wave, lane, oz);
      g5_stage<BKM, BN, BK>(P.B_lo, P.ldb, n0, P.N, k0, P.K, st + 2 * OPA + OPB, wave, lane, oz);
    }
  };
  bf16x8 ahi[FM], alo[FM], bhi[FN], blo[FN];
  // K step q = (LDS tile kt, step ks of it); its planes in buffer (kt - kt0) & 1
  auto ldA = [&](bf16x8 (&f)[FM], int kt, int ks, int plane) {
    if constexpr (PM == 1) return;
    const uint8_t* pl = lds6 + ((kt - kt0) & 1) * STB + plane * OPA;
#pragma unroll
    for (int i = 0; i < FM; ++i) f[i] = g5_frag<AK, BK>(pl, wr * (BM / 2) + 16 * i, ks, lane);
  };
  auto ldB = [&](bf16x8 (&f)[FN], int kt, int ks, int plane) {
    if constexpr (PM == 1) return;
    const uint8_t* pl = lds6 + ((kt - kt0) & 1) * STB + 2 * OPA + plane * OPB;
#pragma unroll
    for (int j = 0; j < FN; ++j) f[j] = g5_frag<BKM, BK>(pl, wc * (BN / 4) + 16 * j, ks, lane);
  };
  auto step = [&](int kt, int ks, bool more) {
    // the next K step: same tile, or the first step of the next one
    const int nkt = ks + 1 < KS ? kt : kt + 1, nks = ks + 1 < KS ? ks + 1 : 0;
    // pass 1: A hi x B lo; this step's A lo / B hi arrive
    ldA(alo, kt, ks, 1);
    ldB(bhi, kt, ks, 0);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        if constexpr (PM != 1) acc[i][j] = g5_mfma(ahi[i], blo[j], acc[i][j]);
    g6_mix<FM + FN, FM * FN>();
    if (ks == KS - 1) {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");   // tile kt+1 landed; kt read
      __builtin_amdgcn_s_barrier();        // every wave: tile kt+1 visible, tile kt's buffer free
      if (kt + 2 < kt1) stage(kt + 2);
    }
    // pass 2: A hi x B hi; B lo <- the next step's
    if (more) ldB(blo, nkt, nks, 1);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        if constexpr (PM != 1) acc[i][j] = g5_mfma(ahi[i], bhi[j], acc[i][j]);
    if (more) g6_mix<FN, FM * FN>(); else g6_mix<0, FM * FN>();
    // pass 3: A lo x B hi; A hi <- the next step's
    if (more) ldA(ahi, nkt, nks, 0);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        if constexpr (PM != 1) acc[i][j] = g5_mfma(alo[i], bhi[j], acc[i][j]);
    if (more) g6_mix<FM, FM * FN>(); else g6_mix<0, FM * FN>();
  };
  if (kt0 < kt1) {
    stage(kt0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (kt0 + 1 < kt1) stage(kt0 + 1);
    ldA(ahi, kt0, 0, 0);
    ldB(blo, kt0, 0, 1);
    const int nq = (kt1 - kt0) * KS;
    for (int q = 0; q + 1 < nq; ++q) step(kt0 + q / KS, q % KS, true);
    step(kt1 - 1, KS - 1, false);
  }
}

template <bool BKM, int BM, int BN, int BK, bool FOK, int PM = 0>
__global__ __launch_bounds__(512) void gemm6_kernel(const G5Args a) {
  constexpr int FM = BM / 32, FN = BN / 64;           // 16 x 16 fragments of the (BM/2) x (BN/4) wave tile
  extern __shared__ __attribute__((aligned(1024))) uint8_t lds6[];
  int bid;
  {
    const int b = blockIdx.x, x = b & 7, qn = a.total >> 3, r = a.total & 7;
    bid = (x < r ? x * (qn + 1) : r * (qn + 1) + (x - r) * qn) + (b >> 3);
  }
  int pi = 0;
#pragma unroll
  for (int i = 1; i < gm::MAXP; ++i)
    if (i < a.np && bid >= a.item_base[i]) pi = i;
  const GemmProb& P = a.p[pi];
  const int S = a.split[pi];
  const int item = bid - a.item_base[pi];
  int tm, tn, ksp;
  g5_coords(a, pi, S, item, tm, tn, ksp);
  const int tile = tm * P.tiles_n + tn;
  const int m0 = tm * BM, n0 = tn * BN;
  const int nk = (P.K + BK - 1) / BK, per = (nk + S - 1) / S;
  const int kt0 = min(nk, ksp * per), kt1 = min(nk, kt0 + per);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  if constexpr (PM != 0) {
    g6_mainloop<true, BKM, BM, BN, BK, FOK, PM>(P, m0, n0, kt0, kt1, lds6, wave, lane, acc);
  } else if constexpr (BM % 128 == 0) {
    if (P.a_kmajor) g6_mainloop<true, BKM, BM, BN, BK, FOK>(P, m0, n0, kt0, kt1, lds6, wave, lane, acc);
    else g6_mainloop<false, BKM, BM, BN, BK, FOK>(P, m0, n0, kt0, kt1, lds6, wave, lane, acc);
  } else {
    g6_mainloop<true, BKM, BM, BN, BK, FOK>(P, m0, n0, kt0, kt1, lds6, wave, lane, acc);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();            // every wave past its last LDS read before the epilogue
  g5_epilogue<BM, BN>(a, P, pi, tile, ksp, S, m0, n0, acc, lds6, tid, wave, lane);
}

// (gemm7, a deep LDS-DMA ring of 16-deep K tiles on 32x32x16 MFMAs, was measured slower than gemm6
// on every shape and removed: profiles/r05_gemm7_deep_ring_rejected.txt)


template <bool BKM, int BM, int BN, int BK, bool FOK, int PM = 0>
static void g6_kernel_launch(const G5Args& a, hipStream_t s) {
  constexpr int LDS = 2 * 2 * (BM + BN) * BK * 2;
  static_assert(LDS <= 160 * 1024 && 64 * (BN + 16) * 4 + 4 <= LDS, "LDS");
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)gemm6_kernel<BKM, BM, BN, BK, FOK, PM>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    attr = true;
  }
  hipLaunchKernelGGL((gemm6_kernel<BKM, BM, BN, BK, FOK, PM>), dim3(a.total), dim3(512), LDS, s, a);
}
// the fast staging only where it applies (k-major A and B, BK 32, no K tail)
template <bool BKM, int BM, int BN, int BK>
static void g6_launch(const G5Args& a, bool k32, hipStream_t s) {
  if (BKM && BK == 32 && k32) g6_kernel_launch<BKM, BM, BN, BK, true>(a, s);
  else g6_kernel_launch<BKM, BM, BN, BK, false>(a, s);
}

// K-split-major item order (g5_coords); r2_gemm5_set_mode bit 6 = the tile-major order instead
// (the probe's A/B: tools/gemm_order_probe.py, profiles/r05_gemm_item_order.txt -- the group of
// the paper config 94-103 -> 92-96 us, bitwise-equal output).  Other bits are ignored (the gemm5
// and probe modes were removed in round 6).
static int g5_order = 1, g5_probe = 0;
extern "C" int r2_gemm5_set_mode(int m) {
  g5_order = !((m >> 6) & 1);
  g5_probe = (m >> 8) & 3;      // decomposition probe instances (192 x 256 fast tile)
  return 0;
}

// tile configurations: {BM, BN, BK, (unused)}
static const int g5_cfgs[][4] = {{192, 128, 64, 2}, {128, 128, 64, 2}, {256, 128, 32, 3},
                                 {256, 256, 32, 2}, {256, 64, 64, 2}, {128, 64, 64, 2},
                                 {128, 128, 32, 4}, {192, 256, 32, 2}};
static const int g5_ncfg = 8;

static int g5_tiles(const GemmProb& p, int bm, int bn) {
  return ((p.M + bm - 1) / bm) * ((p.N + bn - 1) / bn);
}

// Automatic K splits (split[i] == 0) once the tile is fixed: the problem's split grows while its
// per-item K steps exceed both the longest fixed-split problem's and 2, and the launch's items
// still fit one round on nc CUs.  Small-M launches (the reference config's 80-row dX, 184-row
// x-projection: 7-64 items of 25-32 K steps on 256 CUs) then spread their K over the idle CUs;
// launches that already fill the chip keep split 1.  Splits >= 1 pass through.
static void g5_auto_split(const GemmProb* p, const int* split_in, int np, int cfg, int nc,
                          int* out) {
  const int bm = g5_cfgs[cfg][0], bn = g5_cfgs[cfg][1], bk = g5_cfgs[cfg][2];
  long long items = 0;
  int target = 2;
  for (int i = 0; i < np; ++i) {
    out[i] = split_in && split_in[i] > 0 ? split_in[i] : 1;
    items += (long long)g5_tiles(p[i], bm, bn) * out[i];
    if (split_in && split_in[i] > 0) {
      const int ks = (p[i].K + bk - 1) / bk;
      target = max(target, (ks + out[i] - 1) / out[i]);
    }
  }
  if (!split_in) return;
  // a split pays only when it shortens the launch's longest item: every auto problem at the
  // current maximum grows together (one of them alone leaves the critical path where it was)
  auto per = [&](int i) {
    const int ks = (p[i].K + bk - 1) / bk;
    return (ks + out[i] - 1) / out[i];
  };
  for (;;) {
    int mx = 0;
    for (int i = 0; i < np; ++i) mx = max(mx, per(i));
    if (mx <= target) return;
    long long extra = 0;
    for (int i = 0; i < np; ++i) {
      if (per(i) != mx) continue;
      if (split_in[i] != 0) return;                  // a fixed-split problem sets the pace
      extra += g5_tiles(p[i], bm, bn);
    }
    if (items + extra > nc) return;
    for (int i = 0; i < np; ++i)
      if (per(i) == mx) out[i] += 1;
    items += extra;
  }
}

// descs: np x GEMM_DESC (gemm.hip r2_gemm layout), every operand split (A_lo and B_lo set), one B
// layout per launch.  split: np K splits (null = 1).  cfg: index into g5_cfgs, or -1 = pick by a
// CU-utilisation model for n_cus resident workgroups (one per CU).  Returns the cfg used (>= 0)
// or an error (< 0).
extern "C" int r2_gemm5(const int64_t* descs, const int* split, int np, int cfg, float* ws,
                        long long ws_bytes, unsigned* tickets, int n_tickets, int n_cus, void* stream) {
  if (np < 1 || np > gm::MAXP) return -1;
  G5Args a;
  a.np = np; a.ws = ws; a.tickets = tickets;
  int bkm = -1;
  bool all_k = true;
  for (int i = 0; i < np; ++i) {
    const int rc = gemm_parse_desc(descs + GEMM_DESC * i, a.p[i]);
    if (rc) return rc;
    if (!a.p[i].A_lo || !a.p[i].B_lo) return -10;      // split operands only
    if (bkm < 0) bkm = a.p[i].b_kmajor;
    if (bkm != a.p[i].b_kmajor) return -5;
    all_k = all_k && a.p[i].a_kmajor;
    a.split[i] = split && split[i] > 1 ? split[i] : 1;   // auto (0) counts as 1 for the tile choice
  }
  auto ok = [&](int c) {
    const int bm = g5_cfgs[c][0], bn = g5_cfgs[c][1];
    if (bm % 128 && !all_k) return false;
    if (bn % 128 && !bkm) return false;
    return true;
  };
  if (cfg < 0) {   // smallest (rounds x per-item MFMA work / model efficiency)
    double best = 1e30;
    const int nc = n_cus > 0 ? n_cus : 256;
    for (int c = 0; c < g5_ncfg; ++c) {
      if (!ok(c)) continue;
      const int bm = g5_cfgs[c][0], bn = g5_cfgs[c][1];
      long long items = 0;
      double work = 0;
      for (int i = 0; i < np; ++i) {
        items += (long long)g5_tiles(a.p[i], bm, bn) * a.split[i];
        work = fmax(work, (double)bm * bn * ((a.p[i].K + a.split[i] - 1) / a.split[i]));
      }
      const long long rounds = (items + nc - 1) / nc;
      // operand bytes per MFMA fall with the tile's perimeter / area
      const double eff = 1.0 / (1.0 + 96.0 * (1.0 / bm + 1.0 / bn));
      const double cost = rounds * work / eff;
      if (cost < best) { best = cost; cfg = c; }
    }
  }
  if (cfg < 0 || cfg >= g5_ncfg || !ok(cfg)) return -8;
  {
    int sp[gm::MAXP];
    g5_auto_split(a.p, split, np, cfg, n_cus > 0 ? n_cus : 256, sp);
    for (int i = 0; i < np; ++i) a.split[i] = sp[i];
  }
  const int bm = g5_cfgs[cfg][0], bn = g5_cfgs[cfg][1];
  int items = 0, tks = 0;
  long long slabs = 0;
  for (int i = 0; i < np; ++i) {
    GemmProb& p = a.p[i];
    p.tiles_n = (p.N + bn - 1) / bn;
    const int t = g5_tiles(p, bm, bn);
    a.tiles_m[i] = t / p.tiles_n;
    a.item_base[i] = items;
    a.slab_base[i] = slabs;
    a.ticket_base[i] = tks;
    items += t * a.split[i];
    if (a.split[i] > 1) { slabs += (long long)t * a.split[i]; tks += t; }
  }
  for (int i = np; i < gm::MAXP; ++i) {
    a.p[i] = a.p[0]; a.split[i] = 1; a.item_base[i] = 1 << 30; a.tiles_m[i] = 1;
  }
  a.total = items;
  a.order = g5_order;
  if (slabs * bm * bn * 4 > ws_bytes || tks > n_tickets) return -7;
  hipStream_t s = (hipStream_t)stream;
  bool k32 = true;
  for (int i = 0; i < np; ++i) k32 = k32 && a.p[i].K % 32 == 0;
  switch (cfg * 2 + bkm) {
    case 0: g6_launch<false, 192, 128, 64>(a, k32, s); break;
    case 1: g6_launch<true, 192, 128, 64>(a, k32, s); break;
    case 2: g6_launch<false, 128, 128, 64>(a, k32, s); break;
    case 3: g6_launch<true, 128, 128, 64>(a, k32, s); break;
    case 4: g6_launch<false, 256, 128, 32>(a, k32, s); break;
    case 5: g6_launch<true, 256, 128, 32>(a, k32, s); break;
    case 6: g6_launch<false, 256, 256, 32>(a, k32, s); break;
    case 7: g6_launch<true, 256, 256, 32>(a, k32, s); break;
    case 9: g6_launch<true, 256, 64, 64>(a, k32, s); break;
    case 11: g6_launch<true, 128, 64, 64>(a, k32, s); break;
    case 12: g6_launch<false, 128, 128, 32>(a, k32, s); break;
    case 13: g6_launch<true, 128, 128, 32>(a, k32, s); break;
    // 192 x 256: one round of tiles for the x-projection's 10,560 x 1,024 on 256 CUs (224 items;
    // 192 x 128 took 2.6 rounds)
    case 14: g6_launch<false, 192, 256, 32>(a, k32, s); break;
    case 15:
      if (k32 && all_k && g5_probe == 1) g6_kernel_launch<true, 192, 256, 32, true, 1>(a, s);
      else if (k32 && all_k && g5_probe == 2) g6_kernel_launch<true, 192, 256, 32, true, 2>(a, s);
      else g6_launch<true, 192, 256, 32>(a, k32, s);
      break;
    default: return -8;
  }
  R2_CHECK_LAUNCH();
  return cfg;
}

// bytes of split-K workspace for configuration cfg
extern "C" long long r2_gemm5_ws_bytes_nc(const int64_t* descs, const int* split, int np, int cfg,
                                          int n_cus) {
  if (cfg < 0 || cfg >= g5_ncfg || np < 1 || np > gm::MAXP) return -1;
  GemmProb p[gm::MAXP];
  for (int i = 0; i < np; ++i)
    if (gemm_parse_desc(descs + GEMM_DESC * i, p[i])) return -1;
  int sp[gm::MAXP];
  g5_auto_split(p, split, np, cfg, n_cus > 0 ? n_cus : 256, sp);
  long long b = 0;
  for (int i = 0; i < np; ++i)
    if (sp[i] > 1)
      b += (long long)g5_tiles(p[i], g5_cfgs[cfg][0], g5_cfgs[cfg][1]) * sp[i] * g5_cfgs[cfg][0] *
           g5_cfgs[cfg][1] * 4;
  return b;
}

extern "C" long long r2_gemm5_ws_bytes(const int64_t* descs, const int* split, int np, int cfg) {
  return r2_gemm5_ws_bytes_nc(descs, split, np, cfg, 256);
}
