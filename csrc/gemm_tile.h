// 128x128 MFMA GEMM tile machinery (gfx950) shared by gemm.hip and the kernels that run GEMM
// tiles inside their own launch (lstm_persist.hip: BPTT helper workgroups).  See gemm.hip for
// the operand conventions (k-major / mn-major operands, LDS-DMA staging with source swizzles).
#pragma once
#include "common.h"
#include "split.h"

namespace gm {
constexpr int BM = 128, BN = 128, BK = 64, NT = 256;
constexpr int KS = BK + 8;        // k-major LDS row stride (bf16): 144 B rows (b128 reads conflict-free)
constexpr int MS = BM + 32;       // mn-major LDS row stride (bf16): 320 B = 16 dwords mod 64 banks,
                                  // so the 4 rows x 2 column groups of a tr read hit 8 distinct bank octets
constexpr int LPT = BM * BK / 8 / NT;  // 16-B chunks per thread per operand tile (4)
constexpr int TILE = BM * KS > BK * MS ? BM * KS : BK * MS;  // bf16 per operand tile
constexpr int MAXP = 4;
}  // namespace gm

struct GemmProb {
  const bf16* A;
  const bf16* B;
  void* C;
  const float* bias;   // per output column, or null
  const int* crow;     // output row map, or null
  int M, N, K, lda, ldb, ldc;
  int a_kmajor, b_kmajor, c_f32, accumulate;
  float alpha;
  int tiles_n, tile_base;  // tiles along N; first linear tile index of this problem
  // split precision (split.h): lo planes of A / B (null = operand exact in bf16) and of C (null =
  // C is fp32 or plain bf16).  The K loop runs npass passes over K: (A_lo,B) (A,B_lo) (A,B) with
  // both split, (A_lo,B) (A,B) or (A,B_lo) (A,B) with one.
  const bf16* A_lo;
  const bf16* B_lo;
  bf16* C_lo;
  int npass, pad_;
};

// descriptor words per problem (ops/gemm.py Gemm.desc)
#define GEMM_DESC 20

__device__ __forceinline__ const bf16* gp_a(const GemmProb& P, int pass) {
  return (pass == 0 && P.A_lo) ? P.A_lo : P.A;
}
__device__ __forceinline__ const bf16* gp_b(const GemmProb& P, int pass) {
  if (!P.B_lo) return P.B;
  return pass == (P.A_lo ? 1 : 0) ? P.B_lo : P.B;
}

struct GemmArgs {
  GemmProb p[gm::MAXP];
  int nprob;
};

typedef short gi16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) gi16x4 glds_i16x4;

__device__ __forceinline__ bf16x8 gm_tr8(const bf16* p0, const bf16* p1) {
  const gi16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((glds_i16x4*)p0);
  const gi16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((glds_i16x4*)p1);
  return __builtin_bit_cast(bf16x8, __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7));
}


namespace g2 {
constexpr int BM = 128, BN = 128, BK = 64, NT = 256;
constexpr int TILE_B = 16384;        // bytes per operand tile (both layouts)
constexpr int GPW = 4;               // 1-KB DMA instructions per wave per operand tile
}  // namespace g2

// AUX: cache policy of the DMA loads (16 = sc1, for operands another CU of the SAME launch wrote
// write-through: MI355X_MICROARCH.md hand-off table)
template <bool KMAJ, int AUX = 0>
__device__ __forceinline__ void g2_stage(const bf16* X, int ld, int i0, int imax, int k0,
                                         uint8_t* lds_tile, int wave, int lane) {
#pragma unroll
  for (int j = 0; j < g2::GPW; ++j) {
    const int blk = wave * g2::GPW + j;          // 1-KB block of the tile
    const bf16* src;
    if (KMAJ) {
      const int row = blk * 8 + (lane >> 3), cp = lane & 7;
      const int c = cp ^ ((row >> 1) & 7);
      src = X + (size_t)min(i0 + row, imax - 1) * ld + k0 + c * 8;
    } else {
      const int kr = blk * 4 + (lane >> 4), cp = lane & 15;
      const int c = cp ^ (4 * (kr & 3));
      const int col = i0 + c * 8;
      src = X + (size_t)(k0 + kr) * ld + (col < imax ? col : imax - 8);
    }
    __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(lds_tile + blk * 1024),
                                     16, 0, AUX);
  }
}

template <bool KMAJ>
__device__ __forceinline__ bf16x8 g2_frag(const uint8_t* L, int i0, int ks, int lane) {
  const int l32 = lane & 31, h = lane >> 5;
  if (KMAJ) {
    const int r = i0 + l32, c = 2 * ks + h;
    return *(const bf16x8*)(L + r * 128 + ((c ^ ((r >> 1) & 7)) * 16));
  }
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int c = (i0 >> 3) + 2 * (g & 1) + (p >> 1);
  const int kr = 16 * ks + 8 * h + q;                      // + 4 for the second read
  const uint8_t* b0 = L + kr * 256 + ((c ^ (4 * q)) * 16) + 8 * (p & 1);
  return gm_tr8((const bf16*)b0, (const bf16*)(b0 + 4 * 256));
}


// Epilogue of a 128x128 tile held as acc[2][2] (32x32x16 layout, wave (wm, wn) quadrant):
// C[row][col] = alpha * acc + bias[col], row m stored at crow[m], fp32 or bf16, optional +=.
__device__ __forceinline__ void g2_epilogue(const GemmProb& P, int m0, int n0, int wm, int wn,
                                            int lane, const f32x16 (&acc)[2][2]) {
  const int l32 = lane & 31, h = lane >> 5;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = n0 + wn + 32 * j + l32;
    if (col >= P.N) continue;
    const float bv = P.bias ? P.bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (row >= P.M) continue;
        const int orow = P.crow ? P.crow[row] : row;
        const float v = P.alpha * acc[i][j][r] + bv;
        const size_t o = (size_t)orow * P.ldc + col;
        if (P.c_f32) {
          float* c = (float*)P.C + o;
          *c = P.accumulate ? *c + v : v;
        } else if (P.C_lo) {
          sp_split(v, ((bf16*)P.C)[o], P.C_lo[o]);
        } else {
          bf16* c = (bf16*)P.C + o;
          *c = (bf16)(P.accumulate ? (float)*c + v : v);
        }
      }
  }
}

// The same epilogue staged through LDS (>= 33 KB at `lds`, free: every operand read retired):
// each 64-row half of the tile is written fp32 to LDS in the accumulator layout, then stored
// row-contiguous, 4 columns per thread (one 16-B fp32 / 8-B bf16 store, one crow load per row).
// The register epilogue above unrolls 64 scalar stores per lane behind 4 uniform branches each
// (3.7k instructions, ~10 us per launch at any tile count: tools/gemm_floor_probe.py); this one
// is a short loop.  Threads 0..255 of the workgroup, raw barriers.
__device__ __forceinline__ void g2_epilogue_lds(const GemmProb& P, int m0, int n0, int wm, int wn,
                                                int lane, const f32x16 (&acc)[2][2], uint8_t* lds_raw) {
  constexpr int LS = 136;                      // fp32 row stride: rows r, r+4 on disjoint banks
  float* L = (float*)lds_raw;
  const int tid = threadIdx.x, l32 = lane & 31, h = lane >> 5;
  const bool f32 = P.c_f32 != 0;
  const bool vec = ((uintptr_t)P.C % 16 == 0) && (P.ldc % 4 == 0);
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();              // LDS free (operands, or the previous half)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int lr = (wm >> 6) * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        L[lr * LS + wn + 32 * j + l32] = acc[i][j][r];
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
#pragma unroll 2
    for (int pass = 0; pass < 8; ++pass) {
      const int q = pass * 256 + tid;           // 64 rows x 32 four-column chunks
      const int lr = q >> 5, cc = (q & 31) * 4;
      const int row = m0 + (lr >> 5) * 64 + 32 * i + (lr & 31);
      const int col = n0 + cc;
      if (row >= P.M || col >= P.N) continue;
      const f32x4 a = *(const f32x4*)(L + lr * LS + cc);
      const int orow = P.crow ? P.crow[row] : row;
      const size_t o = (size_t)orow * P.ldc + col;
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = P.alpha * a[e] + (P.bias && col + e < P.N ? P.bias[col + e] : 0.f);
      if (vec && col + 4 <= P.N) {
        if (f32) {
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
      } else {
        for (int e = 0; e < 4 && col + e < P.N; ++e) {
          if (f32) {
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
    }
  }
}

// One 128x128 output tile (tm, tn) of problem P by threads 0..255 (4 waves) of a workgroup,
// usable inside other kernels: 2-stage LDS-DMA ring at `lds` (2 x 32 KB), K tiles visited in
// ascending or descending order; ready(kt) is called by EVERY wave before it issues the DMA of K
// tile kt (a per-wave poll when the operand is produced inside the same launch; then AUX = 16).
// K % 64 == 0.  Raw barriers only (threads >= 256 of the workgroup must have exited).
// acc += the tile's product over K tiles [kt0, kt1) (visited ascending, or descending if desc).
template <bool AK, bool BK_, int AUX, class Ready>
__device__ __forceinline__ void g2_tile_acc(const GemmProb& P, int tm, int tn, uint8_t* lds,
                                            int kt0, int kt1, bool desc, Ready ready,
                                            f32x16 (&acc)[2][2]) {
  using namespace g2;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int m0 = tm * BM, n0 = tn * BN;
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;
  const int nk = kt1 - kt0;
  const int nkp = P.K / BK;           // K tiles per pass (kt counts over npass * nkp)
  auto stage = [&](int i) {
    const int kt = desc ? kt1 - 1 - i : kt0 + i;
    ready(kt);
    const int pass = kt / nkp, kk = kt - pass * nkp;
    uint8_t* st = lds + (i & 1) * (2 * TILE_B);
    g2_stage<AK, AUX>(gp_a(P, pass), P.lda, m0, P.M, kk * BK, st, wave, lane);
    g2_stage<BK_, AUX>(gp_b(P, pass), P.ldb, n0, P.N, kk * BK, st + TILE_B, wave, lane);
  };
  if (nk <= 0) return;
  stage(0);
  if (nk > 1) stage(1);
  for (int i = 0; i < nk; ++i) {
    if (i + 1 < nk) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const uint8_t* la = lds + (i & 1) * (2 * TILE_B);
    const uint8_t* lb = la + TILE_B;
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      bf16x8 fa[2], fb[2];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        fa[q] = g2_frag<AK>(la, wm + 32 * q, ks, lane);
        fb[q] = g2_frag<BK_>(lb, wn + 32 * q, ks, lane);
      }
#pragma unroll
      for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int r = 0; r < 2; ++r) acc[q][r] = mfma32(fa[q], fb[r], acc[q][r]);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();          // every wave is done reading this stage
    if (i + 2 < nk) stage(i + 2);
  }
}

template <bool AK, bool BK_, int AUX, class Ready>
__device__ __forceinline__ void g2_tile(const GemmProb& P, int tm, int tn, uint8_t* lds, bool desc,
                                        Ready ready) {
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  f32x16 acc[2][2] = {};
  g2_tile_acc<AK, BK_, AUX>(P, tm, tn, lds, 0, P.K / g2::BK * P.npass, desc, ready, acc);
  g2_epilogue(P, tm * g2::BM, tn * g2::BN, (wave >> 1) * 64, (wave & 1) * 64, lane, acc);
}

// ---- split precision (split.h) helper tile: one 128 x 128 output tile with A and B both given
// as hi / lo planes, all THREE products (lo.hi, hi.lo, hi.hi) taken per 32-deep K tile from ONE
// staging of the four planes (the multi-pass g2_tile re-stages K per product, so a helper that
// waits on a producer per K tile would run two thirds of its work after the producer ended).
// 4 waves (threads 0..255), wave tile 64 x 64 as 2 x 2 32x32x16 accumulators; NS-stage ring of
// 32-KB stages {A hi, A lo, B hi, B lo} (8 KB planes) at `lds`.  k-major planes are [128][32 k]
// (64-B rows; chunk c of row r at slot c ^ ((r >> 2) & 3), conflict-free fragment reads),
// mn-major planes [32 k][128] (g2_stage / g2_frag's layout).  AUXA / AUXB: DMA cache policy of
// the A / B loads (16 = sc1: operands another CU of the same launch wrote write-through).
namespace g2s {
constexpr int BM = 128, BN = 128, BK = 32, PL = 8192, ST = 4 * PL;
}  // namespace g2s

template <bool KMAJ, int AUX>
__device__ __forceinline__ void g2s_stage(const bf16* X, int ld, int i0, int imax, int k0,
                                          uint8_t* plane, int wave, int lane) {
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int blk = wave * 2 + j;                  // 8 x 1 KB blocks per plane
    const bf16* src;
    if (KMAJ) {
      const int row = blk * 16 + (lane >> 2), c = (lane & 3) ^ ((row >> 2) & 3);
      src = X + (size_t)min(i0 + row, imax - 1) * ld + k0 + c * 8;
    } else {
      const int kr = blk * 4 + (lane >> 4), c = (lane & 15) ^ (4 * (kr & 3));
      const int col = i0 + c * 8;
      src = X + (size_t)(k0 + kr) * ld + (col < imax ? col : imax - 8);
    }
    __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(plane + blk * 1024),
                                     16, 0, AUX);
  }
}

template <bool KMAJ>
__device__ __forceinline__ bf16x8 g2s_frag(const uint8_t* plane, int i0, int ks, int lane) {
  if (KMAJ) {
    const int r = i0 + (lane & 31), c = 2 * ks + (lane >> 5);
    return *(const bf16x8*)(plane + r * 64 + ((c ^ ((r >> 2) & 3)) * 16));
  }
  return g2_frag<false>(plane, i0, ks, lane);      // [32 k][128]: 256-B rows as g2's mn-major
}

// acc += the tile's product over K tiles [kt0, kt1) of 32 (ascending, or descending if desc);
// ready(kt) is called by every wave before it issues K tile kt's DMAs.  K % 32 == 0.
template <bool AK, bool BK_, int AUXA, int AUXB, int NS, class Ready>
__device__ __forceinline__ void g2s_tile_acc(const GemmProb& P, int tm, int tn, uint8_t* lds,
                                             int kt0, int kt1, bool desc, Ready ready,
                                             f32x16 (&acc)[2][2]) {
  using namespace g2s;
  static_assert(NS >= 2 && NS <= 3, "ring depth");
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int m0 = tm * BM, n0 = tn * BN;
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;
  const int nk = kt1 - kt0;
  auto stage = [&](int i) {
    const int kt = desc ? kt1 - 1 - i : kt0 + i;
    ready(kt);
    uint8_t* st = lds + (i % NS) * ST;
    g2s_stage<AK, AUXA>(P.A, P.lda, m0, P.M, kt * BK, st, wave, lane);
    g2s_stage<AK, AUXA>(P.A_lo, P.lda, m0, P.M, kt * BK, st + PL, wave, lane);
    g2s_stage<BK_, AUXB>(P.B, P.ldb, n0, P.N, kt * BK, st + 2 * PL, wave, lane);
    g2s_stage<BK_, AUXB>(P.B_lo, P.ldb, n0, P.N, kt * BK, st + 3 * PL, wave, lane);
  };
  if (nk <= 0) return;
  for (int i = 0; i < NS - 1 && i < nk; ++i) stage(i);
  for (int i = 0; i < nk; ++i) {
    // 8 DMAs per wave per stage: stage i landed once only the stages after it remain
    const int ahead = min(NS - 2, nk - 1 - i);
    if (ahead >= 1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();          // stage i visible; every wave done reading stage i-1
    if (i + NS - 1 < nk) stage(i + NS - 1);
    const uint8_t* st = lds + (i % NS) * ST;
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      bf16x8 ah[2], al[2], bh[2], bl[2];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        ah[q] = g2s_frag<AK>(st, wm + 32 * q, ks, lane);
        al[q] = g2s_frag<AK>(st + PL, wm + 32 * q, ks, lane);
        bh[q] = g2s_frag<BK_>(st + 2 * PL, wn + 32 * q, ks, lane);
        bl[q] = g2s_frag<BK_>(st + 3 * PL, wn + 32 * q, ks, lane);
      }
#pragma unroll
      for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int r = 0; r < 2; ++r) acc[q][r] = mfma32_x3(ah[q], al[q], bh[r], bl[r], acc[q][r]);
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();            // every wave done reading the ring (epilogue reuses it)
}

// Host: parse one 16 x int64 problem descriptor (ops/gemm.py Gemm.desc layout) and check the
// shape rules of the 128x128 paths.  0 = ok.
static inline int gemm_parse_desc(const int64_t* d, GemmProb& p) {
  p.A = (const bf16*)d[0]; p.B = (const bf16*)d[1]; p.C = (void*)d[2];
  p.bias = (const float*)d[3]; p.crow = (const int*)d[4];
  p.M = (int)d[5]; p.N = (int)d[6]; p.K = (int)d[7];
  p.lda = (int)d[8]; p.ldb = (int)d[9]; p.ldc = (int)d[10];
  p.a_kmajor = (int)d[11]; p.b_kmajor = (int)d[12]; p.c_f32 = (int)d[13];
  p.accumulate = (int)d[14];
  const uint32_t ab = (uint32_t)d[15];
  float al;
  __builtin_memcpy(&al, &ab, 4);
  p.alpha = al;
  p.A_lo = (const bf16*)d[16]; p.B_lo = (const bf16*)d[17]; p.C_lo = (bf16*)d[18];
  p.npass = 1 + (p.A_lo != nullptr) + (p.B_lo != nullptr);
  p.pad_ = 0;
  if (p.C_lo && (p.c_f32 || p.accumulate)) return -12;   // split output: plain store only
  if (p.M < 1 || p.N < 1 || p.K < 8 || p.K % 8) return -2;
  if (!p.b_kmajor && (p.N % 8)) return -3;
  if (!p.a_kmajor && (p.M % 8)) return -3;
  if (p.lda % 8 || p.ldb % 8) return -4;
  p.tiles_n = (p.N + gm::BN - 1) / gm::BN;
  p.tile_base = 0;
  return 0;
}
