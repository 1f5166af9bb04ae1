// Batched bf16 MFMA GEMM with fused epilogues for the learner's dense layers (gfx950).
//
// Replaces the library GEMMs of one learner step (reference math: learner.py:99-120 -- the
// LSTM input projection, the dueling head's first layer and their backward products) and the
// copies / gathers around them:
//
//   C[m][n] (=|+=) alpha * sum_k A[m][k] B[k][n]  (+ bias[n])      written fp32 or bf16,
//   row m stored at crow[m] when a row map is given (the LSTM's packed gate order -> torch order)
//
// Each operand is either K-contiguous ("k-major": X[i][k] at X + i*ld + k) or M/N-contiguous
// ("mn-major": X[i][k] at X + k*ld + i).  Up to 4 independent problems per launch (their tiles
// enumerated linearly over blockIdx.x), so e.g. the online and target input projections run as
// one grid.
//
// Tile 128x128x64, 256 threads = 4 waves in 2x2, each wave 64x64 = 2x2 v_mfma_f32_32x32x16_bf16
// accumulators.  Global -> registers (tile t+1) overlaps the MFMAs of tile t; LDS double buffer,
// one barrier per K tile.  LDS images: k-major operands as [row][64 k + 8 pad] read with
// ds_read_b128; mn-major operands as [k][128 + 32 pad] read with ds_read_b64_tr_b16 (the hardware
// transpose hands each lane its 8 consecutive k).  K must be a multiple of 8 (tails zero-filled); M and N are
// arbitrary for k-major operands, multiples of 8 for mn-major ones.
#include "../common.h"

#include "../gemm_tile.h"

// Global -> register staging of one 128 x 64 operand tile (256 threads, 4 x 16 B each).
//   k-major: row r = c / 8, k chunk (c % 8) * 8;  mn-major: k row = c / 16, i chunk (c % 16) * 8
template <bool KMAJ>
__device__ __forceinline__ void gm_load(const bf16* X, int ld, int i0, int imax, int k0, int kmax,
                                        int tid, u32x4 (&r)[gm::LPT]) {
#pragma unroll
  for (int q = 0; q < gm::LPT; ++q) {
    const int c = tid + q * gm::NT;
    if (KMAJ) {
      const int row = min(i0 + (c >> 3), imax - 1), k = k0 + (c & 7) * 8;
      r[q] = k < kmax ? *(const u32x4*)(X + (size_t)row * ld + k) : u32x4{0, 0, 0, 0};
    } else {
      const int k = k0 + (c >> 4), col = i0 + (c & 15) * 8;
      // (imax % 8 == 0) chunks wholly past the edge read a valid chunk; never stored
      const int cc = col < imax ? col : imax - 8;
      r[q] = k < kmax ? *(const u32x4*)(X + (size_t)k * ld + cc) : u32x4{0, 0, 0, 0};
    }
  }
}

template <bool KMAJ>
__device__ __forceinline__ void gm_store(bf16* L, int tid, const u32x4 (&r)[gm::LPT]) {
#pragma unroll
  for (int q = 0; q < gm::LPT; ++q) {
    const int c = tid + q * gm::NT;
    if (KMAJ) *(u32x4*)(L + (c >> 3) * gm::KS + (c & 7) * 8) = r[q];
    else *(u32x4*)(L + (c >> 4) * gm::MS + (c & 15) * 8) = r[q];
  }
}

// MFMA fragment (8 consecutive k of tile row i = i0 + lane&31) for K step ks (0..3) of the tile
template <bool KMAJ>
__device__ __forceinline__ bf16x8 gm_frag(const bf16* L, int i0, int ks, int lane) {
  const int l32 = lane & 31, h = lane >> 5;
  if (KMAJ) return *(const bf16x8*)(L + (i0 + l32) * gm::KS + ks * 16 + h * 8);
  // transposed read: 16-lane group g covers columns i0 + 16(g&1) .. +15; lane 4q+p names row
  // (k) 16ks + 8h + 4r + q, columns 4p .. 4p+3
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const bf16* b = L + (ks * 16 + h * 8 + q) * gm::MS + i0 + 16 * (g & 1) + 4 * p;
  return gm_tr8(b, b + 4 * gm::MS);
}

template <bool AK, bool BK_>
__global__ __launch_bounds__(256) void gemm_kernel(const GemmArgs args) {
  using namespace gm;
  __shared__ __attribute__((aligned(16))) bf16 la[2][TILE];
  __shared__ __attribute__((aligned(16))) bf16 lb[2][TILE];
  // problem of this block (tiles of all problems enumerated linearly)
  int pi = 0;
#pragma unroll
  for (int i = 1; i < MAXP; ++i)
    if (i < args.nprob && (int)blockIdx.x >= args.p[i].tile_base) pi = i;
  const GemmProb& P = args.p[pi];
  if (P.a_kmajor != (int)AK || P.b_kmajor != (int)BK_) return;  // launched per layout combo
  const int t = blockIdx.x - P.tile_base;
  const int tm = t / P.tiles_n, tn = t % P.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  if (m0 >= P.M) return;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;

  f32x16 acc[2][2] = {};
  u32x4 ra[LPT], rb[LPT];
  const int nk = (P.K + BK - 1) / BK;   // the last tile's k >= K chunks are zero-filled
  gm_load<AK>(P.A, P.lda, m0, P.M, 0, P.K, tid, ra);
  gm_load<BK_>(P.B, P.ldb, n0, P.N, 0, P.K, tid, rb);
  gm_store<AK>(la[0], tid, ra);
  gm_store<BK_>(lb[0], tid, rb);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) {
      gm_load<AK>(P.A, P.lda, m0, P.M, (kt + 1) * BK, P.K, tid, ra);
      gm_load<BK_>(P.B, P.ldb, n0, P.N, (kt + 1) * BK, P.K, tid, rb);
    }
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      bf16x8 fa[2], fb[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        fa[i] = gm_frag<AK>(la[cur], wm + 32 * i, ks, lane);
        fb[i] = gm_frag<BK_>(lb[cur], wn + 32 * i, ks, lane);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma32(fa[i], fb[j], acc[i][j]);
    }
    if (kt + 1 < nk) {
      gm_store<AK>(la[cur ^ 1], tid, ra);
      gm_store<BK_>(lb[cur ^ 1], tid, rb);
    }
    __syncthreads();
  }

  // ---- epilogue: C[row][col] with acc[i][j][r] = C[m0+wm+32i + (r&3)+8(r>>2)+4h][n0+wn+32j + l32]
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
        } else {
          bf16* c = (bf16*)P.C + o;
          *c = (bf16)(P.accumulate ? (float)*c + v : v);
        }
      }
  }
}

// ============================================================================================
// v2: LDS-DMA staged (global_load_lds, 16 B/lane), used when every problem has K % 64 == 0.
// 128x128x64 tiles, 2 LDS stages x (A 16 KB + B 16 KB), two raw barriers per K step with the
// next-but-one tile's DMA in flight across them (counted vmcnt, never __syncthreads).
// The DMA writes LDS linearly (wave base + 16 B x lane), so the bank-conflict swizzles are applied
// to the per-lane GLOBAL source addresses and undone on the fragment reads:
//   k-major tile  [128 rows][8 x 16-B chunks]: chunk c of row r stored at c ^ ((r >> 1) & 7)
//   mn-major tile [64 k-rows][16 chunks]:      chunk c of k-row k stored at c ^ (4 (k & 3))
template <bool AK, bool BK_>
__global__ __launch_bounds__(256) void gemm2_kernel(const GemmArgs args) {
  using namespace g2;
  __shared__ __attribute__((aligned(1024))) uint8_t lds[2][2][TILE_B];   // [stage][A/B]
  int pi = 0;
#pragma unroll
  for (int i = 1; i < gm::MAXP; ++i)
    if (i < args.nprob && (int)blockIdx.x >= args.p[i].tile_base) pi = i;
  const GemmProb& P = args.p[pi];
  if (P.a_kmajor != (int)AK || P.b_kmajor != (int)BK_) return;
  const int t = blockIdx.x - P.tile_base;
  const int tm = t / P.tiles_n, tn = t % P.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  if (m0 >= P.M) return;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;
  const int nkp = P.K / BK, nk = nkp * P.npass;   // K tiles per pass x passes (split.h)
  auto stage2 = [&](int kt, int st) {
    const int pass = kt / nkp, kk = kt - pass * nkp;
    g2_stage<AK>(gp_a(P, pass), P.lda, m0, P.M, kk * BK, lds[st][0], wave, lane);
    g2_stage<BK_>(gp_b(P, pass), P.ldb, n0, P.N, kk * BK, lds[st][1], wave, lane);
  };

  f32x16 acc[2][2] = {};
  stage2(0, 0);
  if (nk > 1) stage2(1, 1);
  for (int kt = 0; kt < nk; ++kt) {
    const int st = kt & 1;
    // tile kt has landed once at most the next tile's 2*GPW DMA ops remain outstanding
    if (kt + 1 < nk) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const uint8_t* la = lds[st][0];
    const uint8_t* lb = lds[st][1];
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      bf16x8 fa[2], fb[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        fa[i] = g2_frag<AK>(la, wm + 32 * i, ks, lane);
        fb[i] = g2_frag<BK_>(lb, wn + 32 * i, ks, lane);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma32(fa[i], fb[j], acc[i][j]);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();          // every wave is done reading stage st
    if (kt + 2 < nk) stage2(kt + 2, st);
  }

  g2_epilogue_lds(P, m0, n0, wm, wn, lane, acc, &lds[0][0][0]);
}

// ============================================================================================
// v4: 256 x BN x BK tiles (BN 256 or 128, BK 64 or 32), 8 waves (2 in M x 4 in N, two waves per
// SIMD), each wave 128 x BN/4 as 8 x BN/64 v_mfma_f32_16x16x32_bf16 accumulators.  One LDS array
// = NS buffers x {A, B}, filled by global_load_lds (16 B/lane) with the bank swizzle applied to
// the per-lane SOURCE address and undone on the fragment read; per K tile: counted wait for own
// DMA -> barrier -> DMA of tile k+NS-1 into the buffer everybody just finished -> fragment reads
// -> MFMAs.  The two waves of a SIMD overlap each other's fragment reads and barrier waits with
// MFMAs (cdna_hip_programming.md section 5.5, T3+T4 minimum form); blocks are remapped so
// consecutive tiles (same A rows) share an XCD and its L2.
//   k-major image   [rows][BK], 16-B chunk c of row r at c ^ ((r >> 1) & 7) (BK 64) or
//                   c ^ 3 ((r >> 3) & 1) (BK 32): conflict-free 16x16x32 fragment reads
//   mn-major image  per 128-column half: [BK][128], 256-B rows, chunk c of k-row k at
//                   c ^ 2 ((k & 3) | ((k >> 3) & 1) << 2): conflict-free transposed reads
// K % 8 == 0: 16-B chunks past K are DMA'd from a zero block, so a partial last K tile adds
// zeros; mn-major extents % 8 == 0.
// 16-B chunks past K are fetched from here
__device__ __attribute__((aligned(16))) bf16 g4_zero[8];

__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ int g4_mnswz(int k) { return 2 * ((k & 3) | (((k >> 3) & 1) << 2)); }

template <int BK>
__device__ __forceinline__ int g4_kswz(int r) { return BK == 64 ? ((r >> 1) & 7) : 3 * ((r >> 3) & 1); }

// Stage one R x BK operand tile (R*BK*2/1024 1-KB blocks dealt over the 8 waves).  Addresses are
// rebuilt every K tile from 32-bit offsets (oz = opaque zero): hoisting 64-bit pointers out of the
// K loop costs VGPRs the accumulators need.
template <bool KMAJ, int R, int BK>
__device__ __forceinline__ void g4_stage(const bf16* X, int ld, int i0, int imax, int k0, int kmax,
                                         uint8_t* tile, int wave, int lane, int oz) {
  constexpr int NBLK = R * BK * 2 / 1024, PW = NBLK / 8;
#pragma unroll
  for (int j = 0; j < PW; ++j) {
    const int blk = wave * PW + j;
    int off;
    bool kin;
    if (KMAJ) {
      constexpr int CPR = BK / 8, RPB = 64 / CPR;            // chunks per row, rows per block
      const int row = blk * RPB + lane / CPR, cp = lane % CPR;
      const int c = cp ^ g4_kswz<BK>(row);
      const int k = k0 + c * 8;
      kin = k < kmax;
      off = min(i0 + row, imax - 1) * ld + k;
    } else {
      constexpr int BPH = BK / 4;                            // blocks per 128-column half
      const int h = blk / BPH, kr = (blk % BPH) * 4 + (lane >> 4), cp = lane & 15;
      const int c = cp ^ g4_mnswz(kr);
      const int col = i0 + h * 128 + c * 8;
      kin = k0 + kr < kmax;
      off = (k0 + kr) * ld + (col < imax ? col : imax - 8);
    }
    const bf16* src = kin ? X + (off + oz) : g4_zero;
    __builtin_amdgcn_global_load_lds(src,
                                     (__attribute__((address_space(3))) void*)(tile + blk * 1024),
                                     16, 0, 0);
  }
}

// 16x16x32 fragment (k-step ks of the tile): lane l holds X[i0 + (l & 15)][32 ks + 8 (l >> 4) .. +7]
template <bool KMAJ, int R, int BK>
__device__ __forceinline__ bf16x8 g4_frag(const uint8_t* tile, int i0, int ks, int lane) {
  const int l16 = lane & 15, g = lane >> 4;
  if (KMAJ) {
    const int r = i0 + l16, c = 4 * ks + g;
    return *(const bf16x8*)(tile + r * (BK * 2) + ((c ^ g4_kswz<BK>(r)) * 16));
  }
  // tr read: within the 16-lane group, lane 4q+p addresses k-row (32ks + 8g + q), columns
  // i0 + 4p .. +3; the hardware hands lane i column i0+i's 4 k values (second read: k-rows +4)
  const int q = (lane >> 2) & 3, p = lane & 3;
  const uint8_t* half = tile + (i0 >> 7) * (BK * 256);
  const int kr = 32 * ks + 8 * g + q;
  const int c = ((i0 & 127) >> 3) + (p >> 1);
  const uint8_t* b0 = half + kr * 256 + ((c ^ g4_mnswz(kr)) * 16) + 8 * (p & 1);
  return gm_tr8((const bf16*)b0, (const bf16*)(b0 + 4 * 256));
}

template <int N>
__device__ __forceinline__ void g4_vmwait() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(%0)" :: "n"(N) : "memory");
}

template <bool AK, bool BK_, int BN, int BK, int NS>
__global__ __launch_bounds__(512) void gemm4_kernel(const GemmArgs args, int total_tiles) {
  constexpr int BM = 256, TNW = BN / 64, KS = BK / 32;
  constexpr int OPA = BM * BK * 2, OPB = BN * BK * 2, STB = OPA + OPB;
  constexpr int NDMA = (BM + BN) * BK * 2 / (512 * 16);   // DMA instructions per thread per K tile
  extern __shared__ __attribute__((aligned(1024))) uint8_t lds4[];
  // XCD remap (bijective): blocks b with equal b % 8 share an XCD; give each XCD a contiguous
  // range of tile ids so neighbouring tiles (same A rows) hit one L2
  int bid;
  {
    const int b = blockIdx.x, x = b & 7, qn = total_tiles >> 3, r = total_tiles & 7;
    bid = (x < r ? x * (qn + 1) : r * (qn + 1) + (x - r) * qn) + (b >> 3);
  }
  int pi = 0;
#pragma unroll
  for (int i = 1; i < gm::MAXP; ++i)
    if (i < args.nprob && bid >= args.p[i].tile_base) pi = i;
  const GemmProb& P = args.p[pi];
  if (P.a_kmajor != (int)AK || P.b_kmajor != (int)BK_) return;
  const int t = bid - P.tile_base;
  const int tm = t / P.tiles_n, tn = t % P.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  if (m0 >= P.M) return;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wr = wave >> 2, wc = wave & 3;
  const int nkp = (P.K + BK - 1) / BK, nk = nkp * P.npass;   // K tiles per pass x passes

  f32x4 acc[8][TNW];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < TNW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto stage = [&](int kt) {
    int oz;
    asm volatile("v_mov_b32 %0, 0" : "=v"(oz));
    uint8_t* st = lds4 + (kt % NS) * STB;
    const int pass = kt / nkp, kk = kt - pass * nkp;
    g4_stage<AK, BM, BK>(gp_a(P, pass), P.lda, m0, P.M, kk * BK, P.K, st, wave, lane, oz);
    g4_stage<BK_, BN, BK>(gp_b(P, pass), P.ldb, n0, P.N, kk * BK, P.K, st + OPA, wave, lane, oz);
  };
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < nk) stage(s);
  for (int kt = 0; kt < nk; ++kt) {
    // tile kt has landed once only the DMAs of tiles kt+1 .. kt+NS-2 (those issued) remain
    const int ahead = nk - 1 - kt;
    if (NS >= 4 && ahead >= 2) g4_vmwait<(NS >= 4 ? 2 : 0) * NDMA>();
    else if (NS >= 3 && ahead >= 1) g4_vmwait<(NS >= 3 ? 1 : 0) * NDMA>();
    else g4_vmwait<0>();
    __builtin_amdgcn_s_barrier();     // tile kt visible; everyone finished reading tile kt-1
    if (kt + NS - 1 < nk) stage(kt + NS - 1);
    const uint8_t* la = lds4 + (kt % NS) * STB;
    const uint8_t* lb = la + OPA;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      bf16x8 fa[8], fb[TNW];
#pragma unroll
      for (int j = 0; j < TNW; ++j) fb[j] = g4_frag<BK_, BN, BK>(lb, wc * (BN / 4) + 16 * j, ks, lane);
#pragma unroll
      for (int i = 0; i < 8; ++i) fa[i] = g4_frag<AK, BM, BK>(la, wr * 128 + 16 * i, ks, lane);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < TNW; ++j) acc[i][j] = mfma16(fa[i], fb[j], acc[i][j]);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
    }
  }

  // C[m0 + wr*128 + 16i + 4(l>>4) + e][n0 + wc*BN/4 + 16j + (l&15)] = acc[i][j][e], staged
  // through LDS two i at a time (64 rows x BN fp32) and stored row-contiguous, 4 columns per
  // thread (the per-element register epilogue was 7k instructions behind 800 branches)
  constexpr int LS = BN + 16;                  // fp32 row stride: rows 4g+e on disjoint banks
  float* L = (float*)lds4;
  const int l16 = lane & 15, g = lane >> 4;
  const bool f32 = P.c_f32 != 0;
  const bool vec = ((uintptr_t)P.C % 16 == 0) && (P.ldc % 4 == 0);
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
      for (int j = 0; j < TNW; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          L[(wr * 32 + ii * 16 + 4 * g + e) * LS + wc * (BN / 4) + 16 * j + l16] = acc[2 * p + ii][j][e];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
#pragma unroll 2
    for (int q = tid; q < 64 * (BN / 4); q += 512) {
      const int lr = q / (BN / 4), cc = (q % (BN / 4)) * 4;
      const int row = m0 + (lr >> 5) * 128 + 32 * p + (lr & 31);
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

template <int BN, int BK, int NS>
static int g4_launch(GemmArgs& a, int ak, int bk, hipStream_t s) {
  constexpr int LDS = NS * (256 + BN) * BK * 2;
  static_assert(LDS <= 160 * 1024, "LDS");
  int tiles = 0;
  for (int i = 0; i < a.nprob; ++i) {
    GemmProb& p = a.p[i];
    p.tiles_n = (p.N + BN - 1) / BN;
    p.tile_base = tiles;
    tiles += p.tiles_n * ((p.M + 255) / 256);
  }
  for (int i = a.nprob; i < gm::MAXP; ++i) a.p[i] = a.p[0], a.p[i].tile_base = 1 << 30;
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)gemm4_kernel<true, true, BN, BK, NS>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    hipFuncSetAttribute((const void*)gemm4_kernel<true, false, BN, BK, NS>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    hipFuncSetAttribute((const void*)gemm4_kernel<false, true, BN, BK, NS>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    hipFuncSetAttribute((const void*)gemm4_kernel<false, false, BN, BK, NS>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    attr = true;
  }
  if (ak && bk) hipLaunchKernelGGL((gemm4_kernel<true, true, BN, BK, NS>), dim3(tiles), dim3(512), LDS, s, a, tiles);
  else if (ak) hipLaunchKernelGGL((gemm4_kernel<true, false, BN, BK, NS>), dim3(tiles), dim3(512), LDS, s, a, tiles);
  else if (bk) hipLaunchKernelGGL((gemm4_kernel<false, true, BN, BK, NS>), dim3(tiles), dim3(512), LDS, s, a, tiles);
  else hipLaunchKernelGGL((gemm4_kernel<false, false, BN, BK, NS>), dim3(tiles), dim3(512), LDS, s, a, tiles);
  R2_CHECK_LAUNCH();
  return 0;
}

// ============================================================================================
// v3: the v2 tile (128x128x64, 4 waves, LDS-DMA, swizzled images) with an NS-stage ring: the
// DMA of tile k+NS-1 is issued right after the barrier of tile k into the buffer every wave just
// finished, so each tile has NS-1 tile-times to land (v2's 1-tile prefetch stalled on L2/HBM
// latency at these K: dW_ih at K = 2560 ran at ~16 % of the CU's MFMA rate).  One barrier per K
// tile, counted vmcnt, XCD-aware tile order (consecutive tiles share A rows and one L2).
template <bool AK, bool BK_, int NS>
__global__ __launch_bounds__(256) void gemm3_kernel(const GemmArgs args, int total_tiles) {
  using namespace g2;
  extern __shared__ __attribute__((aligned(1024))) uint8_t lds3[];
  int bid;
  {
    const int b = blockIdx.x, x = b & 7, qn = total_tiles >> 3, r = total_tiles & 7;
    bid = (x < r ? x * (qn + 1) : r * (qn + 1) + (x - r) * qn) + (b >> 3);
  }
  int pi = 0;
#pragma unroll
  for (int i = 1; i < gm::MAXP; ++i)
    if (i < args.nprob && bid >= args.p[i].tile_base) pi = i;
  const GemmProb& P = args.p[pi];
  if (P.a_kmajor != (int)AK || P.b_kmajor != (int)BK_) return;
  const int t = bid - P.tile_base;
  const int tm = t / P.tiles_n, tn = t % P.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  if (m0 >= P.M) return;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;
  const int nk = P.K / BK;
  auto stage = [&](int kt) {
    uint8_t* st = lds3 + (kt % NS) * (2 * TILE_B);
    g2_stage<AK>(P.A, P.lda, m0, P.M, kt * BK, st, wave, lane);
    g2_stage<BK_>(P.B, P.ldb, n0, P.N, kt * BK, st + TILE_B, wave, lane);
  };

  f32x16 acc[2][2] = {};
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < nk) stage(s);
  for (int kt = 0; kt < nk; ++kt) {
    // tile kt has landed once only the stages issued after it (at most NS-2) remain
    const int ahead = min(NS - 2, nk - 1 - kt);
    if (ahead >= 2) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else if (ahead == 1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();       // tile kt visible; every wave done with tile kt-1
    if (kt + NS - 1 < nk) stage(kt + NS - 1);
    const uint8_t* la = lds3 + (kt % NS) * (2 * TILE_B);
    const uint8_t* lb = la + TILE_B;
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      bf16x8 fa[2], fb[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        fa[i] = g2_frag<AK>(la, wm + 32 * i, ks, lane);
        fb[i] = g2_frag<BK_>(lb, wn + 32 * i, ks, lane);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma32(fa[i], fb[j], acc[i][j]);
    }
  }

  g2_epilogue_lds(P, m0, n0, wm, wn, lane, acc, lds3);
}

template <int NS>
static int g3_launch(GemmArgs& a, int ak, int bk, int tiles, hipStream_t s) {
  constexpr int LDS = NS * 2 * g2::TILE_B;
  static_assert(LDS <= 160 * 1024, "LDS");
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)gemm3_kernel<true, true, NS>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    hipFuncSetAttribute((const void*)gemm3_kernel<true, false, NS>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    hipFuncSetAttribute((const void*)gemm3_kernel<false, true, NS>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    hipFuncSetAttribute((const void*)gemm3_kernel<false, false, NS>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    attr = true;
  }
  if (ak && bk) hipLaunchKernelGGL((gemm3_kernel<true, true, NS>), dim3(tiles), dim3(256), LDS, s, a, tiles);
  else if (ak) hipLaunchKernelGGL((gemm3_kernel<true, false, NS>), dim3(tiles), dim3(256), LDS, s, a, tiles);
  else if (bk) hipLaunchKernelGGL((gemm3_kernel<false, true, NS>), dim3(tiles), dim3(256), LDS, s, a, tiles);
  else hipLaunchKernelGGL((gemm3_kernel<false, false, NS>), dim3(tiles), dim3(256), LDS, s, a, tiles);
  R2_CHECK_LAUNCH();
  return 0;
}

// ============================================================================================
// Grouped split-K launch: up to 4 problems with their own A layout (B mn-major) and K split
// in ONE grid, items ordered as given (put the longest first).  A split item computes its K
// range, publishes the fp32 partial tile write-through, takes the tile's ticket; the last
// arriver sums ALL partials in split order (bit-reproducible) and runs the epilogue.  Two
// 64-KB-LDS workgroups fit per CU, so e.g. the learner's weight-gradient products (K = 2560,
// 128 tiles) and dX (260 tiles) share the chip instead of running one after the other.
struct GroupArgs {
  GemmProb p[gm::MAXP];
  int split[gm::MAXP];
  int item_base[gm::MAXP + 1];
  int slab_base[gm::MAXP];     // first partial slab (64 KB) of each problem
  int ticket_base[gm::MAXP];
  int np, total;
  float* ws;
  unsigned* tickets;
};

__global__ __launch_bounds__(256) void gemm_group_kernel(const GroupArgs a) {
  __shared__ __attribute__((aligned(1024))) uint8_t lds[2 * 2 * g2::TILE_B];
  __shared__ int last;
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
  const int tile = item / S, ks = item % S;
  const int tm = tile / P.tiles_n, tn = tile % P.tiles_n;
  const int nk = P.K / g2::BK * P.npass, per = (nk + S - 1) / S;
  const int kt0 = min(nk, ks * per), kt1 = min(nk, kt0 + per);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  f32x16 acc[2][2] = {};
  auto none = [](int) {};
  if (P.a_kmajor) g2_tile_acc<true, false, 0>(P, tm, tn, lds, kt0, kt1, false, none, acc);
  else g2_tile_acc<false, false, 0>(P, tm, tn, lds, kt0, kt1, false, none, acc);
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;
  if (S > 1) {
    // partial slab: 16 x (256 threads x 16 B), lane-major so each b128 store / load of a wave
    // covers 1 KB of whole cache lines (thread-major rows made every write-through store touch
    // 64 lines for 16 B each: 0.1 us per split item)
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(a.ws, 0, 0x7fffffff, 0x00020000);
    const int slab0 = a.slab_base[pi] + tile * S;
    auto off = [&](int s, int q) { return (uint32_t)((((size_t)(slab0 + s) * 16 + q) * 256 + tid) * 16); };
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const f32x4 v = {acc[q >> 3][(q >> 2) & 1][4 * (q & 3)], acc[q >> 3][(q >> 2) & 1][4 * (q & 3) + 1],
                       acc[q >> 3][(q >> 2) & 1][4 * (q & 3) + 2], acc[q >> 3][(q >> 2) & 1][4 * (q & 3) + 3]};
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, off(ks, q), 0, 16);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    unsigned* tk = a.tickets + a.ticket_base[pi] + tile;
    if (tid == 0) last = __hip_atomic_fetch_add(tk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)(S - 1);
    __syncthreads();
    if (!last) return;
    f32x16 sum[2][2] = {};
    for (int s = 0; s < S; ++s) {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        f32x4 v;
        if (s == ks) {
          v = f32x4{acc[q >> 3][(q >> 2) & 1][4 * (q & 3)], acc[q >> 3][(q >> 2) & 1][4 * (q & 3) + 1],
                    acc[q >> 3][(q >> 2) & 1][4 * (q & 3) + 2], acc[q >> 3][(q >> 2) & 1][4 * (q & 3) + 3]};
        } else {
          v = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off(s, q), 0, 16));
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) sum[q >> 3][(q >> 2) & 1][4 * (q & 3) + e] += v[e];
      }
    }
    if (tid == 0) __hip_atomic_store(tk, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    g2_epilogue_lds(P, tm * g2::BM, tn * g2::BN, wm, wn, lane, sum, lds);
    return;
  }
  g2_epilogue_lds(P, tm * g2::BM, tn * g2::BN, wm, wn, lane, acc, lds);
}

// descs: np x 16 int64 (ops/gemm.py layout); split[i] >= 1; ws: sum over split problems of
// tiles * split * 64 KB; tickets: one per tile of split problems, zero at first use.
extern "C" long long r2_gemm_group_ws_bytes(const int64_t* descs, const int* split, int np) {
  long long b = 0;
  for (int i = 0; i < np; ++i) {
    GemmProb p;
    if (gemm_parse_desc(descs + GEMM_DESC * i, p)) return -1;
    if (split[i] > 1) b += (long long)p.tiles_n * ((p.M + 127) / 128) * split[i] * 65536;
  }
  return b;
}

extern "C" int r2_gemm_group(const int64_t* descs, const int* split, int np, float* ws,
                             long long ws_bytes, unsigned* tickets, int n_tickets, void* stream) {
  if (np < 1 || np > gm::MAXP) return -1;
  GroupArgs a;
  a.np = np; a.ws = ws; a.tickets = tickets;
  int items = 0, slabs = 0, tks = 0;
  for (int i = 0; i < np; ++i) {
    GemmProb& p = a.p[i];
    const int rc = gemm_parse_desc(descs + GEMM_DESC * i, p);
    if (rc) return rc;
    if (p.K % 64 || p.b_kmajor || (!p.a_kmajor && p.M % 8)) return -6;
    const int tiles = p.tiles_n * ((p.M + 127) / 128);
    const int S = split[i] < 1 ? 1 : split[i];
    a.split[i] = S;
    a.item_base[i] = items;
    a.slab_base[i] = slabs;
    a.ticket_base[i] = tks;
    items += tiles * S;
    if (S > 1) { slabs += tiles * S; tks += tiles; }
  }
  for (int i = np; i < gm::MAXP; ++i) { a.p[i] = a.p[0]; a.split[i] = 1; a.item_base[i] = 1 << 30; }
  a.item_base[gm::MAXP] = items;
  a.total = items;
  if ((long long)slabs * 65536 > ws_bytes || tks > n_tickets) return -7;
  hipLaunchKernelGGL(gemm_group_kernel, dim3(items), dim3(256), 0, (hipStream_t)stream, a);
  R2_CHECK_LAUNCH();
  return 0;
}

static int g_gemm_version = 2;   // 1 = force the register-staged kernel (tests / A-B)
extern "C" int r2_gemm_set_version(int v) { g_gemm_version = v; return 0; }

// descs: nprob x GEMM_DESC int64 {A, B, C, bias, crow, M, N, K, lda, ldb, ldc, a_kmajor, b_kmajor,
// c_f32, accumulate, alpha_bits, A_lo, B_lo, C_lo, 0} (lo planes: split.h; null = not split).  All problems of one call must share (a_kmajor, b_kmajor).
extern "C" int r2_gemm(const int64_t* descs, int nprob, void* stream) {
  if (nprob < 1 || nprob > gm::MAXP) return -1;
  GemmArgs a;
  a.nprob = nprob;
  int tiles = 0, ak = -1, bk = -1;
  bool any_split = false;
  for (int i = 0; i < nprob; ++i) {
    GemmProb& p = a.p[i];
    const int rc = gemm_parse_desc(descs + GEMM_DESC * i, p);
    if (rc) return rc;
    any_split = any_split || p.npass > 1 || p.C_lo;
    if (ak < 0) { ak = p.a_kmajor; bk = p.b_kmajor; }
    if (ak != p.a_kmajor || bk != p.b_kmajor) return -5;
    p.tiles_n = (p.N + gm::BN - 1) / gm::BN;
    p.tile_base = tiles;
    tiles += p.tiles_n * ((p.M + gm::BM - 1) / gm::BM);
  }
  for (int i = nprob; i < gm::MAXP; ++i) a.p[i] = a.p[0], a.p[i].tile_base = 1 << 30;
  hipStream_t s = (hipStream_t)stream;
  bool k8 = true;
  long t256 = 0;
  for (int i = 0; i < nprob; ++i) {
    k8 = k8 && a.p[i].K % 8 == 0;
    t256 += (long)((a.p[i].M + 255) / 256) * ((a.p[i].N + 255) / 256);
  }
  if (any_split) {
    // split precision runs on the LDS-DMA kernels only (the pass loop lives in their staging)
    if (k8 && (t256 >= 150 || g_gemm_version == 5)) return g4_launch<256, 64, 2>(a, ak, bk, s);
    for (int i = 0; i < nprob; ++i)
      if (a.p[i].K % g2::BK) return g4_launch<128, 64, 3>(a, ak, bk, s);
    if (ak && bk) hipLaunchKernelGGL((gemm2_kernel<true, true>), dim3(tiles), dim3(g2::NT), 0, s, a);
    else if (ak) hipLaunchKernelGGL((gemm2_kernel<true, false>), dim3(tiles), dim3(g2::NT), 0, s, a);
    else if (bk) hipLaunchKernelGGL((gemm2_kernel<false, true>), dim3(tiles), dim3(g2::NT), 0, s, a);
    else hipLaunchKernelGGL((gemm2_kernel<false, false>), dim3(tiles), dim3(g2::NT), 0, s, a);
    R2_CHECK_LAUNCH();
    return 0;
  }
  if (g_gemm_version >= 5 && g_gemm_version <= 8 && k8) {   // forced 8-wave variants (tests / micro-benchmarks)
    switch (g_gemm_version) {
      case 5: return g4_launch<256, 64, 2>(a, ak, bk, s);
      case 6: return g4_launch<256, 32, 4>(a, ak, bk, s);
      case 7: return g4_launch<128, 64, 3>(a, ak, bk, s);
      default: return g4_launch<128, 32, 4>(a, ak, bk, s);
    }
  }
  // auto: launches with enough 256x256 tiles to cover most CUs (the x-projection of both nets:
  // 176) run the 8-wave kernel (70 vs 83 us there); fewer, larger-K tiles stay on 128x128, where
  // per-CU operand traffic, not MFMA issue, bounds all of these shapes (tools/pmc_gemm.sh)
  if (g_gemm_version == 2 && k8 && t256 >= 150) return g4_launch<256, 64, 2>(a, ak, bk, s);
  bool v2 = g_gemm_version >= 2;
  for (int i = 0; i < nprob; ++i) v2 = v2 && a.p[i].K % g2::BK == 0;
  if (v2 && g_gemm_version == 9) return g3_launch<3>(a, ak, bk, tiles, s);
  if (v2 && g_gemm_version == 10) return g3_launch<4>(a, ak, bk, tiles, s);
  if (v2) {
    if (ak && bk) hipLaunchKernelGGL((gemm2_kernel<true, true>), dim3(tiles), dim3(g2::NT), 0, s, a);
    else if (ak) hipLaunchKernelGGL((gemm2_kernel<true, false>), dim3(tiles), dim3(g2::NT), 0, s, a);
    else if (bk) hipLaunchKernelGGL((gemm2_kernel<false, true>), dim3(tiles), dim3(g2::NT), 0, s, a);
    else hipLaunchKernelGGL((gemm2_kernel<false, false>), dim3(tiles), dim3(g2::NT), 0, s, a);
    R2_CHECK_LAUNCH();
    return 0;
  }
  if (ak && bk) hipLaunchKernelGGL((gemm_kernel<true, true>), dim3(tiles), dim3(gm::NT), 0, s, a);
  else if (ak) hipLaunchKernelGGL((gemm_kernel<true, false>), dim3(tiles), dim3(gm::NT), 0, s, a);
  else if (bk) hipLaunchKernelGGL((gemm_kernel<false, true>), dim3(tiles), dim3(gm::NT), 0, s, a);
  else hipLaunchKernelGGL((gemm_kernel<false, false>), dim3(tiles), dim3(gm::NT), 0, s, a);
  R2_CHECK_LAUNCH();
  return 0;
}
