// LDS-DMA fill rate of the split GEMM's operand pattern (gfx950): the x-projection's tiles
// (164 workgroups of 256 A rows x 256 B rows, hi and lo planes, K = 1568 bf16 = 3136 B per row)
// streamed through global_load_lds with W bytes of each row per stage (W = 32 / 64 / 128: the
// 16- / 32- / 64-deep K tiles) and D stages in flight (counted vmcnt).  Nothing is computed; the
// LDS destination cycles over 64 KB (the bytes are not read).  Prints per-CU GB/s.  The same
// stream through VGPRs (global_load_dwordx4 + ds_write_b128, two register stages) for comparison.
//   hipcc --offload-arch=gfx950 -O3 tools/micro/dma_rate.hip -o /tmp/dma_rate && /tmp/dma_rate
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

constexpr int AR = 256, BR = 256, KB = 3136;   // rows per tile, bytes per row

template <int N>
__device__ __forceinline__ void vmw() { asm volatile("s_waitcnt vmcnt(%0)" :: "n"(N) : "memory"); }

template <int W, int D>
__global__ __launch_bounds__(512) void k(const uint8_t* A, const uint8_t* Al, const uint8_t* B,
                                         const uint8_t* Bl, int tiles_n) {
  extern __shared__ __attribute__((aligned(1024))) uint8_t lds[];
  constexpr int LPR = W / 16;                    // lanes per row
  constexpr int RPI = 64 / LPR;                  // rows per DMA instruction
  constexpr int NI = 2 * (AR + BR) / RPI;        // DMA instructions per stage
  constexpr int PW = NI / 8;                     // per wave
  static_assert(NI % 8 == 0, "even");
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int tm = blockIdx.x / tiles_n, tn = blockIdx.x % tiles_n;
  const uint8_t* src[PW];
  for (int i = 0; i < PW; ++i) {
    const int blk = wave * PW + i;
    const int row = blk * RPI + lane / LPR;      // over [A hi | A lo | B hi | B lo] rows
    const uint8_t* base;
    int r;
    if (row < AR) { base = A; r = tm * AR + row; }
    else if (row < 2 * AR) { base = Al; r = tm * AR + row - AR; }
    else if (row < 2 * AR + BR) { base = B; r = tn * BR + row - 2 * AR; }
    else { base = Bl; r = tn * BR + row - 2 * AR - BR; }
    src[i] = base + (size_t)r * KB + 16 * (lane % LPR);
  }
  const int nst = KB / W;
  for (int s = 0; s < nst; ++s) {
#pragma unroll
    for (int i = 0; i < PW; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(src[i] + s * W),
                                       (__attribute__((address_space(3))) void*)(lds + ((s * PW + wave * PW + i) & 63) * 1024),
                                       16, 0, 0);
    if (s >= D) vmw<D * PW>();
  }
  vmw<0>();
}

// the same operand stream through VGPRs: global_load_dwordx4 of stage s+1 issued before the
// ds_write_b128 of stage s (two register stages)
template <int W>
__global__ __launch_bounds__(512) void kr(const uint8_t* A, const uint8_t* Al, const uint8_t* B,
                                          const uint8_t* Bl, int tiles_n) {
  extern __shared__ __attribute__((aligned(1024))) uint8_t lds[];
  constexpr int LPR = W / 16, RPI = 64 / LPR, PW = 128 / RPI, NST = KB / W;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int tm = blockIdx.x / tiles_n, tn = blockIdx.x % tiles_n;
  // wave w: 128 rows of plane w / 2 ([A hi | A lo | B hi | B lo]), rows (w & 1) * 128 + ...
  const int plane = wave >> 1;
  const uint8_t* base = plane == 0 ? A : plane == 1 ? Al : plane == 2 ? B : Bl;
  const int r0 = (plane < 2 ? tm * AR : tn * BR) + (wave & 1) * 128;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)(base + (size_t)r0 * KB), 0, 128 * KB, 0x00020000);
  const int voff = (lane / LPR) * KB + 16 * (lane % LPR);
  int4 b0[PW], b1[PW];
  auto ld = [&](int4* b, int s) {
#pragma unroll
    for (int i = 0; i < PW; ++i)
      b[i] = __builtin_bit_cast(int4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff + i * RPI * KB, s * W, 0));
  };
  auto st = [&](const int4* b, int s) {
#pragma unroll
    for (int i = 0; i < PW; ++i)
      *(int4*)(lds + (((s * PW + wave * PW + i) & 63) * 1024) + lane * 16) = b[i];
  };
  ld(b0, 0);
  for (int s = 0; s < NST; s += 2) {
    if (s + 1 < NST) ld(b1, s + 1);
    st(b0, s);
    if (s + 2 < NST) ld(b0, s + 2);
    if (s + 1 < NST) st(b1, s + 1);
  }
}

template <int W>
void runr(const uint8_t* A, const uint8_t* Al, const uint8_t* B, const uint8_t* Bl) {
  const int tiles_n = 4, grid = 41 * 4;
  hipFuncSetAttribute((const void*)kr<W>, hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((kr<W>), dim3(grid), dim3(512), 65536, 0, A, Al, B, Bl, tiles_n);
  hipEventRecord(e0);
  const int reps = 20;
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((kr<W>), dim3(grid), dim3(512), 65536, 0, A, Al, B, Bl, tiles_n);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double us = ms * 1000.0 / reps;
  const double bytes = (double)grid * 2 * (AR + BR) * KB;
  printf("VGPR path W=%3d B/row-stage  2 register stages  %7.1f us  %6.1f GB/s per CU  %5.2f TB/s\n",
         W, us, bytes / us / 1e3 / grid, bytes / us / 1e6);
}

template <int W, int D>
void run(const uint8_t* A, const uint8_t* Al, const uint8_t* B, const uint8_t* Bl) {
  const int tiles_n = 4, grid = 41 * 4;   // 41 row tiles of 256 (of 10560) x 1024 / 256
  hipFuncSetAttribute((const void*)k<W, D>, hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((k<W, D>), dim3(grid), dim3(512), 65536, 0, A, Al, B, Bl, tiles_n);
  hipEventRecord(e0);
  const int reps = 20;
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((k<W, D>), dim3(grid), dim3(512), 65536, 0, A, Al, B, Bl, tiles_n);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double us = ms * 1000.0 / reps;
  const double bytes = (double)grid * 2 * (AR + BR) * KB;
  const int inflight_kb = D * 2 * (AR + BR) * W / 1024;
  printf("W=%3d B/row-stage  D=%d stages in flight (%3d KB)  %7.1f us  %6.1f GB/s per CU  %5.2f TB/s\n",
         W, D, inflight_kb, us, bytes / us / 1e3 / grid, bytes / us / 1e6);
}

int main() {
  uint8_t *A, *Al, *B, *Bl;
  hipMalloc(&A, (size_t)10560 * KB);
  hipMalloc(&Al, (size_t)10560 * KB);
  hipMalloc(&B, (size_t)1024 * KB);
  hipMalloc(&Bl, (size_t)1024 * KB);
  hipMemset(A, 1, (size_t)10560 * KB);
  hipMemset(Al, 1, (size_t)10560 * KB);
  hipMemset(B, 1, (size_t)1024 * KB);
  hipMemset(Bl, 1, (size_t)1024 * KB);
  run<32, 1>(A, Al, B, Bl);
  run<32, 2>(A, Al, B, Bl);
  run<32, 4>(A, Al, B, Bl);
  run<64, 1>(A, Al, B, Bl);
  run<64, 2>(A, Al, B, Bl);
  run<128, 1>(A, Al, B, Bl);
  run<128, 2>(A, Al, B, Bl);
  runr<32>(A, Al, B, Bl);
  runr<64>(A, Al, B, Bl);
  runr<128>(A, Al, B, Bl);
  hipDeviceSynchronize();
  return 0;
}
