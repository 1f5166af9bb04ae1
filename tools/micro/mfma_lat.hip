// MFMA issue / dependency micro-benchmark (gfx950): cycles per MFMA for chains over 1, 3, 6
// independent accumulators, int8 16x16x64 vs bf16 16x16x32, one wave per SIMD (256 threads).
//   hipcc --offload-arch=gfx950 -O3 tools/micro/mfma_lat.hip -o /tmp/mfma_lat && /tmp/mfma_lat
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

template <int NACC, bool I8>
__global__ void k(long long* out, int* sink, int iters) {
  const int tx = (int)threadIdx.x;
  i32x4 a = {tx, 1, 2, 3}, b = {3, tx, 1, 2};
  i32x4 ai[NACC];
  f32x4 af[NACC];
  bf16x8 x, y;
  for (int e = 0; e < 8; ++e) { x[e] = (__bf16)(float)(threadIdx.x + e); y[e] = (__bf16)(float)e; }
  for (int j = 0; j < NACC; ++j) { ai[j] = i32x4{0, 0, 0, 0}; af[j] = f32x4{0, 0, 0, 0}; }
  long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 12 / NACC; ++r)
#pragma unroll
      for (int j = 0; j < NACC; ++j) {
        if (I8) ai[j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, ai[j], 0, 0, 0);
        else af[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x, y, af[j], 0, 0, 0);
      }
  }
  long long t1 = __builtin_readcyclecounter();
  int s = 0;
  for (int j = 0; j < NACC; ++j) s += ai[j][0] + (int)af[j][0];
  sink[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = t1 - t0;
}

template <int NACC, bool I8>
void run(long long* d, int* sink) {
  const int iters = 1000;
  hipLaunchKernelGGL((k<NACC, I8>), dim3(1), dim3(256), 0, 0, d, sink, iters);
  hipLaunchKernelGGL((k<NACC, I8>), dim3(1), dim3(256), 0, 0, d, sink, iters);
  long long h;
  hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
  printf("%s acc=%d: %.1f cycles per MFMA\n", I8 ? "i8 16x16x64 " : "bf16 16x16x32", NACC, (double)h / (iters * 12));
}

int main() {
  long long* d;
  int* sink;
  hipMalloc(&d, 8);
  hipMalloc(&sink, 4096 * 4);
  run<1, true>(d, sink); run<3, true>(d, sink); run<6, true>(d, sink); run<12, true>(d, sink);
  run<1, false>(d, sink); run<3, false>(d, sink); run<6, false>(d, sink); run<12, false>(d, sink);
  return 0;
}
