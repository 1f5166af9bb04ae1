// Stream placement helpers: CU-masked HIP streams and a placement probe.
//
// The concurrent actor / learner topology (runner.run_native, concurrent=True) runs the batched
// actor's short kernels and the learner's persistent recurrence kernels at the same time on one
// MI355X.  The persistent kernels need their whole grid co-resident (one workgroup per CU), so the
// two roles get DISJOINT CU sets: each role's stream is created with a CU mask
// (hipExtStreamCreateWithCUMask) and the learner sizes its persistent grids to the CUs of its mask
// (r2_set_num_cus).  The probe reports (XCC id, HW_ID) of every workgroup of a launch so the mask
// bit -> (XCD, CU) mapping can be measured on the device instead of assumed.
#include "../common.h"

// mask: nwords 32-bit words, bit i = logical CU i.  Returns 0 and the stream in *out.
extern "C" int r2_stream_create_cumask(const uint32_t* mask, int nwords, void** out) {
  if (!mask || nwords <= 0 || !out) return -1;
  hipStream_t s = nullptr;
  const hipError_t e = hipExtStreamCreateWithCUMask(&s, (uint32_t)nwords, mask);
  if (e != hipSuccess) return -(int)e - 100;
  *out = (void*)s;
  return 0;
}

extern "C" int r2_stream_get_cumask(void* stream, uint32_t* mask, int nwords) {
  return hipExtStreamGetCUMask((hipStream_t)stream, (uint32_t)nwords, mask) == hipSuccess ? 0 : -1;
}

extern "C" int r2_stream_destroy(void* stream) {
  return hipStreamDestroy((hipStream_t)stream) == hipSuccess ? 0 : -1;
}

__global__ void cu_probe_kernel(int* out, int spin) {
  if (threadIdx.x == 0) {
    unsigned x, hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    out[2 * blockIdx.x] = (int)(x & 15);
    out[2 * blockIdx.x + 1] = (int)hw;
  }
  for (int i = 0; i < spin; ++i) __builtin_amdgcn_s_sleep(127);
}

// out: 2 ints per block {xcc, HW_ID}; spin keeps each block resident a while (forces spreading)
extern "C" int r2_cu_probe(int* out, int nblocks, int spin, void* stream) {
  if (nblocks <= 0) return -1;
  hipLaunchKernelGGL(cu_probe_kernel, dim3(nblocks), dim3(64), 0, (hipStream_t)stream, out, spin);
  R2_CHECK_LAUNCH();
  return 0;
}

// Async host -> device copy (pinned or registered host memory) on `stream`; the ingest path's
// staging copy (engine/ingest.py).  Kept here so the ingest needs no torch allocation per record.
extern "C" int r2_memcpy_h2d_async(void* dst, const void* src, long long bytes, void* stream) {
  if (bytes <= 0) return 0;
  return hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyHostToDevice, (hipStream_t)stream) ==
                 hipSuccess ? 0 : -1;
}

extern "C" int r2_host_register(void* p, long long bytes) {
  return hipHostRegister(p, (size_t)bytes, hipHostRegisterDefault) == hipSuccess ? 0 : -1;
}

extern "C" int r2_host_unregister(void* p) {
  return hipHostUnregister(p) == hipSuccess ? 0 : -1;
}
