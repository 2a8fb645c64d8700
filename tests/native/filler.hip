// Test-only helper (NOT part of libaaa.so): a "filler" kernel that keeps
// ``wgs`` workgroups resident for ``usec`` microseconds, each holding 96 KB of
// LDS and 256 threads, so no frame-resident ConvLSTM workgroup (> 80 KB of LDS,
// one wave per SIMD at full register use) can share its CU.  tests/
// test_gpu_coresidency.py launches it on a second stream just before a
// multi-workgroup frame-resident launch to check that partners which cannot be
// placed until the filler drains are waited for (no timeout, same results)
// rather than stranded -- the situation a collective kernel beside such a
// launch would create.
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ void __launch_bounds__(256) k_filler(long ticks, float* sink) {
  __shared__ float pad[24576];   // 96 KB
  pad[threadIdx.x * 96] = (float)threadIdx.x;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < (uint64_t)ticks) __builtin_amdgcn_s_sleep(32);
  __syncthreads();
  if (sink && threadIdx.x == 0) sink[blockIdx.x] = pad[(blockIdx.x & 255) * 96];
}

extern "C" int aaa_test_filler(int wgs, long usec, float* sink, hipStream_t st) {
  if (wgs < 1 || wgs > 4096 || usec < 0 || usec > 2000000) return -1;
  hipLaunchKernelGGL(k_filler, dim3(wgs), dim3(256), 0, st, usec * 100, sink);   // 100-MHz real-time counter
  return hipGetLastError() == hipSuccess ? 0 : -3;
}
