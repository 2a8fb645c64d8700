// Diagnostic: does fp32 VALU FMA work run beside fp32 MFMA (v_mfma_f32_32x32x2_f32)
// on the same SIMD, or do they share the f32 multipliers?  512-thread workgroups,
// two waves per SIMD: waves 0-3 issue MFMAs, waves 4-7 issue v_fma_f32 / v_pk_fma_f32
// chains (independent registers).  Reports each role alone and both together.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

typedef float f16v __attribute__((ext_vector_type(16)));
typedef float f2v __attribute__((ext_vector_type(2)));

// mode bit0: MFMA waves active, bit1: VALU waves active, bit2: VALU uses v_pk_fma_f32,
// bit3: same wave does both (all 8 waves, interleaved)
__global__ __launch_bounds__(512) void k_coexec(int iters, int mode, float* out) {
  const int wave = threadIdx.x >> 6;
  const bool mf_role = (mode & 8) ? true : wave < 4;
  const bool va_role = (mode & 8) ? true : wave >= 4;
  float a = threadIdx.x * 1e-3f, b = 1.0001f;
  f16v acc[4];
  for (int i = 0; i < 4; ++i) acc[i] = f16v{0};
  float v[16];
  f2v pv[8];
  for (int i = 0; i < 16; ++i) v[i] = a + i;
  for (int i = 0; i < 8; ++i) pv[i] = f2v{a + i, a - i};
  const f2v pb = f2v{b, b}, pc = f2v{1e-7f, 1e-7f};
  const bool do_mf = (mode & 1) && mf_role, do_va = (mode & 2) && va_role, pk = mode & 4;
  for (int it = 0; it < iters; ++it) {
    if (do_mf) {
#pragma unroll
      for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[i], 0, 0, 0);
    }
    if (do_va) {
      if (pk) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
#pragma unroll
          for (int i = 0; i < 8; ++i) asm volatile("v_pk_fma_f32 %0, %1, %2, %3" : "+v"(pv[i]) : "v"(pv[i]), "v"(pb), "v"(pc));
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r)
#pragma unroll
          for (int i = 0; i < 16; ++i) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(v[i]) : "v"(v[i]), "v"(b));
      }
    }
  }
  float s = 0;
  for (int i = 0; i < 4; ++i) for (int j = 0; j < 16; ++j) s += acc[i][j];
  for (int i = 0; i < 16; ++i) s += v[i];
  for (int i = 0; i < 8; ++i) s += pv[i][0] + pv[i][1];
  out[blockIdx.x * 512 + threadIdx.x] = s;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 4000;
  const int grid = 256 * 2;
  float* out;
  CK(hipMalloc(&out, (size_t)grid * 512 * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const char* names[] = {"", "mfma only (waves 0-3)", "v_fma_f32 only (waves 4-7)", "mfma || v_fma_f32 (split waves)", "",
                         "", "v_pk_fma_f32 only (waves 4-7)", "mfma || v_pk_fma_f32 (split waves)"};
  const int modes[] = {1, 2, 3, 6, 7, 1 | 8, 3 | 8, 7 | 8};
  for (int m : modes) {
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(k_coexec, dim3(grid), dim3(512), 0, 0, iters / 10, m, out);
    CK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(k_coexec, dim3(grid), dim3(512), 0, 0, iters, m, out);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    const int nw_mf = (m & 8) ? 8 : 4, nw_va = (m & 8) ? 8 : 4;
    double fl_mf = (m & 1) ? 2.0 * 32 * 32 * 2 * 8 * (double)iters * nw_mf * grid : 0;
    double fl_va = (m & 2) ? 64.0 * 2 * 16 * 16 * (m & 4 ? 1 : 1) * (double)iters * nw_va * grid : 0;
    printf("mode %2d %-40s %8.3f ms  mfma %7.1f TF  valu %7.1f TF  total %7.1f TF\n", m,
           (m & 8) ? ((m & 2) ? ((m & 4) ? "same wave: mfma + v_pk_fma_f32" : "same wave: mfma + v_fma_f32") : "mfma only (all 8 waves)")
                   : names[m],
           ms, fl_mf / ms / 1e9, fl_va / ms / 1e9, (fl_mf + fl_va) / ms / 1e9);
  }
  return 0;
}
