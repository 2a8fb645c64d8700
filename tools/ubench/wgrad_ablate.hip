// Ablation microbenchmark of the bf16 ConvLSTM weight gradient at C3 size
// (B=256, T=20, 11x11: 619520 pixels of K): D[512][1728] += dZ^T * im2col(XH)
// on the LDS-DMA ring with transposed fragment reads (runtime.hip
// AAA_WGRAD_PIPE), with parts removed (glds.h ABL bits).  Diagnostic only.
//   tools/ubench/build.sh wgrad_ablate.hip && tools/ubench/wgrad_ablate [B] [T]
#include <algorithm>
#include <cstdio>
#include <vector>
#include "glds.h"
#include "epilogues.h"

using namespace aaa;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

template <class F>
static float time_us(F&& launch, int reps = 20) {
  for (int i = 0; i < 3; ++i) launch();
  CK(hipDeviceSynchronize());
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  CK(hipEventRecord(a, 0));
  for (int i = 0; i < reps; ++i) launch();
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  return ms * 1e3f / reps;
}

static __bf16* dev_rand(size_t n, float scale, unsigned seed) {
  std::vector<__bf16> h(n);
  unsigned s = seed;
  for (auto& v : h) { s = s * 1664525u + 1013904223u; v = (__bf16)(scale * (((s >> 8) & 0xffff) / 32768.f - 1.f)); }
  __bf16* d; CK(hipMalloc(&d, n * 2)); CK(hipMemcpy(d, h.data(), n * 2, hipMemcpyHostToDevice));
  return d;
}

template <class C, int NB, int ABL>
static void run_ra(const char* name, const __bf16* dz, const __bf16* xh, float* out, int rows, int h, int w, int wgs) {
  using LA = GRowsT<__bf16, C::BI, C::BK, C::NT>;
  using LB = GIm2colT<__bf16, C::BJ, C::BK, C::NT>;
  typename LA::Params pa{dz, 512, 512, rows};
  typename LB::Params pb{xh, ConvGeo{192, 192, 0, h, w, h, w, 3, 1, 1, 0}.prep(), 1728, (uint32_t)((size_t)rows * 192 * 2)};
  EpiAtomicD ep{{out, 1728, 512, 1728}};
  const int tiles = ((512 + C::BI - 1) / C::BI) * ((1728 + C::BJ - 1) / C::BJ);
  int ns = std::max(1, wgs / tiles);
  int kchunk = (rows + ns - 1) / ns;
  kchunk = (kchunk + C::BK - 1) / C::BK * C::BK;
  ns = (rows + kchunk - 1) / kchunk;
  dim3 grid((1728 + C::BJ - 1) / C::BJ, (512 + C::BI - 1) / C::BI, ns);
  const float us = time_us([&] {
    hipLaunchKernelGGL((gemm_pipe_ra_kernel<C, LA, LB, EpiAtomicD, NB, ABL>), grid, dim3(C::NT), 0, 0, pa, pb, ep, rows,
                       kchunk, tile_map(grid));
  });
  const double flop = 2.0 * 512 * 1728 * rows;
  printf("%-44s %9.1f us  %7.1f TF/s\n", name, us, flop / (us * 1e-6) / 1e12);
#ifdef AAA_STAMPS
  const int nwg = grid.x * grid.y * grid.z;
  std::vector<uint64_t> st((size_t)nwg * 4);
  CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(aaa_stamps), st.size() * 8));
  std::vector<double> ph[3];
  for (int i = 0; i < nwg; ++i)
    for (int k = 0; k < 3; ++k) ph[k].push_back((double)(st[i * 4 + k + 1] - st[i * 4 + k]) * 0.01);
  for (auto& v : ph) std::sort(v.begin(), v.end());
  printf("    phases (median / max us): prologue %.1f/%.1f  K loop %.1f/%.1f  epilogue %.1f/%.1f\n", ph[0][nwg / 2],
         ph[0].back(), ph[1][nwg / 2], ph[1].back(), ph[2][nwg / 2], ph[2].back());
#endif
}

template <class C, int NB, int ABL, int ILV = 0>
static void run(const char* name, const __bf16* dz, const __bf16* xh, float* out, int rows, int h, int w, int wgs) {
  using LA = GRowsT<__bf16, C::BI, C::BK, C::NT>;
  using LB = GIm2colT<__bf16, C::BJ, C::BK, C::NT>;
  typename LA::Params pa{dz, 512, 512, rows};
  typename LB::Params pb{xh, ConvGeo{192, 192, 0, h, w, h, w, 3, 1, 1, 0}.prep(), 1728, (uint32_t)((size_t)rows * 192 * 2)};
  EpiAtomicD ep{{out, 1728, 512, 1728}};
  const int tiles = ((512 + C::BI - 1) / C::BI) * ((1728 + C::BJ - 1) / C::BJ);
  int ns = std::max(1, wgs / tiles);
  int kchunk = (rows + ns - 1) / ns;
  kchunk = (kchunk + C::BK - 1) / C::BK * C::BK;
  ns = (rows + kchunk - 1) / kchunk;
  dim3 grid((1728 + C::BJ - 1) / C::BJ, (512 + C::BI - 1) / C::BI, ns);
  const float us = time_us([&] {
    hipLaunchKernelGGL((gemm_pipe_kernel<C, LA, LB, EpiAtomicD, NB, ABL, ILV>), grid, dim3(C::NT), 0, 0, pa, pb, ep, rows,
                       kchunk, tile_map(grid));
  });
  const double flop = 2.0 * 512 * 1728 * rows;
  printf("%-44s %9.1f us  %7.1f TF/s\n", name, us, flop / (us * 1e-6) / 1e12);
#ifdef AAA_STAMPS
  // medians over workgroups of the last launch: prologue, K loop, epilogue (us)
  const int nwg = grid.x * grid.y * grid.z;
  std::vector<uint64_t> st((size_t)nwg * 4);
  CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(aaa_stamps), st.size() * 8));
  std::vector<double> ph[3];
  uint64_t t0 = ~0ull, t3 = 0;
  for (int i = 0; i < nwg; ++i) {
    for (int k = 0; k < 3; ++k) ph[k].push_back((double)(st[i * 4 + k + 1] - st[i * 4 + k]) * 0.01);
    t0 = std::min(t0, st[i * 4]); t3 = std::max(t3, st[i * 4 + 3]);
  }
  for (auto& v : ph) std::sort(v.begin(), v.end());
  printf("    phases (median / max us): prologue %.1f/%.1f  K loop %.1f/%.1f  epilogue %.1f/%.1f  | span %.1f\n",
         ph[0][nwg / 2], ph[0].back(), ph[1][nwg / 2], ph[1].back(), ph[2][nwg / 2], ph[2].back(), (t3 - t0) * 0.01);
#endif
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 256, T = argc > 2 ? atoi(argv[2]) : 20, h = 11, w = 11;
  const int rows = T * B * h * w;
  __bf16* dz = dev_rand((size_t)rows * 512, 1.f, 3);
  __bf16* xh = dev_rand((size_t)rows * 192, 1.f, 10);
  float* out; CK(hipMalloc(&out, (size_t)512 * 1728 * 4));
  using C8k = GemmCfg<__bf16, 256, 256, 32, 2, 4>;
  run<C8k, 4, 0, 2>("256x256 BK32 ring4 ILV2 (production)", dz, xh, out, rows, h, w, 256);
  run<C8k, 4, 0, 2>("256x256 BK32 ring4 ILV2 (production, again)", dz, xh, out, rows, h, w, 256);
  run<C8k, 4, 4, 2>("  no epilogue", dz, xh, out, rows, h, w, 256);
  run<C8k, 4, 1, 2>("  no in-loop DMA", dz, xh, out, rows, h, w, 256);
  run<C8k, 4, 2, 2>("  no MFMA (DMA + fragment reads)", dz, xh, out, rows, h, w, 256);
  run<C8k, 4, 5, 2>("  MFMA + fragment reads only", dz, xh, out, rows, h, w, 256);
  run<C8k, 4, 3, 2>("  skeleton (no DMA, no MFMA)", dz, xh, out, rows, h, w, 256);
  run<C8k, 3, 0, 2>("256x256 BK32 ring3 ILV2", dz, xh, out, rows, h, w, 256);
  using C8 = GemmCfg<__bf16, 256, 256, 64, 2, 4>;
  run<C8, 2, 0, 2>("256x256 BK64 ring2 ILV2", dz, xh, out, rows, h, w, 256);
  using C16 = GemmCfg<__bf16, 256, 256, 16, 2, 4>;
  run_ra<C16, 8, 0>("read-ahead 256x256 BK16 ring8", dz, xh, out, rows, h, w, 256);
  run_ra<C16, 8, 0>("read-ahead 256x256 BK16 ring8 (again)", dz, xh, out, rows, h, w, 256);
  run_ra<C16, 8, 1>("  no in-loop DMA", dz, xh, out, rows, h, w, 256);
  run_ra<C16, 8, 5>("  no in-loop DMA, no epilogue", dz, xh, out, rows, h, w, 256);
  run_ra<C16, 6, 0>("read-ahead 256x256 BK16 ring6", dz, xh, out, rows, h, w, 256);
  run_ra<C8k, 4, 0>("read-ahead 256x256 BK32 ring4", dz, xh, out, rows, h, w, 256);
  run_ra<C16, 8, 0>("read-ahead 256x256 BK16 ring8, 512 WGs", dz, xh, out, rows, h, w, 512);
  return 0;
}
