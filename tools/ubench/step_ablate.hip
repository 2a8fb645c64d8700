// Ablation microbenchmark of the per-step ConvLSTM GEMMs at C2 size (B=32,
// 11x11): times the production kernels and variants with parts removed
// (glds.h ABL bits) to show where a step's time goes.  Diagnostic only.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -munsafe-fp-atomics -I../../include -I<csrc> step_ablate.hip
#include <cstdio>
#include <type_traits>
#include <vector>
#include "glds.h"
#include "epilogues.h"

using namespace aaa;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

using K4B = GemmCfg<float, 32, 64, 128, 1, 2, 4>;
using CF = GemmCfg<float, 64, 64, 32, 2, 2, 1>;

template <class F>
static float time_us(F&& launch, int reps = 50) {
  for (int i = 0; i < 5; ++i) launch();
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

static float* dev_rand(size_t n, float scale, unsigned seed) {
  std::vector<float> h(n);
  unsigned s = seed;
  for (auto& v : h) { s = s * 1664525u + 1013904223u; v = scale * (((s >> 8) & 0xffff) / 32768.f - 1.f); }
  float* d; CK(hipMalloc(&d, n * 4)); CK(hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice));
  return d;
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 32, h = 11, w = 11, M = B * h * w;
  float* WdT = dev_rand((size_t)128 * 4608, 0.02f, 1);
  float* WpH = dev_rand((size_t)512 * 1152, 0.02f, 2);
  float* dz = dev_rand((size_t)M * 512, 1.f, 3);
  float* gates = dev_rand((size_t)M * 512, 0.5f, 4);
  float* cprev = dev_rand((size_t)M * 128, 1.f, 5);
  float* ccur = dev_rand((size_t)M * 128, 1.f, 6);
  float* dO = dev_rand((size_t)M * 128, 1.f, 7);
  float* dC = dev_rand((size_t)M * 128, 1.f, 8);
  float* dzo = dev_rand((size_t)M * 512, 1.f, 9);
  float* xh = dev_rand((size_t)M * 192 * 2, 1.f, 10);
  float* gt = dev_rand((size_t)M * 512, 1.f, 11);
  float* cn = dev_rand((size_t)M * 128, 1.f, 12);
  float* hs = dev_rand((size_t)M * 128, 1.f, 13);

  const double flop = 2.0 * M * 128 * 4608;
  {  // BPTT step: D[128][M] = WdT[64:192] x gather(dz)
    const ConvGeo g = ConvGeo{512, 512, 0, h, w, h, w, 3, 1, 1, 1}.prep();
    EpiConvLstmBwd<float> ep{nullptr, gates, cprev, ccur, dO, dC, dzo, nullptr, 1, M, 64};
    using LA = GRowsB<float, K4B::BI, K4B::BK, K4B::NT>;
    using LB = GIm2colB<float, K4B::BJ, K4B::BK, K4B::NT>;
    typename LA::Params pa{WdT, 4608, 128};
    typename LB::Params pb{dz, g, M, (uint32_t)((size_t)M * 512 * 4)};
    dim3 grid((M + 63) / 64, 128 / 32, 1);
    auto run = [&](auto kern, const char* name) {
      const float us = time_us([&] { hipLaunchKernelGGL(kern, grid, dim3(K4B::NT), 0, 0, pa, pb, ep, 4608, 4608, tile_map(grid)); });
      printf("bptt %-34s %8.2f us  %6.1f TF/s\n", name, us, flop / (us * 1e-6) / 1e12);
    };
    run(gemm_pipe_kernel<K4B, LA, LB, EpiConvLstmBwd<float>, 3, 0>, "pipe3 full");
    run(gemm_pipe_kernel<K4B, LA, LB, EpiConvLstmBwd<float>, 2, 0>, "pipe2 full");
    run(gemm_pipe_kernel<K4B, LA, LB, EpiConvLstmBwd<float>, 2, 0, true>, "pipe2 interleaved DMA");
    run(gemm_pipe_kernel<K4B, LA, LB, EpiConvLstmBwd<float>, 3, 0, true>, "pipe3 interleaved DMA");
    run(gemm_pipe_kernel<K4B, LA, LB, EpiConvLstmBwd<float>, 3, 1>, "pipe3 no-loop-DMA");
    run(gemm_pipe_kernel<K4B, LA, LB, EpiConvLstmBwd<float>, 3, 2>, "pipe3 no-MFMA");
    run(gemm_pipe_kernel<K4B, LA, LB, EpiConvLstmBwd<float>, 3, 4>, "pipe3 no-epilogue");
    run(gemm_pipe_kernel<K4B, LA, LB, EpiConvLstmBwd<float>, 3, 3>, "pipe3 skeleton (no DMA, no MFMA)");
    run(gemm_pipe_kernel<K4B, LA, LB, EpiConvLstmBwd<float>, 3, 7>, "pipe3 skeleton, no epilogue");
    run(gemm_pipe_kernel<K4B, LA, LB, EpiConvLstmBwd<float>, 3, 5>, "pipe3 MFMA only (no DMA, no epi)");
  }
  {  // forward step: D[512][M] = WpH x gather(h_{t-1}) + fused gates
    const ConvGeo g = ConvGeo{128, 192, 64, h, w, h, w, 3, 1, 1, 0}.prep();
    EpiConvLstmFwd<float> ep{cprev, cn, hs, xh + (size_t)M * 192, gt, M};
    const double fl = 2.0 * M * 512 * 1152;
    auto run = [&](auto cfg, auto nbuf, const char* name) {
      using C = decltype(cfg);
      constexpr int NB = decltype(nbuf)::value;
      using LA = GRowsB<float, C::BI, C::BK, C::NT>;
      using LB = GIm2colB<float, C::BJ, C::BK, C::NT>;
      const float us = time_us([&] {
        CK((launch_pipe<C, LA, LB, EpiConvLstmFwd<float>, NB>(typename LA::Params{WpH, 1152, 512},
                                                               typename LB::Params{xh, g, M, (uint32_t)((size_t)M * 768)},
                                                               ep, 512, M, 1152, 1, 0)));
      });
      printf("fwd  %-40s %8.2f us  %6.1f TF/s\n", name, us, fl / (us * 1e-6) / 1e12);
    };
    using I2 = std::integral_constant<int, 2>;
    using I3 = std::integral_constant<int, 3>;
    run(GemmCfg<float, 64, 64, 32, 2, 2>{}, I2{}, "64x64 BK32 4w pipe2 (current)");
    run(GemmCfg<float, 128, 64, 32, 4, 2>{}, I2{}, "128x64 BK32 8w pipe2");
    run(GemmCfg<float, 128, 64, 32, 4, 2>{}, I3{}, "128x64 BK32 8w pipe3");
    run(GemmCfg<float, 64, 128, 32, 2, 4>{}, I2{}, "64x128 BK32 8w pipe2");
    run(GemmCfg<float, 128, 64, 64, 4, 2>{}, I2{}, "128x64 BK64 8w pipe2");
    run(GemmCfg<float, 128, 64, 32, 2, 2>{}, I2{}, "128x64 BK32 4w (64x32/wave) pipe2");
    run(GemmCfg<float, 128, 64, 64, 2, 2, 2>{}, I2{}, "128x64 BK64 8w 2-way split-K pipe2");
    run(GemmCfg<float, 128, 128, 32, 2, 2>{}, I2{}, "128x128 BK32 4w pipe2");
  }
  {  // BPTT alternatives
    const ConvGeo g = ConvGeo{512, 512, 0, h, w, h, w, 3, 1, 1, 1}.prep();
    EpiConvLstmBwd<float> ep{nullptr, gates, cprev, ccur, dO, dC, dzo, nullptr, 1, M, 64};
    auto run = [&](auto cfg, auto nbuf, auto ilv, const char* name) {
      using C = decltype(cfg);
      constexpr int NB = decltype(nbuf)::value;
      constexpr bool IL = decltype(ilv)::value;
      using LA = GRowsB<float, C::BI, C::BK, C::NT>;
      using LB = GIm2colB<float, C::BJ, C::BK, C::NT>;
      const float us = time_us([&] {
        CK((launch_pipe<C, LA, LB, EpiConvLstmBwd<float>, NB, IL>(typename LA::Params{WdT, 4608, 128},
                                                            typename LB::Params{dz, g, M, (uint32_t)((size_t)M * 2048)},
                                                            ep, 128, M, 4608, 1, 0)));
      });
      printf("bptt %-40s %8.2f us  %6.1f TF/s\n", name, us, flop / (us * 1e-6) / 1e12);
    };
    using I2 = std::integral_constant<int, 2>;
    using I3 = std::integral_constant<int, 3>;
    using T1 = std::true_type;
    using F0 = std::false_type;
    run(GemmCfg<float, 32, 64, 128, 1, 2, 4>{}, I3{}, T1{}, "32x64 BK128 4-way pipe3 ilv (current)");
    run(GemmCfg<float, 32, 64, 64, 1, 2, 4>{}, I3{}, T1{}, "32x64 BK64 4-way pipe3 ilv");
    run(GemmCfg<float, 32, 64, 64, 1, 2, 4>{}, I2{}, F0{}, "32x64 BK64 4-way pipe2");
    run(GemmCfg<float, 64, 32, 128, 2, 1, 4>{}, I3{}, T1{}, "64x32 BK128 4-way pipe3 ilv");
    run(GemmCfg<float, 32, 128, 64, 1, 4, 2>{}, I3{}, T1{}, "32x128 BK64 2-way pipe3 ilv");
  }
  printf("done\n");
  return 0;
}
