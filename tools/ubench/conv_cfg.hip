// Tile/pipeline configurations for the batched vision convs at C2 size
// (640 frames): conv1 (RGBx 84x84 -> 20x20x32, 8x8 s4 p1) and conv2
// (20x20x32 -> 11x11x64, 4x4 s2 p2).  Diagnostic only (tools/ubench/build.sh).
#include <cstdio>
#include <vector>
#include "glds.h"
#include "epilogues.h"

using namespace aaa;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

template <class F>
static float time_us(F&& launch, int reps = 30) {
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
static float* dev_rand(size_t n, float scale, unsigned seed) {
  std::vector<float> h(n);
  unsigned s = seed;
  for (auto& v : h) { s = s * 1664525u + 1013904223u; v = scale * (((s >> 8) & 0xffff) / 32768.f - 1.f); }
  float* d; CK(hipMalloc(&d, n * 4)); CK(hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice));
  return d;
}

template <class C, int NBUF>
static void conv_pipe(const char* name, const float* W, int K, int Cout, const float* x, const ConvGeo& g, int M,
                      uint32_t xb, float* y, const float* bias, double flop) {
  using LA = GRowsB<float, C::BI, C::BK, C::NT>;
  using LB = GIm2colB<float, C::BJ, C::BK, C::NT>;
  EpiStoreT<float> ep{y, Cout, Cout, M, bias, 0};
  const float us = time_us([&] {
    CK((launch_pipe<C, LA, LB, EpiStoreT<float>, NBUF>(typename LA::Params{W, K, Cout}, typename LB::Params{x, g, M, xb},
                                                        ep, Cout, M, K, 1, 0)));
  });
  printf("%-44s %8.2f us  %6.1f TF/s\n", name, us, flop / (us * 1e-6) / 1e12);
}
template <class C>
static void conv_reg(const char* name, const float* W, int K, int Cout, const float* x, const ConvGeo& g, int M,
                     uint32_t xb, float* y, const float* bias, double flop) {
  using LA = LdRowsB<float, float, C::BI, C::BK, C::NT>;
  using LB = LdIm2colB<float, float, C::BJ, C::BK, C::NT>;
  EpiStoreT<float> ep{y, Cout, Cout, M, bias, 0};
  const float us = time_us([&] {
    CK((launch_gemm<C, LA, LB>(typename LA::Params{W, K, Cout}, typename LB::Params{x, g, M, xb}, ep, Cout, M, K, 1, 0)));
  });
  printf("%-44s %8.2f us  %6.1f TF/s\n", name, us, flop / (us * 1e-6) / 1e12);
}

int main() {
  const int F = 640;
  {
    const int M = F * 400, K = 256;
    float* W = dev_rand(32 * 256, 0.05f, 1);
    float* x = dev_rand((size_t)F * 84 * 84 * 4, 1.f, 2);
    float* y = dev_rand((size_t)M * 32, 1.f, 3);
    float* b = dev_rand(32, 1.f, 4);
    const ConvGeo g = ConvGeo{4, 4, 0, 84, 84, 20, 20, 8, 4, 1, 0}.prep();
    const uint32_t xb = (uint32_t)((size_t)F * 84 * 84 * 16);
    const double fl = 2.0 * M * 32 * K;
    conv_reg<GemmCfg<float, 32, 64, 32, 1, 2>>("conv1 reg 32x64 BK32 (current)", W, K, 32, x, g, M, xb, y, b, fl);
    conv_pipe<GemmCfg<float, 32, 64, 32, 1, 2>, 2>("conv1 pipe2 32x64 BK32", W, K, 32, x, g, M, xb, y, b, fl);
    conv_pipe<GemmCfg<float, 32, 64, 32, 1, 2>, 3>("conv1 pipe3 32x64 BK32", W, K, 32, x, g, M, xb, y, b, fl);
    conv_pipe<GemmCfg<float, 32, 128, 32, 1, 2>, 2>("conv1 pipe2 32x128 BK32", W, K, 32, x, g, M, xb, y, b, fl);
    conv_pipe<GemmCfg<float, 32, 128, 32, 1, 4>, 2>("conv1 pipe2 32x128 BK32 4 waves", W, K, 32, x, g, M, xb, y, b, fl);
    conv_pipe<GemmCfg<float, 32, 64, 64, 1, 2>, 2>("conv1 pipe2 32x64 BK64", W, K, 32, x, g, M, xb, y, b, fl);
    conv_pipe<GemmCfg<float, 32, 128, 64, 1, 4>, 2>("conv1 pipe2 32x128 BK64 4 waves", W, K, 32, x, g, M, xb, y, b, fl);
    conv_pipe<GemmCfg<float, 32, 256, 32, 1, 4>, 2>("conv1 pipe2 32x256 BK32 4 waves", W, K, 32, x, g, M, xb, y, b, fl);
  }
  {
    const int M = F * 121, K = 512;
    float* W = dev_rand(64 * 512, 0.05f, 5);
    float* x = dev_rand((size_t)F * 400 * 32, 1.f, 6);
    float* y = dev_rand((size_t)M * 64, 1.f, 7);
    float* b = dev_rand(64, 1.f, 8);
    const ConvGeo g = ConvGeo{32, 32, 0, 20, 20, 11, 11, 4, 2, 2, 0}.prep();
    const uint32_t xb = (uint32_t)((size_t)F * 400 * 32 * 4);
    const double fl = 2.0 * M * 64 * K;
    conv_reg<GemmCfg<float, 64, 64, 32, 2, 2>>("conv2 reg 64x64 BK32 (current)", W, K, 64, x, g, M, xb, y, b, fl);
    conv_pipe<GemmCfg<float, 64, 64, 32, 2, 2>, 2>("conv2 pipe2 64x64 BK32", W, K, 64, x, g, M, xb, y, b, fl);
    conv_pipe<GemmCfg<float, 64, 64, 32, 2, 2>, 3>("conv2 pipe3 64x64 BK32", W, K, 64, x, g, M, xb, y, b, fl);
    conv_pipe<GemmCfg<float, 64, 64, 64, 2, 2>, 2>("conv2 pipe2 64x64 BK64", W, K, 64, x, g, M, xb, y, b, fl);
    conv_pipe<GemmCfg<float, 64, 128, 32, 2, 2>, 2>("conv2 pipe2 64x128 BK32", W, K, 64, x, g, M, xb, y, b, fl);
    conv_pipe<GemmCfg<float, 64, 128, 32, 2, 4>, 2>("conv2 pipe2 64x128 BK32 8 waves", W, K, 64, x, g, M, xb, y, b, fl);
  }
  printf("done\n");
  return 0;
}
