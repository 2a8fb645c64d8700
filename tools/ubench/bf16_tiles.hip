// Tile sweep of the LDS-DMA pipelined GEMM (glds.h) for the bf16 ConvLSTM
// GEMMs at C3 size (B=256, 11x11 grid, M = 30976 pixels): forward step,
// BPTT step (bf16 dZ operand), batched dx and batched x-part.  Epilogue =
// plain fp32 store, to isolate the main loop.  Diagnostic only.
#include <cstdio>
#include <type_traits>
#include <vector>
#include "glds.h"
#include "epilogues.h"

using namespace aaa;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
typedef __bf16 bf;

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

static bf* dev_rand(size_t n, float scale, unsigned seed) {
  std::vector<bf> h(n);
  unsigned s = seed;
  for (auto& v : h) { s = s * 1664525u + 1013904223u; v = (bf)(scale * (((s >> 8) & 0xffff) / 32768.f - 1.f)); }
  bf* d; CK(hipMalloc(&d, n * 2)); CK(hipMemcpy(d, h.data(), n * 2, hipMemcpyHostToDevice));
  return d;
}

template <class C, int NB>
static void run(const char* what, const char* name, const bf* W, int ldw, int Mi, const bf* src, const ConvGeo& g,
                int M, size_t src_elems, int K, float* out, double flop) {
  using LA = GRowsB<bf, C::BI, C::BK, C::NT>;
  using LB = GIm2colB<bf, C::BJ, C::BK, C::NT>;
  EpiStoreT<float> ep{out, Mi, Mi, M, nullptr, 0};
  const float us = time_us([&] {
    CK((launch_pipe<C, LA, LB, EpiStoreT<float>, NB>(typename LA::Params{W, ldw, Mi},
                                                      typename LB::Params{src, g, M, (uint32_t)(src_elems * 2)}, ep, Mi,
                                                      M, K, 1, 0)));
  });
  printf("%-5s %-36s %8.2f us  %7.1f TF/s\n", what, name, us, flop / (us * 1e-6) / 1e12);
}

// Same launch with glds.h ablation bits: 1 no in-loop DMA, 2 no MFMA, 4 no epilogue.
template <class C, int NB, int ABL>
static void abl(const char* name, const bf* W, int ldw, int Mi, const bf* src, const ConvGeo& g, int M,
                size_t src_elems, int K, float* out, double flop) {
  using LA = GRowsB<bf, C::BI, C::BK, C::NT>;
  using LB = GIm2colB<bf, C::BJ, C::BK, C::NT>;
  using EP = EpiStoreT<float>;
  EP ep{out, Mi, Mi, M, nullptr, 0};
  dim3 grid((M + C::BJ - 1) / C::BJ, (Mi + C::BI - 1) / C::BI, 1);
  typename LA::Params pa{W, ldw, Mi};
  typename LB::Params pb{src, g, M, (uint32_t)(src_elems * 2)};
  const TileMap tm = tile_map(grid);
  const float us = time_us([&] {
    hipLaunchKernelGGL((gemm_pipe_kernel<C, LA, LB, EP, NB, ABL, false>), grid, dim3(C::NT), 0, 0, pa, pb, ep, K, K, tm);
    CK(hipGetLastError());
  });
  printf("abl%d %-36s %8.2f us  %7.1f TF/s\n", ABL, name, us, flop / (us * 1e-6) / 1e12);
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 256, h = 11, w = 11, M = B * h * w;
  const int T = 20, FM = T * M;
  bf* WpH = dev_rand((size_t)512 * 1152, 0.02f, 2);
  bf* WdT = dev_rand((size_t)192 * 4608, 0.02f, 1);
  bf* WpX = dev_rand((size_t)512 * 576, 0.02f, 3);
  bf* xh = dev_rand((size_t)FM * 192, 1.f, 10);
  bf* dz = dev_rand((size_t)FM * 512, 1.f, 3);
  float* out; CK(hipMalloc(&out, (size_t)FM * 512 * 4));
  {
    const ConvGeo g = ConvGeo{128, 192, 64, h, w, h, w, 3, 1, 1, 0}.prep();
    const double fl = 2.0 * M * 512 * 1152;
#define FWD(BI, BJ, BK, WI, WJ, WK, NB, NAME) \
    run<GemmCfg<bf, BI, BJ, BK, WI, WJ, WK>, NB>("fwd", NAME, WpH, 1152, 512, xh, g, M, (size_t)2 * M * 192, 1152, out, fl)
    FWD(128, 64, 64, 4, 2, 1, 2, "128x64 BK64 8w (current)");
    using F0 = GemmCfg<bf, 128, 64, 64, 4, 2, 1>;
    abl<F0, 2, 1>("fwd 128x64 no DMA", WpH, 1152, 512, xh, g, M, (size_t)2 * M * 192, 1152, out, fl);
    abl<F0, 2, 2>("fwd 128x64 no MFMA", WpH, 1152, 512, xh, g, M, (size_t)2 * M * 192, 1152, out, fl);
    abl<F0, 2, 4>("fwd 128x64 no epilogue", WpH, 1152, 512, xh, g, M, (size_t)2 * M * 192, 1152, out, fl);
    abl<F0, 2, 5>("fwd 128x64 no DMA, no epi", WpH, 1152, 512, xh, g, M, (size_t)2 * M * 192, 1152, out, fl);
    abl<F0, 2, 6>("fwd 128x64 DMA only", WpH, 1152, 512, xh, g, M, (size_t)2 * M * 192, 1152, out, fl);
    abl<F0, 2, 7>("fwd 128x64 nothing (barriers)", WpH, 1152, 512, xh, g, M, (size_t)2 * M * 192, 1152, out, fl);
    FWD(128, 128, 64, 2, 2, 1, 2, "128x128 BK64 4w");
    FWD(128, 128, 64, 4, 2, 1, 2, "128x128 BK64 8w");
    FWD(256, 128, 64, 4, 2, 1, 2, "256x128 BK64 8w");
    FWD(128, 256, 64, 2, 4, 1, 2, "128x256 BK64 8w");
    FWD(256, 64, 64, 4, 1, 1, 2, "256x64 BK64 4w");
    FWD(128, 128, 64, 2, 2, 1, 3, "128x128 BK64 4w pipe3");
    FWD(128, 128, 128, 2, 2, 2, 2, "128x128 BK128 8w 2-way");
    FWD(128, 64, 64, 4, 2, 1, 3, "128x64 BK64 8w pipe3");
    FWD(128, 64, 64, 4, 2, 1, 4, "128x64 BK64 8w pipe4");
    FWD(128, 128, 64, 4, 2, 1, 3, "128x128 BK64 8w pipe3");
    FWD(256, 64, 64, 4, 1, 1, 3, "256x64 BK64 4w pipe3");
  }
  {
    const ConvGeo g = ConvGeo{512, 512, 0, h, w, h, w, 3, 1, 1, 1}.prep();
    const double fl = 2.0 * M * 128 * 4608;
#define BPTT(BI, BJ, BK, WI, WJ, WK, NB, NAME) \
    run<GemmCfg<bf, BI, BJ, BK, WI, WJ, WK>, NB>("bptt", NAME, WdT + 64 * 4608, 4608, 128, dz, g, M, (size_t)M * 512, 4608, out, fl)
    BPTT(128, 64, 64, 4, 2, 1, 2, "128x64 BK64 8w");
    BPTT(128, 64, 64, 2, 1, 1, 2, "128x64 BK64 2w");
    BPTT(128, 128, 64, 2, 2, 1, 2, "128x128 BK64 4w");
    BPTT(128, 128, 64, 4, 2, 1, 2, "128x128 BK64 8w");
    BPTT(128, 128, 128, 2, 2, 2, 2, "128x128 BK128 8w 2-way");
    using B7 = GemmCfg<bf, 128, 128, 128, 2, 2, 2>;
    abl<B7, 2, 1>("bptt 128x128 no DMA", WdT + 64 * 4608, 4608, 128, dz, g, M, (size_t)M * 512, 4608, out, fl);
    abl<B7, 2, 5>("bptt 128x128 no DMA, no epi", WdT + 64 * 4608, 4608, 128, dz, g, M, (size_t)M * 512, 4608, out, fl);
    abl<B7, 2, 6>("bptt 128x128 DMA only", WdT + 64 * 4608, 4608, 128, dz, g, M, (size_t)M * 512, 4608, out, fl);
    BPTT(128, 64, 128, 2, 1, 2, 2, "128x64 BK128 4w 2-way");
    BPTT(128, 64, 64, 2, 2, 1, 3, "128x64 BK64 4w pipe3");
    BPTT(64, 128, 64, 2, 2, 1, 2, "64x128 BK64 4w");
    BPTT(128, 128, 64, 2, 2, 2, 3, "128x128 BK64 8w 2-way pipe3");
    BPTT(128, 128, 128, 2, 2, 2, 2, "128x128 BK128 8w 2-way (again)");
    BPTT(128, 64, 64, 4, 2, 1, 3, "128x64 BK64 8w pipe3");
    BPTT(128, 64, 64, 4, 2, 1, 4, "128x64 BK64 8w pipe4");
  }
  {
    const ConvGeo g = ConvGeo{512, 512, 0, h, w, h, w, 3, 1, 1, 1}.prep();
    const double fl = 2.0 * FM * 64 * 4608;
#define DX(BI, BJ, BK, WI, WJ, WK, NB, NAME) \
    run<GemmCfg<bf, BI, BJ, BK, WI, WJ, WK>, NB>("dx", NAME, WdT, 4608, 64, dz, g, FM, (size_t)FM * 512, 4608, out, fl)
    DX(64, 64, 64, 2, 2, 1, 2, "64x64 BK64 4w");
    DX(64, 128, 64, 2, 2, 1, 2, "64x128 BK64 4w");
    DX(64, 256, 64, 1, 4, 1, 2, "64x256 BK64 4w");
    DX(64, 256, 64, 2, 4, 1, 2, "64x256 BK64 8w");
    DX(64, 128, 64, 1, 2, 1, 3, "64x128 BK64 2w pipe3");
    DX(64, 128, 64, 2, 2, 1, 3, "64x128 BK64 4w pipe3");
    DX(64, 256, 64, 2, 4, 1, 3, "64x256 BK64 8w pipe3");
  }
  {
    const ConvGeo g = ConvGeo{64, 192, 0, h, w, h, w, 3, 1, 1, 0}.prep();
    const double fl = 2.0 * FM * 512 * 576;
#define XP(BI, BJ, BK, WI, WJ, WK, NB, NAME) \
    run<GemmCfg<bf, BI, BJ, BK, WI, WJ, WK>, NB>("xpart", NAME, WpX, 576, 512, xh, g, FM, (size_t)FM * 192, 576, out, fl)
    XP(64, 64, 64, 2, 2, 1, 2, "64x64 BK64 4w (current)");
    XP(128, 128, 64, 2, 2, 1, 2, "128x128 BK64 4w");
    XP(256, 128, 64, 4, 2, 1, 2, "256x128 BK64 8w");
    XP(128, 256, 64, 2, 4, 1, 2, "128x256 BK64 8w");
    XP(128, 128, 64, 4, 2, 1, 3, "128x128 BK64 8w pipe3");
    XP(128, 64, 64, 4, 2, 1, 3, "128x64 BK64 8w pipe3");
    XP(64, 64, 64, 2, 2, 1, 3, "64x64 BK64 4w pipe3");
  }
  printf("done\n");
  return 0;
}
