// Halo-staged 3x3 conv (halo.h) vs the im2col LDS-DMA ring (glds.h) for the
// bf16 ConvLSTM GEMMs at C3 size (B=256, 11x11 grid): batched x-part, forward
// step (h-part), BPTT step and batched dx.  Epilogue = plain fp32 store, to
// isolate the main loop; each halo variant is also checked against the ring
// kernel's output (max |diff| / max |ref|).  Diagnostic only.
#include <cmath>
#include <cstdio>
#include <vector>
#include "halo.h"
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

static double max_rel(const float* a, const float* b, size_t n) {
  std::vector<float> x(n), y(n);
  CK(hipMemcpy(x.data(), a, n * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(y.data(), b, n * 4, hipMemcpyDeviceToHost));
  double d = 0, m = 0;
  for (size_t i = 0; i < n; ++i) { d = fmax(d, fabs((double)x[i] - y[i])); m = fmax(m, fabs((double)y[i])); }
  return d / (m > 0 ? m : 1);
}

template <class C>
static void ring(const char* what, const char* name, const bf* W, int ldw, int Mi, const bf* src, const ConvGeo& g,
                 int M, size_t src_elems, int K, float* out, double flop) {
  using LA = GRowsB<bf, C::BI, C::BK, C::NT>;
  using LB = GIm2colB<bf, C::BJ, C::BK, C::NT>;
  EpiStoreT<float> ep{out, Mi, Mi, M, nullptr, 0};
  const float us = time_us([&] {
    CK((launch_pipe<C, LA, LB, EpiStoreT<float>, 2>(typename LA::Params{W, ldw, Mi},
                                                     typename LB::Params{src, g, M, (uint32_t)(src_elems * 2)}, ep, Mi,
                                                     M, K, 1, 0)));
  });
  printf("%-5s ring %-34s %8.2f us  %7.1f TF/s\n", what, name, us, flop / (us * 1e-6) / 1e12);
}

template <class C>
static void halo(const char* what, const char* name, const HaloParams& p, float* out, const float* ref, double flop) {
  const int M = p.nframes * p.h * p.w;
  EpiStoreT<float> ep{out, p.Mi, p.Mi, M, nullptr, 0};
  CK(hipMemset(out, 0, (size_t)M * p.Mi * 4));
  CK((launch_halo<C>(p, ep, 0)));
  CK(hipDeviceSynchronize());
  const double err = max_rel(out, ref, (size_t)M * p.Mi);
  const float us = time_us([&] { CK((launch_halo<C>(p, ep, 0))); });
  printf("%-5s halo %-34s %8.2f us  %7.1f TF/s   max rel diff vs ring %.2e\n", what, name, us,
         flop / (us * 1e-6) / 1e12, err);
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 256, h = 11, w = 11, M = B * h * w;
  const int T = 20, F = T * B, FM = T * M;
  bf* WpH = dev_rand((size_t)512 * 1152, 0.02f, 2);
  bf* WdT = dev_rand((size_t)192 * 4608, 0.02f, 1);
  bf* WpX = dev_rand((size_t)512 * 576, 0.02f, 3);
  bf* xh = dev_rand((size_t)FM * 192, 1.f, 10);
  bf* dz = dev_rand((size_t)FM * 512, 1.f, 3);
  float *out, *ref;
  CK(hipMalloc(&out, (size_t)FM * 512 * 4));
  CK(hipMalloc(&ref, (size_t)FM * 512 * 4));
  {  // x-part: all frames, Cin 64 of XH (one channel chunk)
    const ConvGeo g = ConvGeo{64, 192, 0, h, w, h, w, 3, 1, 1, 0}.prep();
    const double fl = 2.0 * FM * 512 * 576;
    ring<GemmCfg<bf, 128, 128, 64, 2, 2, 1>>("xpart", "128x128 BK64 4w", WpX, 576, 512, xh, g, FM, (size_t)FM * 192,
                                             576, ref, fl);
    HaloParams p{WpX, 576, 512, xh, 192, 0, 64, (uint32_t)((size_t)FM * 192 * 2), h, w, F, 0};
    halo<HaloCfg<bf, 128, 128, 64, 2, 2, 1, 192>>("xpart", "128x128(1 fr) 4w", p, out, ref, fl);
    halo<HaloCfg<bf, 256, 128, 64, 4, 2, 1, 192>>("xpart", "256x128(1 fr) 8w", p, out, ref, fl);
    halo<HaloCfg<bf, 128, 256, 64, 2, 2, 2, 352>>("xpart", "128x256(2 fr) 4w", p, out, ref, fl);
    halo<HaloCfg<bf, 128, 256, 64, 2, 4, 2, 384>>("xpart", "128x256(2 fr) 8w", p, out, ref, fl);
  }
  {  // forward step h-part: one step's frames, Cin 128 at channel 64 of XH
    const ConvGeo g = ConvGeo{128, 192, 64, h, w, h, w, 3, 1, 1, 0}.prep();
    const double fl = 2.0 * M * 512 * 1152;
    ring<GemmCfg<bf, 128, 64, 64, 4, 2, 1>>("fwd", "128x64 BK64 8w (current)", WpH, 1152, 512, xh, g, M,
                                            (size_t)2 * M * 192, 1152, ref, fl);
    HaloParams p{WpH, 1152, 512, xh, 192, 64, 128, (uint32_t)((size_t)2 * M * 192 * 2), h, w, B, 0};
    halo<HaloCfg<bf, 128, 128, 64, 2, 2, 1, 192>>("fwd", "128x128(1 fr) 4w", p, out, ref, fl);
    halo<HaloCfg<bf, 256, 128, 64, 4, 2, 1, 192>>("fwd", "256x128(1 fr) 8w", p, out, ref, fl);
    halo<HaloCfg<bf, 64, 128, 64, 1, 2, 1, 176>>("fwd", "64x128(1 fr) 2w", p, out, ref, fl);
  }
  {  // BPTT step: dh rows (128) of the transposed conv over dz (Cin 512)
    const ConvGeo g = ConvGeo{512, 512, 0, h, w, h, w, 3, 1, 1, 1}.prep();
    const double fl = 2.0 * M * 128 * 4608;
    ring<GemmCfg<bf, 128, 128, 128, 2, 2, 2>>("bptt", "128x128 BK128 8w 2-way (current)", WdT + 64 * 4608, 4608, 128,
                                              dz, g, M, (size_t)M * 512, 4608, ref, fl);
    HaloParams p{WdT + 64 * 4608, 4608, 128, dz, 512, 0, 512, (uint32_t)((size_t)M * 512 * 2), h, w, B, 1};
    halo<HaloCfg<bf, 128, 128, 64, 2, 2, 1, 192>>("bptt", "128x128(1 fr) 4w", p, out, ref, fl);
    halo<HaloCfg<bf, 64, 128, 64, 1, 2, 1, 176>>("bptt", "64x128(1 fr) 2w", p, out, ref, fl);
  }
  {  // batched dx: 64 rows over all frames
    const ConvGeo g = ConvGeo{512, 512, 0, h, w, h, w, 3, 1, 1, 1}.prep();
    const double fl = 2.0 * FM * 64 * 4608;
    ring<GemmCfg<bf, 64, 64, 64, 2, 2, 1>>("dx", "64x64 BK64 4w (current)", WdT, 4608, 64, dz, g, FM,
                                           (size_t)FM * 512, 4608, ref, fl);
    HaloParams p{WdT, 4608, 64, dz, 512, 0, 512, (uint32_t)((size_t)FM * 512 * 2), h, w, F, 1};
    halo<HaloCfg<bf, 64, 128, 64, 1, 2, 1, 176>>("dx", "64x128(1 fr) 2w", p, out, ref, fl);
    halo<HaloCfg<bf, 64, 256, 64, 1, 4, 2, 352>>("dx", "64x256(2 fr) 4w", p, out, ref, fl);
  }
  printf("done\n");
  return 0;
}
