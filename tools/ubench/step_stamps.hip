// Per-workgroup phase timing of the step kernels (build with -DAAA_STAMPS):
// dispatch skew, prologue, K loop, epilogue, from s_memrealtime stamps.
#include <algorithm>
#include <cstdio>
#include <vector>
#include "glds.h"
#include "epilogues.h"

using namespace aaa;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

static float* dev_rand(size_t n, float scale, unsigned seed) {
  std::vector<float> h(n);
  unsigned s = seed;
  for (auto& v : h) { s = s * 1664525u + 1013904223u; v = scale * (((s >> 8) & 0xffff) / 32768.f - 1.f); }
  float* d; CK(hipMalloc(&d, n * 4)); CK(hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice));
  return d;
}

static void report(const char* name, int nwg) {
  std::vector<uint64_t> st((size_t)nwg * 4);
  CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(aaa_stamps), st.size() * 8));
  uint64_t t0 = ~0ull, t1 = 0;
  for (int w = 0; w < nwg; ++w) { t0 = std::min(t0, st[w * 4]); t1 = std::max(t1, st[w * 4 + 3]); }
  std::vector<double> ent, pro, loop, epi, exitv;
  for (int w = 0; w < nwg; ++w) {
    const uint64_t* s = &st[w * 4];
    ent.push_back((s[0] - t0) * 0.01); pro.push_back((s[1] - s[0]) * 0.01);
    loop.push_back((s[2] - s[1]) * 0.01); epi.push_back((s[3] - s[2]) * 0.01); exitv.push_back((s[3] - t0) * 0.01);
  }
  auto pct = [](std::vector<double> v, double p) { std::sort(v.begin(), v.end()); return v[(size_t)(p * (v.size() - 1))]; };
  printf("%s: span %.2f us over %d WGs (us: p0 / p50 / p100)\n", name, (t1 - t0) * 0.01, nwg);
  printf("  entry offset %6.2f %6.2f %6.2f\n", pct(ent, 0), pct(ent, .5), pct(ent, 1));
  printf("  prologue     %6.2f %6.2f %6.2f\n", pct(pro, 0), pct(pro, .5), pct(pro, 1));
  printf("  K loop       %6.2f %6.2f %6.2f\n", pct(loop, 0), pct(loop, .5), pct(loop, 1));
  printf("  epilogue     %6.2f %6.2f %6.2f\n", pct(epi, 0), pct(epi, .5), pct(epi, 1));
  printf("  exit         %6.2f %6.2f %6.2f\n", pct(exitv, 0), pct(exitv, .5), pct(exitv, 1));
}

int main() {
  const int B = 32, h = 11, w = 11, M = B * h * w;
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
  float* junk = dev_rand((size_t)64 << 20, 1.f, 14);   // 256 MB to flush L2/MALL between runs
  for (int rep = 0; rep < 2; ++rep) {
    const bool cold = rep == 1;
    {
      using K4B = GemmCfg<float, 32, 64, 128, 1, 2, 4>;
      const ConvGeo g = ConvGeo{512, 512, 0, h, w, h, w, 3, 1, 1, 1}.prep();
      EpiConvLstmBwd ep{nullptr, gates, cprev, ccur, dO, dC, dzo, nullptr, 1, M, 64};
      using LA = GRowsB<float, K4B::BI, K4B::BK, K4B::NT>;
      using LB = GIm2colB<float, K4B::BJ, K4B::BK, K4B::NT>;
      for (int i = 0; i < 3; ++i) {
        if (cold) CK(hipMemsetAsync(junk, i, (size_t)256 << 20, 0));
        CK((launch_pipe<K4B, LA, LB, EpiConvLstmBwd, 3, true>(typename LA::Params{WdT, 4608, 128},
                                                               typename LB::Params{dz, g, M, (uint32_t)((size_t)M * 2048)},
                                                               ep, 128, M, 4608, 1, 0)));
      }
      CK(hipDeviceSynchronize());
      report(cold ? "BPTT step (after 256 MB flush)" : "BPTT step (warm)", ((M + 63) / 64) * 4);
    }
    {
      using CF = GemmCfg<float, 64, 64, 32, 2, 2, 1>;
      const ConvGeo g = ConvGeo{128, 192, 64, h, w, h, w, 3, 1, 1, 0}.prep();
      EpiConvLstmFwd<float> ep{cprev, cn, hs, xh + (size_t)M * 192, gt, M};
      using LA = GRowsB<float, CF::BI, CF::BK, CF::NT>;
      using LB = GIm2colB<float, CF::BJ, CF::BK, CF::NT>;
      for (int i = 0; i < 3; ++i) {
        if (cold) CK(hipMemsetAsync(junk, i, (size_t)256 << 20, 0));
        CK((launch_pipe<CF, LA, LB, EpiConvLstmFwd<float>, 2>(typename LA::Params{WpH, 1152, 512},
                                                               typename LB::Params{xh, g, M, (uint32_t)((size_t)M * 768)},
                                                               ep, 512, M, 1152, 1, 0)));
      }
      CK(hipDeviceSynchronize());
      report(cold ? "fwd step (after 256 MB flush)" : "fwd step (warm)", ((M + 63) / 64) * 8);
    }
  }
  printf("done\n");
  return 0;
}
