// Winograd F(2x2,3x3) ConvLSTM kernels (csrc/wino.h) vs the direct implicit
// GEMMs at C2 size: checks each Winograd launch against the direct kernel on the
// same random operands (transformed weights built on the host in fp64 from one
// random ConvLSTM weight), then times both with the production epilogues.
// Diagnostic only:  tools/ubench/build.sh wino.hip && tools/ubench/wino [B]
#include <cmath>
#include <cstdio>
#include <type_traits>
#include <vector>
#include "glds.h"
#include "epilogues.h"
#include "wino.h"   // tools/ubench/wino.h (diagnostic; not in the library)

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

static std::vector<float> host_rand(size_t n, float scale, unsigned seed) {
  std::vector<float> h(n);
  unsigned s = seed;
  for (auto& v : h) { s = s * 1664525u + 1013904223u; v = scale * (((s >> 8) & 0xffff) / 32768.f - 1.f); }
  return h;
}
static float* up(const std::vector<float>& h) {
  float* d; CK(hipMalloc(&d, h.size() * 4)); CK(hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  return d;
}
static float* dzeros(size_t n) { float* d; CK(hipMalloc(&d, n * 4)); CK(hipMemset(d, 0, n * 4)); return d; }
static std::vector<float> down(const float* d, size_t n) {
  std::vector<float> h(n); CK(hipMemcpy(h.data(), d, n * 4, hipMemcpyDeviceToHost)); return h;
}
static double relerr(const std::vector<float>& a, const std::vector<float>& b) {
  double m = 0, r = 0;
  for (size_t i = 0; i < a.size(); ++i) { m = std::max(m, (double)std::fabs(b[i])); r = std::max(r, (double)std::fabs(a[i] - b[i])); }
  return r / (m > 0 ? m : 1);
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 32, T = 20, h = 11, w = 11, P = h * w, M = B * P, F = B * T, R = F * P;
  // ConvLSTM weight w[n][ky][kx][c'], n = 4ch + gate, c' over [x (64) | h (128)]
  const auto wt = host_rand((size_t)512 * 9 * 192, 0.05f, 1);
  auto W = [&](int n, int ky, int kx, int c) { return wt[((size_t)n * 9 + ky * 3 + kx) * 192 + c]; };
  std::vector<float> WpX(512 * 576), WpH(512 * 1152), WdT((size_t)192 * 4608), Uf((size_t)16 * 512 * 192),
      Ud((size_t)16 * 192 * 512);
  for (int n = 0; n < 512; ++n)
    for (int t = 0; t < 9; ++t)
      for (int c = 0; c < 192; ++c) {
        const float v = W(n, t / 3, t % 3, c);
        if (c < 64) WpX[(size_t)n * 576 + t * 64 + c] = v;
        else WpH[(size_t)n * 1152 + t * 128 + c - 64] = v;
        WdT[(size_t)c * 4608 + t * 512 + n] = v;
      }
  const double G[4][3] = {{1, 0, 0}, {.5, .5, .5}, {.5, -.5, .5}, {0, 0, 1}};
  for (int e = 0; e < 16; ++e)
    for (int n = 0; n < 512; ++n)
      for (int c = 0; c < 192; ++c) {
        double sf = 0, sd = 0;
        for (int k = 0; k < 3; ++k)
          for (int l = 0; l < 3; ++l) {
            sf += G[e >> 2][k] * G[e & 3][l] * W(n, k, l, c);
            sd += G[e >> 2][k] * G[e & 3][l] * W(n, 2 - k, 2 - l, c);
          }
        Uf[((size_t)e * 512 + n) * 192 + c] = (float)sf;
        Ud[((size_t)e * 192 + c) * 512 + n] = (float)sd;
      }
  float *dWpX = up(WpX), *dWpH = up(WpH), *dWdT = up(WdT), *dUf = up(Uf), *dUd = up(Ud);
  float* XH = up(host_rand((size_t)R * 192, 1.f, 2));
  float* dZ = up(host_rand((size_t)R * 512, 1.f, 3));
  float* o1 = dzeros((size_t)R * 512);
  float* o2 = dzeros((size_t)R * 512);
  const uint32_t xhb = (uint32_t)((size_t)R * 192 * 4), dzb = (uint32_t)((size_t)R * 512 * 4);

  using CD = GemmCfg<float, 64, 64, 32, 2, 2>;
  using CD64 = GemmCfg<float, 64, 64, 64, 2, 2>;
  using CBP = GemmCfg<float, 32, 32, 64, 1, 1, 4>;
  auto direct = [&](auto cfg, auto nb, const float* Wd, int ldw, int wrows, const float* src, const ConvGeo& g, int rows,
                    uint32_t sb, const auto& ep, int Mi, int K) {
    using C = decltype(cfg);
    using LA = GRowsB<float, C::BI, C::BK, C::NT>;
    using LB = GIm2colB<float, C::BJ, C::BK, C::NT>;
    using EP = std::decay_t<decltype(ep)>;
    CK((launch_pipe<C, LA, LB, EP, decltype(nb)::value>(typename LA::Params{Wd, ldw, wrows},
                                                        typename LB::Params{src, g, rows, sb}, ep, Mi, rows, K, 1, 0)));
  };
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;

  using P1 = WinoCfg<32, 2, 2, 1, 8>;    // 64x32, 4 waves
  using P2 = WinoCfg<16, 2, 2, 1, 8>;    // 32x32, 4 waves
  using P3 = WinoCfg<32, 2, 4, 1, 8>;    // 64x64, 8 waves
  using P4 = WinoCfg<16, 2, 1, 2, 8>;    // 32x16, 2-way split-K
  using P5 = WinoCfg<16, 2, 2, 1, 16>;   // 32x32, BK16
  using P6 = WinoCfg<32, 1, 2, 2, 8>;    // 32x32, 2-way split-K, 32-row waves
  using P7 = WinoCfg<16, 2, 2, 2, 8>;    // 32x32, 2-way split-K, 8 waves
  using I1 = std::integral_constant<int, 1>;
  (void)sizeof(I1);
  auto wl = [&](auto cfg, auto nb, const float* U, int ldu, int urows, int urow0, int uoff, const float* src,
                const WinoGeo& g, const auto& ep, int Mi, int K) {
    using C = decltype(cfg);
    using EP = std::decay_t<decltype(ep)>;
    CK((launch_wino<C, EP, decltype(nb)::value>(U, ldu, urows, urow0, uoff, src, g, ep, Mi, K, 0)));
  };
  // ---------------- correctness: raw conv outputs
  auto check = [&](const char* name, auto cfg, auto nb, const float* U, int ldu, int urows, int urow0, int uoff,
                   const float* src, int cs, int coff, int frames, uint32_t sb, int Mi, int K, auto ref_launch) {
    const int rows = frames * P;
    CK(hipMemset(o1, 0, (size_t)rows * Mi * 4));
    CK(hipMemset(o2, 0, (size_t)rows * Mi * 4));
    ref_launch(EpiStoreT<float>{o1, Mi, Mi, rows, nullptr, 0});
    const WinoGeo g = wino_geo(h, w, frames, cs, coff, sb);
    wl(cfg, nb, U, ldu, urows, urow0, uoff, src, g, EpiStoreT<float>{o2, Mi, Mi, rows, nullptr, 0}, Mi, K);
    CK(hipDeviceSynchronize());
    const double e = relerr(down(o2, (size_t)rows * Mi), down(o1, (size_t)rows * Mi));
    printf("check %-44s rel max err %.3e %s\n", name, e, e < 1e-5 ? "ok" : "MISMATCH");
  };
  const ConvGeo gx = ConvGeo{64, 192, 0, h, w, h, w, 3, 1, 1, 0}.prep();
  const ConvGeo gh = ConvGeo{128, 192, 64, h, w, h, w, 3, 1, 1, 0}.prep();
  const ConvGeo gd = ConvGeo{512, 512, 0, h, w, h, w, 3, 1, 1, 1}.prep();
  const uint32_t sbh = (uint32_t)(M * 768), sbz = (uint32_t)(M * 2048);
  auto refx = [&](auto ep) { direct(CD{}, I2{}, dWpX, 576, 512, XH, gx, R, xhb, ep, 512, 576); };
  auto refh = [&](auto ep) { direct(CD{}, I2{}, dWpH, 1152, 512, XH, gh, M, sbh, ep, 512, 1152); };
  auto refb = [&](auto ep) { direct(CD{}, I2{}, dWdT + 64 * 4608, 4608, 128, dZ, gd, M, sbz, ep, 128, 4608); };
  auto refd = [&](auto ep) { direct(CD{}, I2{}, dWdT, 4608, 64, dZ, gd, R, dzb, ep, 64, 4608); };
  check("x-part P1", P1{}, I2{}, dUf, 192, 512, 0, 0, XH, 192, 0, F, xhb, 512, 64, refx);
  check("x-part P3", P3{}, I2{}, dUf, 192, 512, 0, 0, XH, 192, 0, F, xhb, 512, 64, refx);
  check("h-part P2", P2{}, I2{}, dUf, 192, 512, 0, 64, XH, 192, 64, B, sbh, 512, 128, refh);
  check("h-part P5 (BK16)", P5{}, I2{}, dUf, 192, 512, 0, 64, XH, 192, 64, B, sbh, 512, 128, refh);
  check("h-part P6", P6{}, I2{}, dUf, 192, 512, 0, 64, XH, 192, 64, B, sbh, 512, 128, refh);
  check("dh P4", P4{}, I2{}, dUd, 512, 192, 64, 0, dZ, 512, 0, B, sbz, 128, 512, refb);
  check("dh P7", P7{}, I2{}, dUd, 512, 192, 64, 0, dZ, 512, 0, B, sbz, 128, 512, refb);
  check("dx P1", P1{}, I3{}, dUd, 512, 192, 0, 0, dZ, 512, 0, F, dzb, 64, 512, refd);

  // ---------------- timing with production epilogues
  float* bias = up(host_rand(512, 0.1f, 4));
  float* gates = up(host_rand((size_t)M * 512, 0.5f, 5));
  float* cprev = up(host_rand((size_t)M * 128, 1.f, 6));
  float* ccur = up(host_rand((size_t)M * 128, 1.f, 7));
  float* dO = up(host_rand((size_t)M * 128, 1.f, 8));
  float* dC = up(host_rand((size_t)M * 128, 1.f, 9));
  float* hs = dzeros((size_t)M * 128);
  float* part = dzeros((size_t)4096 * 512);
  float* gb = dzeros(512);
  const double fx = 2.0 * R * 512 * 576, fs = 2.0 * M * 512 * 1152, fb = 2.0 * M * 128 * 4608, fd = 2.0 * R * 64 * 4608;
  auto rep = [&](const char* name, double fl, float us) {
    printf("%-52s %8.2f us  %6.1f TF/s direct-equivalent, %6.1f Winograd MFMA\n", name, us, fl / (us * 1e-6) / 1e12,
           fl * (16.0 * 36 / 121 / 9) / (us * 1e-6) / 1e12);
  };
  {
    EpiStoreT<float> ep{o1, 512, 512, R, bias, 0};
    rep("x-part direct 64x64 BK32 pipe2", fx, time_us([&] { refx(ep); }));
    const WinoGeo g = wino_geo(h, w, F, 192, 0, xhb);
    auto t = [&](const char* n, auto c, auto nb) { rep(n, fx, time_us([&] { wl(c, nb, dUf, 192, 512, 0, 0, XH, g, ep, 512, 64); })); };
    t("x-part P1 64x32 r2", P1{}, I2{});
    t("x-part P1 64x32 r3", P1{}, I3{});
    t("x-part P2 32x32 r2", P2{}, I2{});
    t("x-part P2 32x32 r3", P2{}, I3{});
    t("x-part P3 64x64 8w r2", P3{}, I2{});
    t("x-part P5 32x32 BK16 r2", P5{}, I2{});
  }
  {
    EpiConvLstmFwd<float> ep{cprev, ccur, hs, XH + (size_t)M * 192, gates, M};
    rep("fwd step direct 64x64 BK64 pipe2 (tile 6)", fs, time_us([&] { direct(CD64{}, I2{}, dWpH, 1152, 512, XH, gh, M, sbh, ep, 512, 1152); }));
    const WinoGeo g = wino_geo(h, w, B, 192, 64, sbh);
    auto t = [&](const char* n, auto c, auto nb) { rep(n, fs, time_us([&] { wl(c, nb, dUf, 192, 512, 0, 64, XH, g, ep, 512, 128); })); };
    t("fwd P1 64x32 r2", P1{}, I2{});
    t("fwd P2 32x32 r2", P2{}, I2{});
    t("fwd P2 32x32 r3", P2{}, I3{});
    t("fwd P4 32x16 2-way r2", P4{}, I2{});
    t("fwd P5 32x32 BK16 r2", P5{}, I2{});
    t("fwd P6 32x32 2-way r2", P6{}, I2{});
    t("fwd P7 32x32 2-way 8w r2", P7{}, I2{});
  }
  {
    float* dzo = o2;
    EpiConvLstmBwd<float, float> ep{nullptr, gates, cprev, ccur, dO, dC, dzo, nullptr, 1, M, 64, part};
    rep("bptt direct 32x32 BK64 4-way pipe3 (tile 16)", fb, time_us([&] { direct(CBP{}, I3{}, dWdT + 64 * 4608, 4608, 128, dZ, gd, M, sbz, ep, 128, 4608); }));
    const WinoGeo g = wino_geo(h, w, B, 512, 0, sbz);
    auto t = [&](const char* n, auto c, auto nb) { rep(n, fb, time_us([&] { wl(c, nb, dUd, 512, 192, 64, 0, dZ, g, ep, 128, 512); })); };
    t("bptt P2 32x32 r2", P2{}, I2{});
    t("bptt P2 32x32 r3", P2{}, I3{});
    t("bptt P4 32x16 2-way r2", P4{}, I2{});
    t("bptt P4 32x16 2-way r3", P4{}, I3{});
    t("bptt P6 32x32 2-way r2", P6{}, I2{});
    t("bptt P7 32x32 2-way 8w r2", P7{}, I2{});
  }
  {
    EpiStoreBiasT<float> ep{o1, 64, 64, R, gb};
    rep("dx direct 64x64 BK32 pipe2", fd, time_us([&] { refd(ep); }));
    const WinoGeo g = wino_geo(h, w, F, 512, 0, dzb);
    auto t = [&](const char* n, auto c, auto nb) { rep(n, fd, time_us([&] { wl(c, nb, dUd, 512, 192, 0, 0, dZ, g, ep, 64, 512); })); };
    t("dx P1 64x32 r2", P1{}, I2{});
    t("dx P1 64x32 r3", P1{}, I3{});
    t("dx P3 64x64 8w r2", P3{}, I2{});
    t("dx P6 32x32 2-way r2", P6{}, I2{});
  }
  {  // ablations (x-part, C2 rows): where does a stage's time go
    EpiStoreT<float> ep{o1, 512, 512, R, bias, 0};
    const WinoGeo g = wino_geo(h, w, F, 192, 0, xhb);
    auto ab = [&](const char* n, auto c, auto abl) {
      using Cc = decltype(c);
      rep(n, fx, time_us([&] { CK((launch_wino<Cc, EpiStoreT<float>, 2, decltype(abl)::value>(dUf, 192, 512, 0, 0, XH, g, ep, 512, 64, 0))); }));
    };
    using A0 = std::integral_constant<int, 0>;
    using A1 = std::integral_constant<int, 1>;
    using A2 = std::integral_constant<int, 2>;
    using A4 = std::integral_constant<int, 4>;
    using A5 = std::integral_constant<int, 5>;
    using A6 = std::integral_constant<int, 6>;
    ab("abl P2 full", P2{}, A0{});
    ab("abl P2 no transform", P2{}, A1{});
    ab("abl P2 no MFMA", P2{}, A2{});
    ab("abl P2 no LDS frag reads", P2{}, A4{});
    ab("abl P2 no reads, no transform", P2{}, A5{});
    ab("abl P2 no reads, no MFMA (DMA + epilogue)", P2{}, A6{});
    ab("abl P3 full", P3{}, A0{});
    ab("abl P3 no transform", P3{}, A1{});
    ab("abl P3 no MFMA", P3{}, A2{});
    ab("abl P3 no LDS frag reads", P3{}, A4{});
    ab("abl P3 no reads, no MFMA (DMA + epilogue)", P3{}, A6{});
  }
  printf("done\n");
  return 0;
}
