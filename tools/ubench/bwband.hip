// Microbenchmark of the bf16 frame-resident ConvLSTM BPTT (csrc/recur_bwd.h) on
// random operands: the band kernel at config 5's shape (B = 64, T = 50, 21x21
// grid, 4 bands) and the single-workgroup kernel at config 3's (B = 256, T = 20,
// 11x11), plus the split-role kernel (tools/ubench/recur_bwd_split.h, a rejected variant kept out of libaaa.so) at both.  Device
// time per launch of the production kernels and of their ablations (ABL bits
// in recur_bwd.h) and -- built with -DAAA_STAMPS -- per-step phase times.
// Timing only: the results are not checked (tests/test_gpu_band.py,
// tests/test_gpu_parity.py are).
//   EXTRA="-DAAA_STAMPS -DAAA_ABLATION" tools/ubench/build.sh bwband.hip && tools/ubench/bwband
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "recur.h"
#include "recur_bwd.h"

using namespace aaa;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

template <typename T>
static T* dev_rand(size_t n, float scale, unsigned seed) {
  std::vector<T> h(n);
  unsigned s = seed;
  for (auto& v : h) { s = s * 1664525u + 1013904223u; v = (T)(scale * (((s >> 8) & 0xffff) / 32768.f - 1.f)); }
  T* d; CK(hipMalloc(&d, n * sizeof(T))); CK(hipMemcpy(d, h.data(), n * sizeof(T), hipMemcpyHostToDevice));
  return d;
}

static double timeit(const void* k, int grid, int block, RecBwdParams& p, bool resident, int reps, const char* name) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  double best = 1e30, sum = 0;
  for (int r = 0; r < reps + 2; ++r) {
    CK(hipMemset(p.flags, 0, (size_t)p.B * kRecBands * 4));
    CK(hipEventRecord(a, 0));
    if (resident) CK(launch_resident(k, grid, block, p, 0));
    else { void* args[] = {&p}; CK(hipLaunchKernel(k, dim3(grid), dim3(block), args, 0, 0)); }
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    if (r >= 2) { best = std::min(best, (double)ms); sum += ms; }
  }
  printf("%-44s best %8.1f us  mean %8.1f us  (%.1f us/step)\n", name, best * 1e3, sum / reps * 1e3, best * 1e3 / p.T);
  return best;
}

#ifdef AAA_STAMPS
static void phases(int nblk, int B, int T, bool band) {
  std::vector<uint64_t> st((size_t)1024 * 64 * 8);
  CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(aaa_bw_stamps), st.size() * 8));
  const char* nm[7] = {"halo", "chunk0", "chunk1", "chunk2", "chunk3", "dx", "epilogue"};
  std::vector<double> tot(7, 0.0);
  int n = 0;
  for (int t = T - 2; t >= 1; --t) {   // interior steps
    std::vector<double> ph[7];
    for (int w = 0; w < nblk; ++w) {
      if (band) { const int loc = w >> 3, b = (w & 7) + 8 * (loc / kRecBands); if (b >= B) continue; }
      const uint64_t* s = &st[((size_t)w * 64 + t) * 8];
      for (int k = 0; k < 7; ++k) ph[k].push_back((double)(s[k + 1] - s[k]) * 0.01);
    }
    for (int k = 0; k < 7; ++k) {
      std::sort(ph[k].begin(), ph[k].end());
      tot[k] += ph[k][ph[k].size() / 2];
    }
    ++n;
  }
  printf("  per-step phase medians (us):");
  double all = 0;
  for (int k = 0; k < 7; ++k) { printf("  %s %.2f", nm[k], tot[k] / n); all += tot[k] / n; }
  printf("  | sum %.2f\n", all);
}
#endif

static void bench(int B, int T, int h, int w, bool band) {
  const int P = h * w;
  const size_t M = (size_t)B * P;
  RecBwdParams p{};
  p.Wb = dev_rand<__bf16>((size_t)6 * kBwKSP * 64 * 8, 0.02f, 1);
  p.dO = dev_rand<float>((size_t)T * M * 128, 0.1f, 2);
  p.Gt = dev_rand<_Float16>((size_t)T * M * 512, 0.5f, 3);
  p.Cst = dev_rand<float>((size_t)(T + 1) * M * 128, 1.f, 4);
  p.dhT = nullptr;
  p.dC = dev_rand<float>(M * 128, 0.1f, 5);
  p.dZ = dev_rand<__bf16>((size_t)T * M * 512, 0.1f, 6);
  CK(hipMalloc(&p.part, (size_t)T * B * kRecBands * 512 * 4));
  p.dh0 = nullptr;
  p.dY2 = dev_rand<__bf16>((size_t)T * M * 64, 0.1f, 7);
  CK(hipMalloc(&p.dxb, (size_t)B * 64 * 4));
  CK(hipMalloc(&p.flags, (size_t)B * kRecBands * 4));
  int* hrep = nullptr;
  CK(hipHostMalloc(&hrep, 64, hipHostMallocMapped | hipHostMallocCoherent));
  CK(hipHostGetDevicePointer((void**)&p.report, hrep, 0));
  p.spin = 1 << 24;
  p.T = T; p.B = B; p.h = h; p.w = w; p.P = P;
  const int reps = 6;
  const int grid = band ? 8 * kRecBands * ((B + 7) / 8) : B;
  printf("%s: B=%d T=%d %dx%d\n", band ? "band" : "frame", B, T, h, w);
#define RUN(ABL, name)                                                                                              \
  timeit(band ? reinterpret_cast<const void*>(&k_convlstm_bwd_frames<ABL, true>)                                   \
              : reinterpret_cast<const void*>(&k_convlstm_bwd_frames<ABL, false>),                                 \
         grid, 256, p, band, reps, name)
  RUN(0, "production");
#ifdef AAA_STAMPS
  phases(grid, B, T, band);
#endif
  RUN(2, "no epilogue HBM loads/stores");
  RUN(32, "no dZ stores");
  RUN(64, "no epilogue loads");
  RUN(1, "no A loads");
  RUN(4, "no MFMA");
  RUN(8, "no chunk-3 DMA");
  RUN(128, "coalesced epilogue loads (same bytes)");
  RUN(160, "coalesced epilogue loads, no dZ stores");
  if (band) RUN(16, "no halo exchange");
  timeit(band ? reinterpret_cast<const void*>(&k_convlstm_bwd_frames<0, true, true>)
              : reinterpret_cast<const void*>(&k_convlstm_bwd_frames<0, false, false>),
         grid, 256, p, band, reps, band ? "dO in the accumulators (band)" : "dO in the ring (frame)");
  printf("timeout reports: %d\n", *hrep);
}

#ifdef AAA_STAMPS
static void phases_fwd(int nblk, int B, int T, int G, bool band) {
  std::vector<uint64_t> st((size_t)1024 * 64 * 8);
  CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(aaa_fw_stamps), st.size() * 8));
  const char* nm[5] = {"x-part", "exchange", "h-part", "epilogue", "h store/publish"};
  std::vector<double> tot(5, 0.0);
  int n = 0;
  for (int t = 1; t < T - 1; ++t) {
    std::vector<double> ph[5];
    for (int w = 0; w < nblk; ++w) {
      if (band) { const int loc = w >> 3, b = (w & 7) + 8 * (loc / kRecBands); if (b >= B) continue; }
      const uint64_t* s = &st[((size_t)w * 64 + t) * 8];
      for (int k = 0; k < 5; ++k) ph[k].push_back((double)(s[k + 1] - s[k]) * 0.01);
    }
    for (int k = 0; k < 5; ++k) {
      std::sort(ph[k].begin(), ph[k].end());
      tot[k] += ph[k][ph[k].size() / 2];
    }
    ++n;
  }
  printf("  per-step phase medians (us):");
  double all = 0;
  for (int k = 0; k < 5; ++k) { printf("  %s %.2f", nm[k], tot[k] / n); all += tot[k] / n; }
  printf("  | sum %.2f\n", all);
}
#endif

// the bf16 frame-resident forward (recur.h): G = 1, G = 2 (paired) or band mode;
// ABL ablations (timing only): 1 no A loads, 2 no epilogue HBM stores, 4 no MFMAs,
// 8 no B fragment reads; cqm = the slice layout mask, hs = keep the fp32 h copy
template <int ABL = 0>
static void bench_fwd(int B, int T, int h, int w, int G, bool band, int cqm = 3, bool hs = false,
                      const char* what = "production") {
  const int P = h * w;
  const size_t M = (size_t)B * P;
  RecFwdParams<_Float16> p{};
  p.Wf = dev_rand<__bf16>((size_t)16 * kRecKSP * 64 * 8, 0.02f, 11);
  p.bias = dev_rand<float>(512, 0.1f, 12);
  p.XH = dev_rand<__bf16>((size_t)(T + 1) * M * 192, 1.f, 13);
  p.Cst = dev_rand<float>((size_t)(T + 1) * M * 128, 1.f, 14);
  p.Hs = hs ? dev_rand<float>((size_t)T * M * 128, 1.f, 15) : nullptr;
  p.cqm = cqm;
  p.Gt = dev_rand<_Float16>((size_t)T * M * 512, 1.f, 16);
  CK(hipMalloc(&p.flags, (size_t)B * kRecBands * 4));
  int* hrep = nullptr;
  CK(hipHostMalloc(&hrep, 64, hipHostMallocMapped | hipHostMallocCoherent));
  CK(hipHostGetDevicePointer((void**)&p.report, hrep, 0));
  p.spin = 1 << 24;
  p.T = T; p.B = B; p.h = h; p.w = w; p.P = P;
  for (int c = 0; c < 128; ++c) {
    const int pp = c < P ? c : P - 1;
    p.colpp[c] = (short)(c < P ? c : -1);
    p.colhb[c] = (short)((pp / w) * (w + 2) + pp % w);
  }
  const int grid = band ? 8 * kRecBands * ((B + 7) / 8) : G * B;
  const void* k = band ? reinterpret_cast<const void*>(&k_convlstm_fwd_frames<_Float16, 1, ABL, true>)
                  : G == 2 ? reinterpret_cast<const void*>(&k_convlstm_fwd_frames<_Float16, 2, ABL>)
                           : reinterpret_cast<const void*>(&k_convlstm_fwd_frames<_Float16, 1, ABL>);
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  double best = 1e30;
  for (int r = 0; r < 8; ++r) {
    CK(hipMemset(p.flags, 0, (size_t)B * kRecBands * 4));
    CK(hipEventRecord(a, 0));
    CK(launch_resident(k, grid, 256, p, 0));
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    if (r >= 2) best = std::min(best, (double)ms);
  }
  printf("forward %s G=%d: B=%d T=%d %dx%d  %-34s best %8.1f us (%.1f us/step)\n", band ? "band" : "frame", G, B, T,
         h, w, what, best * 1e3, best * 1e3 / T);
#ifdef AAA_STAMPS
  if (ABL == 0) phases_fwd(grid, B, T, G, band);
#endif
  printf("timeout reports: %d\n", *hrep);
}

int main(int argc, char** argv) {
  const int which = argc > 1 ? atoi(argv[1]) : 0;
  if (which == 0 || which == 5) bench(64, 50, 21, 21, true);
  if (which == 0 || which == 3) bench(256, 20, 11, 11, false);
  if (which == 0 || which == 5) bench_fwd(64, 50, 21, 21, 1, true);
  if (which == 0 || which == 3) bench_fwd(256, 20, 11, 11, 1, false);
  if (which == 6) {   // forward ablations at C3's shape
    bench_fwd(256, 20, 11, 11, 1, false, 0, false, "row-major slices");
    bench_fwd(256, 20, 11, 11, 1, false, 3, false, "quad-major c + gates");
    bench_fwd(256, 20, 11, 11, 1, false, 3, true, "quad-major, fp32 h copy");
    bench_fwd<2>(256, 20, 11, 11, 1, false, 3, false, "no epilogue HBM stores");
    bench_fwd<1>(256, 20, 11, 11, 1, false, 3, false, "no A loads");
    bench_fwd<4>(256, 20, 11, 11, 1, false, 3, false, "no MFMAs");
    bench_fwd<8>(256, 20, 11, 11, 1, false, 3, false, "no B fragment reads");
    bench_fwd(64, 50, 21, 21, 1, true, 0, false, "band row-major slices");
    bench_fwd(64, 50, 21, 21, 1, true, 3, false, "band quad-major");
    bench_fwd<2>(64, 50, 21, 21, 1, true, 3, false, "band no epilogue HBM stores");
  }
  if (which == 0 || which == 4) bench_fwd(128, 20, 11, 11, 2, false);
  return 0;
}
