// Microbenchmark of the PRE-SPLIT fp32 frame-group ConvLSTM forward
// (csrc/recur_f32.h k_convlstm_fwd_f32ps) at config 2's shape (B = 32, T = 20,
// 11x11 grid, G = 8) on random operands: device time per launch of the
// production kernel and its ablations (ABL bits: 1 no epilogue, 4 no partner
// exchange, 8 no MFMAs, 32 no A-stream loads), beside the in-loop-split kernel
// it replaces, and -- built with -DAAA_STAMPS -- per-step phase times.
// Timing only: the results are not checked (tests/test_gpu_f32_frames.py is).
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "recur_bwd_f32.h"
#include "recur_f32.h"

using namespace aaa;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

static float* dev_rand(size_t n, float scale, unsigned seed) {
  std::vector<float> h(n);
  unsigned s = seed;
  for (auto& v : h) { s = s * 1664525u + 1013904223u; v = scale * (((s >> 8) & 0xffff) / 32768.f - 1.f); }
  float* d; CK(hipMalloc(&d, n * 4)); CK(hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice));
  return d;
}


template <class K>
static double run_k(K k, RecF32Params p, int reps, const char* name) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  double best = 1e30, sum = 0;
  for (int r = 0; r < reps + 2; ++r) {
    CK(hipMemset(p.flags, 0, (size_t)p.B * 8 * 4));
    CK(hipEventRecord(a, 0));
    CK(launch_resident(reinterpret_cast<const void*>(k), f32_grid(p.B, 8), 256, p, 0));
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    if (r >= 2) { best = std::min(best, (double)ms); sum += ms; }
  }
  printf("%-44s best %8.1f us  mean %8.1f us\n", name, best * 1e3, sum / reps * 1e3);
  return best;
}

#ifdef AAA_STAMPS
static void phases(int B, int T) {
  const int nwg = f32_grid(B, 8);
  std::vector<uint64_t> st((size_t)512 * 64 * 5);
  CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(aaa_f32_stamps), st.size() * 8));
  const char* nm[4] = {"x-part+exch", "h-part", "epilogue", "x store+publish"};
  std::vector<double> tot(4, 0.0);
  double span = 0;
  for (int t = 0; t < T; ++t) {
    std::vector<double> ph[4];
    for (int w = 0; w < nwg; ++w) {
      const int xcd = w & 7, loc = w >> 3, b = xcd + 8 * (loc / 8);
      if (b >= B) continue;
      const uint64_t* s = &st[((size_t)w * 64 + t) * 5];
      for (int k = 0; k < 4; ++k) ph[k].push_back((s[k + 1] - s[k]) * 0.01);
    }
    if (t % 4 == 1) printf("  t=%2d", t);
    for (int k = 0; k < 4; ++k) {
      std::sort(ph[k].begin(), ph[k].end());
      const double med = ph[k][ph[k].size() / 2];
      tot[k] += med;
      if (t % 4 == 1) printf("  %s %6.2f (max %6.2f)", nm[k], med, ph[k].back());
    }
    if (t % 4 == 1) printf("\n");
  }
  printf("  sum of medians:");
  for (int k = 0; k < 4; ++k) printf("  %s %.1f", nm[k], tot[k]);
  printf("\n");
}
#endif

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 32, T = argc > 2 ? atoi(argv[2]) : 20, h = 11, w = 11, P = h * w;
  const size_t M = (size_t)B * P;
  RecF32Params p{};
  p.Wf = dev_rand((size_t)16 * kF32QP * 256, 0.02f, 1);
  p.bias = dev_rand(512, 0.1f, 2);
  p.XH = dev_rand((size_t)(T + 1) * M * 192, 1.f, 3);
  p.Cst = dev_rand((size_t)(T + 1) * M * 128, 1.f, 4);
  p.Hs = dev_rand((size_t)T * M * 128, 1.f, 5);
  p.Gt = dev_rand((size_t)T * M * 512, 1.f, 6);
  CK(hipMalloc(&p.flags, (size_t)B * 8 * 4));
  int* hrep = nullptr;
  CK(hipHostMalloc(&hrep, 64, hipHostMallocMapped | hipHostMallocCoherent));
  CK(hipHostGetDevicePointer((void**)&p.report, hrep, 0));
  p.spin = 1 << 24;
  p.T = T; p.B = B; p.h = h; p.w = w; p.P = P; p.h0_zero = 1;
  for (int c = 0; c < 128; ++c) {
    const int pp = c < P ? c : P - 1;
    p.colhb[c] = (short)((pp / w) * (w + 2) + pp % w);
  }
  void* w6;
  CK(hipMalloc(&w6, (size_t)16 * kF32QP * 64 * 24));
  CK(split_frag(p.Wf, w6, 16 * kF32QP * 64, 0));
  p.Wf6 = reinterpret_cast<const u32x2*>(w6);
  const int reps = 10;
  for (int rep = 0; rep < 2; ++rep) {   // the arms twice, in opposite orders (clock drift)
    if (rep == 1) run_k(&k_convlstm_fwd_f32<8, 0, true, true, 4>, p, reps, "in-loop split (r04 production)");
    run_k(&k_convlstm_fwd_f32ps<0, 1, 8>, p, reps, "pre-split MAP1 PD8 (production)");
#ifdef AAA_STAMPS
    if (rep == 0) phases(B, T);
#endif
    run_k(&k_convlstm_fwd_f32ps<0, 1, 4>, p, reps, "pre-split MAP1 PD4");
    run_k(&k_convlstm_fwd_f32ps<0, 0, 4>, p, reps, "pre-split MAP0 PD4 (4 waves per A quad)");
    run_k(&k_convlstm_fwd_f32ps<0, 0, 8>, p, reps, "pre-split MAP0 PD8");
    run_k(&k_convlstm_fwd_f32ps<1, 1>, p, reps, "MAP1, no epilogue");
    run_k(&k_convlstm_fwd_f32ps<4, 1>, p, reps, "MAP1, no exchange");
    run_k(&k_convlstm_fwd_f32ps<8, 1>, p, reps, "MAP1, no MFMA");
    run_k(&k_convlstm_fwd_f32ps<32, 1>, p, reps, "MAP1, no A loads");
    run_k(&k_convlstm_fwd_f32ps<5, 1>, p, reps, "MAP1, no epilogue, no exchange");
    run_k(&k_convlstm_fwd_f32ps<37, 1>, p, reps, "MAP1, no epi/exch/A loads (MFMA+B)");
    run_k(&k_convlstm_fwd_f32ps<13, 1>, p, reps, "MAP1, no epi/exch/MFMA (A+B loads)");
    run_k(&k_convlstm_fwd_f32ps<45, 1>, p, reps, "MAP1, no epi/exch/MFMA/A (B reads)");

    if (rep == 0) run_k(&k_convlstm_fwd_f32<8, 0, true, true, 4>, p, reps, "in-loop split (r04 production)");
  }
  printf("timeout reports: %d\n", *hrep);
  return 0;
}
