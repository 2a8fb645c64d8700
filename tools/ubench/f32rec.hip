// Microbenchmark of the fp32 frame-group ConvLSTM recurrence (csrc/recur_f32.h)
// at config 2's shape (B = 32, T = 20, 11x11 grid, G = 8) on random operands:
// device time per launch of the production kernel and of its ablations
// (ABL bits: 1 no epilogue, 2 no epilogue HBM stores, 4 no partner exchange,
// 8 no MFMAs), and -- built with -DAAA_STAMPS -- per-step phase times.
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

template <int G, int ABL, bool S6 = false, bool WIDE = false, int PDW = kF32PD>
static double run(RecF32Params p, int reps, const char* name) {
  const void* k = reinterpret_cast<const void*>(&k_convlstm_fwd_f32<G, ABL, S6, WIDE, PDW>);
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  double best = 1e30, sum = 0;
  for (int r = 0; r < reps + 2; ++r) {
    CK(hipMemset(p.flags, 0, (size_t)p.B * G * 4));
    CK(hipEventRecord(a, 0));
    CK(launch_resident(k, f32_grid(p.B, G), 256, p, 0));
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    if (r >= 2) { best = std::min(best, (double)ms); sum += ms; }
  }
  printf("%-34s G=%d  best %8.1f us  mean %8.1f us\n", name, G, best * 1e3, sum / reps * 1e3);
  return best;
}

#ifdef AAA_STAMPS
static void phases(int G, int B, int T) {
  const int nwg = f32_grid(B, G);
  std::vector<uint64_t> st((size_t)512 * 64 * 5);
  CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(aaa_f32_stamps), st.size() * 8));
  // per step: median over live workgroups of each phase
  const char* nm[4] = {"x-part+exch", "h-part", "epilogue", "publish"};
  std::vector<double> tot(4, 0.0);
  for (int t = 0; t < T; ++t) {
    std::vector<double> ph[4], span;
    for (int w = 0; w < nwg; ++w) {
      const int xcd = w & 7, loc = w >> 3, b = xcd + 8 * (loc / G);
      if (b >= B) continue;
      const uint64_t* s = &st[((size_t)w * 64 + t) * 5];
      for (int k = 0; k < 4; ++k) ph[k].push_back((s[k + 1] - s[k]) * 0.01);
      if (t + 1 < T) span.push_back((st[((size_t)w * 64 + t + 1) * 5] - s[0]) * 0.01);
    }
    printf("  t=%2d", t);
    for (int k = 0; k < 4; ++k) {
      std::sort(ph[k].begin(), ph[k].end());
      const double med = ph[k][ph[k].size() / 2];
      tot[k] += med;
      printf("  %s %6.2f (max %6.2f)", nm[k], med, ph[k].back());
    }
    printf("\n");
  }
  {  // in-kernel shader clock over the h-parts (stamps 1 -> 2), median over workgroups and steps 1..T-1
    std::vector<uint64_t> ck((size_t)512 * 64 * 5);
    CK(hipMemcpyFromSymbol(ck.data(), HIP_SYMBOL(aaa_f32_clocks), ck.size() * 8));
    std::vector<double> ghz;
    for (int w = 0; w < nwg; ++w) {
      const int xcd = w & 7, loc = w >> 3, b = xcd + 8 * (loc / G);
      if (b >= B) continue;
      for (int t = 1; t < T; ++t) {
        const size_t i = ((size_t)w * 64 + t) * 5;
        ghz.push_back((double)(ck[i + 2] - ck[i + 1]) / ((st[i + 2] - st[i + 1]) * 10.0));
      }
    }
    std::sort(ghz.begin(), ghz.end());
    printf("  shader clock over h-parts: p10 %.3f  p50 %.3f  p90 %.3f GHz\n", ghz[ghz.size() / 10], ghz[ghz.size() / 2],
           ghz[ghz.size() * 9 / 10]);
  }
  printf("  sum of medians:");
  for (int k = 0; k < 4; ++k) printf("  %s %.1f", nm[k], tot[k]);
  printf("\n");
}
#endif

template <int ABL, bool S6 = false, int PDS = kB32PD>
static double run_bwd(RecBwdF32Params p, int reps, const char* name) {
  const void* k = reinterpret_cast<const void*>(&k_convlstm_bwd_f32<ABL, S6, PDS>);
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  double best = 1e30, sum = 0;
  for (int r = 0; r < reps + 2; ++r) {
    CK(hipMemset(p.flags, 0, (size_t)p.B * 8 * 4));
    CK(hipEventRecord(a, 0));
    CK(launch_resident(k, f32_grid(p.B, 8), 256, p, 0));
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    if (r >= 2) { best = std::min(best, (double)ms); sum += ms; }
  }
  printf("BPTT %-29s G=8  best %8.1f us  mean %8.1f us\n", name, best * 1e3, sum / reps * 1e3);
  return best;
}

#ifdef AAA_STAMPS
static void phases_bwd(int B, int T) {
  const int nwg = f32_grid(B, 8);
  std::vector<uint64_t> st((size_t)512 * 64 * 4);
  CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(aaa_b32_stamps), st.size() * 8));
  const char* nm[3] = {"K loop", "publish+wait", "sum+gate bwd"};
  std::vector<double> tot(3, 0.0);
  for (int it = 0; it < T - 1; ++it) {
    std::vector<double> ph[3];
    for (int w = 0; w < nwg; ++w) {
      const int xcd = w & 7, loc = w >> 3, b = xcd + 8 * (loc / 8);
      if (b >= B) continue;
      const uint64_t* s = &st[((size_t)w * 64 + it) * 4];
      for (int k = 0; k < 3; ++k) ph[k].push_back((s[k + 1] - s[k]) * 0.01);
    }
    if (it % 4 == 1) printf("  it=%2d", it);
    for (int k = 0; k < 3; ++k) {
      std::sort(ph[k].begin(), ph[k].end());
      const double med = ph[k][ph[k].size() / 2];
      tot[k] += med;
      if (it % 4 == 1) printf("  %s %6.2f (max %6.2f)", nm[k], med, ph[k].back());
    }
    if (it % 4 == 1) printf("\n");
  }
  printf("  BPTT sum of medians:");
  for (int k = 0; k < 3; ++k) printf("  %s %.1f", nm[k], tot[k]);
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
  const int reps = 10;
  run<8, 0>(p, reps, "production");
#ifdef AAA_STAMPS
  phases(8, B, T);
#endif
  run<8, 2>(p, reps, "no epilogue HBM stores");
  run<8, 4>(p, reps, "no partner exchange");
  run<8, 1>(p, reps, "no epilogue");
  run<8, 5>(p, reps, "no epilogue, no exchange");
  run<8, 13>(p, reps, "no epilogue/exchange/MFMA");
  run<4, 0>(p, reps, "production");
  {  // the split-product (bf16x6) kernel, the production fp32 path since round 4
    void* w6;
    CK(hipMalloc(&w6, (size_t)16 * kF32QP * 64 * 24));
    CK(split_frag(p.Wf, w6, 16 * kF32QP * 64, 0));
    p.Wf6 = reinterpret_cast<const u32x2*>(w6);
    for (int rep = 0; rep < 2; ++rep) {   // the arms twice, in opposite orders (clock drift)
      if (rep == 1) {
        run<8, 0, true, true, 4>(p, reps, "S6 WIDE, 4 A quads in flight (production)");
        run<8, 0, true, false, 4>(p, reps, "S6, 4 A quads in flight");
        run<8, 0, true, true>(p, reps, "S6 WIDE (1 wave per column block)");
      }
      run<8, 0, true>(p, reps, "S6 2 column blocks per wave, 8 in flight");
      run<8, 16, true>(p, reps, "S6 no B split (hi only)");
      run<8, 1, true>(p, reps, "S6 no epilogue");
      if (rep == 0) {
        run<8, 0, true, true>(p, reps, "S6 WIDE (1 wave per column block)");
        run<8, 0, true, false, 4>(p, reps, "S6, 4 A quads in flight");
        run<8, 0, true, true, 4>(p, reps, "S6 WIDE, 4 A quads in flight (production)");
      }
    }
  }
  {  // the frame-group BPTT at the same shape
    RecBwdF32Params q{};
    q.Wb = dev_rand((size_t)8 * kB32QP * 4 * 256, 0.02f, 7);
    q.dO = dev_rand((size_t)T * M * 128, 0.1f, 8);
    q.Gt = dev_rand((size_t)T * M * 512, 0.5f, 9);
    q.Cst = p.Cst;
    q.dC = dev_rand(M * 128, 0.1f, 10);
    q.dZ = dev_rand((size_t)T * M * 512, 0.1f, 11);
    q.part = dev_rand((size_t)T * B * 512, 1.f, 12);
    q.dh0 = nullptr;
    CK(hipMalloc(&q.xp, b32_xpart_floats(B) * 4));
    q.flags = p.flags; q.report = p.report; q.spin = p.spin;
    q.T = T; q.B = B; q.h = h; q.w = w; q.P = P;
    for (int c = 0; c < 128; ++c) q.colhb[c] = p.colhb[c];
    run_bwd<0>(q, reps, "production");
#ifdef AAA_STAMPS
    phases_bwd(B, T);
#endif
    run_bwd<1>(q, reps, "no partner waits");
    run_bwd<9>(q, reps, "no exchange");
    run_bwd<11>(q, reps, "no exchange, no MFMA");
    void* w6;
    CK(hipMalloc(&w6, (size_t)8 * kB32QP * 4 * 64 * 24));
    CK(split_frag(q.Wb, w6, 8 * kB32QP * 4 * 64, 0));
    q.Wb6 = reinterpret_cast<const u32x2*>(w6);
    for (int rep = 0; rep < 2; ++rep) {
      if (rep == 1) run_bwd<0, true, 4>(q, reps, "S6, 4 A quads in flight (production)");
      run_bwd<0, true>(q, reps, "S6, 8 A quads in flight");
      run_bwd<16, true>(q, reps, "S6 no B split (hi only)");
      if (rep == 0) run_bwd<0, true, 4>(q, reps, "S6, 4 A quads in flight (production)");
    }

  }
  printf("timeout reports: %d\n", *hrep);
  return 0;
}
