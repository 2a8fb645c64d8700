// Phase stamps of the attention readout backward (csrc/misc.hip k_attn_bwd) at
// config 5's shape (F = 3200 frames of a 21x21 grid, nq = 8) and config 3's
// (5120 frames of 11x11, nq = 4), on random operands, reading O as fp32 rows
// of 128 (fp32 path) or as the bf16 h half of XH rows (bf16 path); the
// forward readout timed beside it.  Timing only.
//   EXTRA=-DAAA_STAMPS tools/ubench/build.sh attn_stamps.hip && tools/ubench/attn_stamps
#include <algorithm>
#include <cstdio>
#include <vector>
#include "misc.hip"

using namespace aaa;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

static float* dev_rand(size_t n, float lo, float hi, unsigned seed) {
  std::vector<float> h(n);
  unsigned s = seed;
  for (auto& v : h) { s = s * 1664525u + 1013904223u; v = lo + (hi - lo) * (((s >> 8) & 0xffff) / 65536.f); }
  float* d; CK(hipMalloc(&d, n * 4)); CK(hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice));
  return d;
}

__global__ void k_to_xh(const float* h, __bf16* xh, long n) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += gridDim.x * 256L)
    xh[(i >> 7) * 192 + 64 + (i & 127)] = (__bf16)h[i];
}

static void run(int F, int P, int nq, bool bf) {
  const int da_ld = 256 * nq + 2;
  float* Hs = dev_rand((size_t)F * P * 128, -1.f, 1.f, 1);
  __bf16* XH;
  CK(hipMalloc(&XH, (size_t)F * P * 192 * 2));
  hipLaunchKernelGGL(k_to_xh, dim3(4096), dim3(256), 0, 0, Hs, XH, (long)F * P * 128);
  const OSrc O = bf ? o_bf16(XH + 64, 192) : o_f32(Hs);
  float *SQ, *ans;
  CK(hipMalloc(&SQ, (size_t)P * nq * 4));
  CK(hipMalloc(&ans, (size_t)F * da_ld * 4));
  float* S = dev_rand((size_t)P * 64, -1.f, 1.f, 2);
  float* Q = dev_rand((size_t)nq * 72, -0.5f, 0.5f, 3);
  float* Am = dev_rand((size_t)F * P * nq, 0.f, 2.f / P, 4);
  float* dAns = dev_rand((size_t)F * da_ld, -1.f, 1.f, 5);
  float *dO, *dQ;
  CK(hipMalloc(&dO, (size_t)F * P * 128 * 4));
  CK(hipMalloc(&dQ, (size_t)F * nq * 72 * 4));
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  float best = 1e30f;
  for (int r = 0; r < 8; ++r) {
    CK(hipEventRecord(a, 0));
    CK(attn_bwd(O, S, Q, Am, dAns, da_ld, F, P, nq, dO, dQ, 0, 0, 0));
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    if (r >= 2) best = std::min(best, ms);
  }
  const double oe = bf ? 2.0 : 4.0;
  const double bytes = F * (oe * 128 * P + 4.0 * (128.0 * P + nq * P + 184.0 * nq + 72.0 * nq));
  printf("attn_bwd %s F=%d P=%d nq=%d: %.1f us  %.2f TB/s\n", bf ? "bf16 O" : "fp32 O", F, P, nq, best * 1e3,
         bytes / (best * 1e-3) / 1e12);
  CK(query_sq(S, Q, P, nq, SQ, 0));
  float bestf = 1e30f;
  for (int r = 0; r < 8; ++r) {
    CK(hipEventRecord(a, 0));
    CK(attn_fwd(O, S, Q, SQ, nullptr, nullptr, F, P, nq, Am, ans, da_ld, 0));
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    if (r >= 2) bestf = std::min(bestf, ms);
  }
  const double fbytes = F * (oe * 128 * P + 4.0 * (nq * P + da_ld));
  printf("attn_fwd %s: %.1f us  %.2f TB/s\n", bf ? "bf16 O" : "fp32 O", bestf * 1e3, fbytes / (bestf * 1e-3) / 1e12);
#ifdef AAA_STAMPS
  const int n = std::min(F, 16384);
  std::vector<uint64_t> st((size_t)n * 8);
  CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(aaa_attn_stamps), st.size() * 8));
  const char* nm[6] = {"loads", "dA chunks", "softmax bwd", "dO", "dQ partials", "dQ sum"};
  std::vector<double> ph[6], life;
  uint64_t t0 = ~0ull, t1 = 0;
  for (int i = 0; i < n; ++i) {
    for (int k = 0; k < 6; ++k) ph[k].push_back((st[i * 8 + k + 1] - st[i * 8 + k]) * 0.01);
    life.push_back((st[i * 8 + 6] - st[i * 8]) * 0.01);
    t0 = std::min(t0, st[i * 8]); t1 = std::max(t1, st[i * 8 + 6]);
  }
  printf("  phase medians (us):");
  for (int k = 0; k < 6; ++k) { std::sort(ph[k].begin(), ph[k].end()); printf("  %s %.2f", nm[k], ph[k][n / 2]); }
  std::sort(life.begin(), life.end());
  printf("  | workgroup lifetime %.2f, span %.1f\n", life[n / 2], (t1 - t0) * 0.01);
#endif
}

int main() {
  for (int bf = 0; bf < 2; ++bf) {
    run(3200, 441, 8, bf);
    run(5120, 121, 4, bf);
  }
  return 0;
}
