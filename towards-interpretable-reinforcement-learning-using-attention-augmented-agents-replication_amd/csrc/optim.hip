// Fused multi-tensor Adam step: the optimizer the
// reference builds at main_mp.py:92 (torch.optim.Adam(policy.parameters(),
// lr=1e-3)) and steps at main_mp.py:78, as ONE launch over every parameter
// tensor instead of torch's per-op foreach kernels (lerp, mul, addcmul, sqrt,
// div, add, addcdiv = 7 passes over the optimizer state).
//
// Per element, in the op order of torch's _multi_tensor_adam (fp32 opmath):
//   g  = grad (+ weight_decay * p)          (-grad when maximize)
//   m  = lerp(m, g, 1 - beta1)
//   v  = v * beta2 + (1 - beta2) * g * g
//   vm = max(vmax, v) when amsgrad (vmax <- vm), else v
//   p  = p + (-lr / (1 - beta1^step)) * m / (sqrt(vm) / sqrt(1 - beta2^step) + eps)
// The step-dependent scalars are computed in double and rounded to fp32 once,
// as torch does: on the host from the caller's step, or -- with a device step
// counter (aaa_adam_step_counted) -- by each workgroup from that counter, so a
// step the guard skipped does not advance the bias corrections.  HBM traffic: 16 B read + 12 B written per element
// (20 + 16 with amsgrad) -- the kernel is bound by HBM (or Infinity Cache)
// bandwidth, so it streams 16-byte vectors, 4 per thread.
#include <cmath>

#include "common.h"
#include "optim.h"

namespace aaa {

struct AdamScalars {
  float wd, one_m_b1, b2, one_m_b2, step_size_neg, bc2_sqrt, eps;
  int amsgrad, maximize;
  const float* guard;   // skip the whole update when *guard != 0 (aaa_adam_step_guarded), or nullptr
  const int* step_dev;  // device step counter (aaa_adam_step_counted), or nullptr: the scalars above hold
  double lr, beta1, beta2;   // the host's doubles (torch's Python floats), read only with step_dev
};

// Bias-corrected scalars of update number *step_dev + 1, in double as on the host.
__device__ __forceinline__ void adam_device_step(AdamScalars& s) {
  const double step = (double)(*s.step_dev) + 1.0;
  s.step_size_neg = (float)(-(s.lr / (1.0 - pow(s.beta1, step))));
  s.bc2_sqrt = (float)sqrt(1.0 - pow(s.beta2, step));
}

__device__ __forceinline__ float adam_elem(float& p, float g, float& m, float& v, float* vmax, const AdamScalars& s) {
  if (s.maximize) g = -g;
  if (s.wd != 0.f) g = g + s.wd * p;
  // torch lerp: weight < 0.5 -> self + w * (end - self)
  m = m + s.one_m_b1 * (g - m);
  v = v * s.b2;
  v = v + s.one_m_b2 * g * g;
  float vv = v;
  if (vmax) { vv = fmaxf(*vmax, v); *vmax = vv; }
  const float denom = sqrtf(vv) / s.bc2_sqrt + s.eps;
  p = p + s.step_size_neg * (m / denom);
  return p;
}

constexpr int kAdamThreads = 256;
constexpr int kAdamVec = 4;                                   // floats per 16-byte access
constexpr int kAdamChunk = kAdamThreads * kAdamVec * 4;       // elements per workgroup

// Workgroup -> (tensor, chunk) through the chunk prefix table; tensors whose
// pointers are all 16-byte aligned use 16-byte vectors, the rest scalars.
__global__ void __launch_bounds__(kAdamThreads) k_adam(AdamTable tab, AdamScalars s) {
  if (s.guard && *s.guard != 0.f) return;   // gradients of a stranded launch: no update on any rank
  if (s.step_dev) adam_device_step(s);
  const int b = blockIdx.x;
  int t = 0;
  while (t + 1 < tab.n && tab.chunk0[t + 1] <= b) ++t;
  const size_t n = tab.numel[t];
  const size_t base = (size_t)(b - tab.chunk0[t]) * kAdamChunk;
  float* __restrict__ P = tab.p[t];
  const float* __restrict__ G = tab.g[t];
  float* __restrict__ M = tab.m[t];
  float* __restrict__ V = tab.v[t];
  float* __restrict__ X = tab.vmax[t];
  const bool vec = tab.vec[t];
  if (vec) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const size_t i = base + ((size_t)r * kAdamThreads + threadIdx.x) * kAdamVec;
      if (i + kAdamVec <= n) {
        f32x4 p = *reinterpret_cast<const f32x4*>(P + i);
        const f32x4 g = *reinterpret_cast<const f32x4*>(G + i);
        f32x4 m = *reinterpret_cast<const f32x4*>(M + i);
        f32x4 v = *reinterpret_cast<const f32x4*>(V + i);
        f32x4 x = X ? *reinterpret_cast<const f32x4*>(X + i) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float pe = p[e], me = m[e], ve = v[e], xe = x[e];
          adam_elem(pe, g[e], me, ve, X ? &xe : nullptr, s);
          p[e] = pe; m[e] = me; v[e] = ve; x[e] = xe;
        }
        *reinterpret_cast<f32x4*>(P + i) = p;
        *reinterpret_cast<f32x4*>(M + i) = m;
        *reinterpret_cast<f32x4*>(V + i) = v;
        if (X) *reinterpret_cast<f32x4*>(X + i) = x;
      } else {
        for (size_t j = i; j < n; ++j) adam_elem(P[j], G[j], M[j], V[j], X ? X + j : nullptr, s);
      }
    }
  } else {
    for (int r = 0; r < kAdamVec * 4; ++r) {
      const size_t j = base + (size_t)r * kAdamThreads + threadIdx.x;
      if (j < n) adam_elem(P[j], G[j], M[j], V[j], X ? X + j : nullptr, s);
    }
  }
}

// After k_adam in stream order: count the update iff the guard let it through.
__global__ void k_adam_advance(const float* __restrict__ guard, int* __restrict__ step_dev) {
  if (threadIdx.x == 0 && !(guard && *guard != 0.f)) step_dev[0] = step_dev[0] + 1;
}

hipError_t adam_launch(const AdamTable& tab, int nchunks, const AdamHost& h, hipStream_t st, bool advance) {
  AdamScalars s;
  s.wd = (float)h.weight_decay;
  s.one_m_b1 = (float)(1.0 - h.beta1);
  s.b2 = (float)h.beta2;
  s.one_m_b2 = (float)(1.0 - h.beta2);
  s.step_size_neg = (float)(-(h.lr / (1.0 - std::pow(h.beta1, (double)h.step))));
  s.bc2_sqrt = (float)std::sqrt(1.0 - std::pow(h.beta2, (double)h.step));
  s.eps = (float)h.eps;
  s.amsgrad = h.amsgrad;
  s.maximize = h.maximize;
  s.guard = h.guard;
  s.step_dev = h.step_dev;
  s.lr = h.lr;
  s.beta1 = h.beta1;
  s.beta2 = h.beta2;
  if (nchunks > 0) hipLaunchKernelGGL(k_adam, dim3(nchunks), dim3(kAdamThreads), 0, st, tab, s);
  if (h.step_dev && advance) hipLaunchKernelGGL(k_adam_advance, dim3(1), dim3(64), 0, st, h.guard, h.step_dev);
  return hipGetLastError();
}

// The partner timeouts of the frame-resident kernels reported since the last
// k_pair_flag on this device, as one float, in stream order: the report word
// is monotonic (rt_core.hip), ``base`` is this reader's own snapshot of it.
__global__ void k_pair_flag(const int* __restrict__ report, int* __restrict__ base, float* __restrict__ dst) {
  if (threadIdx.x == 0) {
    const int cur = __hip_atomic_load(report, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const int b = __hip_atomic_load(base, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    dst[0] = (float)(unsigned)(cur - b);
    __hip_atomic_store(base, cur, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

hipError_t pair_flag_launch(const int* report, int* base, float* dst, hipStream_t st) {
  hipLaunchKernelGGL(k_pair_flag, dim3(1), dim3(64), 0, st, report, base, dst);
  return hipGetLastError();
}

int adam_chunks(size_t numel) { return (int)((numel + kAdamChunk - 1) / kAdamChunk); }

}  // namespace aaa
