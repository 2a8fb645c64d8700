// Policy.forward's action draw for one row of logits (main_mp.py:54-58:
// softmax -> Categorical -> sample -> log_prob), shared by the sampler kernel
// (loss.hip, aaa_sample_actions) and the actor chain's heads kernel
// (actor.hip, aaa_actor_step) so both draw bit-identical actions:
//   p_k  = exp(l_k - max l) / Z
//   a    = first k with cumsum_k(exp(l - max)) > u * Z,  u = rng(seed, counter, row) in [0, 1)
//   logp = log(clamp(p_a, eps, 1 - eps))       (Categorical(probs) clamps, as k_reinforce)
//   jac_k = d logp / d l_k = 1[k == a] - p_k   (0 where the clamp is active)
// rng: two rounds of the splitmix64 finaliser over (seed, counter, row); the
// top 24 bits give an exactly representable fp32 uniform.
#pragma once
#include <cfloat>
#include <cmath>

#include "common.h"

namespace aaa {

__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ float sample_uniform(uint64_t seed, uint64_t ctr, uint64_t row) {
  const uint64_t x = mix64(mix64(seed) ^ (ctr * 0xD1B54A32D192ED03ull + row));
  return (float)(x >> 40) * (1.0f / 16777216.0f);
}

__device__ __forceinline__ float smp_wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float smp_wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// One wavefront draws row ``row`` of the logits l[0..A) (any memory space).
template <typename LP>
__device__ __forceinline__ void draw_row(LP l, int A, uint64_t seed, uint64_t ctr, int row, int* actions,
                                         float* logp, float* jac) {
  const int lane = threadIdx.x & 63;
  float mx = -INFINITY;
  for (int k = lane; k < A; k += 64) mx = fmaxf(mx, l[k]);
  mx = smp_wave_max(mx);
  float z = 0.f;
  for (int k = lane; k < A; k += 64) z += expf(l[k] - mx);
  z = smp_wave_sum(z);
  int a = 0;
  if (lane == 0) {   // inverse CDF, sequential (A is the action count: 18 for Seaquest)
    const float target = sample_uniform(seed, ctr, (uint64_t)row) * z;
    float cum = 0.f;
    a = -1;
    int last = 0;
    for (int k = 0; k < A; ++k) {
      const float e = expf(l[k] - mx);
      if (e > 0.f) last = k;
      cum += e;
      if (a < 0 && cum > target) a = k;
    }
    if (a < 0) a = last;   // u*Z rounded past the total: the last action with mass
  }
  a = __shfl(a, 0, 64);
  const float pa = expf(l[a] - mx) / z;
  const float eps = FLT_EPSILON;
  const bool clamped = !(pa >= eps && pa <= 1.f - eps);
  if (lane == 0) {
    actions[row] = a;
    if (logp) logp[row] = logf(fminf(fmaxf(pa, eps), 1.f - eps));
  }
  if (jac)
    for (int k = lane; k < A; k += 64)
      jac[(size_t)row * A + k] = clamped ? 0.f : (k == a ? 1.f : 0.f) - expf(l[k] - mx) / z;
}

}  // namespace aaa
