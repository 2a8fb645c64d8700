// REINFORCE loss on device: the reference's
// finish_episode (main_mp.py:62-77) for B independent episodes of T steps,
// fused into one kernel that also produces the loss cotangent the learner's
// backward consumes -- so an episode update needs no host round trip for the
// returns and no autograd graph over T per-step Categorical objects.
//
// Per episode b (one workgroup):
//   R_t  = r_t + gamma * R_{t+1}               (Python float = double in the reference, :66-68)
//   R^_t = (R_t - mean R) / (std R + eps)      (float32 tensor ops, unbiased std, eps = f32 eps, :69-70)
//   logp = log(clamp(p_{a_t}, eps, 1 - eps)),  p = softmax(logits_t) / sum   (Categorical(probs=..)
//          as built at main_mp.py:55-58: probs_to_logits clamps the probabilities)
//   loss_b = sum_t -logp_t * R^_t               (:71-73, :76)
//   dlogits[t][b][k] = -R^_t * (1[k == a_t] - p_k), zero where the clamp is active.
// The discounted return is a linear recurrence, so it runs as a parallel scan
// of affine maps x -> r + gamma x (in double) over the workgroup's threads.
#include <cfloat>
#include <cmath>

#include "common.h"
#include "sampling.h"

namespace aaa {

constexpr int kRfThreads = 256;

__device__ __forceinline__ double wg_sum_d(double v, double* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  double t = 0.0;
#pragma unroll
  for (int w = 0; w < kRfThreads / 64; ++w) t += red[w];
  return t;
}

// rn: (T, B) scratch for the normalised returns (always written).
__global__ void __launch_bounds__(kRfThreads)
k_reinforce(int T, int B, int A, const float* __restrict__ logits, const int* __restrict__ actions,
            const float* __restrict__ rewards, double gamma, float* __restrict__ loss, float* __restrict__ rn,
            float* __restrict__ dlogits) {
  __shared__ double sa[kRfThreads], sb[kRfThreads];   // affine map of each thread's chunk: R_in -> a*R_in + b
  __shared__ double red[kRfThreads / 64];
  const int b = blockIdx.x, tid = threadIdx.x;
  const int per = (T + kRfThreads - 1) / kRfThreads;
  const int t0 = min(T, tid * per), t1 = min(T, t0 + per);
  // 1. chunk-local backward scan: R_t = r_t + gamma R_{t+1} with R_{t1} = x  ->  R_{t0} = a x + b
  double ca = 1.0, cb = 0.0;
  for (int t = t1 - 1; t >= t0; --t) {
    cb = (double)rewards[(size_t)t * B + b] + gamma * cb;
    ca *= gamma;
  }
  sa[tid] = ca;
  sb[tid] = cb;
  __syncthreads();
  // 2. incoming return of every chunk: compose the maps of the chunks to its right
  //    (one thread; kRfThreads affine compositions)
  if (tid == 0) {
    double x = 0.0;
    for (int k = kRfThreads - 1; k >= 0; --k) {
      const double nx = sa[k] * x + sb[k];
      sa[k] = x;          // R entering chunk k from the right
      x = nx;
    }
  }
  __syncthreads();
  // 3. returns of this chunk (double -> float32 as torch.tensor(returns) does)
  double x = sa[tid], s1 = 0.0;
  for (int t = t1 - 1; t >= t0; --t) {
    x = (double)rewards[(size_t)t * B + b] + gamma * x;
    const float rf = (float)x;
    rn[(size_t)t * B + b] = rf;
    s1 += (double)rf;
  }
  const double mean = wg_sum_d(s1, red) / (double)T;
  double s2 = 0.0;
  for (int t = t0; t < t1; ++t) {
    const double d = (double)rn[(size_t)t * B + b] - mean;
    s2 += d * d;
  }
  const double var = wg_sum_d(s2, red) / (double)(T - 1);   // T == 1 -> nan, as torch.std
  const float sd = (float)sqrt(var);
  const float meanf = (float)mean;
  const float eps = FLT_EPSILON;
  // 4. per-step softmax, clamped log-prob and cotangent (each thread its chunk of steps)
  double lsum = 0.0;
  for (int t = t0; t < t1; ++t) {
    const float Rh = (rn[(size_t)t * B + b] - meanf) / (sd + eps);
    rn[(size_t)t * B + b] = Rh;
    const float* l = logits + ((size_t)t * B + b) * A;
    float* dl = dlogits + ((size_t)t * B + b) * A;
    float mx = -INFINITY;
    for (int k = 0; k < A; ++k) mx = fmaxf(mx, l[k]);
    float z = 0.f;
    for (int k = 0; k < A; ++k) z += expf(l[k] - mx);
    const int a = actions[(size_t)t * B + b];
    const float pa = expf(l[a] - mx) / z;
    const bool clamped = !(pa >= eps && pa <= 1.f - eps);   // clamp's backward passes at the bounds
    const float lp = logf(fminf(fmaxf(pa, eps), 1.f - eps));
    lsum += (double)(-lp * Rh);
    for (int k = 0; k < A; ++k) {
      const float pk = expf(l[k] - mx) / z;
      dl[k] = clamped ? 0.f : -Rh * ((k == a ? 1.f : 0.f) - pk);
    }
  }
  const double tot = wg_sum_d(lsum, red);
  if (tid == 0) loss[b] = (float)tot;
}

hipError_t reinforce_launch(int T, int B, int A, const float* logits, const int* actions, const float* rewards,
                            double gamma, float* loss, float* rn, float* dlogits, hipStream_t st) {
  hipLaunchKernelGGL(k_reinforce, dim3(B), dim3(kRfThreads), 0, st, T, B, A, logits, actions, rewards, gamma, loss,
                     rn, dlogits);
  return hipGetLastError();
}

}  // namespace aaa

namespace aaa {

// ------------------------------------------------------ actor sampling ---
// Policy.forward's action draw for B rows of logits, on device, one wavefront
// per row (the per-row draw is draw_row, sampling.h).  The draw index
// ``counter`` lives in device memory and is advanced by one per launch, so a
// captured graph replays fresh draws without a host round trip.
constexpr int kSmpThreads = 256;

__global__ void __launch_bounds__(kSmpThreads)
k_sample_actions(int B, int A, const float* __restrict__ logits, uint64_t seed, unsigned long long* counter,
                 int* __restrict__ actions, float* __restrict__ logp, float* __restrict__ jac) {
  const int wave = threadIdx.x >> 6;
  const uint64_t ctr = counter ? (uint64_t)*counter : 0ull;
  for (int b = wave; b < B; b += kSmpThreads / 64) draw_row(logits + (size_t)b * A, A, seed, ctr, b, actions, logp, jac);
  __syncthreads();   // every wave has read the counter
  if (counter && threadIdx.x == 0) *counter = ctr + 1ull;
}

hipError_t sample_launch(int B, int A, const float* logits, uint64_t seed, unsigned long long* counter, int* actions,
                         float* logp, float* jac, hipStream_t st) {
  hipLaunchKernelGGL(k_sample_actions, dim3(1), dim3(kSmpThreads), 0, st, B, A, logits, seed, counter, actions, logp,
                     jac);
  return hipGetLastError();
}

}  // namespace aaa
