#pragma once
#include "common.h"

namespace aaa {

constexpr int kAdamMaxTensors = 48;   // per launch (kernel-argument table)

struct AdamTable {
  float* p[kAdamMaxTensors];
  const float* g[kAdamMaxTensors];
  float* m[kAdamMaxTensors];
  float* v[kAdamMaxTensors];
  float* vmax[kAdamMaxTensors];
  size_t numel[kAdamMaxTensors];
  int chunk0[kAdamMaxTensors];        // first workgroup of each tensor
  unsigned char vec[kAdamMaxTensors]; // all four pointers 16-byte aligned
  int n;
};

struct AdamHost {
  double lr, beta1, beta2, eps, weight_decay;
  long step;
  int amsgrad, maximize;
  const float* guard = nullptr;   // device float: skip the update when != 0
  int* step_dev = nullptr;        // device step counter (aaa_adam_step_counted): step = *step_dev + 1,
                                  // advanced in stream order only when the update was applied
};

int adam_chunks(size_t numel);
// advance: count this update on h.step_dev after the launch (the last table of a step)
hipError_t adam_launch(const AdamTable& tab, int nchunks, const AdamHost& h, hipStream_t st, bool advance);
hipError_t pair_flag_launch(const int* report, int* base, float* dst, hipStream_t st);

// loss.hip: REINFORCE (finish_episode) loss + logits cotangent, one workgroup per episode
hipError_t reinforce_launch(int T, int B, int A, const float* logits, const int* actions, const float* rewards,
                            double gamma, float* loss, float* rn, float* dlogits, hipStream_t st);
hipError_t sample_launch(int B, int A, const float* logits, uint64_t seed, unsigned long long* counter, int* actions,
                         float* logp, float* jac, hipStream_t st);

}  // namespace aaa
