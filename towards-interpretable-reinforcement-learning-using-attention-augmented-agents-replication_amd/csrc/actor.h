// Actor step chain (aaa_actor_step): one environment step of the agent for a
// few rows (the acting half of main_mp.py:49-59 / test_model.py:42-73), fp32,
// as six launches sized for B <= 16 instead of the learner's whole-batch
// kernels.  Pointers are resolved by the runtime from the aaa_cfg layout.
#pragma once
#include "common.h"

namespace aaa {

struct ActorParams {
  // geometry
  int B, H, W, H1, W1, h, w, P, nq, A, ldy, ans_in, ans_ld, u8;
  // inputs
  const void* frames;        // (B, H, W, 3) uint8 or fp32
  const float* basis;        // (P, 64)
  const float* prev_reward;  // (B) or NULL
  const float* prev_action;  // (B) or NULL
  // packed / flat weights
  const float *Wp1, *b1;     // conv1 [32][256] RGBx, bias (32)
  const float *Wp2, *b2;     // conv2 [64][512], bias (64)
  const float *WpXH, *bl;    // ConvLSTM [512][1728] rows 4ch+g, bias [512]
  const float* Q;            // constant query (nq*72)
  const float *W1p, *a0b;    // answer_processor.0 [512][ans_ld], bias
  const float *A2W, *a2b;    // answer_processor.2 [256][512], bias
  const float *Wihp, *blc;   // LSTMCell [1024][256] rows 4u+g, b_ih + b_hh
  const float *Whd, *bhd;    // heads [ldy][256], bias
  // state (in place) and outputs
  float *hst, *cst;          // (B, P, 128) state in (and out, in place, unless hout / cout)
  float *hout, *cout;        // (B, P, 128) the step's h_t / c_t, or NULL (written into hst / cst)
  float *logits, *values;    // (B, A)
  float* attn;               // (B, P, nq) or NULL
  float* gates;              // (B, P, 512) gate activations, row 4ch+g, or NULL
  // workspace
  float *X, *Hs, *hid1, *AO, *LH;
  // action draw (actions == NULL: none)
  unsigned long long seed;
  unsigned long long* counter;
  int* actions;
  float* logp;
  float* jac;
};

hipError_t actor_launch(const ActorParams& p, hipStream_t st);

// Dynamic LDS of the attention-readout launch (k_act_attn): the logits of all P
// positions x nq queries, the queries, the readout's partial sums, the answer
// row.  Above 64 KB the launch raises the kernel's limit; above kActLdsMax the
// chain does not apply (actor_layout refuses it: such grids use aaa_forward).
constexpr size_t kActLdsMax = 160 * 1024;
size_t actor_attn_lds(int P, int nq, int ans_ld);

}  // namespace aaa
