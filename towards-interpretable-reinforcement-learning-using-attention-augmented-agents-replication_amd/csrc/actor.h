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
  float* Zp;                 // ConvLSTM split-K partial tiles (B, 8 * npt, kActLstmKS, 4096)
  int* zcnt;                 // (B, 8 * npt) arrival counters of those tiles, (B) of the readout
                             // chunks, 1 of the LSTMCell; all zeroed by the vision launch
  float* Lg;                 // (B, P, nq) attention logits (for the map)
  float* Apart;              // (B, nch, nq, kAttnPart) readout partials of position chunks
  float* arow;               // (B, ans_ld) answer_processor input row
  // action draw (actions == NULL: none)
  unsigned long long seed;
  unsigned long long* counter;
  int* actions;
  float* logp;
  float* jac;
};

hipError_t actor_launch(const ActorParams& p, hipStream_t st);

// Attention readout geometry: kAttnChunk positions per workgroup, each
// chunk's (query) partial = 184 readout sums + its max + its sum (+2 pad); at
// most kActMaxChunks chunks per frame (the combining workgroup's LDS), so the
// chain applies to P <= kAttnChunk * kActMaxChunks (larger grids: aaa_forward).
constexpr int kAttnChunk = 16;
constexpr int kAttnPart = 188;
constexpr int kActMaxChunks = 128;
__host__ __device__ inline int actor_chunks(int P) { return (P + kAttnChunk - 1) / kAttnChunk; }

// ConvLSTM launch geometry: 64 gate rows x 64 pixels per tile, 8 row tiles
// (one per XCD), ceil(P / 64) pixel tiles, K (1728) cut into kActLstmKS slices.
constexpr int kActLstmKS = 6;
__host__ __device__ inline int actor_pix_tiles(int P) { return (P + 63) / 64; }
size_t actor_attn_lds(int P, int nq, int ans_ld);

}  // namespace aaa
