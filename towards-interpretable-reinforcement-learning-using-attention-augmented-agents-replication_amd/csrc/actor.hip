// Actor step chain (aaa_actor_step): one environment step of the agent for a
// few rows -- the acting half of the reference's loop (Policy.forward,
// main_mp.py:49-59; test_model.py:42-73 rollouts): vision CNN -> ConvLSTM
// step with carried state -> constant-query attention readout -> answer MLP
// -> LSTMCell (zero state, Q1) -> policy/value heads -> action draw.
//
// The learner's kernels are whole-batch GEMMs; at B = 1 they run as ~25
// latency-bound launches (188-226 us graph-replayed, profiles/r01).  Here each
// stage is split across the chip by its OUTPUT (conv2 pixels, ConvLSTM
// channel x pixel tiles, answer rows, LSTMCell units), so every stage is a
// few microseconds, and the chain is six launches.  Six launches and not one
// persistent kernel: a seam inside one launch costs a grid barrier (~4-5 us,
// MI355X_MICROARCH.md 'barrier-xcd'), a kernel boundary ~1.2-1.5 us
// ('boundary'); the answer MLP / LSTMCell / heads seams are all-to-all.
//
// Numerics: fp32 throughout (the ConvLSTM and conv1 on exact-fp32
// v_mfma_f32_16x16x4_f32, the rest fp32 FMA); only the summation order
// differs from the learner path (tests/test_gpu_actor.py compares both at
// 1e-4).  The action draw is draw_row (sampling.h), bit-identical to
// aaa_sample_actions on the same logits, seed and counter.
#include "actor.h"
#include "epilogues.h"
#include "sampling.h"

namespace aaa {

namespace {

__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
__device__ __forceinline__ float dot4(const f32x4& a, const f32x4& b) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2] + a[3] * b[3];
}
__device__ __forceinline__ float wsum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wmax(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ f32x4 mfma4(float a, float b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// ------------------------------------------------------------ vision ------
// One workgroup per (conv2 output pixel, frame): VisionNetwork.vision_cnn
// (attention.py:155-170 on X.transpose(1,3), Q3: the packed weights carry
// the transposed kernel orientation).  conv2 (4x4, stride 2, pad 2) of pixel
// (oy, ox) reads the 4x4 window of conv1 outputs at rows 2oy-2.., which read
// frame rows 8oy-9 .. 8oy+10: that 20x20 RGB patch is staged in LDS once
// (conv1's zero padding included), conv1 runs on the window as a 32x16x256
// MFMA GEMM (rows = channels, columns = window pixels, K = 64 taps x RGBx;
// 4 waves split K), conv1 outputs outside the H1 x W1 map are conv2's zero
// padding, and conv2 is 64 dot products of length 512 (4 waves x 16
// channels, lanes along K).
constexpr int kPatchLd = 81;   // floats per patch row: 4*81 = 4 (mod 64) spreads the 4 window rows over banks

template <typename TI>
__global__ void __launch_bounds__(256) k_act_vision(ActorParams p) {
  __shared__ float patch[20 * kPatchLd];
  __shared__ __attribute__((aligned(16))) float red[4][2][64][4];
  __shared__ __attribute__((aligned(16))) float y1w[16 * 32];
  __shared__ float red2[4][16][65];
  const int pix = blockIdx.x, f = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int oy = pix / p.w, ox = pix - oy * p.w;
  // conv2 weights of this wave's 16 channels, lane's 8 K values: issued first
  f32x4 w2a[16], w2b[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const float* wr = p.Wp2 + (size_t)(wv * 16 + j) * 512 + 8 * lane;
    w2a[j] = ld4(wr);
    w2b[j] = ld4(wr + 4);
  }
  // conv1 weights: A[i = lane&15][k = lane>>4] of the wave's 16 taps, both row tiles
  const int r = lane & 15, q = lane >> 4;
  float w1a[16], w1b[16];
#pragma unroll
  for (int t = 0; t < 16; ++t) {
    const int tap = wv * 16 + t;
    w1a[t] = p.Wp1[r * 256 + tap * 4 + q];
    w1b[t] = p.Wp1[(16 + r) * 256 + tap * 4 + q];
  }
  {
    const int r0 = 8 * oy - 9, c0 = 8 * ox - 9;
    const TI* fr = (const TI*)p.frames + (size_t)f * p.H * p.W * 3;
    for (int i = tid; i < 400; i += 256) {
      const int pr = i / 20, pc = i - pr * 20, iy = r0 + pr, ix = c0 + pc;
      float v0 = 0.f, v1 = 0.f, v2 = 0.f;
      if (iy >= 0 && iy < p.H && ix >= 0 && ix < p.W) {
        const TI* s = fr + ((size_t)iy * p.W + ix) * 3;
        v0 = (float)s[0]; v1 = (float)s[1]; v2 = (float)s[2];
      }
      float* d = patch + pr * kPatchLd + pc * 4;
      d[0] = v0; d[1] = v1; d[2] = v2; d[3] = 0.f;
    }
  }
  __syncthreads();
  {
    const int a = r >> 2, b = r & 3;   // B operand: window pixel r = lane&15, channel q of the tap
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const int tap = wv * 16 + t, ky = tap >> 3, kx = tap & 7;
      const float bv = patch[(4 * a + ky) * kPatchLd + (4 * b + kx) * 4 + q];
      acc0 = mfma4(w1a[t], bv, acc0);
      acc1 = mfma4(w1b[t], bv, acc1);
    }
    *reinterpret_cast<f32x4*>(red[wv][0][lane]) = acc0;
    *reinterpret_cast<f32x4*>(red[wv][1][lane]) = acc1;
  }
  __syncthreads();
  if (tid < 128) {   // D[row 4(l>>4)+v][col l&15] of row tile ``tile``: sum the 4 K quarters, bias, padding
    const int tile = tid >> 6, l = tid & 63, wp = l & 15, o0 = tile * 16 + 4 * (l >> 4);
    f32x4 s = *reinterpret_cast<const f32x4*>(red[0][tile][l]);
#pragma unroll
    for (int k = 1; k < 4; ++k) s += *reinterpret_cast<const f32x4*>(red[k][tile][l]);
    const int iy = 2 * oy - 2 + (wp >> 2), ix = 2 * ox - 2 + (wp & 3);
    const bool ok = iy >= 0 && iy < p.H1 && ix >= 0 && ix < p.W1;
#pragma unroll
    for (int v = 0; v < 4; ++v) y1w[wp * 32 + o0 + v] = ok ? s[v] + p.b1[o0 + v] : 0.f;
  }
  __syncthreads();
  {   // conv2: y1w index (a*4 + b)*32 + ci is the packed K order (tap*32 + ci)
    const f32x4 ya = *reinterpret_cast<const f32x4*>(y1w + 8 * lane);
    const f32x4 yb = *reinterpret_cast<const f32x4*>(y1w + 8 * lane + 4);
#pragma unroll
    for (int j = 0; j < 16; ++j) red2[wv][j][lane] = dot4(w2a[j], ya) + dot4(w2b[j], yb);
  }
  __syncthreads();
  {
    const int j = lane >> 2, part = lane & 3;
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) s += red2[wv][j][part * 16 + i];
    s += __shfl_xor(s, 1, 64);
    s += __shfl_xor(s, 2, 64);
    const int o = wv * 16 + j;
    if (part == 0) p.X[((size_t)f * p.P + pix) * 64 + o] = s + p.b2[o];
  }
}

// ---------------------------------------------------------- ConvLSTM ------
// ConvLSTMCell step (attention.py:110-126, zero peepholes) as an implicit
// GEMM D[512 gate rows][P pixels] = W[.][1728] * [x | h_{t-1}] (3x3 taps),
// cut into 16-row x 16-pixel tiles (4 channels x 4 gates, gate-interleaved
// rows) so that B = 1 still spreads over 32 x ceil(P/16) workgroups (256 at
// 84x84).  Eight waves split K (108 blocks of 16; each lane prefetches its
// weight and input float4 of every block before the first MFMA), the
// partials meet in LDS, and wave 0 holds, per lane, the four gates of one
// (channel, pixel): the cell update runs there (c in place; h to Hs, which
// the attention kernel copies into the state after reading it).
// blockIdx -> tile is XCD-aware: the ceil(P/16) pixel tiles of a channel group
// share an XCD (blockIdx % 8), so its 110 KB weight slab is read into one L2.
constexpr int kLstmWaves = 8;
constexpr int kLstmBlocks = 1728 / 16;                                         // 108
constexpr int kLstmPer = (kLstmBlocks + kLstmWaves - 1) / kLstmWaves;          // 14

__global__ void __launch_bounds__(512) k_act_convlstm(ActorParams p, int npg) {
  __shared__ __attribute__((aligned(16))) float red[kLstmWaves][64][4];
  const int f = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int bid = blockIdx.x, xcd = bid & 7, slot = bid >> 3;
  const int chg = xcd * 4 + slot / npg, pxg = slot - (slot / npg) * npg;
  const int r = lane & 15, q = lane >> 4;
  const int pix = pxg * 16 + r;
  const bool pin = pix < p.P;
  const int pc = pin ? pix : 0, y = pc / p.w, x = pc - y * p.w;
  const float* wrow = p.WpXH + (size_t)(chg * 16 + r) * 1728 + 4 * q;
  const float* Xf = p.X + (size_t)f * p.P * 64;
  const float* Hf = p.hst + (size_t)f * p.P * 128;
  f32x4 wk[kLstmPer], xk[kLstmPer];
  bool ok[kLstmPer];
#pragma unroll
  for (int i = 0; i < kLstmPer; ++i) {
    const int kb = wv + kLstmWaves * i;
    const int kbc = kb < kLstmBlocks ? kb : kLstmBlocks - 1;
    const int tap = kbc / 12, c0 = (kbc - tap * 12) * 16 + 4 * q;
    const int ky = tap / 3, kx = tap - ky * 3, ny = y + ky - 1, nx = x + kx - 1;
    ok[i] = pin && kb < kLstmBlocks && ny >= 0 && ny < p.h && nx >= 0 && nx < p.w;
    const int np = ok[i] ? ny * p.w + nx : 0;
    xk[i] = c0 < 64 ? ld4(Xf + (size_t)np * 64 + c0) : ld4(Hf + (size_t)np * 128 + (c0 - 64));
    wk[i] = ld4(wrow + kbc * 16);
  }
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < kLstmPer; ++i) {
    const f32x4 xv = ok[i] ? xk[i] : zero;   // padding taps, the ragged last pixel tile, K past 1728
    acc0 = mfma4(wk[i][0], xv[0], acc0);
    acc1 = mfma4(wk[i][1], xv[1], acc1);
    acc0 = mfma4(wk[i][2], xv[2], acc0);
    acc1 = mfma4(wk[i][3], xv[3], acc1);
  }
  *reinterpret_cast<f32x4*>(red[wv][lane]) = acc0 + acc1;
  __syncthreads();
  if (wv == 0 && pin) {
    f32x4 z = *reinterpret_cast<const f32x4*>(red[0][lane]);
#pragma unroll
    for (int k = 1; k < kLstmWaves; ++k) z += *reinterpret_cast<const f32x4*>(red[k][lane]);
    const int ch = chg * 4 + q;
    const f32x4 b = ld4(p.bl + 4 * ch);
    const size_t si = ((size_t)f * p.P + pix) * 128 + ch;
    float gi, gf, gc, go, c, h;
    GateFwd::run(z[0] + b[0], z[1] + b[1], z[2] + b[2], z[3] + b[3], p.cst[si], gi, gf, gc, go, c, h);
    (p.cout ? p.cout : p.cst)[si] = c;
    p.Hs[si] = h;
    if (p.gates) *reinterpret_cast<f32x4*>(p.gates + ((size_t)f * p.P + pix) * 512 + 4 * ch) = f32x4{gi, gf, gc, go};
  }
}

// ------------------------------------------- attention + answer layer 0 ---
// Every workgroup of a frame recomputes the frame's attention readout
// (attention.py:319-348 with the constant query, Q1: logits K.Q with
// K = [O[:8] | S], softmax over the P positions, readout of V = [O[8:] | S],
// answer row [a | Q | r | a_prev]) -- 93 KB of L2 reads and ~0.1 MFLOP, cheaper
// than a seam -- then computes 512 / gridDim.x rows of answer_processor.0 +
// ReLU (attention.py:277-282, 350) from it, one wave per row.  Workgroup 0
// also writes the attention map; each workgroup copies its slice of h_t into
// the carried state.
constexpr int kActAttnSlices = 5;   // 46 column groups x 5 position slices = 230 readout threads

template <int NQ>
__global__ void __launch_bounds__(256) k_act_attn(ActorParams p) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int P = p.P;
  float* L = sm;                                   // P*NQ
  float* Qs = L + P * NQ;                          // NQ*72
  float* red = Qs + NQ * 72;                       // SL*NQ*184
  float* ans = red + kActAttnSlices * NQ * 184;    // ans_ld
  const int f = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const float* O = p.Hs + (size_t)f * P * 128;
  const float* S = p.basis;
  // this wave's row of answer_processor.0 (gridDim.x * 4 = 512 rows), requested first: its
  // loads run under the attention readout instead of after it
  constexpr int NIT = (NQ * 256 + 2 + 7) / 8 * 8 / 256 + 1;   // float4 slices per lane over ans_ld
  const int row = blockIdx.x * 4 + wv;
  f32x4 w1r[NIT];
#pragma unroll
  for (int i = 0; i < NIT; ++i) {
    const int k = min(4 * lane + 256 * i, p.ans_ld - 4);
    w1r[i] = ld4(p.W1p + (size_t)row * p.ans_ld + k);
  }
  const float a0 = p.a0b[row];
  for (int i = tid; i < NQ * 72; i += 256) Qs[i] = p.Q[i];
  {   // this workgroup's slice of h_t -> the carried state (read by the next step's ConvLSTM kernel)
    const int n4 = P * 32, per = (n4 + gridDim.x - 1) / gridDim.x;
    const f32x4* src = reinterpret_cast<const f32x4*>(O);
    f32x4* dst = reinterpret_cast<f32x4*>((p.hout ? p.hout : p.hst) + (size_t)f * P * 128);
    for (int i = blockIdx.x * per + tid; i < min(n4, (int)(blockIdx.x + 1) * per); i += 256) dst[i] = src[i];
  }
  __syncthreads();
  for (int pp = tid; pp < P; pp += 256) {
    const f32x4 k0 = ld4(O + pp * 128), k1 = ld4(O + pp * 128 + 4);
    float acc[NQ];
#pragma unroll
    for (int qq = 0; qq < NQ; ++qq) {
      const float* Qq = Qs + qq * 72;
      acc[qq] = k0[0] * Qq[0] + k0[1] * Qq[1] + k0[2] * Qq[2] + k0[3] * Qq[3] + k1[0] * Qq[4] + k1[1] * Qq[5] +
                k1[2] * Qq[6] + k1[3] * Qq[7];
    }
#pragma unroll 4
    for (int c = 0; c < 16; ++c) {
      const f32x4 v = ld4(S + pp * 64 + 4 * c);
#pragma unroll
      for (int qq = 0; qq < NQ; ++qq) {
        const float* Qq = Qs + qq * 72 + 8 + 4 * c;
        acc[qq] += v[0] * Qq[0] + v[1] * Qq[1] + v[2] * Qq[2] + v[3] * Qq[3];
      }
    }
#pragma unroll
    for (int qq = 0; qq < NQ; ++qq) L[pp * NQ + qq] = acc[qq];
  }
  __syncthreads();
  for (int qq = wv; qq < NQ; qq += 4) {   // spatial_softmax over the P positions (attention.py:235-241)
    float m = -INFINITY;
    for (int pp = lane; pp < P; pp += 64) m = fmaxf(m, L[pp * NQ + qq]);
    m = wmax(m);
    float s = 0.f;
    for (int pp = lane; pp < P; pp += 64) {
      const float e = expf(L[pp * NQ + qq] - m);
      L[pp * NQ + qq] = e;
      s += e;
    }
    const float inv = 1.f / wsum(s);
    for (int pp = lane; pp < P; pp += 64) {
      const float a = L[pp * NQ + qq] * inv;
      L[pp * NQ + qq] = a;
      if (blockIdx.x == 0 && p.attn) p.attn[((size_t)f * P + pp) * NQ + qq] = a;
    }
  }
  __syncthreads();
  if (tid < 46 * kActAttnSlices) {   // readout (apply_alpha, attention.py:244-254)
    const int g = tid % 46, sl = tid / 46;
    const float* src = g < 30 ? O + 8 + 4 * g : S + 4 * (g - 30);
    const int ld = g < 30 ? 128 : 64;
    float acc[NQ][4];
#pragma unroll
    for (int qq = 0; qq < NQ; ++qq) acc[qq][0] = acc[qq][1] = acc[qq][2] = acc[qq][3] = 0.f;
#pragma unroll 4
    for (int pp = sl; pp < P; pp += kActAttnSlices) {
      const f32x4 v = ld4(src + (size_t)pp * ld);
#pragma unroll
      for (int qq = 0; qq < NQ; ++qq) {
        const float a = L[pp * NQ + qq];
        acc[qq][0] += a * v[0]; acc[qq][1] += a * v[1]; acc[qq][2] += a * v[2]; acc[qq][3] += a * v[3];
      }
    }
#pragma unroll
    for (int qq = 0; qq < NQ; ++qq)
      *reinterpret_cast<f32x4*>(red + (sl * NQ + qq) * 184 + 4 * g) =
          f32x4{acc[qq][0], acc[qq][1], acc[qq][2], acc[qq][3]};
  }
  __syncthreads();
  for (int i = tid; i < p.ans_ld; i += 256) {   // [a_0..a_nq-1 | Q | r | a_prev | 0-pad]
    float v = 0.f;
    if (i < NQ * 184) {
#pragma unroll
      for (int s2 = 0; s2 < kActAttnSlices; ++s2) v += red[s2 * NQ * 184 + i];
    } else if (i < NQ * 256) {
      v = Qs[i - NQ * 184];
    } else if (i == NQ * 256) {
      v = p.prev_reward ? p.prev_reward[f] : 0.f;
    } else if (i == NQ * 256 + 1) {
      v = p.prev_action ? p.prev_action[f] : 0.f;
    }
    ans[i] = v;
  }
  __syncthreads();
  {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
      const int k = 4 * lane + 256 * i;
      if (k < p.ans_ld) s += dot4(w1r[i], *reinterpret_cast<const f32x4*>(ans + k));
    }
    s = wsum(s) + a0;
    if (lane == 0) p.hid1[(size_t)f * 512 + row] = fmaxf(s, 0.f);
  }
}

// ------------------------------------------- answer layer 2 (linear) -----
// answer_processor.2 (attention.py:277-282): AO = W2 hid1 + b2, one wave per
// output row (weights read once into registers), all B frames.
__global__ void __launch_bounds__(256) k_act_ans2(ActorParams p) {
  const int lane = threadIdx.x & 63, row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const float* wr = p.A2W + (size_t)row * 512 + 8 * lane;
  const f32x4 w0 = ld4(wr), w1 = ld4(wr + 4);
  for (int f = 0; f < p.B; ++f) {
    const float* x = p.hid1 + (size_t)f * 512 + 8 * lane;
    const float s = wsum(dot4(w0, ld4(x)) + dot4(w1, ld4(x + 4)));
    if (lane == 0) p.AO[(size_t)f * 256 + row] = s + p.a2b[row];
  }
}

// ------------------------------------------------- LSTMCell (zero state) --
// policy_core from zero state (attention.py:354-355, Q1): one wave per unit u,
// its four gate rows 4u..4u+3 of the interleaved [1024][256] weights;
// c = i*g~ (+ f*0), h = o*tanh(c) -- the learner's EpiLstmCellFwd.
__global__ void __launch_bounds__(256) k_act_lstmcell(ActorParams p) {
  const int lane = threadIdx.x & 63, u = blockIdx.x * 4 + (threadIdx.x >> 6);
  f32x4 w[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) w[g] = ld4(p.Wihp + (size_t)(4 * u + g) * 256 + 4 * lane);
  const f32x4 b = ld4(p.blc + 4 * u);
  for (int f = 0; f < p.B; ++f) {
    const f32x4 x = ld4(p.AO + (size_t)f * 256 + 4 * lane);
    float z[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) z[g] = wsum(dot4(w[g], x));
    if (lane == 0) {
      const float gi = sigm_acc(z[0] + b[0]), gf = sigm_acc(z[1] + b[1]);
      const float gc = tanhf(z[2] + b[2]), go = sigm_acc(z[3] + b[3]);
      const float c = gf * 0.f + gi * gc;
      p.LH[(size_t)f * 256 + u] = go * tanhf(c);
    }
  }
}

// --------------------------------------------------- heads + action draw --
// policy_head / values_head (attention.py:365-367) and Policy.forward's draw
// (main_mp.py:54-58) in one workgroup: rows o < A -> logits, A <= o < 2A ->
// values, then one wave per frame runs draw_row on the logits it just wrote
// (the device counter is read by every wave before the single increment).
__global__ void __launch_bounds__(256) k_act_heads(ActorParams p) {
  __shared__ float lg[16 * 256];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, A = p.A, R = 2 * A;
  // rows in chunks of 8 per wave, each chunk's weight and state loads issued before its math
  for (int o0 = wv * 8; o0 < R; o0 += 32) {
    f32x4 w[8];
    float b[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int o = min(o0 + j, R - 1);
      w[j] = ld4(p.Whd + (size_t)o * 256 + 4 * lane);
      b[j] = p.bhd[o];
    }
    for (int f = 0; f < p.B; ++f) {
      const f32x4 x = ld4(p.LH + (size_t)f * 256 + 4 * lane);
      float s[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] = dot4(w[j], x);
#pragma unroll
      for (int o = 32; o > 0; o >>= 1)
#pragma unroll
        for (int j = 0; j < 8; ++j) s[j] += __shfl_xor(s[j], o, 64);
      if (lane < 8 && o0 + lane < R) {   // lane j stores row o0 + j
        float v = s[0] + b[0];
#pragma unroll
        for (int j = 1; j < 8; ++j) v = lane == j ? s[j] + b[j] : v;
        const int o = o0 + lane;
        if (o < A) {
          p.logits[(size_t)f * A + o] = v;
          lg[f * A + o] = v;
        } else {
          p.values[(size_t)f * A + o - A] = v;
        }
      }
    }
  }
  if (!p.actions) return;
  __syncthreads();
  const uint64_t ctr = p.counter ? (uint64_t)*p.counter : 0ull;
  for (int f = wv; f < p.B; f += 4) draw_row(lg + f * A, A, p.seed, ctr, f, p.actions, p.logp, p.jac);
  __syncthreads();   // every wave has read the counter
  if (p.counter && tid == 0) *p.counter = ctr + 1ull;
}

}  // namespace

size_t actor_attn_lds(int P, int nq, int ans_ld) {
  return sizeof(float) * ((size_t)P * nq + (size_t)nq * 72 + (size_t)kActAttnSlices * nq * 184 + ans_ld);
}

hipError_t actor_launch(const ActorParams& p, hipStream_t st) {
  if (p.B < 1 || p.B > 16 || (p.nq != 4 && p.nq != 8) || p.A < 1 || p.A > 256) return hipErrorInvalidValue;
  const size_t lds = actor_attn_lds(p.P, p.nq, p.ans_ld);
  if (lds > kActLdsMax) return hipErrorInvalidValue;
  if (lds > 64 * 1024) {   // beyond the default dynamic-LDS limit: raise it for this launch's kernel
    const void* k = p.nq == 4 ? reinterpret_cast<const void*>(&k_act_attn<4>) : reinterpret_cast<const void*>(&k_act_attn<8>);
    const hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  if (p.u8)
    hipLaunchKernelGGL(k_act_vision<uint8_t>, dim3(p.P, p.B), dim3(256), 0, st, p);
  else
    hipLaunchKernelGGL(k_act_vision<float>, dim3(p.P, p.B), dim3(256), 0, st, p);
  const int npg = (p.P + 15) / 16;
  hipLaunchKernelGGL(k_act_convlstm, dim3(32 * npg, p.B), dim3(512), 0, st, p, npg);
  if (p.nq == 4)
    hipLaunchKernelGGL(k_act_attn<4>, dim3(128, p.B), dim3(256), lds, st, p);
  else
    hipLaunchKernelGGL(k_act_attn<8>, dim3(128, p.B), dim3(256), lds, st, p);
  hipLaunchKernelGGL(k_act_ans2, dim3(64), dim3(256), 0, st, p);
  hipLaunchKernelGGL(k_act_lstmcell, dim3(64), dim3(256), 0, st, p);
  hipLaunchKernelGGL(k_act_heads, dim3(1), dim3(256), 0, st, p);
  return hipGetLastError();
}

}  // namespace aaa
