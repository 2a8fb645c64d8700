// Frame-resident ConvLSTM recurrence (bf16 operands, fp32 accumulate).
//
// The recurrence of one frame depends only on that frame (attention.py:110-126:
// the gate convs are 3x3 over the frame's own grid, no batch coupling), so one
// workgroup owns a frame for ALL T steps of the unroll: the zero-bordered
// images of x_t and h_{t-1} live in LDS, the cell state c in registers, and a
// step is one 512 x P x 1728 GEMM whose B operand (the im2col of [x_t | h_{t-1}])
// is read straight out of the LDS images by all nine taps -- no per-step launch,
// no prologue, no re-gathering of the pixel operand from L2, and the epilogue's
// HBM stores of step t drain under the MFMAs of step t+1.
//
// Geometry: 8 waves; wave w owns gate rows [64w, 64w+64) (row = 4*channel +
// gate, i.e. channels 16w..16w+15) for all P <= 128 pixel columns (4 column
// blocks of 32), acc 2x4 v_mfma_f32_32x32x16_bf16 tiles.  Lane (r32, hh) of
// block (rr, cb) holds rows 8g + 4hh + e: the four gates of channel
// 16w + 8rr + 2g + hh at pixel 32cb + r32 -- the whole cell update is lane-local.
//
// A operand (weights): fragment-order copy of the packed [512][1728] matrix
// (k_pack_wfrag), one contiguous 1 KB wave load per (row block, k step),
// streamed from L2 continuously across steps (the prefetch wraps into the next
// step's first k steps).  K order k = tap*192 + c, c < 64 from the x image,
// c >= 64 from the h image, exactly as the implicit GEMM of fused_step.
#pragma once
#include <cstdlib>
#include "common.h"
#include "epilogues.h"
#include "glds.h"

namespace aaa {

constexpr int kRecKS = 1728 / 16;   // k steps of one [x|h] step GEMM
constexpr int kRecPD = 3;           // A k steps in flight (registers); 12 % kRecPD == 0
constexpr int kRecKSP = kRecKS + kRecPD - 1;   // packed k steps per row block: the first PD-1 repeated at
                                               // the end, so the prefetch runs into the next step unwrapped
constexpr int kRecNPH = 169;        // LDS image pixels: (h+2)*(w+2) <= 169 (11x11 grids: 84x84 frames)
constexpr int kRecXB = 22 * 1024;   // x image bytes per buffer: 169 pixels x 128 B, whole 1-KB DMA pieces
constexpr int kRecHS = 136;         // h image pixel pitch (bf16): 128 + 8 pad (272 B = 17 x 16 B)

// Wf[((rb*kRecKSP + ks)*64 + lane)*8 + e] = W[rb*32 + lane%32][(ks % kRecKS)*16 + (lane/32)*8 + e]
__global__ void __launch_bounds__(256) k_pack_wfrag(const __bf16* __restrict__ W, __bf16* __restrict__ Wf) {
  const int c = blockIdx.x * 256 + (int)threadIdx.x;   // one 16-B chunk
  if (c >= 16 * kRecKSP * 64) return;
  const int lane = c & 63, rk = c >> 6, ks = rk % kRecKSP, rb = rk / kRecKSP;
  const int row = rb * 32 + (lane & 31), k = (ks % kRecKS) * 16 + (lane >> 5) * 8;
  *reinterpret_cast<bf16x8*>(Wf + (size_t)c * 8) = *reinterpret_cast<const bf16x8*>(W + (size_t)row * 1728 + k);
}

// Branch-free gate math for the bf16 path (operands already rounded to 8
// mantissa bits): sigma(x) = 1 / (1 + 2^(-x log2 e)) on v_exp_f32 / v_rcp_f32,
// tanh(x) = 2 sigma(2x) - 1 (absolute error ~1e-7).
__device__ __forceinline__ float sigm_fast(float x) {
  return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-1.4426950408889634f * x));
}
__device__ __forceinline__ float tanh_fast(float x) { return 2.0f * sigm_fast(2.0f * x) - 1.0f; }

inline hipError_t pack_wfrag(const __bf16* W, __bf16* Wf, hipStream_t st) {
  hipLaunchKernelGGL(k_pack_wfrag, dim3((16 * kRecKSP * 64 + 255) / 256), dim3(256), 0, st, W, Wf);
  return hipGetLastError();
}

// Whether a grid runs on the frame-resident kernels.
inline bool rec_fits(int h, int w) { return h * w <= 128 && (h + 2) * (w + 2) <= kRecNPH; }

template <typename GT>
struct RecFwdParams {
  const __bf16* Wf;    // fragment-order [x|h] weights
  const float* bias;   // [512] gate-interleaved x-conv biases
  __bf16* XH;          // (T+1, B, P, 192): slot t = [x_t | h_{t-1}]; writes h_t into slot t+1
  float* Cst;          // (T+1, B, P, 128): slot 0 = c_0 (read), slot t+1 <- c_t
  float* Hs;           // (T, B, P, 128) <- h_t (fp32)
  GT* Gt;              // (T, B, P, 512) <- gate activations (i, f, c~, o)
  int T, B, h, w, P;
};

// ABL (diagnostic A/B only, AAA_REC_ABL): bit 0 = no A loads in the K loop,
// bit 1 = no epilogue HBM stores, bit 2 = no MFMAs, bit 3 = no B fragment reads.
template <typename GT, int ABL = 0>
__global__ void __launch_bounds__(512) k_convlstm_fwd_frames(RecFwdParams<GT> p) {
  __shared__ __attribute__((aligned(16))) unsigned char xim[2 * kRecXB];
  __shared__ __attribute__((aligned(16))) __bf16 him[2 * kRecNPH * kRecHS];
  __shared__ __attribute__((aligned(16))) float sbias[512];
  const int b = blockIdx.x, tid = (int)threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r32 = lane & 31, hh = lane >> 5;
  const int P = p.P, W2 = p.w + 2, NPH = (p.h + 2) * W2;
  const size_t M = (size_t)p.B * P;
  auto hidx = [&](int pp) { return (pp / p.w + 1) * W2 + pp % p.w + 1; };   // interior pixel -> image index

  {  // zero the h images (their borders stay zero), bias into LDS
    u32x4* z = reinterpret_cast<u32x4*>(him);
    for (int i = tid; i < 2 * kRecNPH * kRecHS / 8; i += 512) z[i] = u32x4{0u, 0u, 0u, 0u};
    sbias[tid] = p.bias[tid];
  }
  // x image of step t (XH slot t, channels 0..63) by LDS-DMA, border included:
  // image pixel ip holds its 8 16-B channel chunks at slots q ^ xswz(ip) (the
  // fragment reads of 16 consecutive pixels then hit 16 distinct bank groups);
  // border pixels read outside the descriptor and land as zeros.  Wave w issues
  // the 1-KB pieces w, w+8, ... of the 22 (8 pixels each).
  auto dma_x = [&](int t, int buf) {
    const __amdgpu_buffer_rsrc_t rs =
        make_rsrc(p.XH + ((size_t)t * M + (size_t)b * P) * 192, (uint32_t)(P * 192 * 2));
    for (int i = wave; i < kRecXB / 1024; i += 8) {
      const int sl = i * 64 + lane, ip = sl >> 3, q = (sl & 7) ^ ((ip >> 1) & 7);
      const int py = ip / W2 - 1, px = ip % W2 - 1;
      const bool v = ip < NPH && (unsigned)py < (unsigned)p.h && (unsigned)px < (unsigned)p.w;
      dma16(rs, xim + buf * kRecXB + i * 1024, v ? (uint32_t)(((py * p.w + px) * 192 + q * 8) * 2) : kOOB);
    }
  };
  dma_x(0, 0);
  __syncthreads();   // h images zeroed
  {  // h_0 (slot 0, channels 64..191) into image 0
    const __bf16* src = p.XH + (size_t)b * P * 192 + 64;
    for (int i = tid; i < P * 16; i += 512)
      *reinterpret_cast<u32x4*>(him + hidx(i >> 4) * kRecHS + (i & 15) * 8) =
          *reinterpret_cast<const u32x4*>(src + (size_t)(i >> 4) * 192 + (i & 15) * 8);
  }

  // per-lane B fragment bases: top-left image pixel of each column block's 3x3
  // window (columns >= P read pixel P-1: their outputs are never stored)
  int hb[4];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) {
    const int pp = min(cb * 32 + r32, P - 1);
    hb[cb] = (pp / p.w) * W2 + pp % p.w;
  }
  const __bf16* A0 = p.Wf + ((size_t)(2 * wave) * kRecKSP * 64 + lane) * 8;
  const __bf16* A1 = A0 + (size_t)kRecKSP * 64 * 8;
  constexpr int PD = kRecPD;
  bf16x8 af[PD][2];
#pragma unroll
  for (int s = 0; s < PD - 1; ++s) {
    af[s][0] = *reinterpret_cast<const bf16x8*>(A0 + s * 512);
    af[s][1] = *reinterpret_cast<const bf16x8*>(A1 + s * 512);
  }
  __syncthreads();   // images of step 0 complete

  for (int t = 0; t < p.T; ++t) {
    const int cur = t & 1, nxt = cur ^ 1;
    // x_{t+1} into the other image (last read in step t-1); the wave's later A
    // loads retire after it (vmcnt is in order), so it has landed by the end of the K loop
    if (t + 1 < p.T) dma_x(t + 1, nxt);
    f32x16 acc[2][4];
#pragma unroll
    for (int rr = 0; rr < 2; ++rr)
#pragma unroll
      for (int cb = 0; cb < 4; ++cb)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[rr][cb][e] = 0.f;
    const unsigned char* xb = xim + cur * kRecXB;
    int hbs[4];   // laundered per step: no per-tap address tables hoisted out of the step loop
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      hbs[cb] = hb[cb];
      asm volatile("" : "+v"(hbs[cb]));
    }
    const __bf16* hbp = him + cur * NPH * kRecHS + hh * 8;
    // B fragments of k step ks (image, tap offset, channel chunk c16 of 12: 4 from x, 8 from h)
    auto ldb = [&](int toff, int c16, bf16x8 (&bf)[4]) {
#pragma unroll
      for (int cb = 0; cb < 4; ++cb)
      {
        const int ip = hbs[cb] + toff;
        bf[cb] = c16 < 4 ? *reinterpret_cast<const bf16x8*>(xb + ip * 128 + (((2 * c16 + hh) ^ ((ip >> 1) & 7)) << 4))
                         : *reinterpret_cast<const bf16x8*>(hbp + ip * kRecHS + (c16 - 4) * 16);
      }
    };
    bf16x8 bfr[2][4];
    ldb(0, 0, bfr[0]);
    for (int tap = 0; tap < 9; ++tap) {
      const int toff = (tap / 3) * W2 + tap % 3;
      const int tnext = tap < 8 ? ((tap + 1) / 3) * W2 + (tap + 1) % 3 : 0;
      int ko = tap * 12 * 512;   // laundered: one base per tap, immediate offsets inside (no hoisted address table)
      asm volatile("" : "+s"(ko));
      const __bf16* a0 = A0 + ko;
      const __bf16* a1 = A1 + ko;
#pragma unroll
      for (int c16 = 0; c16 < 12; ++c16) {
        // A fragments of k step ks + PD - 1 (the packed copy runs on into the next step's first ones)
        if constexpr (!(ABL & 1)) {
          af[(c16 + PD - 1) % PD][0] = *reinterpret_cast<const bf16x8*>(a0 + (c16 + PD - 1) * 512);
          af[(c16 + PD - 1) % PD][1] = *reinterpret_cast<const bf16x8*>(a1 + (c16 + PD - 1) * 512);
        }
        // B fragments one k step ahead (the last k step's are this step's last use)
        if constexpr (!(ABL & 8)) {
          if (c16 < 11) ldb(toff, c16 + 1, bfr[(c16 + 1) & 1]);
          else if (tap < 8) ldb(tnext, 0, bfr[0]);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) {
          if constexpr (ABL & 4) {
            acc[0][cb][0] += (float)af[c16 % PD][0][0] * (float)bfr[c16 & 1][cb][0];
          } else {
            acc[0][cb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[c16 % PD][0], bfr[c16 & 1][cb], acc[0][cb], 0, 0, 0);
            acc[1][cb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[c16 % PD][1], bfr[c16 & 1][cb], acc[1][cb], 0, 0, 0);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // gate math + cell update (lane-local), h_t into the other h image.  The
    // lane's pixel is laundered per step so the compiler recomputes the 32
    // epilogue addresses from one base instead of hoisting them all out of the
    // step loop into (spilled) registers.
    int pl = r32;
    asm volatile("" : "+v"(pl));
    const size_t rowt = (size_t)t * M + (size_t)b * P;   // this frame's rows of step t (Hs, Gt; Cst slot t)
    const int c0 = 16 * wave + hh;                       // + 8*rr + 2*g
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      const int pp = cb * 32 + pl;
      if (pp >= P) continue;
      const size_t row = rowt + pp;
      const float* cprev = p.Cst + row * 128 + c0;       // c_{t-1}: the lane's own stores of step t-1 (slot 0: c_0)
      float* cnext = p.Cst + (row + M) * 128 + c0;
      float* hout = p.Hs + row * 128 + c0;
      GT* gout = p.Gt + row * 512 + 4 * c0;
      __bf16* hl = him + (nxt * NPH + hidx(pp)) * kRecHS + c0;
      float cp[2][4];
#pragma unroll
      for (int rr = 0; rr < 2; ++rr)
#pragma unroll
        for (int g = 0; g < 4; ++g) cp[rr][g] = cprev[8 * rr + 2 * g];
#pragma unroll
      for (int rr = 0; rr < 2; ++rr)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int co = 8 * rr + 2 * g;
          const f32x4 bz = *reinterpret_cast<const f32x4*>(sbias + 4 * (c0 + co));
          const float gi = sigm_fast(acc[rr][cb][4 * g] + bz[0]);
          const float gf = sigm_fast(acc[rr][cb][4 * g + 1] + bz[1]);
          const float gc = tanh_fast(acc[rr][cb][4 * g + 2] + bz[2]);
          const float go = sigm_fast(acc[rr][cb][4 * g + 3] + bz[3]);
          const float c = gf * cp[rr][g] + gi * gc;
          const float h = go * tanh_fast(c);
          if constexpr (!(ABL & 2)) {
            cnext[co] = c;
            hout[co] = h;
            store_gates(gout + 4 * co, f32x4{gi, gf, gc, go});
          }
          hl[co] = (__bf16)h;
        }
      __builtin_amdgcn_sched_barrier(0);   // one column block at a time (register pressure)
    }
    barrier_lds();   // step t+1's images complete; every wave is done with step t's (VM stores stay in flight)
    // h_t (bf16) into XH slot t+1 channels 64..191 (the weight-gradient operand), from the image
    const size_t rown = rowt + M;                        // slot t+1
    for (int i = tid; i < ((ABL & 2) ? 0 : P * 16); i += 512)
      *reinterpret_cast<u32x4*>(p.XH + (rown + (i >> 4)) * 192 + 64 + (i & 15) * 8) =
          *reinterpret_cast<const u32x4*>(him + (nxt * NPH + hidx(i >> 4)) * kRecHS + (i & 15) * 8);
  }
}

template <typename GT>
inline hipError_t convlstm_fwd_frames(const RecFwdParams<GT>& p, hipStream_t st) {
  if (!rec_fits(p.h, p.w) || p.P != p.h * p.w || p.B < 1 || p.T < 1) return hipErrorInvalidValue;
  const char* e = getenv("AAA_REC_ABL");
  switch (e ? atoi(e) : 0) {
#define AAA_REC_CASE(a) \
  case a: hipLaunchKernelGGL((k_convlstm_fwd_frames<GT, a>), dim3(p.B), dim3(512), 0, st, p); break;
    AAA_REC_CASE(1) AAA_REC_CASE(2) AAA_REC_CASE(3) AAA_REC_CASE(4) AAA_REC_CASE(8) AAA_REC_CASE(12)
#undef AAA_REC_CASE
    default: hipLaunchKernelGGL((k_convlstm_fwd_frames<GT, 0>), dim3(p.B), dim3(512), 0, st, p); break;
  }
  return hipGetLastError();
}

}  // namespace aaa
