// Frame-group-resident ConvLSTM recurrence, fp32 (exact v_mfma_f32_32x32x2_f32).
//
// The reference's recurrence (attention.py:117-125) couples a frame's pixels
// only through the 3x3 gate convs over that frame's own h_{t-1}; frames never
// interact.  The fp32 learner's batch (config 2: B = 32 frames, 84x84 -> 11x11
// grid) is far below the CU count, so here G workgroups (G = 8 or 4) own
// one frame for all T steps, each a slice of 512/G gate-interleaved rows
// (128/G channels), and exchange only h_t: each publishes its channels
// of h_t (XH slot t+1, written anyway as the weight-gradient operand) with
// write-through stores and a flag, and reads the other G-1 slices back into
// its LDS h image under the next step's x-part.  This
// replaces the 19 per-step launches of the h-part GEMM AND the batched x-part
// GEMM (one K = 1728 [x | h] GEMM per step, as the bf16 frame-resident kernel
// in recur.h does), with no launch boundary, prologue or operand re-gather.
//
// Workgroup (b, kh): 4 waves; gate rows [512 kh / G, 512 (kh+1) / G) =
// NRB = 16 / G row blocks of 32; the frame's P <= 128 pixels are 4 column
// blocks of 32.  Wave w: row blocks (w & 1) * RPW .. + RPW (RPW = NRB / 2),
// column blocks 2 (w >> 1), 2 (w >> 1) + 1.  The G workgroups of a frame get
// block indices of equal residue mod 8 (one XCD under round-robin placement),
// so the hand-off runs through one L2.
//
// K order of a step: 216 "quads" of 4 MFMA k-steps (8 channels of one tap):
// x-part 9 taps x 8 quads, then h-part 9 taps x 16 quads.  Within a quad,
// lane half hh covers channels 4hh..4hh+3 and k-step j channel 4hh+j, so one
// ds_read_b128 of the B image and one 16-B load of the fragment-order weights
// (k_pack_wf32) feed four MFMAs.
//
// LDS images (zero border), 16-B chunk q of image pixel (y, x) at slot q ^ (key & 15),
// key = y * w + x (border pixels: y or x = -1 / h or w): consecutive columns --
// the lanes of a fragment read -- have consecutive keys under every tap, row ends
// included, so 8 consecutive lanes hit 8 distinct bank groups (keyed by the bordered
// index ip instead, the 2-pixel jump at each row end collided: PMC conflict rate
// 0.54 on the C2 forward):
//   x image: 169 pixels x 64 fp32 (256 B),  DMA-filled from XH slot t+1 under the epilogue
//   h image: 169 pixels x 128 fp32 (512 B), own channels from the epilogue, the
//            partners' from XH slot t.
#pragma once
#include "common.h"
#include "epilogues.h"
#include "glds.h"
#include "recur.h"

namespace aaa {

constexpr int kF32QX = 72;                 // x-part quads (9 taps x 8)
constexpr int kF32Q = 216;                 // quads per step
constexpr int kF32PD = 8;                  // A quads in flight (register slots); divides 8, 16 and kF32Q
constexpr int kF32QP = kF32Q + kF32PD - 1;  // packed quads per row block: the first PD-1 repeated at the end
constexpr int kF32PP = (kF32Q + kF32PD) / 2;  // packed quad PAIRS per row block (the pre-split kernel's stream)
constexpr int kF32XB = 44 * 1024;          // x image bytes: 169 x 256 B rounded up to whole 1-KB DMA pieces
constexpr int kF32HB = 169 * 512;          // h image bytes
constexpr int kF32GP = 144;                // epilogue staging: gate tile pixel pitch (128 B + 16)
constexpr int kF32SG = 32 * kF32GP;        // ... c / h tiles after it, pixel pitch 48 B (32 B + 16)
constexpr int kF32STG = kF32SG + 2 * 32 * 48;   // staging bytes per wave (7.5 KB)

// element offset k (= tap * 192 + channel) of quad q's channel 0 for lane half 0
__host__ __device__ constexpr int f32_k(int q) {
  return q < kF32QX ? (q >> 3) * 192 + (q & 7) * 8 : ((q - kF32QX) >> 4) * 192 + 64 + ((q - kF32QX) & 15) * 8;
}

// Wf[((rb * kF32QP + q) * 64 + lane) * 4 + j] = W[32 rb + lane % 32][f32_k(q % kF32Q) + 4 (lane / 32) + j]
static __global__ void __launch_bounds__(256) k_pack_wf32(const float* __restrict__ W, float* __restrict__ Wf) {
  const int c = blockIdx.x * 256 + (int)threadIdx.x;   // one 16-B chunk
  if (c >= 16 * kF32QP * 64) return;
  const int lane = c & 63, rq = c >> 6, q = rq % kF32QP, rb = rq / kF32QP;
  const int row = rb * 32 + (lane & 31), k = f32_k(q % kF32Q) + (lane >> 5) * 4;
  *reinterpret_cast<f32x4*>(Wf + (size_t)c * 4) = *reinterpret_cast<const f32x4*>(W + (size_t)row * 1728 + k);
}

// S6 (bf16x6) copy of a fragment-order fp32 weight stream: chunk c = g * 64 + lane
// (16 B = 4 fp32) -> three 8-B parts (hi, mid, lo: 4 bf16 each, gemm.h split3_bf16's
// split) at [(g * 3 + part) * 64 + lane], so a wave's load of one part is 512 contiguous
// bytes and the kernels assemble their bf16x8 operands from two quads without VALU work.
static __global__ void __launch_bounds__(256) k_split_frag(const f32x4* __restrict__ src, u32x2* __restrict__ dst,
                                                           int nchunks) {
  const int c = blockIdx.x * 256 + (int)threadIdx.x;
  if (c >= nchunks) return;
  const f32x4 x = src[c];
  u32x2 part[3];
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    uint32_t h2[2], m2[2], l2[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const float v = x[2 * e + k];
      const __bf16 hi = (__bf16)v;
      const float r = v - (float)hi;
      const __bf16 mid = (__bf16)r;
      const __bf16 lo = (__bf16)(r - (float)mid);
      h2[k] = __builtin_bit_cast(uint16_t, hi);
      m2[k] = __builtin_bit_cast(uint16_t, mid);
      l2[k] = __builtin_bit_cast(uint16_t, lo);
    }
    part[0][e] = h2[0] | (h2[1] << 16);
    part[1][e] = m2[0] | (m2[1] << 16);
    part[2][e] = l2[0] | (l2[1] << 16);
  }
  const int g = c >> 6, lane = c & 63;
#pragma unroll
  for (int p = 0; p < 3; ++p) dst[(g * 3 + p) * 64 + lane] = part[p];
}

inline hipError_t split_frag(const float* src, void* dst, int nchunks, hipStream_t st) {
  hipLaunchKernelGGL(k_split_frag, dim3((nchunks + 255) / 256), dim3(256), 0, st,
                     reinterpret_cast<const f32x4*>(src), reinterpret_cast<u32x2*>(dst), nchunks);
  return hipGetLastError();
}

inline hipError_t pack_wf32(const float* W, float* Wf, hipStream_t st) {
  hipLaunchKernelGGL(k_pack_wf32, dim3((16 * kF32QP * 64 + 255) / 256), dim3(256), 0, st, W, Wf);
  return hipGetLastError();
}

struct RecF32Params {
  const float* Wf;     // fragment-order [x|h] weights (k_pack_wf32)
  const float* bias;   // [512] gate-interleaved x-conv biases
  float* XH;           // (T+1, B, P, 192): slot t = [x_t | h_{t-1}]; h_t -> slot t+1
  float* Cst;          // (T+1, B, P, 128): slot 0 = c_0 (read), slot t+1 <- c_t
  float* Hs;           // (T, B, P, 128) <- h_t
  float* Gt;           // (T, B, P, 512) <- gate activations (i, f, c~, o)
  int* flags;          // [B][G] count of published h steps (zeroed by the caller)
  int* report;         // partner-timeout report word (pair_wait)
  int spin;            // partner-wait budget, 100-MHz ticks (pair_wait)
  int T, B, h, w, P;
  int h0_zero;         // slot 0's h part is zero (reset()): the t = 0 h-part is skipped
  short colhb[128];    // column -> top-left image pixel of its 3x3 window (padding columns: pixel P-1's)
  const u32x2* Wf6 = nullptr;   // S6: the three-way split of Wf (k_split_frag)
  const u32x4* Wf6p = nullptr;  // the pre-split kernel's stream: quads 2j, 2j+1 of a part side by side per lane
};

// Blocks of the launch: 8 * G * ceil(B / 8) (XCD-local frame groups).
inline int f32_grid(int B, int G) { return 8 * G * ((B + 7) / 8); }

#ifdef AAA_STAMPS
// Diagnostic builds only (tools/ubench/f32rec): per (workgroup, step) phase
// stamps (s_memrealtime, 100 MHz): step start, x-part done (partners' h in),
// h-part done, epilogue done, flag published.
__device__ uint64_t aaa_f32_stamps[512 * 64 * 5];
__device__ uint64_t aaa_f32_clocks[512 * 64 * 5];   // s_memtime (shader clock) at the same points
#define AAA_F32_STAMP(t, k)                                                                          \
  do {                                                                                               \
    if (tid == 0 && (t) < 64) {                                                                      \
      aaa_f32_stamps[(blk * 64 + (t)) * 5 + (k)] = __builtin_amdgcn_s_memrealtime();                  \
      aaa_f32_clocks[(blk * 64 + (t)) * 5 + (k)] = __builtin_amdgcn_s_memtime();                      \
    }                                                                                                \
  } while (0)
#else
#define AAA_F32_STAMP(t, k) do {} while (0)
#endif

// ABL (diagnostic builds only, tools/ubench/f32rec; production launches use 0):
// bit 0 = no epilogue (gate math, stores), bit 1 = no epilogue HBM stores,
// bit 2 = no partner exchange, bit 3 = no MFMAs, bit 4 (S6) = no three-way
// split of the B fragments (hi part only: the split's cost, wrong numerics).
// S6: the MFMAs on the bf16 MFMA at fp32 accuracy (gemm.h SPLIT6): two quads
// (16 channels) per v_mfma_f32_32x32x16_bf16 k-step -- lane half hh's 8 k-slots
// are channels 4hh..4hh+3 of the first quad, then of the second, in the same
// order for A and B -- each operand split three ways, six MFMAs (6 x 32
// cycles) where the fp32 MFMA takes eight (8 x 64).
//
// WIDE (S6, G = 8 only): wave w takes both row blocks and column block w, so each
// B fragment is split by one wave instead of two (the split is VALU work the MFMAs
// wait on: tools/ubench/f32rec "S6 no B split"), at twice the per-wave A stream
// (the four waves of a workgroup then read the same A quads).  PDW: A quads in flight.
template <int G, int ABL = 0, bool S6 = false, bool WIDE = false, int PDW = kF32PD>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
k_convlstm_fwd_f32(RecF32Params p) {
  static_assert(!WIDE || (S6 && G == 8), "WIDE: the S6 kernel at G = 8");
  constexpr int NRB = 16 / G;                      // row blocks per workgroup
  constexpr int RPW = WIDE ? NRB : NRB / 2;        // ... per wave
  constexpr int NCB = WIDE ? 1 : 2;                // column blocks per wave
  constexpr int CPG = 32 / G;                      // 16-B h chunks (4 channels) per workgroup slice
  constexpr int NPL = (128 * (G - 1) * CPG + 255) / 256;   // partner chunks per thread (P <= 128)
  static_assert(G == 4 || G == 8, "G");
  __shared__ __attribute__((aligned(16))) unsigned char xim[kF32XB];
  __shared__ __attribute__((aligned(16))) unsigned char him[kF32HB];
  __shared__ __attribute__((aligned(16))) unsigned char stgall[4 * kF32STG];   // per-wave epilogue staging

  const int blk = (int)blockIdx.x, xcd = blk & 7, loc = blk >> 3;
  const int b = xcd + 8 * (loc / G), kh = loc % G;
  if (b >= p.B) return;   // padding group of the last XCD column (never a partner of a live frame)
  const int tid = (int)threadIdx.x, lane = tid & 63;
  uint64_t wdl = 0;   // partner-wait deadline (common.h wait_expired), set by the first wait that polls
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r32 = lane & 31, hh = lane >> 5;
  const int P = p.P, W2 = p.w + 2, NPH = (p.h + 2) * W2;
  const size_t M = (size_t)p.B * P;
  const int rw = WIDE ? 0 : wave & 1;
  auto cbk = [&](int c) { return WIDE ? wave : 2 * (wave >> 1) + c; };   // the wave's column block c
  const int rbg0 = kh * NRB + rw * RPW;            // the wave's first global row block
  auto hidx = [&](int pp) { return (pp / p.w + 1) * W2 + pp % p.w + 1; };
  auto sw16 = [](int q, int key) { return (q ^ (key & 15)) << 4; };
  unsigned char* stg = stgall + wave * kF32STG;

  {  // zero both images (borders stay zero)
    u32x4* z = reinterpret_cast<u32x4*>(xim);
    for (int i = tid; i < kF32XB / 16; i += 256) z[i] = u32x4{0u, 0u, 0u, 0u};
    z = reinterpret_cast<u32x4*>(him);
    for (int i = tid; i < kF32HB / 16; i += 256) z[i] = u32x4{0u, 0u, 0u, 0u};
  }
  __syncthreads();
  // x image of step t by LDS-DMA (XH slot t, channels 0..63): piece i of 44
  // covers image bytes [1024 i, 1024 i + 1024) = pixels 4i + lane / 16, slot
  // lane % 16, which holds chunk slot ^ (key & 15); border pixels land as zeros.
  auto dma_x = [&](int t) {
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(p.XH + ((size_t)t * M + (size_t)b * P) * 192, (uint32_t)(P * 192 * 4));
    for (int i = wave; i < kF32XB / 1024; i += 4) {
      const int ip = i * 4 + (lane >> 4);
      const int py = ip / W2 - 1, px = ip % W2 - 1, q = (lane & 15) ^ ((py * p.w + px) & 15);
      const bool v = ip < NPH && (unsigned)py < (unsigned)p.h && (unsigned)px < (unsigned)p.w;
      dma16(rs, xim + i * 1024, v ? (uint32_t)(((py * p.w + px) * 192 + q * 4) * 4) : kOOB);
    }
  };
  dma_x(0);
  if (!p.h0_zero) {   // h_{-1} (XH slot 0, all 128 channels) into the h image
    const float* src = p.XH + (size_t)b * P * 192 + 64;
    for (int i = tid; i < P * 32; i += 256) {
      const int px = i >> 5, q = i & 31, ip = hidx(px);
      *reinterpret_cast<u32x4*>(him + ip * 512 + sw16(q, px)) = *reinterpret_cast<const u32x4*>(src + (size_t)px * 192 + q * 4);
    }
  }

  // per-lane state: bias of the lane's rows, c of its (pixel, channel) pairs
  // tile (r, c) lane (r32, hh): element 4g + e = row 8g + 4hh + e of row block
  // rbg0 + r = gate e of channel 8 (rbg0 + r) + 2g + hh, at column 32 cbk(c) + r32
  f32x4 bz[RPW][4];
  float cst[RPW][NCB][4];
  int pcol[NCB], hb[NCB], sb[NCB];   // sb: swizzle key of the window's top-left pixel
#pragma unroll
  for (int c = 0; c < NCB; ++c) {
    const int col = 32 * cbk(c) + r32;
    pcol[c] = col < P ? col : -1;
    hb[c] = p.colhb[col];
    sb[c] = (col < P ? col : P - 1) - p.w - 1;
  }
#pragma unroll
  for (int r = 0; r < RPW; ++r)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int ch = 8 * (rbg0 + r) + 2 * g + hh;
      bz[r][g] = *reinterpret_cast<const f32x4*>(p.bias + 4 * ch);
#pragma unroll
      for (int c = 0; c < NCB; ++c) cst[r][c][g] = pcol[c] >= 0 ? p.Cst[((size_t)b * P + pcol[c]) * 128 + ch] : 0.f;
    }

  // A stream: the wave's RPW row blocks, quad q at soffset (rb * kF32QP + q) * 1 KB
  const __amdgpu_buffer_rsrc_t rsw = make_rsrc(p.Wf, (uint32_t)(16 * kF32QP * 1024));
  auto lda = [&](int q, int r) {
    return __builtin_bit_cast(f32x4,
                              __builtin_amdgcn_raw_buffer_load_b128(rsw, lane * 16, ((rbg0 + r) * kF32QP + q) * 1024, 0));
  };
  constexpr int PD = S6 ? PDW : kF32PD;
  static_assert(8 % PD == 0 && PD >= 4 && PD <= kF32PD, "PD");   // slot = quad % PD; a pair never wraps
  f32x4 af[PD][RPW];
  // S6: the pre-split stream, quad q's part p of row block rb at ((rb * kF32QP + q) * 3 + p) * 512 B
  const __amdgpu_buffer_rsrc_t rsw6 = make_rsrc(p.Wf6, S6 ? (uint32_t)(16 * kF32QP * 3 * 512) : 0u);
  auto lda6 = [&](int q, int r, int part) {
    return __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(
                                         rsw6, lane * 8, (((rbg0 + r) * kF32QP + q) * 3 + part) * 512, 0));
  };
  u32x2 a6[S6 ? PD : 1][RPW][3];
  auto preload = [&] {
#pragma unroll
    for (int s = 0; s < PD - 1; ++s)
#pragma unroll
      for (int r = 0; r < RPW; ++r) {
        if constexpr (S6) {
#pragma unroll
          for (int part = 0; part < 3; ++part) a6[s][r][part] = lda6(s, r, part);
        } else {
          af[s][r] = lda(s, r);
        }
      }
  };
  preload();
  __syncthreads();   // h_{-1} image written; this wave's x DMA is waited for below
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();   // every wave's x_0 DMA landed

  for (int t = 0; t < p.T; ++t) {
    f32x16 acc[RPW][NCB];
#pragma unroll
    for (int r = 0; r < RPW; ++r)
#pragma unroll
      for (int c = 0; c < NCB; ++c)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[r][c][e] = 0.f;
    int hbs[NCB], sbs[NCB];
#pragma unroll
    for (int c = 0; c < NCB; ++c) {
      hbs[c] = hb[c];
      sbs[c] = sb[c];
      asm volatile("" : "+v"(hbs[c]), "+v"(sbs[c]));
    }
    // a tap's image-pixel offset and swizzle-key offset, packed (key offset << 16 | pixel offset)
    auto tapoff = [&](int tap) { return (((tap / 3) * p.w + tap % 3) << 16) | ((tap / 3) * W2 + tap % 3); };
    // B fragments of a quad: image pixel hbs[c] + toff, 16-B chunk q (x: 0..15, h: 0..31) + hh
    auto ldb = [&](const unsigned char* img, int pitch, int toff, int q, f32x4 (&bf)[NCB]) {
#pragma unroll
      for (int c = 0; c < NCB; ++c) {
        const int ip = hbs[c] + (toff & 0xffff);
        bf[c] = *reinterpret_cast<const f32x4*>(img + ip * pitch + sw16(q + hh, sbs[c] + (toff >> 16)));
      }
    };
    // one quad: A prefetch PD-1 ahead, next B fragments, 4 k-steps x RPW x 2 MFMAs
    auto quad = [&](int qn, int slot, f32x4 (&bc)[NCB], auto&& load_next_b) {
#pragma unroll
      for (int r = 0; r < RPW; ++r) af[(slot + PD - 1) % PD][r] = lda(qn + PD - 1, r);
      load_next_b();
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < RPW; ++r)
#pragma unroll
          for (int c = 0; c < NCB; ++c) {
            if constexpr (ABL & 8)
              acc[r][c][j] += af[slot][r][j] * bc[c][j];
            else
              acc[r][c] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[slot][r][j], bc[c][j], acc[r][c], 0, 0, 0);
          }
      __builtin_amdgcn_sched_barrier(0);
    };
    // S6: quads qn, qn + 1 (slot even: PD is even), B fragments of both in b0 / b1;
    // the A operand's parts come pre-split (k_split_frag): two quads' 8-B parts side by side
    auto pair = [&](int qn, int slot, f32x4 (&b0)[NCB], f32x4 (&b1)[NCB], auto&& load_next_b) {
      bf16x8 a3[RPW][3];
#pragma unroll
      for (int r = 0; r < RPW; ++r)
#pragma unroll
        for (int part = 0; part < 3; ++part)
          a3[r][part] = __builtin_bit_cast(bf16x8, u32x4{a6[slot][r][part].x, a6[slot][r][part].y,
                                                         a6[slot + 1][r][part].x, a6[slot + 1][r][part].y});
#pragma unroll
      for (int r = 0; r < RPW; ++r)
#pragma unroll
        for (int part = 0; part < 3; ++part) {
          a6[(slot + PD - 1) % PD][r][part] = lda6(qn + PD - 1, r, part);
          a6[slot][r][part] = lda6(qn + PD, r, part);
        }
      load_next_b();
      __builtin_amdgcn_sched_barrier(0);
      bf16x8 bh[NCB], bm[NCB], bl[NCB];
#pragma unroll
      for (int c = 0; c < NCB; ++c) {
        const float b8[8] = {b0[c][0], b0[c][1], b0[c][2], b0[c][3], b1[c][0], b1[c][1], b1[c][2], b1[c][3]};
        if constexpr ((ABL & 16) != 0) {   // ablation: hi part only (the split's VALU cost, wrong numerics)
#pragma unroll
          for (int e = 0; e < 8; ++e) bh[c][e] = (__bf16)b8[e];
          bm[c] = bh[c];
          bl[c] = bh[c];
        } else {
          split3_bf16(b8, bh[c], bm[c], bl[c]);
        }
      }
#pragma unroll
      for (int r = 0; r < RPW; ++r) {
        const bf16x8 ah = a3[r][0], am = a3[r][1], al = a3[r][2];
#pragma unroll
        for (int c = 0; c < NCB; ++c) {
          acc[r][c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh[c], acc[r][c], 0, 0, 0);
          acc[r][c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl[c], acc[r][c], 0, 0, 0);
          acc[r][c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bm[c], acc[r][c], 0, 0, 0);
          acc[r][c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bh[c], acc[r][c], 0, 0, 0);
          acc[r][c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bm[c], acc[r][c], 0, 0, 0);
          acc[r][c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh[c], acc[r][c], 0, 0, 0);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    };
    f32x4 bfr[2][NCB];
    f32x4 bp[4][NCB];   // S6: B fragments of two pairs of quads
    // partners' slices of h_{t-1} (XH slot t): loaded into registers mid x-part
    u32x4 pv[NPL];
    const bool exch = G > 1 && t > 0 && !(ABL & 4);
    AAA_F32_STAMP(t, 0);
    auto partner_issue = [&] {
      wave_wait_flags(p.flags + b * G, ((1ull << G) - 1) & ~(1ull << kh), t, p.report, p.spin, wdl);
      const __amdgpu_buffer_rsrc_t rs = make_rsrc(p.XH + ((size_t)t * M + (size_t)b * P) * 192, (uint32_t)(P * 192 * 4));
#pragma unroll
      for (int n = 0; n < NPL; ++n) {
        const int i = tid + 256 * n, px = i / ((G - 1) * CPG), rem = i % ((G - 1) * CPG);
        const int pj = rem / CPG, kq = (pj < kh ? pj : pj + 1) * CPG + rem % CPG;
        pv[n] = __builtin_amdgcn_raw_buffer_load_b128(rs, px < P ? (uint32_t)((px * 192 + 64 + kq * 4) * 4) : kOOB, 0,
                                                      kSC1);
      }
    };
    auto partner_store = [&] {
#pragma unroll
      for (int n = 0; n < NPL; ++n) {
        const int i = tid + 256 * n, px = i / ((G - 1) * CPG), rem = i % ((G - 1) * CPG);
        const int pj = rem / CPG, kq = (pj < kh ? pj : pj + 1) * CPG + rem % CPG;
        if (px < P) {
          const int ip = hidx(px);
          *reinterpret_cast<u32x4*>(him + ip * 512 + sw16(kq, px)) = pv[n];
        }
      }
    };

    // ---- x-part: 9 taps x 8 quads over the x image
    if constexpr (S6) {
      ldb(xim, 256, 0, 0, bp[0]);
      ldb(xim, 256, 0, 2, bp[1]);
    } else {
      ldb(xim, 256, 0, 0, bfr[0]);
    }
    for (int tap = 0; tap < 9; ++tap) {
      const int toff = tapoff(tap), tn = tap < 8 ? tapoff(tap + 1) : 0;
      int qt = tap * 8;
      asm volatile("" : "+s"(qt));
      if (tap == 2 && exch) partner_issue();
      if constexpr (S6) {
#pragma unroll
        for (int c8 = 0; c8 < 8; c8 += 2) {
          const int pb = (c8 >> 1) & 1, nb = pb ^ 1;
          pair(qt + c8, c8 % PD, bp[2 * pb], bp[2 * pb + 1], [&] {
            if (c8 < 6) {
              ldb(xim, 256, toff, 2 * (c8 + 2), bp[2 * nb]);
              ldb(xim, 256, toff, 2 * (c8 + 3), bp[2 * nb + 1]);
            } else if (tap < 8) {
              ldb(xim, 256, tn, 0, bp[2 * nb]);
              ldb(xim, 256, tn, 2, bp[2 * nb + 1]);
            }
          });
        }
      } else {
#pragma unroll
        for (int c8 = 0; c8 < 8; ++c8)
          quad(qt + c8, c8 % PD, bfr[c8 & 1], [&] {
            if (c8 < 7) ldb(xim, 256, toff, 2 * (c8 + 1), bfr[(c8 + 1) & 1]);
            else if (tap < 8) ldb(xim, 256, tn, 0, bfr[0]);
          });
      }
    }
    const bool hpart = t > 0 || !p.h0_zero;
    if (exch) partner_store();
    barrier_lds();   // every wave is done with x_t; the partners' h_{t-1} is in the image
    AAA_F32_STAMP(t, 1);
    if (hpart) {
      // ---- h-part: 9 taps x 16 quads over the h image
      if constexpr (S6) {
        ldb(him, 512, 0, 0, bp[0]);
        ldb(him, 512, 0, 2, bp[1]);
      } else {
        ldb(him, 512, 0, 0, bfr[0]);
      }
      for (int tap = 0; tap < 9; ++tap) {
        const int toff = tapoff(tap), tn = tap < 8 ? tapoff(tap + 1) : 0;
        int qt = kF32QX + tap * 16;
        asm volatile("" : "+s"(qt));
        if constexpr (S6) {
#pragma unroll
          for (int c16 = 0; c16 < 16; c16 += 2) {
            const int pb = (c16 >> 1) & 1, nb = pb ^ 1;
            pair(qt + c16, c16 % PD, bp[2 * pb], bp[2 * pb + 1], [&] {
              if (c16 < 14) {
                ldb(him, 512, toff, 2 * (c16 + 2), bp[2 * nb]);
                ldb(him, 512, toff, 2 * (c16 + 3), bp[2 * nb + 1]);
              } else if (tap < 8) {
                ldb(him, 512, tn, 0, bp[2 * nb]);
                ldb(him, 512, tn, 2, bp[2 * nb + 1]);
              }
            });
          }
        } else {
#pragma unroll
          for (int c16 = 0; c16 < 16; ++c16)
            quad(qt + c16, c16 % PD, bfr[c16 & 1], [&] {
              if (c16 < 15) ldb(him, 512, toff, 2 * (c16 + 1), bfr[(c16 + 1) & 1]);
              else if (tap < 8) ldb(him, 512, tn, 0, bfr[0]);
            });
        }
      }
    } else {   // the prefetched A quads are the h-part's: restart the stream at quad 0
      preload();
    }
    barrier_lds();   // every wave is done with h_{t-1}: the epilogue overwrites its own channels
    AAA_F32_STAMP(t, 2);
    // x_{t+1} lands under the epilogue: issued here, not under the h-part, because
    // vmcnt retires in order -- every later A-stream wait would queue behind the DMA
    if (t + 1 < p.T) dma_x(t + 1);

    // ---- epilogue: gate math + cell update lane-local; h_t into the image;
    // the HBM outputs staged through the wave's LDS scratch one 32 x 32 tile
    // at a time, so every store instruction writes whole pixel rows (Gt:
    // 128 B of the 32 gate rows, c / h: 32 B of the 8 channels).
    const size_t rowt = (size_t)t * M + (size_t)b * P;   // this frame's rows of step t
#pragma unroll
    for (int r = 0; r < RPW; ++r)
#pragma unroll
      for (int c = 0; c < NCB; ++c) {
        const int pp = pcol[c];
        if constexpr ((ABL & 1) != 0) {   // keep the accumulators alive, no epilogue work
          if (pp < 0) *reinterpret_cast<float*>(him) = acc[r][c][0] + acc[r][c][15];
          continue;
        }
        const int ip = hidx(max(pp, 0));
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int chl = 2 * g + hh, ch = 8 * (rbg0 + r) + chl;
          float gi, gf, gc, go, cc, h;
          GateFwd::run(acc[r][c][4 * g] + bz[r][g][0], acc[r][c][4 * g + 1] + bz[r][g][1],
                       acc[r][c][4 * g + 2] + bz[r][g][2], acc[r][c][4 * g + 3] + bz[r][g][3], cst[r][c][g], gi, gf,
                       gc, go, cc, h);
          cst[r][c][g] = cc;
          *reinterpret_cast<f32x4*>(stg + r32 * kF32GP + 16 * chl) = f32x4{gi, gf, gc, go};
          *reinterpret_cast<float*>(stg + kF32SG + r32 * 48 + 4 * chl) = cc;
          *reinterpret_cast<float*>(stg + kF32SG + 32 * 48 + r32 * 48 + 4 * chl) = h;
          if (pp >= 0) *reinterpret_cast<float*>(him + ip * 512 + sw16(ch >> 2, pp) + (ch & 3) * 4) = h;
        }
        __builtin_amdgcn_wave_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if constexpr (!(ABL & 2)) {
          const int col0 = 32 * cbk(c);
#pragma unroll
          for (int k = 0; k < 4; ++k) {   // Gt: 32 pixels x 8 chunks of 16 B (rows 32 rbg .. + 32)
            const int q = k * 64 + lane, px = q >> 3, ch16 = q & 7, pix = col0 + px;
            const u32x4 v = *reinterpret_cast<const u32x4*>(stg + px * kF32GP + 16 * ch16);
            if (pix < P) *reinterpret_cast<u32x4*>(p.Gt + (rowt + pix) * 512 + 32 * (rbg0 + r) + 4 * ch16) = v;
          }
          {  // c_t, h_t: 32 pixels x 2 chunks of 16 B (channels 8 rbg .. + 8)
            const int px = lane >> 1, half = lane & 1, pix = col0 + px;
            const u32x4 vc = *reinterpret_cast<const u32x4*>(stg + kF32SG + px * 48 + 16 * half);
            const u32x4 vh = *reinterpret_cast<const u32x4*>(stg + kF32SG + 32 * 48 + px * 48 + 16 * half);
            if (pix < P) {
              *reinterpret_cast<u32x4*>(p.Cst + (rowt + M + pix) * 128 + 8 * (rbg0 + r) + 4 * half) = vc;
              *reinterpret_cast<u32x4*>(p.Hs + (rowt + pix) * 128 + 8 * (rbg0 + r) + 4 * half) = vh;
            }
          }
        }
        __builtin_amdgcn_wave_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
    barrier_lds();   // this workgroup's channels of h_t are in the image
    {  // ... and from there into XH slot t+1 (the partners' and the weight gradient's operand):
       // 16-B write-through (sc1) stores, whole chunks
      const __amdgpu_buffer_rsrc_t rs = make_rsrc(p.XH + (rowt + M) * 192, (uint32_t)(P * 192 * 4));
      for (int i = tid; i < P * CPG; i += 256) {
        const int px = i / CPG, q = kh * CPG + i % CPG, ip = hidx(px);
        __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const u32x4*>(him + ip * 512 + sw16(q, px)), rs,
                                               (uint32_t)((px * 192 + 64 + q * 4) * 4), 0, kSC1);
      }
    }
    AAA_F32_STAMP(t, 3);
    // publish h_t: every wave's stores (and its x_{t+1} DMA) retired, a barrier, one flag store
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    barrier_lds();
    if (G > 1 && tid == 0) __hip_atomic_store(p.flags + b * G + kh, t + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    AAA_F32_STAMP(t, 4);
  }
}

// ---------------------------------------------------------------------------
// Pre-split frame-group forward (S6, G = 8): the same recurrence, mapping and A
// stream as k_convlstm_fwd_f32<8, 0, true, true, 4>, but the B operand -- the
// LDS images of x_t and h_{t-1} -- is held ALREADY split into its three bf16
// parts, so the K loop does no splitting at all (tools/ubench/f32rec: the
// in-loop split of the B fragments was 19 % of the launch, "S6 no B split").
// Each value is split once per step where it enters the image: x_{t+1} and the
// partners' h slices as they are loaded from XH, the workgroup's own h_t in the
// epilogue.  The split images are 1.5x the fp32 bytes, so they drop the zero
// border: a lane whose 3x3 neighbour is off the grid (or whose column is a
// padding column) reads the all-zero pixel P instead (per-lane tap mask).
//
// Image layout (both): pixel p at p * pitch; its 16-channel group g (the two
// quads of one S6 k-step) holds, per part (hi, mid, lo) and lane half hh, the
// 8 bf16 of channels 16g + {4hh..4hh+3, 8+4hh..8+4hh+3} -- exactly a lane's
// bf16x8 operand -- at chunk (part * NG + g) * 2 + hh (16 B each; NG = 8 groups
// for h, 4 for x).  Pitches 784 / 400 B are odd multiples of 16: the 16 lanes of
// a ds_read_b128 group (consecutive columns = consecutive pixels under every
// tap) hit 16 distinct bank groups, and a k-step's three parts are immediate
// offsets from one per-tap lane address.  The epilogue's staging aliases the x
// image (x_{t+1} is written after the epilogue).
//
// The zero pixel (round 6: at the END of the image, index kPsZP): an off-grid
// tap reads it.  At P (round 5) it sat inside the x image's aliased epilogue
// staging for grids with P < 88 (e.g. 64x64 frames: an 8x8 grid), which
// overwrote it after the first step -- logits 6.8e-2 off the oracle
// (test_f32_frames_small_grid_vs_oracle).  Off-grid lanes all read that one
// pixel, so a ds_read_b128 group with such lanes takes a second pass where
// their slot meets an on-grid lane's (LDS conflict rate 0.34 forward, 0.26
// BPTT at C2); a slot-matched pair of zero pixels (each off-grid lane at the
// slot its on-grid address would have had) removed the conflicts and measured
// SLOWER (C2 forward 745 -> 770 us, BPTT 836 -> 845: the per-tap slot
// arithmetic costs more than the second pass; profiles/r06/ab/zero_slot/).
constexpr int kPsHP = 784, kPsXP = 400;                 // pixel pitches (B)
constexpr int kPsNP = 129;                              // pixels (P <= kPsZP) + the zero pixel
constexpr int kPsZP = kPsNP - 1;                        // the zero pixel
__device__ __forceinline__ uint32_t ps_tap_base(bool valid, int nb, int pitch, int hh) {
  return (uint32_t)((valid ? nb : kPsZP) * pitch + hh * 16);
}
constexpr int kPsHB = kPsNP * kPsHP, kPsXB = kPsNP * kPsXP;
constexpr int kPsGT = 0, kPsCT = 32 * 144;               // per-wave staging: gate tile, c tile
constexpr int kPsSTG = kPsCT + 32 * 48;                  // 6 KB per wave
constexpr int kPsHT = 4 * kPsSTG;                        // the workgroup's h_t tile: 128 pixels x 16 channels, pitch 80 B
static_assert(kPsHT + 128 * 80 <= kPsXB, "staging aliases the x image");
static_assert(kPsHT + 128 * 80 <= kPsZP * kPsXP, "the staging must not reach the zero pixel");


// split 16 fp32 channels of one pixel (group order) into the image's 6 chunks
__device__ __forceinline__ void ps_store_group(unsigned char* img, int pix_off, int NG, int g, const f32x4 (&v)[4]) {
#pragma unroll
  for (int hh = 0; hh < 2; ++hh) {
    const float x8[8] = {v[hh][0], v[hh][1], v[hh][2], v[hh][3], v[2 + hh][0], v[2 + hh][1], v[2 + hh][2], v[2 + hh][3]};
    bf16x8 hi, mid, lo;
    split3_bf16(x8, hi, mid, lo);
    *reinterpret_cast<bf16x8*>(img + pix_off + ((0 * NG + g) * 2 + hh) * 16) = hi;
    *reinterpret_cast<bf16x8*>(img + pix_off + ((1 * NG + g) * 2 + hh) * 16) = mid;
    *reinterpret_cast<bf16x8*>(img + pix_off + ((2 * NG + g) * 2 + hh) * 16) = lo;
  }
}

// ABL (diagnostic builds only, tools/ubench/f32ps; production launches use 0): bit 0 = no
// epilogue math / HBM stores, bit 2 = no partner exchange, bit 3 = no MFMAs, bit 5 = no
// A-stream loads in the K loop.
// MAP: wave -> tiles.  0: wave w takes both row blocks and column block w (each A quad is
// streamed by all four waves); 1: wave w takes row block w & 1 and column blocks
// 2 (w >> 1), +1 (each A quad streamed by two waves, each B part read by two).  The A stream
// (L2 -> L1 -> VGPR, no LDS room left beside the split images) is the kernel's bound
// (tools/ubench/f32ps: no A loads -29 %), so MAP 1 halves its L1 traffic.
template <int ABL = 0, int MAP = 1, int PD = 8>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
k_convlstm_fwd_f32ps(RecF32Params p) {
  static_assert(8 % PD == 0 && PD >= 4 && PD <= kF32PD, "PD");   // slot = quad % PD; a pair never wraps
  constexpr int G = 8, NPU = (128 * 7 + 255) / 256, NXU = (128 * 4 + 255) / 256;
  constexpr int RPW = MAP ? 1 : 2, NCB = MAP ? 2 : 1;
  __shared__ __attribute__((aligned(16))) unsigned char him[kPsHB];
  __shared__ __attribute__((aligned(16))) unsigned char xim[kPsXB];

  const int blk = (int)blockIdx.x, xcd = blk & 7, loc = blk >> 3;
  const int b = xcd + 8 * (loc / G), kh = loc % G;
  if (b >= p.B) return;   // padding group of the last XCD column (never a partner of a live frame)
  const int tid = (int)threadIdx.x, lane = tid & 63;
  uint64_t wdl = 0;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r32 = lane & 31, hh = lane >> 5;
  const int P = p.P, W = p.w;
  const size_t M = (size_t)p.B * P;
  const int rw = MAP ? (wave & 1) : 0;
  const int rbg0 = 2 * kh + rw;                 // the wave's first global row block
  auto cbk = [&](int c) { return MAP ? 2 * (wave >> 1) + c : wave; };
  unsigned char* stg = xim + wave * kPsSTG;

  // per lane and column block: the column, its 3x3 validity mask (padding columns: none valid)
  int colc[NCB], vmask[NCB];
#pragma unroll
  for (int c = 0; c < NCB; ++c) {
    colc[c] = 32 * cbk(c) + r32;
    vmask[c] = 0;
    if (colc[c] < P) {
      const int y = colc[c] / W, x = colc[c] % W;
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int yy = y + tap / 3 - 1, xx = x + tap % 3 - 1;
        if ((unsigned)yy < (unsigned)p.h && (unsigned)xx < (unsigned)W) vmask[c] |= 1 << tap;
      }
    }
  }
  // lane byte address of tap ``tap``'s neighbour pixel (or the zero pixel) in an image of ``pitch``
  auto tapbase = [&](int c, int tap, int pitch) -> uint32_t {
    const int nb = colc[c] + (tap / 3 - 1) * W + (tap % 3 - 1);
    return ps_tap_base((vmask[c] >> tap) & 1, nb, pitch, hh);
  };

  // XH slot loads of 16-channel groups: unit u = (pixel, group) -> 4 x 16 B (sc1 for partner slices)
  auto xh_rsrc = [&](int slot) {
    return make_rsrc(p.XH + ((size_t)slot * M + (size_t)b * P) * 192, (uint32_t)(P * 192 * 4));
  };
  auto ld_group = [&](__amdgpu_buffer_rsrc_t rs, int px, int chan0, bool sc1, f32x4 (&v)[4]) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t off = px < P ? (uint32_t)((px * 192 + chan0 + 4 * k) * 4) : kOOB;
      v[k] = __builtin_bit_cast(f32x4, sc1 ? __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, kSC1)
                                           : __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
    }
  };
  f32x4 xv[NXU][4];
  auto x_issue = [&](int slot) {   // x_slot: units (pixel, group 0..3)
    const __amdgpu_buffer_rsrc_t rs = xh_rsrc(slot);
#pragma unroll
    for (int n = 0; n < NXU; ++n) {
      const int u = tid + 256 * n;
      ld_group(rs, u >> 2, 16 * (u & 3), false, xv[n]);
    }
  };
  auto x_store = [&] {
#pragma unroll
    for (int n = 0; n < NXU; ++n) {
      const int u = tid + 256 * n, px = u >> 2;
      if (px < P) ps_store_group(xim, px * kPsXP, 4, u & 3, xv[n]);
    }
  };

  {  // the zero pixel of both images
    u32x4* z = reinterpret_cast<u32x4*>(him + kPsZP * kPsHP);
    for (int i = tid; i < kPsHP / 16; i += 256) z[i] = u32x4{0u, 0u, 0u, 0u};
    z = reinterpret_cast<u32x4*>(xim + kPsZP * kPsXP);
    for (int i = tid; i < kPsXP / 16; i += 256) z[i] = u32x4{0u, 0u, 0u, 0u};
  }
  x_issue(0);
  x_store();
  if (!p.h0_zero) {   // h_{-1} (XH slot 0, all 8 groups) into the h image
    const __amdgpu_buffer_rsrc_t rs = xh_rsrc(0);
    for (int u = tid; u < P * 8; u += 256) {
      f32x4 v[4];
      ld_group(rs, u >> 3, 64 + 16 * (u & 7), false, v);
      ps_store_group(him, (u >> 3) * kPsHP, 8, u & 7, v);
    }
  }

  // per-lane state: bias of the lane's rows, c of its (pixel, channel) pairs -- tile (r, c)
  // lane (r32, hh): element 4g + e = gate e of channel 8 (rbg0 + r) + 2g + hh at column colc[c]
  f32x4 bz[RPW][4];
  float cst[RPW][NCB][4];
#pragma unroll
  for (int r = 0; r < RPW; ++r)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int ch = 8 * (rbg0 + r) + 2 * g + hh;
      bz[r][g] = *reinterpret_cast<const f32x4*>(p.bias + 4 * ch);
#pragma unroll
      for (int c = 0; c < NCB; ++c) cst[r][c][g] = colc[c] < P ? p.Cst[((size_t)b * P + colc[c]) * 128 + ch] : 0.f;
    }

  // A stream (pre-split fragment-order weights, k_pack_frag_f32's paired stream): per lane one 16-B
  // load brings a part of both quads of a pair (half the load instructions of two 8-B loads);
  // PD / 2 pairs in flight
  const __amdgpu_buffer_rsrc_t rsw6 = make_rsrc(p.Wf6p, (uint32_t)(16 * kF32PP * 3 * 1024));
  auto lda6 = [&](int pj, int r, int part) {
    return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                         rsw6, lane * 16, (((rbg0 + r) * kF32PP + pj) * 3 + part) * 1024, 0));
  };
  u32x4 a6[PD / 2][RPW][3];
  auto preload = [&] {
#pragma unroll
    for (int s = 0; s < PD / 2; ++s)
#pragma unroll
      for (int r = 0; r < RPW; ++r)
#pragma unroll
        for (int part = 0; part < 3; ++part) a6[s][r][part] = lda6(s, r, part);
  };
  preload();
  __syncthreads();   // x_0 / h_{-1} images and the zero pixels written

  for (int t = 0; t < p.T; ++t) {
    f32x16 acc[RPW][NCB];
#pragma unroll
    for (int r = 0; r < RPW; ++r)
#pragma unroll
      for (int c = 0; c < NCB; ++c)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[r][c][e] = 0.f;
    // B parts of group g at the lane addresses ``base``: three immediate offsets per column block
    auto ldb = [&](const unsigned char* img, const uint32_t (&base)[NCB], int NG, int g, bf16x8 (&bv)[NCB][3]) {
#pragma unroll
      for (int c = 0; c < NCB; ++c)
#pragma unroll
        for (int part = 0; part < 3; ++part)
          bv[c][part] = *reinterpret_cast<const bf16x8*>(img + base[c] + (part * NG + g) * 32);
    };
    // quads qn, qn + 1 (slot even): A parts pre-split in the stream, B parts pre-split in the image
    auto pair = [&](int qn, int slot, const bf16x8 (&bv)[NCB][3], auto&& load_next_b) {
      bf16x8 a3[RPW][3];
#pragma unroll
      for (int r = 0; r < RPW; ++r)
#pragma unroll
        for (int part = 0; part < 3; ++part) a3[r][part] = __builtin_bit_cast(bf16x8, a6[slot / 2][r][part]);
      if constexpr (!(ABL & 32)) {   // refill the slot pair with pair qn / 2 + PD / 2 (the stream wraps)
#pragma unroll
        for (int r = 0; r < RPW; ++r)
#pragma unroll
          for (int part = 0; part < 3; ++part) a6[slot / 2][r][part] = lda6(qn / 2 + PD / 2, r, part);
      }
      load_next_b();
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int r = 0; r < RPW; ++r) {
        const bf16x8 ah = a3[r][0], am = a3[r][1], al = a3[r][2];
#pragma unroll
        for (int c = 0; c < NCB; ++c) {
          if constexpr ((ABL & 8) != 0) {   // keep every operand alive, no MFMA
            acc[r][c][0] += (float)ah[0] * (float)bv[c][0][0] + (float)am[1] * (float)bv[c][1][1] +
                            (float)al[2] * (float)bv[c][2][2];
          } else {
            acc[r][c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bv[c][0], acc[r][c], 0, 0, 0);
            acc[r][c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bv[c][2], acc[r][c], 0, 0, 0);
            acc[r][c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bv[c][1], acc[r][c], 0, 0, 0);
            acc[r][c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bv[c][0], acc[r][c], 0, 0, 0);
            acc[r][c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bv[c][1], acc[r][c], 0, 0, 0);
            acc[r][c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bv[c][0], acc[r][c], 0, 0, 0);
          }
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    };
    bf16x8 bp[2][NCB][3];
    // partners' groups of h_{t-1} (XH slot t): loaded into registers mid x-part
    f32x4 pv[NPU][4];
    const bool exch = t > 0 && !(ABL & 4);
    AAA_F32_STAMP(t, 0);
    auto partner_issue = [&] {
      wave_wait_flags(p.flags + b * G, ((1ull << G) - 1) & ~(1ull << kh), t, p.report, p.spin, wdl);
      const __amdgpu_buffer_rsrc_t rs = xh_rsrc(t);
#pragma unroll
      for (int n = 0; n < NPU; ++n) {
        const int u = tid + 256 * n, px = u / 7, j = u % 7, g = j < kh ? j : j + 1;
        ld_group(rs, px, 64 + 16 * g, true, pv[n]);
      }
    };
    auto partner_store = [&] {
#pragma unroll
      for (int n = 0; n < NPU; ++n) {
        const int u = tid + 256 * n, px = u / 7, j = u % 7, g = j < kh ? j : j + 1;
        if (px < P) ps_store_group(him, px * kPsHP, 8, g, pv[n]);
      }
    };
    auto bases = [&](int tap, int pitch, uint32_t (&o)[NCB]) {
#pragma unroll
      for (int c = 0; c < NCB; ++c) o[c] = tapbase(c, tap, pitch);
    };

    // ---- x-part: 9 taps x 4 groups over the x image
    {
      uint32_t xb[NCB], xn[NCB];
      bases(0, kPsXP, xb);
      ldb(xim, xb, 4, 0, bp[0]);
      for (int tap = 0; tap < 9; ++tap) {
        bases(tap < 8 ? tap + 1 : 8, kPsXP, xn);
        int qt = tap * 8;
        asm volatile("" : "+s"(qt));
        if (tap == 2 && exch) partner_issue();
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          pair(qt + 2 * g, (2 * g) % PD, bp[g & 1], [&] {
            if (g < 3) ldb(xim, xb, 4, g + 1, bp[(g + 1) & 1]);
            else if (tap < 8) ldb(xim, xn, 4, 0, bp[0]);
          });
        }
#pragma unroll
        for (int c = 0; c < NCB; ++c) xb[c] = xn[c];
      }
    }
    const bool hpart = t > 0 || !p.h0_zero;
    if (exch) partner_store();
    barrier_lds();   // every wave is done with x_t; the partners' h_{t-1} is in the image
    AAA_F32_STAMP(t, 1);
    if (hpart) {
      // ---- h-part: 9 taps x 8 groups over the h image
      uint32_t hb[NCB], hn[NCB];
      bases(0, kPsHP, hb);
      ldb(him, hb, 8, 0, bp[0]);
      for (int tap = 0; tap < 9; ++tap) {
        bases(tap < 8 ? tap + 1 : 8, kPsHP, hn);
        int qt = kF32QX + tap * 16;
        asm volatile("" : "+s"(qt));
#pragma unroll
        for (int g = 0; g < 8; ++g) {
          pair(qt + 2 * g, (2 * g) % PD, bp[g & 1], [&] {
            if (g < 7) ldb(him, hb, 8, g + 1, bp[(g + 1) & 1]);
            else if (tap < 8) ldb(him, hn, 8, 0, bp[0]);
          });
        }
#pragma unroll
        for (int c = 0; c < NCB; ++c) hb[c] = hn[c];
      }
    } else {   // the prefetched A quads are the h-part's: restart the stream at quad 0
      preload();
    }
    barrier_lds();   // every wave is done with both images: staging (aliasing x) and h_t may be written
    AAA_F32_STAMP(t, 2);
    if (t + 1 < p.T) x_issue(t + 1);   // x_{t+1} lands under the epilogue

    // ---- epilogue: gate math + cell update lane-local; Gt / c_t staged per wave through its
    // LDS tiles (whole pixel rows per store instruction); h_t into the workgroup's h tile
    const size_t rowt = (size_t)t * M + (size_t)b * P;
    if constexpr ((ABL & 1) != 0) {
#pragma unroll
      for (int r = 0; r < RPW; ++r)
#pragma unroll
        for (int c = 0; c < NCB; ++c)   // keep the accumulators alive: one value each into the h tile
          *reinterpret_cast<float*>(xim + kPsHT + (colc[c] & 127) * 80 + 4 * r) = acc[r][c][0] + acc[r][c][15];
    } else {
#pragma unroll
      for (int r = 0; r < RPW; ++r)
#pragma unroll
        for (int c = 0; c < NCB; ++c) {
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int chl = 2 * g + hh;
            float gi, gf, gc, go, cc, h;
            GateFwd::run(acc[r][c][4 * g] + bz[r][g][0], acc[r][c][4 * g + 1] + bz[r][g][1],
                         acc[r][c][4 * g + 2] + bz[r][g][2], acc[r][c][4 * g + 3] + bz[r][g][3], cst[r][c][g], gi, gf,
                         gc, go, cc, h);
            cst[r][c][g] = cc;
            *reinterpret_cast<f32x4*>(stg + kPsGT + r32 * 144 + 16 * chl) = f32x4{gi, gf, gc, go};
            *reinterpret_cast<float*>(stg + kPsCT + r32 * 48 + 4 * chl) = cc;
            *reinterpret_cast<float*>(xim + kPsHT + colc[c] * 80 + 4 * (8 * (rbg0 + r - 2 * kh) + chl)) = h;
          }
          __builtin_amdgcn_wave_barrier();
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          const int col0 = 32 * cbk(c);
#pragma unroll
          for (int k = 0; k < 4; ++k) {   // Gt: 32 pixels x 8 chunks of 16 B (rows 32 rbg .. + 32)
            const int q = k * 64 + lane, px = q >> 3, ch16 = q & 7, pix = col0 + px;
            const u32x4 v = *reinterpret_cast<const u32x4*>(stg + kPsGT + px * 144 + 16 * ch16);
            if (pix < P) *reinterpret_cast<u32x4*>(p.Gt + (rowt + pix) * 512 + 32 * (rbg0 + r) + 4 * ch16) = v;
          }
          {  // c_t: 32 pixels x 2 chunks of 16 B (channels 8 rbg .. + 8)
            const int px = lane >> 1, half = lane & 1, pix = col0 + px;
            const u32x4 vc = *reinterpret_cast<const u32x4*>(stg + kPsCT + px * 48 + 16 * half);
            if (pix < P) *reinterpret_cast<u32x4*>(p.Cst + (rowt + M + pix) * 128 + 8 * (rbg0 + r) + 4 * half) = vc;
          }
          __builtin_amdgcn_wave_barrier();
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
    }
    barrier_lds();   // the workgroup's h_t tile is complete
    if constexpr (!(ABL & 1)) {
      // h_t, the workgroup's 16 channels: Hs, XH slot t+1 (sc1: the partners' and the weight
      // gradient's operand) and the own group of the split h image; thread = (pixel, half)
      const int px = tid >> 1, half = tid & 1;
      if (px < P) {
        const unsigned char* ht = xim + kPsHT + px * 80;
        const u32x4 h0 = *reinterpret_cast<const u32x4*>(ht + 32 * half);
        const u32x4 h1 = *reinterpret_cast<const u32x4*>(ht + 32 * half + 16);
        float* hs = p.Hs + (rowt + px) * 128 + 16 * kh + 8 * half;
        *reinterpret_cast<u32x4*>(hs) = h0;
        *reinterpret_cast<u32x4*>(hs + 4) = h1;
        const __amdgpu_buffer_rsrc_t rs = xh_rsrc(t + 1);
        const uint32_t off = (uint32_t)((px * 192 + 64 + 16 * kh + 8 * half) * 4);
        __builtin_amdgcn_raw_buffer_store_b128(h0, rs, off, 0, kSC1);
        __builtin_amdgcn_raw_buffer_store_b128(h1, rs, off + 16, 0, kSC1);
        // the split image's lane half ``half`` holds channels {4 half .. +3, 8 + 4 half .. +3}
        const f32x4 va = *reinterpret_cast<const f32x4*>(ht + 16 * half);
        const f32x4 vb = *reinterpret_cast<const f32x4*>(ht + 32 + 16 * half);
        const float x8[8] = {va[0], va[1], va[2], va[3], vb[0], vb[1], vb[2], vb[3]};
        bf16x8 hi, mid, lo;
        split3_bf16(x8, hi, mid, lo);
        unsigned char* dst = him + px * kPsHP + half * 16;
        *reinterpret_cast<bf16x8*>(dst + (0 * 8 + kh) * 32) = hi;
        *reinterpret_cast<bf16x8*>(dst + (1 * 8 + kh) * 32) = mid;
        *reinterpret_cast<bf16x8*>(dst + (2 * 8 + kh) * 32) = lo;
      }
    }
    barrier_lds();   // every wave is done with the staging and the h tile (they alias the x image)
    AAA_F32_STAMP(t, 3);
    if (t + 1 < p.T) x_store();
    // publish h_t: every wave's stores retired, a barrier (also: x_{t+1} in the image), one flag store
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    barrier_lds();
    if (tid == 0) __hip_atomic_store(p.flags + b * G + kh, t + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    AAA_F32_STAMP(t, 4);
  }
}

inline bool f32_rec_fits(int h, int w) { return rec_fits(h, w); }

// Workgroups per frame for B frames on a device of ``cus`` CUs (0: does not fit one residency wave).
inline int f32_rec_g(int B, int cus) {
  for (int G : {8, 4})   // (G = 2 spills at 1 wave per SIMD: 8 row blocks x 2 column blocks per wave)
    if (f32_grid(B, G) <= cus) return G;
  return 0;
}

// Whether convlstm_fwd_f32 runs the pre-split kernel (k_convlstm_fwd_f32ps) for this launch.
inline bool f32_fwd_presplit(bool s6, int G, int P) {
#ifdef AAA_ABLATION
  if (std::getenv("AAA_F32_PRESPLIT") != nullptr) return false;
#endif
  return s6 && G == 8 && P <= kPsZP;
}

inline hipError_t convlstm_fwd_f32(RecF32Params& p, int G, hipStream_t st, bool s6 = false) {
  if (!f32_rec_fits(p.h, p.w) || p.P != p.h * p.w || p.B < 1 || p.T < 1 || !p.flags || !p.report || p.spin < 0)
    return hipErrorInvalidValue;
  for (int c = 0; c < 128; ++c) {
    const int pp = c < p.P ? c : p.P - 1;
    p.colhb[c] = (short)((pp / p.w) * (p.w + 2) + pp % p.w);
  }
  // G = 8, S6: the WIDE mapping with 4 A quads in flight (tools/ubench/f32rec: 7-10% under
  // the two-column-block mapping with 8, most of it from the shallower prefetch)
  // G = 8, S6, P <= 128: the pre-split images (k_convlstm_fwd_f32ps); larger grids the in-loop
  // split (AAA_F32_PRESPLIT=0 selects it everywhere in ablation builds)
  const bool ps = f32_fwd_presplit(s6, G, p.P);
  const void* k = ps       ? reinterpret_cast<const void*>(&k_convlstm_fwd_f32ps<0, 1, 8>)
                  : G == 8 ? (s6 ? reinterpret_cast<const void*>(&k_convlstm_fwd_f32<8, 0, true, true, 4>)
                                 : reinterpret_cast<const void*>(&k_convlstm_fwd_f32<8>))
                  : G == 4 ? (s6 ? reinterpret_cast<const void*>(&k_convlstm_fwd_f32<4, 0, true>)
                                 : reinterpret_cast<const void*>(&k_convlstm_fwd_f32<4>))
                           : nullptr;
  if (!k) return hipErrorInvalidValue;
  return launch_resident(k, f32_grid(p.B, G), 256, p, st);
}

}  // namespace aaa
