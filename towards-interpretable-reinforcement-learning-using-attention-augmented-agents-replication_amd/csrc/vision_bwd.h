// Frame-resident bf16 vision-encoder BACKWARD (round 6): the backward of
// VisionNetwork.vision_cnn (attention.py:153-170 on X.transpose(1,3), :179)
// for one frame at a time, all three products in one persistent workgroup:
//
//   conv2 dgrad   dY1 = conv2^T(dY2)           (4 stride-2 parity classes)
//   conv2 wgrad   gW2 += dY2^T x im2col(Y1)     [64][512 = (ky*4+kx)*32 + ci]
//   conv1 wgrad   gW1 += dY1^T x im2col(Xp)     [32][256 = (ky*8+kx)*4 + c]
//
// It replaces three launches (halo-staged conv2 dgrad, conv2 / conv1 weight
// gradients on the LDS-DMA rings: C3 135 + 103 + 127 us) whose operands went
// through HBM: dY1 (written by the dgrad, re-read by conv1's wgrad: 262 MB at
// C3) and Xp (the bordered RGBx frames the forward wrote for conv1's wgrad:
// 303 MB).  Here dY1 never leaves LDS and the RGBx image is rebuilt from the
// observation (uint8, 21 KB per 84x84 frame), as the forward's encoder does.
// uint8 observations only (the environment's dtype, main_mp.py:53 casts them
// on the host): an fp32-observation variant spilled 46 registers and computed
// conv1's weight gradient wrong (tools/dbg/vbwd_diag.py), so fp32 frames keep
// the layered launches.
//
// Per frame, LDS holds: the frame's RGBx bf16 image (bordered, as k_vision_fwd),
// the Y1 image (bordered by 2 for conv2's pad), the dY2 image (one row of 64
// channels per grid pixel, 16-B chunks XOR-keyed by pixel pair so the dgrad's
// B-fragment reads of 16 consecutive pixels hit 16 bank groups), and dY1
// ([pixels][32 channels], the conv1 weight gradient's A operand by transposed
// reads).  Waves:
//   dgrad        wave w = parity class w (32 rows of WdT2), all 4 column
//                blocks of the class grid, K = 4 taps x 64 channels
//   conv2 wgrad  wave w = taps 4w .. 4w+3 (one 32-column block each: ci), both
//                64-row blocks, K = the frame's pixels; A (dY2^T) and B
//                (im2col Y1) by ds_read_b64_tr_b16 transposed reads
//   conv1 wgrad  wave w = ky 2w, 2w+1 (one column block each: kx x c), K = the
//                conv1 output pixels; A (dY1) and B (RGBx) by transposed reads
// The weight-gradient accumulators (128 + 32 per lane) stay in registers for
// all of a workgroup's frames; each workgroup writes one partial of gW2 / gW1
// / the conv1 bias grad, summed in workgroup order by k_vbwd_reduce (no
// atomics: the result is deterministic).  The next frame's dY2 and Y1 are
// LDS-DMA'd and its observation loaded while conv1's weight gradient runs.
#pragma once
#include "vision.h"

namespace aaa {

constexpr int kVbDN = 128;                       // dY2 image pixels: grid pixels < kVbDN - 1, pixel kVbDN - 1 zero
constexpr int kVbDB = kVbDN * 128;               // dY2 image bytes (64 bf16 per pixel)
constexpr int kVbYB = 36864;                     // Y1 image bytes: (H1+4)(W1+4) pixels x 64 B (24 x 24 at 84x84)
constexpr int kVbK1 = 416;                       // conv1-wgrad K (conv1 output pixels, padded to 16)
constexpr int kVbTB = kVbK1 * 64;                // dY1 image bytes: [pixel][32 channels] bf16
constexpr int kVbPart = 64 * 512 + 32 * 256 + 32;   // floats of one workgroup partial: gW2, gW1, conv1 bias

struct VisBwdParams {
  const void* frames;   // (F, H, W, 3) uint8: the observation the forward read
  const __bf16* dY2;    // (F, P, 64) conv2 output gradient
  const __bf16* Y1;     // (F, P1, 32) conv1 output (forward)
  const __bf16* WdT2;   // [128 = class*32 + c][256 = tap*64 + o]: conv2 dgrad weights (k_WdT2)
  float* part;          // [gridDim.x][kVbPart] <- per-workgroup partials
  int F, H, W, H1, W1, h, w;
};

// Whether the fused backward applies (it also needs the frame-resident forward's RGBx image).
inline bool vbwd_fits(int H, int W, int H1, int W1, int h, int w) {
  const int Ha = (H1 + 1) / 2, Wa = (W1 + 1) / 2;
  return vis_fits(H, W, H1, W1, h, w) && h * w <= kVbDN - 1 && H1 * W1 <= kVbK1 && Ha * Wa <= 128 && w < 128 &&
         (H1 + 4) * (W1 + 4) * 64 <= kVbYB && Ha <= h && Wa <= w && W1 > 16;
}

// dY2 image: 16-B chunk q (channels 8q .. 8q+7) of pixel pix at slot q ^ ((pix >> 1) & 7)
__device__ __forceinline__ int vb_dofs(int pix, int ch) {
  return pix * 128 + ((((ch >> 3) ^ (pix >> 1)) & 7) << 4) + (ch & 7) * 2;
}

// ds_read_b64_tr_b16 pair (glds.h frag_rc): the lane's 8 k values of its row from two 8-B pieces
__device__ __forceinline__ bf16x8 vb_tr(const unsigned char* lds, int o0, int o1) {
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(const_cast<unsigned char*>(lds + o0)));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(const_cast<unsigned char*>(lds + o1)));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// ABL (ablation builds only, AAA_VBWD_ABL): bit 0 = no conv2 dgrad, 1 = no conv2 wgrad, 2 = no conv1 wgrad,
// 3 = no next-frame loads (every frame recomputes the first frame's inputs)
template <int ABL = 0>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) k_vision_bwd_frames(VisBwdParams p) {
  __shared__ __attribute__((aligned(16))) unsigned char xim[kVisXB];   // RGBx image (bordered), as k_vision_fwd
  __shared__ __attribute__((aligned(16))) unsigned char yim[kVbYB];    // Y1 image, interior at (+2, +2)
  __shared__ __attribute__((aligned(16))) unsigned char dim[kVbDB];    // dY2 image
  __shared__ __attribute__((aligned(16))) unsigned char tim[kVbTB];   // dY1 [pixel][32 c] (transposed reads)
  const int tid = (int)threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r32 = lane & 31, hh = lane >> 5;
  const int li = lane & 15, tq = li >> 2, tp = li & 3;   // transposed-read lane roles (glds.h frag_rc)
  const int Wp = p.W + 2, W1p = p.W1 + 4, P = p.h * p.w, P1 = p.H1 * p.W1;
  const int Ha = (p.H1 + 1) / 2, Wa = (p.W1 + 1) / 2, NA = Ha * Wa;
  const int G4 = p.H * p.W / 4;
  const int KS1 = (P1 + 15) / 16;   // conv1-wgrad k steps

  {  // zero every image once: borders, pads and the zero pixel stay zero
    u32x4* z = reinterpret_cast<u32x4*>(xim);
    for (int i = tid; i < kVisXB / 16; i += 256) z[i] = u32x4{0u, 0u, 0u, 0u};
    z = reinterpret_cast<u32x4*>(yim);
    for (int i = tid; i < kVbYB / 16; i += 256) z[i] = u32x4{0u, 0u, 0u, 0u};
    z = reinterpret_cast<u32x4*>(dim);
    for (int i = tid; i < kVbDB / 16; i += 256) z[i] = u32x4{0u, 0u, 0u, 0u};
    z = reinterpret_cast<u32x4*>(tim);
    for (int i = tid; i < kVbTB / 16; i += 256) z[i] = u32x4{0u, 0u, 0u, 0u};
  }
  __syncthreads();

  // ---- loads of frame f: dY2 and Y1 by LDS-DMA (lane-linear 1-KB pieces, the image layouts applied
  // on the source side; border / pad positions read outside the descriptor and land as zeros), the
  // observation into registers (converted into the RGBx image by build())
  auto dma_frame = [&](int f) {
    {  // dY2: piece i covers image pixels 8i .. 8i+7 (8 chunks each)
      const __amdgpu_buffer_rsrc_t rs = make_rsrc(p.dY2 + (size_t)f * P * 64, (uint32_t)(P * 64 * 2));
      for (int i = wave; i < kVbDB / 1024; i += 4) {
        const int sl = i * 64 + lane, pix = sl >> 3, q = ((sl & 7) ^ (pix >> 1)) & 7;
        dma16a(rs, dim + i * 1024, pix < P ? (uint32_t)((pix * 64 + 8 * q) * 2) : kOOB);
      }
    }
    {  // Y1: piece i covers image pixels 16i .. 16i+15 (4 chunks each)
      const __amdgpu_buffer_rsrc_t rs = make_rsrc(p.Y1 + (size_t)f * P1 * 32, (uint32_t)(P1 * 32 * 2));
      const int n = ((p.H1 + 4) * W1p * 64 + 1023) / 1024;
      for (int i = wave; i < n; i += 4) {
        const int sl = i * 64 + lane, ip = sl >> 2, iy = ip / W1p, ix = ip - iy * W1p, y = iy - 2, x = ix - 2;
        const bool v = (unsigned)y < (unsigned)p.H1 && (unsigned)x < (unsigned)p.W1;
        dma16a(rs, yim + i * 1024, v ? (uint32_t)(((y * p.W1 + x) * 32 + 8 * (sl & 3)) * 2) : kOOB);
      }
    }
  };
  uint32_t raw[kVisNG][3];   // the next frame's pixels (uint8), prefetched
  auto fetch = [&](int f) {
    const uint32_t* src =
        reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(p.frames) + (size_t)f * p.H * p.W * 3);
#pragma unroll
    for (int i = 0; i < kVisNG; ++i) {
      const int g = min(tid + 256 * i, G4 - 1);
#pragma unroll
      for (int q = 0; q < 3; ++q) raw[i][q] = src[(size_t)g * 3 + q];
    }
  };
  auto build = [&]() {   // as k_vision_fwd: bf16 RGBx, channel 3 zero
#pragma unroll
    for (int i = 0; i < kVisNG; ++i) {
      const int g = tid + 256 * i;
      if (g < G4) {
        const int pix = 4 * g, y = pix / p.W, x = pix - y * p.W;
        unsigned char* d = xim + ((y + 1) * Wp + x + 1) * 8;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float v[3];
#pragma unroll
          for (int c = 0; c < 3; ++c) {
            const int e = 3 * j + c;
            v[c] = (float)((raw[i][e >> 2] >> (8 * (e & 3))) & 255u);
          }
          *reinterpret_cast<bf16x4*>(d + j * 8) = bf16x4{(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)0.f};
        }
      }
    }
  };

  // ---- frame-invariant lane geometry
  // dgrad B: class-grid column n = 32 cb + r32 -> dY2 pixel (a, b) (+ tap t: (t >> 1, t & 1)) and the taps that
  // stay on the grid (bit t); off-grid taps and padding columns read the zero pixel
  int dpb[4], dvm[4];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) {
    const int n = 32 * cb + r32, a = n / Wa, b = n - a * Wa;
    dpb[cb] = a * p.w + b;
    dvm[cb] = 0;
#pragma unroll
    for (int t = 0; t < 4; ++t)
      if (n < NA && a + (t >> 1) < p.h && b + (t & 1) < p.w) dvm[cb] |= 1 << t;
  }
  auto dpix = [&](int cb, int t) { return (dvm[cb] >> t) & 1 ? dpb[cb] + (t >> 1) * p.w + (t & 1) : kVbDN - 1; };
  // conv2 wgrad: k-row (pixel) -> the Y1 image offset of its window origin (pix / w by a 16-bit reciprocal:
  // exact for pix < 128, w < 128)
  const int rw16 = (65536 + p.w - 1) / p.w;
  auto ypo = [&](int pix) {
    pix = pix < P ? pix : 0;   // (A is zero past the grid: any finite B)
    const int y2 = (pix * rw16) >> 16, x2 = pix - y2 * p.w;
    return (2 * y2 * W1p + 2 * x2) * 64;
  };

  f32x16 acc2[2][4], acc1[2];
#pragma unroll
  for (int e = 0; e < 16; ++e) {
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc2[r][j][e] = 0.f;
    acc1[0][e] = acc1[1][e] = 0.f;
  }
  float bsum[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) bsum[i] = 0.f;
  const int py = wave >> 1, px = wave & 1;   // the wave's dgrad parity class

  int f = blockIdx.x;
  if (f < p.F) {
    dma_frame(f);
    fetch(f);
  }
  const __bf16* wa = p.WdT2 + (size_t)(32 * wave + r32) * 256 + 8 * hh;   // the dgrad's A rows (class = wave)
  for (; f < p.F; f += gridDim.x) {
    bf16x8 af[16];   // issued first: their (L2) latency hides under build()
    auto load_af = [&] {
#pragma unroll
      for (int s = 0; s < 16; ++s) af[s] = *reinterpret_cast<const bf16x8*>(wa + 16 * s);
    };
    load_af();
    build();   // the frame's RGBx image (xim free: the previous conv1 wgrad is done)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this frame's dY2 / Y1 DMA
    __syncthreads();

    // ---- conv2 dgrad (wave = parity class): D[32 c][class grid] = WdT2[class rows] x dY2 gather
    if constexpr (!(ABL & 1)) {
      f32x16 acc[4];
#pragma unroll
      for (int cb = 0; cb < 4; ++cb)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[cb][e] = 0.f;
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const int t = s >> 2, ch = 16 * (s & 3) + 8 * hh;
        bf16x8 bf[4];
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) bf[cb] = *reinterpret_cast<const bf16x8*>(dim + vb_dofs(dpix(cb, t), ch));
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) acc[cb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[s], bf[cb], acc[cb], 0, 0, 0);
      }
      // dY1 (class pixels) into the dY1 image in bf16 (the HBM path's rounding); the bias sums from fp32
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
        const int n = 32 * cb + r32, a = n / Wa, b = n - a * Wa, y1 = 2 * a + py, x1 = 2 * b + px;
        if (n < NA && y1 < p.H1 && x1 < p.W1) {
          const int p1 = y1 * p.W1 + x1;
#pragma unroll
          for (int g = 0; g < 4; ++g) {   // channels 8g + 4hh .. +3: one 8-B store
            const float v0 = acc[cb][4 * g], v1 = acc[cb][4 * g + 1], v2 = acc[cb][4 * g + 2], v3 = acc[cb][4 * g + 3];
            bsum[4 * g] += v0; bsum[4 * g + 1] += v1; bsum[4 * g + 2] += v2; bsum[4 * g + 3] += v3;
            *reinterpret_cast<bf16x4*>(tim + p1 * 64 + (8 * g + 4 * hh) * 2) =
                bf16x4{(__bf16)v0, (__bf16)v1, (__bf16)v2, (__bf16)v3};
          }
        }
      }
    }

    // ---- conv2 wgrad: gW2[64 o][tap 4w + j, ci] += sum_pixels dY2[pix][o] Y1[window(pix, tap)][ci]
#pragma unroll
    for (int s = 0; s < ((ABL & 2) ? 0 : 8); ++s) {
      bf16x8 a2[2], b2[4];
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) {   // A: rows o = 32 rb + (r32 & 16) + 4 tp .. +3 at pixels 16 s + 8 hh + tq (+4)
        const int o0 = 32 * rb + (r32 & 16) + 4 * tp, k0 = 16 * s + 8 * hh + tq;
        a2[rb] = vb_tr(dim, vb_dofs(k0, o0), vb_dofs(k0 + 4, o0));
      }
      const int y0 = ypo(16 * s + 8 * hh + tq), y1o = ypo(16 * s + 8 * hh + tq + 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) {   // B: rows ci = (r32 & 16) + 4 tp .. +3 of tap (ky, kx)
        const int tap = 4 * wave + j, ky = tap >> 2, kx = tap & 3;
        const int off = (ky * W1p + kx) * 64 + ((r32 & 16) + 4 * tp) * 2;
        b2[j] = vb_tr(yim, y0 + off, y1o + off);
      }
#pragma unroll
      for (int rb = 0; rb < 2; ++rb)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc2[rb][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2[rb], b2[j], acc2[rb][j], 0, 0, 0);
    }
    __syncthreads();   // the dY1 image complete; the dY2 and Y1 images are free

    const int fn = f + (int)gridDim.x;
    if (fn < p.F && !(ABL & 8)) {   // the next frame's loads land under conv1's weight gradient
      dma_frame(fn);
      fetch(fn);
    }

    // ---- conv1 wgrad: gW1[32 o][ky = 2w + j, kx, c] += sum_pixels dY1[pix][o] X[4 oy + ky][4 ox + kx][c]
    if constexpr (!(ABL & 4)) {
      int oy[2], ox[2];   // the k-rows' conv1 output pixels, advanced 16 per k step
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int pix = 8 * hh + tq + 4 * u;
        oy[u] = pix / p.W1;
        ox[u] = pix - oy[u] * p.W1;
      }
      // A: rows o = (r32 & 16) + 4 tp .. +3 of the dY1 image at the k-rows; B: the lane's RGBx piece,
      // kx = (r32 & 16) / 4 + tp, channels 0..3
      const int ao = 8 * hh * 64 + tq * 64 + ((r32 & 16) + 4 * tp) * 2;
      const int kxo = (((r32 & 16) >> 2) + tp) * 8;
      auto frags = [&](int s, bf16x8& a1, bf16x8 (&b1)[2]) {
        a1 = vb_tr(tim, ao + 16 * s * 64, ao + 16 * s * 64 + 4 * 64);
        int xo[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const bool ok = 16 * s + 8 * hh + tq + 4 * u < P1;   // past P1: the dY1 rows are zero, any finite B
          xo[u] = ok ? (4 * oy[u] * Wp + 4 * ox[u]) * 8 + kxo : kxo;
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) b1[j] = vb_tr(xim, xo[0] + (2 * wave + j) * Wp * 8, xo[1] + (2 * wave + j) * Wp * 8);
#pragma unroll
        for (int u = 0; u < 2; ++u) {   // k += 16: W1 > 16, so at most one row wrap
          ox[u] += 16;
          if (ox[u] >= p.W1) { ox[u] -= p.W1; ++oy[u]; }
        }
      };
      bf16x8 ac, bc[2];
      frags(0, ac, bc);
      for (int s = 0; s < KS1; ++s) {   // the next step's reads issued before this step's MFMAs
        bf16x8 an, bn[2];
        if (s + 1 < KS1) frags(s + 1, an, bn);
#pragma unroll
        for (int j = 0; j < 2; ++j) acc1[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ac, bc[j], acc1[j], 0, 0, 0);
        ac = an;
        bc[0] = bn[0];
        bc[1] = bn[1];
      }
    }
    __syncthreads();   // every wave is done with xim and the dY1 image
  }

  // ---- this workgroup's partials: gW2, gW1 (plain stores, disjoint per wave), conv1 bias
  float* pt = p.part + (size_t)blockIdx.x * kVbPart;
#pragma unroll
  for (int rb = 0; rb < 2; ++rb)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          pt[(32 * rb + 8 * g + 4 * hh + e) * 512 + 32 * (4 * wave + j) + r32] = acc2[rb][j][4 * g + e];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        pt[32768 + (8 * g + 4 * hh + e) * 256 + 32 * (2 * wave + j) + r32] = acc1[j][4 * g + e];
  float* red = reinterpret_cast<float*>(xim);   // (free: the loop ended on a barrier)
#pragma unroll
  for (int i = 0; i < 16; ++i) red[(wave * 64 + lane) * 16 + i] = bsum[i];
  __syncthreads();
  if (tid < 32) {   // channel c = 8 g + 4 hh + e: rows 4 g + e of the lanes with that hh, every class
    const int g = tid >> 3, h2 = (tid >> 2) & 1, e = tid & 3;
    float t = 0.f;
    for (int w = 0; w < 4; ++w)
      for (int l = 0; l < 32; ++l) t += red[(w * 64 + 32 * h2 + l) * 16 + 4 * g + e];
    pt[40960 + tid] = t;
  }
}

// Sum of the workgroups' partials into the packed gradients: 64 columns per block, each wave summing a
// quarter of the workgroups (8 loads in flight per lane), the quarters added in order (deterministic).
static __global__ void __launch_bounds__(256) k_vbwd_reduce(const float* __restrict__ part, int nwg, float* gW2,
                                                            float* gW1, float* gb1) {
  __shared__ float q4[4][64];
  const int lane = threadIdx.x & 63, qw = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + lane;
  const int k0 = (nwg * qw) / 4, k1 = (nwg * (qw + 1)) / 4;
  float s = 0.f;
  if (i < kVbPart) {
    int k = k0;
    for (; k + 8 <= k1; k += 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = part[(size_t)(k + u) * kVbPart + i];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; k < k1; ++k) s += part[(size_t)k * kVbPart + i];
  }
  q4[qw][lane] = s;
  __syncthreads();
  if (qw == 0 && i < kVbPart) {
    const float t = ((q4[0][lane] + q4[1][lane]) + q4[2][lane]) + q4[3][lane];
    if (i < 32768) gW2[i] += t;
    else if (i < 40960) gW1[i - 32768] += t;
    else gb1[i - 40960] += t;
  }
}

// Workgroups for F frames: at most one per CU and at least 8 frames each, so the partials (164 KB per
// workgroup) fit in the F frames' dY1 buffer (25.6 KB per frame at 84x84) the caller lends them.
inline int vbwd_groups(int F, int cus) { return std::max(1, std::min(cus, F / 8)); }

inline hipError_t vision_bwd_frames(const VisBwdParams& p, int cus, float* gW2, float* gW1, float* gb1,
                                    hipStream_t st) {
  if (!vbwd_fits(p.H, p.W, p.H1, p.W1, p.h, p.w) || p.F < 1) return hipErrorInvalidValue;
  const int nwg = vbwd_groups(p.F, cus);
#ifdef AAA_ABLATION
  const char* e = std::getenv("AAA_VBWD_ABL");
  switch (e ? std::atoi(e) : 0) {
#define AAA_VB_CASE(a) \
  case a: hipLaunchKernelGGL((k_vision_bwd_frames<a>), dim3(nwg), dim3(256), 0, st, p); break;
    AAA_VB_CASE(1) AAA_VB_CASE(2) AAA_VB_CASE(4) AAA_VB_CASE(8) AAA_VB_CASE(7) AAA_VB_CASE(6) AAA_VB_CASE(5) AAA_VB_CASE(3)
#undef AAA_VB_CASE
    default: hipLaunchKernelGGL((k_vision_bwd_frames<0>), dim3(nwg), dim3(256), 0, st, p);
  }
#else
  hipLaunchKernelGGL((k_vision_bwd_frames<0>), dim3(nwg), dim3(256), 0, st, p);
#endif
  hipLaunchKernelGGL(k_vbwd_reduce, dim3((kVbPart + 63) / 64), dim3(256), 0, st, p.part, nwg, gW2, gW1, gb1);
  return hipGetLastError();
}

}  // namespace aaa
