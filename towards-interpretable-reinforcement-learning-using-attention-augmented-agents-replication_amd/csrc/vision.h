// Frame-resident bf16 vision encoder forward (VisionNetwork.vision_cnn,
// attention.py:153-170, on X.transpose(1,3), :179): one workgroup runs a frame
// end to end -- the observation (uint8 or fp32 (H, W, 3)) into a zero-bordered
// RGBx bf16 image in LDS, conv1 (8x8 / 4, pad 1) from that image into a
// zero-bordered Y1 image in LDS, conv2 (4x4 / 2, pad 2) from it into the
// ConvLSTM operand slot -- and writes the bordered frame image (Xp) and Y1 to
// HBM only as the weight-gradient operands.  It replaces the three launches of
// the layered path (frames_rgbx, conv1, conv2: C3 107 + 221 + 125 us), whose
// im2col tiles re-read every frame pixel from L2 four (conv1) to sixteen times.
//
// Workgroups are persistent (one per CU, frames strided over the grid); the
// weights stay on chip for the whole launch (conv1's 32x256 as 16 fragments in
// LDS, conv2's 64x512 in registers, split by 32-row block: 32 fragments per
// wave), and the next frame's pixels are loaded while the current one computes.
// GEMMs (v_mfma_f32_32x32x16_bf16, fp32 accumulate):
//   conv1: D[32 ch][P1 px] = W1[32][256 = (ky*8+kx)*4 + c] x im2col(Xp): wave w
//          takes column blocks w, w+4, ...; a lane's B fragment (8 k = 2 taps x
//          4 channels) is one 16-B read of the RGBx image.
//   conv2: D[64 ch][P px] = W2[64][512 = (ky*4+kx)*32 + c] x im2col(Y1): wave w
//          takes row block w%2 over column blocks 2(w/2), 2(w/2)+1.
#pragma once
#include "glds.h"

namespace aaa {

constexpr int kVisXB = 59392;   // RGBx image bytes: (H+2)(W+2) x 8 B <= 58 KB (86 x 86 for 84x84 frames)
constexpr int kVisYP = 80;      // Y1 image pixel pitch (bytes): 32 bf16 + 16 B pad (conflict-free-ish gathers)
constexpr int kVisYB = 46080;   // Y1 image bytes: (H1+4)(W1+4) x 80 B (24 x 24 for 20x20)
constexpr int kVisNG = 7;       // 4-pixel groups per thread: H*W <= 7 x 256 x 4

struct VisFwdParams {
  const void* frames;   // (F, H, W, 3) uint8 or fp32
  const __bf16* Wc1;    // packed conv1 [32][256] (k_pack_conv1_rgbx)
  const float* b1;      // [32]
  const __bf16* Wc2;    // packed conv2 [64][512] (k_pack_conv)
  const float* b2;      // [64]
  __bf16* Xp;           // (F, H+2, W+2, 4) <- bordered RGBx frames (conv1's weight-gradient operand), or null
  __bf16* Y1;           // (F, H1*W1, 32) <- conv1 output
  __bf16* out;          // (F, h*w, out_ld) <- conv2 output, channels 0..63
  int out_ld, F, H, W, H1, W1, h, w;
};

// Whether a geometry runs on the frame-resident vision kernel.
inline bool vis_fits(int H, int W, int H1, int W1, int h, int w) {
  return (H + 2) * (W + 2) * 8 <= kVisXB && (H1 + 4) * (W1 + 4) * kVisYP <= kVisYB && W % 4 == 0 &&
         H * W <= kVisNG * 256 * 4 && H1 * W1 <= 16 * 32 && h * w <= 128;
}

template <typename TI>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) k_vision_fwd(VisFwdParams p) {
  __shared__ __attribute__((aligned(16))) unsigned char xim[kVisXB];
  __shared__ __attribute__((aligned(16))) unsigned char yim[kVisYB];
  __shared__ __attribute__((aligned(16))) bf16x8 w1s[16 * 64];   // conv1 weights, fragment order [ks][lane]
  __shared__ float sb[96];
  const int tid = (int)threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r32 = lane & 31, hh = lane >> 5;
  const int Wp = p.W + 2, W1p = p.W1 + 4;
  const int P1 = p.H1 * p.W1, P = p.h * p.w, NC1 = (P1 + 31) / 32, G4 = p.H * p.W / 4;

  {  // zero both images (their borders are never written), biases into LDS
    u32x4* z = reinterpret_cast<u32x4*>(xim);
    for (int i = tid; i < kVisXB / 16; i += 256) z[i] = u32x4{0u, 0u, 0u, 0u};
    z = reinterpret_cast<u32x4*>(yim);
    for (int i = tid; i < kVisYB / 16; i += 256) z[i] = u32x4{0u, 0u, 0u, 0u};
    if (tid < 32) sb[tid] = p.b1[tid];
    else if (tid < 96) sb[tid] = p.b2[tid - 32];
    // weight fragments: lane (r32, hh) of k step ks holds row r32 of its row block, k = 16 ks + 8 hh .. +7
    for (int i = tid; i < 16 * 64; i += 256) {
      const int ks = i >> 6, l = i & 63;
      w1s[i] = *reinterpret_cast<const bf16x8*>(p.Wc1 + (l & 31) * 256 + ks * 16 + (l >> 5) * 8);
    }
  }
  // conv2's weights stay in registers (its wave's 32-row block); conv1's are read from LDS
  bf16x8 a2[32];
  const int rb = wave & 1, cb2 = 2 * (wave >> 1);
#pragma unroll
  for (int ks = 0; ks < 32; ++ks)
    a2[ks] = *reinterpret_cast<const bf16x8*>(p.Wc2 + (32 * rb + r32) * 512 + ks * 16 + hh * 8);

  // the frame's pixels, 4 at a time (12 channel values: 3 dwords of uint8 or 3 x 16 B of fp32)
  constexpr int RW = sizeof(TI) == 1 ? 1 : 4;   // 4-byte words per 4 channel values
  uint32_t raw[kVisNG][3 * RW];
  auto fetch = [&](int f) {
    const uint32_t* src =
        reinterpret_cast<const uint32_t*>(reinterpret_cast<const TI*>(p.frames) + (size_t)f * p.H * p.W * 3);
#pragma unroll
    for (int i = 0; i < kVisNG; ++i) {   // unconditional (clamped) loads: no branch for the waits to gather at
      const int g = min(tid + 256 * i, G4 - 1);
      if constexpr (RW == 4) {
#pragma unroll
        for (int q = 0; q < 12; q += 4) {
          const u32x4 v = *reinterpret_cast<const u32x4*>(src + (size_t)g * 12 + q);
          raw[i][q] = v[0]; raw[i][q + 1] = v[1]; raw[i][q + 2] = v[2]; raw[i][q + 3] = v[3];
        }
      } else {
#pragma unroll
        for (int q = 0; q < 3; ++q) raw[i][q] = src[(size_t)g * 3 + q];
      }
    }
  };
  auto chan = [&](int i, int c) -> float {   // channel value c (0..11) of group i
    if constexpr (RW == 4) return __builtin_bit_cast(float, raw[i][c]);
    else return (float)((raw[i][c >> 2] >> (8 * (c & 3))) & 255u);
  };
  auto build = [&]() {   // the fetched group pixels into the RGBx image
#pragma unroll
    for (int i = 0; i < kVisNG; ++i) {
      const int g = tid + 256 * i;
      if (g < G4) {
        const int pix = 4 * g, y = pix / p.W, x = pix - y * p.W;
        unsigned char* d = xim + ((y + 1) * Wp + x + 1) * 8;
#pragma unroll
        for (int j = 0; j < 4; ++j)
          *reinterpret_cast<bf16x4*>(d + j * 8) =
              bf16x4{(__bf16)chan(i, 3 * j), (__bf16)chan(i, 3 * j + 1), (__bf16)chan(i, 3 * j + 2), (__bf16)0.f};
      }
    }
  };

  int f = blockIdx.x;
  if (f < p.F) fetch(f);
  __syncthreads();   // images zeroed, biases in
  for (; f < p.F; f += gridDim.x) {
    build();
    if (f + (int)gridDim.x < p.F) fetch(f + gridDim.x);   // next frame's pixels, under this one's convs
    barrier_lds();   // RGBx image complete (and the previous frame's conv2 done with the Y1 image); the
                     // next frame's loads stay in flight (no vmcnt drain, unlike __syncthreads)
    if (p.Xp) {        // the bordered frame for conv1's weight gradient
      u32x4* xo = reinterpret_cast<u32x4*>(p.Xp + (size_t)f * (p.H + 2) * Wp * 4);
      const int n = (p.H + 2) * Wp / 2;
      for (int i0 = 0; i0 < n; i0 += 1024) {   // 4 pieces in flight per thread
        u32x4 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = reinterpret_cast<const u32x4*>(xim)[min(i0 + tid + 256 * k, n - 1)];
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (i0 + tid + 256 * k < n) xo[i0 + tid + 256 * k] = v[k];
      }
    }
    // conv1 -> Y1 image (interior at +2, +2)
    for (int cb = wave; cb < NC1; cb += 4) {
      const int pp = min(cb * 32 + r32, P1 - 1), oy = pp / p.W1, ox = pp - oy * p.W1;
      const unsigned char* bb = xim + (4 * oy * Wp + 4 * ox) * 8 + hh * 16;
      int wl = lane;   // laundered: the A fragments are re-read per column block, not hoisted into 64 VGPRs
      asm volatile("" : "+v"(wl));
      f32x16 acc;
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[e] = 0.f;
#pragma unroll
      for (int k0 = 0; k0 < 16; k0 += 8) {   // 8 k steps of A and B fragments in flight
        bf16x8 a[8], b[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int ks = k0 + k;
          a[k] = w1s[ks * 64 + wl];
          b[k] = *reinterpret_cast<const bf16x8*>(bb + ((ks >> 1) * Wp + (ks & 1) * 4) * 8);
        }
        __builtin_amdgcn_sched_barrier(0);   // the 16 reads issue before the MFMAs (their latency overlaps)
#pragma unroll
        for (int k = 0; k < 8; ++k) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[k], b[k], acc, 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
      if (cb * 32 + r32 < P1) {
        unsigned char* yd = yim + ((oy + 2) * W1p + ox + 2) * kVisYP;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int c = 8 * g + 4 * hh;
          *reinterpret_cast<bf16x4*>(yd + c * 2) =
              bf16x4{(__bf16)(acc[4 * g] + sb[c]), (__bf16)(acc[4 * g + 1] + sb[c + 1]),
                     (__bf16)(acc[4 * g + 2] + sb[c + 2]), (__bf16)(acc[4 * g + 3] + sb[c + 3])};
        }
      }
    }
    barrier_lds();   // Y1 image complete
    {  // Y1 to HBM (conv2's weight-gradient operand): whole 64-B pixel rows
      u32x4* yo = reinterpret_cast<u32x4*>(p.Y1 + (size_t)f * P1 * 32);
      for (int i0 = 0; i0 < P1 * 4; i0 += 1024) {
        u32x4 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int i = min(i0 + tid + 256 * k, P1 * 4 - 1), pp = i >> 2, oy = pp / p.W1, ox = pp - oy * p.W1;
          v[k] = *reinterpret_cast<const u32x4*>(yim + ((oy + 2) * W1p + ox + 2) * kVisYP + (i & 3) * 16);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (i0 + tid + 256 * k < P1 * 4) yo[i0 + tid + 256 * k] = v[k];
      }
    }
    // conv2 -> the ConvLSTM operand slot
    f32x16 acc2[2];
    int yb[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
#pragma unroll
      for (int e = 0; e < 16; ++e) acc2[j][e] = 0.f;
      const int pp = min((cb2 + j) * 32 + r32, P - 1), y2 = pp / p.w, x2 = pp - y2 * p.w;
      yb[j] = (2 * y2 * W1p + 2 * x2) * kVisYP + hh * 16;
    }
#pragma unroll
    for (int k0 = 0; k0 < 32; k0 += 4) {   // 4 k steps x 2 column blocks of B fragments in flight
      bf16x8 b[4][2];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int ks = k0 + k, tap = ks >> 1, off = ((tap >> 2) * W1p + (tap & 3)) * kVisYP + (ks & 1) * 32;
#pragma unroll
        for (int j = 0; j < 2; ++j) b[k][j] = *reinterpret_cast<const bf16x8*>(yim + yb[j] + off);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc2[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2[k0 + k], b[k][j], acc2[j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int pp = (cb2 + j) * 32 + r32;
      if (pp < P) {
        __bf16* o = p.out + ((size_t)f * P + pp) * p.out_ld + 32 * rb;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int c = 8 * g + 4 * hh;
          const float* bz = sb + 32 + 32 * rb + c;
          *reinterpret_cast<bf16x4*>(o + c) =
              bf16x4{(__bf16)(acc2[j][4 * g] + bz[0]), (__bf16)(acc2[j][4 * g + 1] + bz[1]),
                     (__bf16)(acc2[j][4 * g + 2] + bz[2]), (__bf16)(acc2[j][4 * g + 3] + bz[3])};
        }
      }
    }
  }
}

template <typename TI>
inline hipError_t vision_fwd_frames(const VisFwdParams& p, int cus, hipStream_t st) {
  if (!vis_fits(p.H, p.W, p.H1, p.W1, p.h, p.w) || p.F < 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL((k_vision_fwd<TI>), dim3(std::min(p.F, cus)), dim3(256), 0, st, p);
  return hipGetLastError();
}

// Banded conv1 for frames too large for the frame-resident encoder (C5's
// 168x168): one workgroup per (frame, band of kBandRows conv1 output rows).
// It builds the band's 4*rows+4 padded-image rows as a zero-bordered RGBx bf16
// image in LDS straight from the observation (uint8 or fp32), writes the
// bordered rows it owns to Xp (conv1's weight-gradient operand; band b owns
// padded rows [4*y0, 4*(y0+rows)), the last band also the 4 below), and runs
// conv1 on the band from LDS exactly as k_vision_fwd does -- replacing the
// frames_rgbx pass and conv1's im2col GEMM, which re-read every pixel of the
// 740 MB bordered image four times through L2 (C5: 260 + 550 us).
constexpr int kBandRows = 8;        // conv1 output rows per band
constexpr int kBandXB = 50 * 1024;  // band image bytes: (4*kBandRows+4) rows x (W+2) x 8 B (36 x 170 x 8 = 48960)

struct VisBandParams {
  const void* frames;   // (F, H, W, 3) uint8 or fp32
  const __bf16* Wc1;    // packed conv1 [32][256]
  const float* b1;      // [32]
  __bf16* Xp;           // (F, H+2, W+2, 4) <- bordered RGBx rows 0 .. 4*H1+3, or null
  __bf16* Y1;           // (F, H1*W1, 32) <- conv1 output
  int F, H, W, H1, W1;
};

inline bool band_fits(int H, int W, int H1, int W1) {
  return (4 * kBandRows + 4) * (W + 2) * 8 <= kBandXB && 4 * H1 + 4 <= H + 2 && H1 >= 1 && W1 >= 1 && W % 4 == 0;
}

template <typename TI>
__global__ void __launch_bounds__(256) k_vision_conv1_band(VisBandParams p) {
  __shared__ __attribute__((aligned(16))) unsigned char xim[kBandXB];
  __shared__ __attribute__((aligned(16))) bf16x8 w1s[16 * 64];   // conv1 weights, fragment order [ks][lane]
  __shared__ float sb[32];
  const int tid = (int)threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r32 = lane & 31, hh = lane >> 5;
  const int nb = (p.H1 + kBandRows - 1) / kBandRows;
  const int f = (int)blockIdx.x / nb, band = (int)blockIdx.x - f * nb;
  const int y0 = band * kBandRows, ny = min(kBandRows, p.H1 - y0);
  const int Wp = p.W + 2, r0 = 4 * y0, nr = 4 * ny + 4;   // padded rows r0 .. r0+nr-1
  if (tid < 32) sb[tid] = p.b1[tid];
  for (int i = tid; i < 16 * 64; i += 256) {
    const int ks = i >> 6, l = i & 63;
    w1s[i] = *reinterpret_cast<const bf16x8*>(p.Wc1 + (l & 31) * 256 + ks * 16 + (l >> 5) * 8);
  }
  {  // the band image: padded pixel (r0 + rr, px) = frame pixel (r0 + rr - 1, px - 1), zero outside.
     // Border columns and rows outside the frame are zeroed; the interior goes in groups of 4
     // pixels (12 channel values: 3 dwords of uint8 or 3 x 16 B of fp32), every group's loads
     // of a batch issued before its stores (the fill is otherwise one latency per pixel).
    for (int i = tid; i < nr * Wp; i += 256) {
      const int rr = i / Wp, px = i - rr * Wp, iy = r0 + rr - 1;
      if ((unsigned)iy >= (unsigned)p.H || px == 0 || px == Wp - 1)
        *reinterpret_cast<uint2*>(xim + (size_t)i * 8) = uint2{0u, 0u};
    }
    constexpr int RW = sizeof(TI) == 1 ? 1 : 4;   // 4-byte words per 4 channel values
    constexpr int NG = 8;                          // groups per thread per batch
    const uint32_t* fr = reinterpret_cast<const uint32_t*>(reinterpret_cast<const TI*>(p.frames) +
                                                           (size_t)f * p.H * p.W * 3);
    const int G4 = p.W / 4, ry0 = max(r0 - 1, 0), ry1 = min(r0 + nr - 1, p.H);   // frame rows [ry0, ry1)
    const int ng = (ry1 - ry0) * G4;
    for (int g0 = 0; g0 < ng; g0 += 256 * NG) {
      uint32_t raw[NG][3 * RW];
#pragma unroll
      for (int k = 0; k < NG; ++k) {
        const int g = min(g0 + tid + 256 * k, ng - 1), iy = ry0 + g / G4, gx = g - (g / G4) * G4;
        const uint32_t* src = fr + ((size_t)iy * p.W + 4 * gx) * 3 * RW / 4;
#pragma unroll
        for (int q = 0; q < 3 * RW; ++q) raw[k][q] = src[q];
      }
#pragma unroll
      for (int k = 0; k < NG; ++k) {
        const int g = g0 + tid + 256 * k;
        if (g < ng) {
          const int iy = ry0 + g / G4, gx = g - (g / G4) * G4;
          unsigned char* d = xim + ((size_t)(iy + 1 - r0) * Wp + 4 * gx + 1) * 8;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            float v[3];
#pragma unroll
            for (int c = 0; c < 3; ++c) {
              const int e = 3 * j + c;
              if constexpr (RW == 4) v[c] = __builtin_bit_cast(float, raw[k][e]);
              else v[c] = (float)((raw[k][e >> 2] >> (8 * (e & 3))) & 255u);
            }
            *reinterpret_cast<bf16x4*>(d + j * 8) = bf16x4{(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)0.f};
          }
        }
      }
    }
  }
  __syncthreads();
  if (p.Xp) {  // the rows this band owns into Xp (16 B = 2 pixels per store)
    const int rows = 4 * ny + (y0 + ny == p.H1 ? 4 : 0);
    u32x4* xo = reinterpret_cast<u32x4*>(p.Xp + ((size_t)f * (p.H + 2) + r0) * Wp * 4);
    const int n = rows * Wp / 2;
    for (int i = tid; i < n; i += 256) xo[i] = reinterpret_cast<const u32x4*>(xim)[i];
  }
  // conv1 on the band: D[32 ch][ny*W1 px] = W1[32][256 = (ky*8+kx)*4 + c] x im2col(band)
  const int NP = ny * p.W1, NC = (NP + 31) / 32, P1 = p.H1 * p.W1;
  for (int cb = wave; cb < NC; cb += 4) {
    const int pp = min(cb * 32 + r32, NP - 1), oy = pp / p.W1, ox = pp - oy * p.W1;
    const unsigned char* bb = xim + (4 * oy * Wp + 4 * ox) * 8 + hh * 16;
    f32x16 acc;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = 0.f;
#pragma unroll
    for (int k0 = 0; k0 < 16; k0 += 8) {
      bf16x8 a[8], b[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int ks = k0 + k;
        a[k] = w1s[ks * 64 + lane];
        b[k] = *reinterpret_cast<const bf16x8*>(bb + ((ks >> 1) * Wp + (ks & 1) * 4) * 8);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[k], b[k], acc, 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (cb * 32 + r32 < NP) {
      __bf16* yd = p.Y1 + ((size_t)f * P1 + (size_t)(y0 + oy) * p.W1 + ox) * 32;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int c = 8 * g + 4 * hh;
        *reinterpret_cast<bf16x4*>(yd + c) =
            bf16x4{(__bf16)(acc[4 * g] + sb[c]), (__bf16)(acc[4 * g + 1] + sb[c + 1]),
                   (__bf16)(acc[4 * g + 2] + sb[c + 2]), (__bf16)(acc[4 * g + 3] + sb[c + 3])};
      }
    }
  }
}

template <typename TI>
inline hipError_t vision_conv1_band(const VisBandParams& p, hipStream_t st) {
  if (!band_fits(p.H, p.W, p.H1, p.W1) || p.F < 1) return hipErrorInvalidValue;
  const int nb = (p.H1 + kBandRows - 1) / kBandRows;
  hipLaunchKernelGGL((k_vision_conv1_band<TI>), dim3(p.F * nb), dim3(256), 0, st, p);
  return hipGetLastError();
}

// Banded conv2 (4x4, stride 2, pad 2) for the same frames: one workgroup per (frame, band of
// kBand2Rows conv2 output rows); the band's 2*rows+2 conv1 output rows are staged once as a
// zero-bordered bf16 image in LDS (pixel pitch kVisYP, interior at +2, +2) and all 16 taps read
// their B fragments from it -- the im2col ring GEMM gathered every Y1 pixel four times through L2.
// Waves: row block wave % 2 (32 of the 64 channels, weights in registers), column blocks
// wave / 2, wave / 2 + 2, ...
constexpr int kBand2Rows = 8;
constexpr int kBand2YB = 72 * 1024;   // (2*kBand2Rows+2) rows x (W1+4) x kVisYP bytes (18 x 45 x 80 = 64800)

struct VisBand2Params {
  const __bf16* Y1;     // (F, H1*W1, 32)
  const __bf16* Wc2;    // packed conv2 [64][512]
  const float* b2;      // [64]
  __bf16* out;          // (F, h*w, out_ld), channels 0..63
  int out_ld, F, H1, W1, h, w;
};

inline bool band2_fits(int H1, int W1, int h, int w) {
  return (2 * kBand2Rows + 2) * (W1 + 4) * kVisYP <= kBand2YB && h >= 1 && w >= 1 && 2 * (h - 1) + 1 <= H1 + 1;
}

static __global__ void __launch_bounds__(256) k_vision_conv2_band(VisBand2Params p) {
  __shared__ __attribute__((aligned(16))) unsigned char yim[kBand2YB];
  __shared__ float sb[64];
  const int tid = (int)threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r32 = lane & 31, hh = lane >> 5;
  const int nb = (p.h + kBand2Rows - 1) / kBand2Rows;
  const int f = (int)blockIdx.x / nb, band = (int)blockIdx.x - f * nb;
  const int o0 = band * kBand2Rows, n2 = min(kBand2Rows, p.h - o0);
  const int W1p = p.W1 + 4, nr = 2 * n2 + 2, iy0 = 2 * o0 - 2, P1 = p.H1 * p.W1;
  const int rb = wave & 1;
  bf16x8 a2[32];   // this wave's 32-row block of the conv2 weights, all 32 k steps
#pragma unroll
  for (int ks = 0; ks < 32; ++ks)
    a2[ks] = *reinterpret_cast<const bf16x8*>(p.Wc2 + (32 * rb + r32) * 512 + ks * 16 + hh * 8);
  if (tid < 64) sb[tid] = p.b2[tid];
  {  // the band's Y1 rows iy0 .. iy0+nr-1 (zero outside the map), 16-B pieces, 4 per pixel
    const u32x4* src = reinterpret_cast<const u32x4*>(p.Y1 + (size_t)f * P1 * 32);
    const int n = nr * W1p * 4;
    constexpr int NB2 = 16;   // pieces in flight per thread (a C5 band is ~13 per thread: one batch)
    for (int i0 = 0; i0 < n; i0 += 256 * NB2) {
      u32x4 v[NB2];
#pragma unroll
      for (int k = 0; k < NB2; ++k) {
        const int i = i0 + tid + 256 * k, px = i >> 2, br = px / W1p, bc = px - br * W1p;
        const int iy = iy0 + br, ix = bc - 2;
        const bool ok = i < n && (unsigned)iy < (unsigned)p.H1 && (unsigned)ix < (unsigned)p.W1;
        v[k] = ok ? src[((size_t)iy * p.W1 + ix) * 4 + (i & 3)] : u32x4{0u, 0u, 0u, 0u};
      }
#pragma unroll
      for (int k = 0; k < NB2; ++k) {
        const int i = i0 + tid + 256 * k;
        if (i < n) *reinterpret_cast<u32x4*>(yim + (i >> 2) * kVisYP + (i & 3) * 16) = v[k];
      }
    }
  }
  __syncthreads();
  const int NP = n2 * p.w, NC = (NP + 31) / 32;
  for (int cb = wave >> 1; cb < NC; cb += 2) {
    const int pp = min(cb * 32 + r32, NP - 1), y2 = pp / p.w, x2 = pp - y2 * p.w;
    // output (o0 + y2, x2) reads Y1 rows 2(o0+y2)-2+ky = iy0 + 2 y2 + ky: band row 2 y2 + ky, column 2 x2 + kx
    const unsigned char* yb = yim + (2 * y2 * W1p + 2 * x2) * kVisYP + hh * 16;
    f32x16 acc;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = 0.f;
#pragma unroll
    for (int k0 = 0; k0 < 32; k0 += 8) {
      bf16x8 b[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int ks = k0 + k, tap = ks >> 1;
        b[k] = *reinterpret_cast<const bf16x8*>(yb + ((tap >> 2) * W1p + (tap & 3)) * kVisYP + (ks & 1) * 32);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2[k0 + k], b[k], acc, 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (cb * 32 + r32 < NP) {
      __bf16* o = p.out + ((size_t)f * p.h * p.w + (size_t)(o0 + y2) * p.w + x2) * p.out_ld + 32 * rb;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int c = 8 * g + 4 * hh;
        const float* bz = sb + 32 * rb + c;
        *reinterpret_cast<bf16x4*>(o + c) = bf16x4{(__bf16)(acc[4 * g] + bz[0]), (__bf16)(acc[4 * g + 1] + bz[1]),
                                                   (__bf16)(acc[4 * g + 2] + bz[2]), (__bf16)(acc[4 * g + 3] + bz[3])};
      }
    }
  }
}

inline hipError_t vision_conv2_band(const VisBand2Params& p, hipStream_t st) {
  if (!band2_fits(p.H1, p.W1, p.h, p.w) || p.F < 1) return hipErrorInvalidValue;
  const int nb = (p.h + kBand2Rows - 1) / kBand2Rows;
  hipLaunchKernelGGL(k_vision_conv2_band, dim3(p.F * nb), dim3(256), 0, st, p);
  return hipGetLastError();
}

}  // namespace aaa
