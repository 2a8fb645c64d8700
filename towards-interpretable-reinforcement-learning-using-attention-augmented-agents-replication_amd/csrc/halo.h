// 3x3, stride-1, pad-1 convolutions over the ConvLSTM's small grids (11x11 at
// 84x84 frames) as an implicit GEMM whose pixel operand is staged ONCE per
// channel chunk as a zero-bordered LDS "halo" image of FR whole frames and
// then read by all nine taps:
//
//   D[i][j] = sum_{tap, c} W[i][tap*Cin + c] * X[frame(j)][pixel(j) + off(tap)][c]
//
// off(tap) = (ky-1, kx-1) for the forward gather, (1-ky, 1-kx) for the dgrad
// (transposed) gather; rows i are output channels (gate-interleaved for the
// ConvLSTM), columns j output pixels, frame-major, so a tile of FR frames is a
// contiguous column range and the epilogues of glds.h apply unchanged.
//
// Why: the im2col ring of glds.h fetches every input pixel nine times through
// L2 and issues one LDS-DMA piece per 1 KiB -- for bf16 MFMAs that DMA issue
// and L2 traffic, not the matrix pipe, set the pace.  Here the pixel operand
// costs one DMA pass per channel chunk and only the weight tile streams per
// tap (ring of NBUF = 3 stages, one tap in flight across every barrier).
//
// LDS images are lane-linear (LDS-DMA writes base + lane*16); the XOR swizzle
// that keeps the fragment reads conflict-free is applied on the source side:
// physical 16-B slot pc of halo row R holds logical chunk pc ^ halo_swz(R),
// and the weight tile uses lds_swz as in glds.h.  Halo rows outside the frame
// (the zero border) and beyond the tile's frames read through the buffer
// descriptor's range check and land as zeros.
#pragma once
#include "glds.h"

namespace aaa {

// Halo tile geometry: FR frames of h x w output pixels (h, w <= GH, GW at compile time).
template <typename T, int BI_, int BJ_, int CK_, int WI_, int WJ_, int FR_, int HMAX_>
struct HaloCfg {
  using type = T;
  static constexpr int BI = BI_, BJ = BJ_, CK = CK_, WI = WI_, WJ = WJ_, WK = 1, FR = FR_;
  static constexpr int NT = WI * WJ * 64;
  static constexpr int BK = CK;                   // one tap x one channel chunk per K step
  static constexpr int HMAX = HMAX_;              // halo rows (>= FR*(h+2)*(w+2) + 1 zero row)
};

// fp32 at fp32 accuracy on the bf16 MFMA (gemm.h SPLIT6): three-way split operands, six products
template <int BI_, int BJ_, int CK_, int WI_, int WJ_, int FR_, int HMAX_>
struct HaloCfgS6 : HaloCfg<float, BI_, BJ_, CK_, WI_, WJ_, FR_, HMAX_> {
  static constexpr bool SPLIT3 = true, SPLIT6 = true;
};

struct HaloParams {
  const void* wt;       // weights [Mi][9*Cin] (row stride ldw elements), tap-major k
  int ldw, Mi;
  const void* x;        // pixels [F*P][cs] (element stride cs), channels coff .. coff+Cin
  int cs, coff, Cin;
  uint32_t x_bytes;     // buffer range of x
  int h, w, nframes;
  int transposed;       // dgrad gather
  int oh, ow;           // output grid per frame (0: the input grid); KS = 2 convs only
};

// The halo rows a ds_read_b128 lane group (16 lanes, one 256-B bank row) reads
// are 16 mostly-consecutive pixels; with 128-B bf16 rows two of them share a
// bank row, so the XOR must rotate per PAIR of rows ((R/2) & 7, i.e. lds_swz)
// for the 16 reads to land on 16 distinct 16-B slots.  (R & 7 leaves every
// group at least 2-way conflicted: 50.7 % SQ_LDS_BANK_CONFLICT at C3.)
template <int RS>
__device__ __forceinline__ int halo_swz(int row) { return lds_swz<RS>(row); }

// KS = 3: the 3x3 / pad-1 conv above.  KS = 2: a 2x2 stride-1 conv whose
// output (a, b) on an oh x ow grid reads input pixels (a + ky, b + kx), rows
// past the input grid reading the zero border -- conv2's dgrad classes
// (runtime.hip conv2_dgrad: all four parity classes share this gather).
template <class C, class EP, int NBUF = 3, int KS = 3>
__global__ void __launch_bounds__(C::NT) conv3_halo_kernel(HaloParams p, EP ep, TileMap tm) {
  using T = typename C::type;
  constexpr int BI = C::BI, BJ = C::BJ, CK = C::CK, WI = C::WI, WJ = C::WJ, NT = C::NT;
  constexpr int WTI = BI / WI, WTJ = BJ / WJ, MI = WTI / 32, MJ = WTJ / 32;
  constexpr int VG = 16 / (int)sizeof(T);
  constexpr int RS = CK / VG;                       // 16-B slots per row (halo and weight tile)
  constexpr int AEL = BI * CK;                      // weight tile elements
  constexpr int HEL = C::HMAX * CK;                 // halo image elements
  constexpr int PA = BI * RS / NT;                  // weight DMA pieces per wave per step
  constexpr int PH = C::HMAX * RS / NT;             // halo DMA pieces per wave per chunk
  static_assert(MI >= 1 && MJ >= 1 && CK % 16 == 0, "tile shape");
  static_assert((BI * RS) % NT == 0 && (C::HMAX * RS) % NT == 0, "every wave must issue the same number of DMA pieces");
  constexpr int ELD = BI + 4;
  constexpr int EPI_T = (int)((BJ / epi_chunks<C>() * ELD * sizeof(float) + sizeof(T) - 1) / sizeof(T));
  constexpr int RING = NBUF * AEL + 2 * HEL;
  __shared__ __attribute__((aligned(16))) T smem[RING > EPI_T ? RING : EPI_T];
  static_assert(!has_acc<EP>::value || NT * 16 * sizeof(float) <= sizeof(smem), "accumulator reduction");
  T* const As = smem;                               // NBUF weight stages
  T* const Hs = smem + NBUF * AEL;                  // two halo images

  int ti, tj, tz;
  tile_of(tm, ti, tj, tz);
  constexpr int NTAP = KS * KS;
  const int P = p.h * p.w, Hp = p.h + 2, Wp = p.w + 2, HP = Hp * Wp;
  const int ow = KS == 2 && p.ow ? p.ow : p.w, PO = KS == 2 && p.oh ? p.oh * ow : P;   // output grid
  const int i0 = ti * BI, f0 = tj * C::FR, j0 = f0 * PO;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wi = wave / WJ, wj = wave - wi * WJ;
  const int r32 = lane & 31, hh = lane >> 5;

  // ---- weight tile DMA: rows i0.., k = tap*Cin + c0 + logical chunk
  const __amdgpu_buffer_rsrc_t wr = make_rsrc(p.wt, (uint32_t)((size_t)p.Mi * p.ldw * sizeof(T)));
  uint32_t avoff[PA];
#pragma unroll
  for (int c = 0; c < PA; ++c) {
    const int ch = threadIdx.x + c * NT, lr = ch / RS, lc = (ch % RS) ^ lds_swz<RS>(lr), row = i0 + lr;
    avoff[c] = row < p.Mi ? (uint32_t)((row * p.ldw + lc * VG) * (int)sizeof(T)) : kOOB;
  }
  const int wofs = __builtin_amdgcn_readfirstlane((int)(threadIdx.x & ~63u) * VG);
  auto issue_a = [&](int step, int cc) {         // step = chunk*NTAP + tap
    const int tap = step - NTAP * cc;
    const int ko = __builtin_amdgcn_readfirstlane((tap * p.Cin + cc * CK) * (int)sizeof(T));
    T* dst = As + (step % NBUF) * AEL;
#pragma unroll
    for (int c = 0; c < PA; ++c) dma16a(wr, dst + c * NT * VG + wofs, avoff[c], ko);
  };
  // ---- halo DMA: halo row R = (frame fl, padded y, padded x); border / absent frames -> zeros
  const __amdgpu_buffer_rsrc_t xr = make_rsrc(p.x, p.x_bytes);
  uint32_t hvoff[PH];
#pragma unroll
  for (int c = 0; c < PH; ++c) {
    const int ch = threadIdx.x + c * NT, R = ch / RS, lc = (ch % RS) ^ halo_swz<RS>(R);
    const int fl = R / HP, rr = R - fl * HP, py = rr / Wp, px = rr - py * Wp;
    const int y = py - 1, xx = px - 1, f = f0 + fl;
    const bool ok = fl < C::FR && f < p.nframes && y >= 0 && y < p.h && xx >= 0 && xx < p.w;
    hvoff[c] = ok ? (uint32_t)(((size_t)(f * P + y * p.w + xx) * p.cs + p.coff + lc * VG) * sizeof(T)) : kOOB;
  }
  auto issue_h = [&](int cc) {
    const int co = __builtin_amdgcn_readfirstlane(cc * CK * (int)sizeof(T));
    T* dst = Hs + (cc & 1) * HEL;
#pragma unroll
    for (int c = 0; c < PH; ++c) dma16a(xr, dst + c * NT * VG + wofs, hvoff[c], co);
  };
  // ---- per-lane halo row of each B column block (tap (1,1)); padding columns read the zero row
  int hrow[MJ];
#pragma unroll
  for (int b = 0; b < MJ; ++b) {
    const int j = wj * WTJ + b * 32 + r32;          // tile-local output pixel
    const int fl = j / PO, q = j - fl * PO, y = q / ow, xx = q - y * ow;
    hrow[b] = j < C::FR * PO ? fl * HP + (y + 1) * Wp + (xx + 1) : C::HMAX - 1;
  }
  const int sg = p.transposed ? -1 : 1;

  f32x16 acc[MI][MJ];
#pragma unroll
  for (int a = 0; a < MI; ++a)
#pragma unroll
    for (int b = 0; b < MJ; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.f;

  using PL = EpiPlan<C, EP, has_pre<EP>::value>;
  typename PL::PreT pre[PL::PD];
  const int jn = min(C::FR, p.nframes - f0) * PO;   // valid tile columns (whole frames)
  epilogue_prefetch<C, EP, PL>(ep, i0, j0, jn, pre);

  const int nc = p.Cin / CK, ns = NTAP * nc;
  issue_h(0);
#pragma unroll
  for (int s = 0; s < NBUF - 1; ++s)
    if (s < ns) issue_a(s, s / NTAP);

  for (int s = 0; s < ns; ++s) {
    const int cc = s / NTAP, tap = s - NTAP * cc;
    // A(s) is the oldest weight stage in flight; the next chunk's halo, issued
    // at this chunk's first step right after A(9cc+NBUF-1), is younger than
    // A(s) for the steps 9cc+1 .. 9cc+NBUF-1 (it must not be waited for there).
    const bool h_younger = cc + 1 < nc && tap >= 1 && tap <= NBUF - 1;
    if (s + NBUF - 2 < ns) {
      if (h_younger) wait_vmcnt<PA * (NBUF - 2) + PH>();
      else wait_vmcnt<PA * (NBUF - 2)>();
    } else {
      wait_vmcnt<0>();
    }
    barrier_lds();
    if (s + NBUF - 1 < ns) issue_a(s + NBUF - 1, (s + NBUF - 1) / NTAP);
    if (tap == 0 && cc + 1 < nc) issue_h(cc + 1);
    const T* Ac = As + (s % NBUF) * AEL;
    const T* Hc = Hs + (cc & 1) * HEL;
    const int ky = tap / KS, kx = tap - KS * ky;
    const int toff = KS == 3 ? sg * ((ky - 1) * Wp + (kx - 1)) : ky * Wp + kx;
#pragma unroll
    for (int s2 = 0; s2 < CK / 16; ++s2) {
      const int kofs = 16 * s2 + 8 * hh;
      if constexpr (is_f32<T>::value) {
        float af[MI][8], bfr[MJ][8];
#pragma unroll
        for (int a = 0; a < MI; ++a) frag_sw<CK>(Ac, wi * WTI + a * 32 + r32, kofs, af[a]);
#pragma unroll
        for (int b = 0; b < MJ; ++b) {
          const int R = hrow[b] + toff, g = halo_swz<RS>(R), c0 = kofs >> 2;
          const f32x4 x = *reinterpret_cast<const f32x4*>(Hc + R * CK + ((c0 ^ g) << 2));
          const f32x4 y = *reinterpret_cast<const f32x4*>(Hc + R * CK + (((c0 + 1) ^ g) << 2));
          bfr[b][0] = x[0]; bfr[b][1] = x[1]; bfr[b][2] = x[2]; bfr[b][3] = x[3];
          bfr[b][4] = y[0]; bfr[b][5] = y[1]; bfr[b][6] = y[2]; bfr[b][7] = y[3];
        }
        if constexpr (split6_of<C>::value) {
          bf16x8 ah[MI], am[MI], al[MI], bh[MJ], bm[MJ], bl[MJ];
#pragma unroll
          for (int a = 0; a < MI; ++a) split3_bf16(af[a], ah[a], am[a], al[a]);
#pragma unroll
          for (int b = 0; b < MJ; ++b) split3_bf16(bfr[b], bh[b], bm[b], bl[b]);
#pragma unroll
          for (int a = 0; a < MI; ++a)
#pragma unroll
            for (int b = 0; b < MJ; ++b) {
              acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[a], bh[b], acc[a][b], 0, 0, 0);
              acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[a], bl[b], acc[a][b], 0, 0, 0);
              acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am[a], bm[b], acc[a][b], 0, 0, 0);
              acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am[a], bh[b], acc[a][b], 0, 0, 0);
              acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[a], bm[b], acc[a][b], 0, 0, 0);
              acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[a], bh[b], acc[a][b], 0, 0, 0);
            }
        } else {
#pragma unroll
          for (int kk = 0; kk < 8; ++kk)
#pragma unroll
            for (int a = 0; a < MI; ++a)
#pragma unroll
              for (int b = 0; b < MJ; ++b)
                acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[a][kk], bfr[b][kk], acc[a][b], 0, 0, 0);
        }
      } else {
        bf16x8 af[MI], bfr[MJ];
#pragma unroll
        for (int a = 0; a < MI; ++a) af[a] = frag_sw<CK>(Ac, wi * WTI + a * 32 + r32, kofs);
#pragma unroll
        for (int b = 0; b < MJ; ++b) {
          const int R = hrow[b] + toff;
          bfr[b] = *reinterpret_cast<const bf16x8*>(Hc + R * CK + (((kofs >> 3) ^ halo_swz<RS>(R)) << 3));
        }
#pragma unroll
        for (int a = 0; a < MI; ++a)
#pragma unroll
          for (int b = 0; b < MJ; ++b)
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[a], bfr[b], acc[a][b], 0, 0, 0);
      }
    }
  }
  staged_epilogue<C, EP, PL>(ep, smem, acc, i0, j0, jn, tj, pre);
}

// Whether an h x w grid with Cin channels fits tile config C.
template <class C>
inline bool halo_fits(int h, int w, int Cin) {
  return C::FR * h * w <= C::BJ && C::FR * (h + 2) * (w + 2) + 1 <= C::HMAX && Cin % C::CK == 0 && Cin >= C::CK;
}

// Host launcher: Mi output rows, nframes frames of h x w pixels.  Returns
// hipErrorInvalidValue when the geometry does not fit the compile-time tile.
template <class C, class EP, int KS = 3, int NBUF = 3>
inline hipError_t launch_halo(const HaloParams& p, const EP& ep, hipStream_t st) {
  const int Hp = p.h + 2, Wp = p.w + 2;
  const int PO = KS == 2 && p.oh ? p.oh * p.ow : p.h * p.w;
  if (p.Mi <= 0 || p.nframes <= 0) return hipSuccess;
  if (C::FR * PO > C::BJ || C::FR * Hp * Wp + 1 > C::HMAX || p.Cin % C::CK || p.Cin < C::CK)
    return hipErrorInvalidValue;
  if (KS == 2 && p.oh && (p.oh > p.h || p.ow > p.w)) return hipErrorInvalidValue;
  if ((size_t)p.nframes * p.h * p.w * p.cs * sizeof(typename C::type) > 0x7fffffffu) return hipErrorInvalidValue;
  dim3 grid((p.nframes + C::FR - 1) / C::FR, (p.Mi + C::BI - 1) / C::BI, 1);
  hipLaunchKernelGGL((conv3_halo_kernel<C, EP, NBUF, KS>), grid, dim3(C::NT), 0, st, p, ep, tile_map(grid));
  return hipGetLastError();
}

}  // namespace aaa
