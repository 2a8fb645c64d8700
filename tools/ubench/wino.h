// Winograd F(2x2, 3x3) engine for the fp32 ConvLSTM convolutions (3x3,
// stride 1, pad 1 on the h x w grid): the batched x-part, the recurrent h-part
// step, the BPTT dh step and the batched dx (attention.py:110-126 and its
// autograd).  Lavin & Gray 2016, correlation form:
//
//   Y(2x2 tile) = A^T [ (G g G^T) (.) (B^T d B) ] A,   d = the tile's 4x4 input patch
//   G = [1 0 0; .5 .5 .5; .5 -.5 .5; 0 0 1]
//   B^T = [1 0 -1 0; 0 1 1 0; 0 -1 1 0; 0 1 0 -1],  A^T = [1 1 1 0; 0 1 -1 -1]
//
// The 16 Winograd-domain products are 16 independent GEMMs
//   M_e[row][tile] = sum_c U_e[row][c] * V_e[c][tile],   e = 4a + b,
// 4 multiplies per output pixel instead of 9 (1.89x fewer on the 11x11 grid,
// whose 6x6 tiles cover 12x12).  U (the transformed weights, [16][rows][K]) is
// packed once per weight update (k_pack_wino); V is transformed on the fly from
// the raw 4x4 input patches when the fragments are read out of LDS.  Every wave owns ALL 16 e of its
// (rows x 16 tiles) output block, so the inverse transform is lane-local: the
// v_mfma_f32_16x16x4_f32 accumulator gives a lane 4 consecutive rows (one
// channel's 4 gates, row = 4*ch + gate) of one tile column for every e.
//
// Operands are exact fp32 (the MFMA is an fmaf chain); the transforms add a few
// roundings (B^T d B: sums of 4 inputs with +-1; A^T M A: sums of 9), which the
// 1e-4 parity tolerance absorbs (tools/ubench/wino.hip checks each launch against the direct kernel).
//
// k ordering: a lane group q = lane/16 reads BK/4 consecutive k of a BK-slice
// (b64 at BK = 8, b128 at BK = 16) and MFMA s takes its component s, i.e. MFMA s
// sums k = (BK/4) q + s over q: the slice is covered in a permuted order, which
// a sum over k does not see.
#pragma once
#include <type_traits>
#include "glds.h"

namespace aaa {

struct WinoGeo {
  int H, W;            // grid (output grid = input grid)
  int TW, TP;          // tiles per row = ceil(W/2), tiles per frame
  int ntiles;          // frames x TP
  int cs, coff;        // input pixel stride and first channel (floats)
  uint32_t src_bytes;  // bytes of the input the descriptor may address
  FastDiv dTP, dTW;
};

inline WinoGeo wino_geo(int H, int W, int frames, int cs, int coff, size_t src_bytes) {
  WinoGeo g;
  g.H = H; g.W = W;
  g.TW = (W + 1) / 2;
  g.TP = ((H + 1) / 2) * g.TW;
  g.ntiles = frames * g.TP;
  g.cs = cs; g.coff = coff;
  g.src_bytes = (uint32_t)src_bytes;
  g.dTP = FastDiv((uint32_t)g.TP);
  g.dTW = FastDiv((uint32_t)g.TW);
  return g;
}

// Wave tile WTI rows x 16 tiles (x 16 e); WI x WJ waves tile the workgroup,
// WK wave groups split each stage's K (intra-workgroup split-K, partial
// outputs summed in the epilogue).  BK = channels per wave group per stage.
template <int WTI_, int WI_, int WJ_, int WK_, int BK_>
struct WinoCfg {
  static constexpr int WTI = WTI_, WI = WI_, WJ = WJ_, WK = WK_, BK = BK_;
  static constexpr int BI = WTI * WI, BJ = 16 * WJ, NT = 64 * WI * WJ * WK;
  static constexpr int MB = WTI / 16;   // 16-row MFMA blocks per wave
  static constexpr int KS = BK * WK;    // channels per stage
  static_assert(WTI % 16 == 0 && (BK == 8 || BK == 16), "wave tile / stage depth");
};

// 4x4 input patch -> V = B^T d B (in place order: v[4a + b]).
__device__ __forceinline__ void wino_in(const float (&d)[16], float (&v)[16]) {
  float t[16];
#pragma unroll
  for (int s = 0; s < 4; ++s) {   // rows: B^T along the patch's row index
    t[0 * 4 + s] = d[0 * 4 + s] - d[2 * 4 + s];
    t[1 * 4 + s] = d[1 * 4 + s] + d[2 * 4 + s];
    t[2 * 4 + s] = d[2 * 4 + s] - d[1 * 4 + s];
    t[3 * 4 + s] = d[1 * 4 + s] - d[3 * 4 + s];
  }
#pragma unroll
  for (int a = 0; a < 4; ++a) {   // columns
    v[a * 4 + 0] = t[a * 4 + 0] - t[a * 4 + 2];
    v[a * 4 + 1] = t[a * 4 + 1] + t[a * 4 + 2];
    v[a * 4 + 2] = t[a * 4 + 2] - t[a * 4 + 1];
    v[a * 4 + 3] = t[a * 4 + 1] - t[a * 4 + 3];
  }
}

// Winograd-domain 4x4 -> 2x2 outputs y[2i + j] = (A^T M A)[i][j].
__device__ __forceinline__ void wino_out(const float (&m)[16], float (&y)[4]) {
  float u[8];
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    u[a * 2 + 0] = m[a * 4 + 0] + m[a * 4 + 1] + m[a * 4 + 2];
    u[a * 2 + 1] = m[a * 4 + 1] - m[a * 4 + 2] - m[a * 4 + 3];
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    y[0 * 2 + j] = u[0 * 2 + j] + u[1 * 2 + j] + u[2 * 2 + j];
    y[1 * 2 + j] = u[1 * 2 + j] - u[2 * 2 + j] - u[3 * 2 + j];
  }
}

// Transformed weights U[e][row][k] (A) and raw input patches (B) go global ->
// LDS through the LDS-DMA ring of glds.h (NBUF stages, counted vmcnt, one
// barrier per stage).  Per k-wave group a stage holds
//   A: [16 e][BI rows][BK]  -- row = BK floats (RS 16-B slots), slot XOR lds_swz<RS>(row)
//   B: [BJ tiles][16 taps][BK] -- the tile's 4x4 input patch (tap = 4r + s), slot XOR (tile & 15)
// and the B fragment is transformed at read time: a lane reads its tile's 16
// taps for its BK/4 channels and computes V = B^T d B for all 16 e at once.
// ABL (diagnostic builds only, tools/ubench/wino): bit 0 = no B transform
// (raw taps used as V), bit 1 = no MFMA, bit 2 = no LDS fragment reads.
template <class C, class EP, int NBUF, int ABL = 0>
__global__ void __launch_bounds__(C::NT)
wino_kernel(const float* __restrict__ U, int ldu, int urows, int urow0, int uoff, const float* __restrict__ X,
            WinoGeo g, EP ep, int Mi, int K, TileMap tm) {
  constexpr int BI = C::BI, BJ = C::BJ, BK = C::BK, WK = C::WK, NT = C::NT, MB = C::MB, WTI = C::WTI;
  constexpr int RS = BK / 4, KL = BK / 4;       // 16-B slots per row / k values per lane
  constexpr int AEL = 16 * BI * BK;             // floats of A per k-wave group and stage
  constexpr int BEL = 16 * BJ * BK;             // floats of B
  constexpr int GEL = AEL + BEL, STG = WK * GEL;
  constexpr int XA = AEL / 4, XB = BEL / 4;     // 16-B pieces per group
  static_assert(XA % NT == 0 && XB % NT == 0, "every wave issues the same DMA count, one group per piece index");
  constexpr int APER = WK * XA / NT, BPER = WK * XB / NT, PIECES = APER + BPER;
  constexpr int ELD = BI + 4;                   // epilogue pitch (pad: conflict-free b128 writes)
  constexpr int EPI = WK * 4 * BJ * ELD;
  constexpr int SM = NBUF * STG > EPI ? NBUF * STG : EPI;
  constexpr bool ACC = has_acc<EP>::value;
  static_assert(!ACC || NT * 16 <= SM, "accumulator reduction does not fit in LDS");
  __shared__ __attribute__((aligned(16))) float smem[SM];

  int ti, tj, tz;
  tile_of(tm, ti, tj, tz);
  const int i0 = ti * BI, j0 = tj * BJ;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wk = wave / (C::WI * C::WJ), wr = wave - wk * (C::WI * C::WJ);
  const int wi = wr / C::WJ, wj = wr - wi * C::WJ;
  const int l16 = lane & 15, q = lane >> 4;
  const int wofs = __builtin_amdgcn_readfirstlane((int)(tid & ~63) * 4);

  // ---- DMA piece offsets (fixed along K; the stage's k0 goes in soffset)
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(U, (uint32_t)((size_t)16 * urows * ldu * 4));
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(X, g.src_bytes);
  uint32_t avo[APER], bvo[BPER];
#pragma unroll
  for (int c = 0; c < APER; ++c) {
    const int ch = c * NT + tid, kw = ch / XA, rem = ch - kw * XA;
    const int row16 = rem / RS, e = row16 / BI, r = row16 - e * BI;
    const int ls = (rem % RS) ^ lds_swz<RS>(r);
    avo[c] = i0 + r < Mi ? (uint32_t)(((e * urows + urow0 + i0 + r) * ldu + uoff + kw * BK + ls * 4) * 4) : kOOB;
  }
#pragma unroll
  for (int c = 0; c < BPER; ++c) {
    const int ch = c * NT + tid, kw = ch / XB, rem = ch - kw * XB;
    const int tl = rem / (16 * RS), ls = (rem % (16 * RS)) ^ (tl & 15);
    const int tap = ls / RS, cg = ls - tap * RS;
    const int t = j0 + tl;
    bool v = t < g.ntiles;
    const int f = v ? (int)g.dTP.div((uint32_t)t) : 0, rr = t - f * g.TP;
    const int ty = v ? (int)g.dTW.div((uint32_t)rr) : 0, tx = rr - ty * g.TW;
    const int y = 2 * ty - 1 + (tap >> 2), x = 2 * tx - 1 + (tap & 3);
    v = v && (unsigned)y < (unsigned)g.H && (unsigned)x < (unsigned)g.W;
    bvo[c] = v ? (uint32_t)((((f * g.H + y) * g.W + x) * g.cs + g.coff + kw * BK + cg * 4) * 4) : kOOB;
  }
  auto issue = [&](float* st, int k0) {
    const int so = __builtin_amdgcn_readfirstlane(k0 * 4);
#pragma unroll
    for (int c = 0; c < APER; ++c) {
      const int ch0 = c * NT, kw = ch0 / XA;
      dma16(ra, st + kw * GEL + (ch0 - kw * XA) * 4 + wofs, avo[c], so);
    }
#pragma unroll
    for (int c = 0; c < BPER; ++c) {
      const int ch0 = c * NT, kw = ch0 / XB;
      dma16(rb, st + kw * GEL + AEL + (ch0 - kw * XB) * 4 + wofs, bvo[c], so);
    }
  };

  f32x4 acc[16][MB];
#pragma unroll
  for (int e = 0; e < 16; ++e)
#pragma unroll
    for (int m = 0; m < MB; ++m) acc[e][m] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment offsets inside this wave group's part of a stage (e = 0 / tap = 0)
  const int ksl = KL == 2 ? (q >> 1) : q, kh = KL == 2 ? (q & 1) * 2 : 0;
  int aof[MB];
#pragma unroll
  for (int m = 0; m < MB; ++m) {
    const int rr = wi * WTI + m * 16 + l16;
    aof[m] = wk * GEL + rr * BK + ((ksl ^ lds_swz<RS>(rr)) << 2) + kh;
  }
  const int brr = wj * 16 + l16;
  const int bof = wk * GEL + AEL + brr * 16 * BK + kh;
  const int bsw = brr & 15;

  const int nk = K / C::KS;
#pragma unroll
  for (int s = 0; s < NBUF - 1; ++s)
    if (s < nk) issue(smem + s * STG, s * C::KS);
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + NBUF - 2 < nk) wait_vmcnt<PIECES * (NBUF - 2)>();
    else wait_vmcnt<0>();
    barrier_lds();
    if (kt + NBUF - 1 < nk) issue(smem + ((kt + NBUF - 1) % NBUF) * STG, (kt + NBUF - 1) * C::KS);
    const float* st = smem + (kt % NBUF) * STG;
    float v[16][KL];
    {
      float d[16][KL];
#pragma unroll
      for (int tap = 0; tap < 16; ++tap) {
        const float* p = st + bof + (((tap * RS + ksl) ^ bsw) << 2);
        if constexpr ((ABL & 4) != 0) {
#pragma unroll
          for (int kk = 0; kk < KL; ++kk) d[tap][kk] = (float)(tap + kk + kt);
        } else if constexpr (KL == 2) {
          typedef float f32x2 __attribute__((ext_vector_type(2)));
          const f32x2 x = *reinterpret_cast<const f32x2*>(p);
          d[tap][0] = x[0]; d[tap][1] = x[1];
        } else {
          const f32x4 x = *reinterpret_cast<const f32x4*>(p);
          d[tap][0] = x[0]; d[tap][1] = x[1]; d[tap][2] = x[2]; d[tap][3] = x[3];
        }
      }
#pragma unroll
      for (int kk = 0; kk < KL; ++kk) {
        float dd[16], vv[16];
#pragma unroll
        for (int p = 0; p < 16; ++p) dd[p] = d[p][kk];
        if constexpr ((ABL & 1) != 0) {
#pragma unroll
          for (int e = 0; e < 16; ++e) vv[e] = dd[e];
        } else {
          wino_in(dd, vv);
        }
#pragma unroll
        for (int e = 0; e < 16; ++e) v[e][kk] = vv[e];
      }
    }
    float a[16][MB][KL];
#pragma unroll
    for (int e = 0; e < 16; ++e)
#pragma unroll
      for (int m = 0; m < MB; ++m) {
        const float* p = st + aof[m] + e * BI * BK;
        if constexpr ((ABL & 4) != 0) {
#pragma unroll
          for (int kk = 0; kk < KL; ++kk) a[e][m][kk] = (float)(e + kk + m);
        } else if constexpr (KL == 2) {
          typedef float f32x2 __attribute__((ext_vector_type(2)));
          const f32x2 x = *reinterpret_cast<const f32x2*>(p);
          a[e][m][0] = x[0]; a[e][m][1] = x[1];
        } else {
          const f32x4 x = *reinterpret_cast<const f32x4*>(p);
          a[e][m][0] = x[0]; a[e][m][1] = x[1]; a[e][m][2] = x[2]; a[e][m][3] = x[3];
        }
      }
    if constexpr ((ABL & 2) == 0) {
      // consecutive MFMAs on different accumulators (16x16x4: 40-cycle dependent latency, 32 issue)
#pragma unroll
      for (int kk = 0; kk < KL; ++kk)
#pragma unroll
        for (int e = 0; e < 16; ++e)
#pragma unroll
          for (int m = 0; m < MB; ++m)
            acc[e][m] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[e][m][kk], v[e][kk], acc[e][m], 0, 0, 0);
    } else {
#pragma unroll
      for (int e = 0; e < 16; ++e)
#pragma unroll
        for (int m = 0; m < MB; ++m) acc[e][m][0] += a[e][m][0] * v[e][0];
    }
  }
  __syncthreads();   // every wave is done reading the last stage

  // ---- epilogue: inverse transform in registers, partial outputs through LDS
  float* E = smem;
#pragma unroll
  for (int m = 0; m < MB; ++m) {
    float y[4][4];   // [reg r = row 4q + r][pixel ij]
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float mm[16], yy[4];
#pragma unroll
      for (int e = 0; e < 16; ++e) mm[e] = acc[e][m][r];
      wino_out(mm, yy);
#pragma unroll
      for (int ij = 0; ij < 4; ++ij) y[r][ij] = yy[ij];
    }
    const int row = wi * WTI + m * 16 + 4 * q;
#pragma unroll
    for (int ij = 0; ij < 4; ++ij)
      *reinterpret_cast<f32x4*>(E + (wk * 4 * BJ + (wj * 16 + l16) * 4 + ij) * ELD + row) =
          f32x4{y[0][ij], y[1][ij], y[2][ij], y[3][ij]};
  }
  __syncthreads();
  constexpr int G4 = BI / 4, NG = G4 * 4 * BJ, NPT = (NG + NT - 1) / NT;
  static_assert(!ACC || NT % G4 == 0, "fixed row group per thread for the accumulator reduction");
  typename acc_of<EP, ACC>::type eacc{};
#pragma unroll
  for (int qq = 0; qq < NPT; ++qq) {
    const int c = qq * NT + tid;
    if (NG % NT != 0 && c >= NG) break;
    const int r4 = c % G4, ps = c / G4;
    const int t = j0 + (ps >> 2);
    if (t >= g.ntiles) continue;
    const int f = (int)g.dTP.div((uint32_t)t), rr = t - f * g.TP;
    const int ty = (int)g.dTW.div((uint32_t)rr), tx = rr - ty * g.TW;
    const int y = 2 * ty + ((ps >> 1) & 1), x = 2 * tx + (ps & 1);
    if (y >= g.H || x >= g.W) continue;
    f32x4 v = *reinterpret_cast<const f32x4*>(E + ps * ELD + 4 * r4);
#pragma unroll
    for (int w = 1; w < WK; ++w) {
      const f32x4 u = *reinterpret_cast<const f32x4*>(E + (w * 4 * BJ + ps) * ELD + 4 * r4);
      v[0] += u[0]; v[1] += u[1]; v[2] += u[2]; v[3] += u[3];
    }
    const int i = i0 + 4 * r4, j = (f * g.H + y) * g.W + x;
    if constexpr (ACC) ep.finish(i, j, v[0], v[1], v[2], v[3], ep.prefetch(i, j), &eacc);
    else ep(i, j, v[0], v[1], v[2], v[3]);
  }
  if constexpr (ACC) {
    __syncthreads();   // every thread is done reading E
    ep.template flush<G4, NT>(eacc, E, i0, tj);
  }
}

template <class C, class EP, int NBUF = 2, int ABL = 0>
inline hipError_t launch_wino(const float* U, int ldu, int urows, int urow0, int uoff, const float* X,
                              const WinoGeo& g, const EP& ep, int Mi, int K, hipStream_t st) {
  if (Mi <= 0 || g.ntiles <= 0 || K <= 0) return hipSuccess;
  if (K % C::KS || urow0 + Mi > urows || uoff + K > ldu) return hipErrorInvalidValue;
  dim3 grid((g.ntiles + C::BJ - 1) / C::BJ, (Mi + C::BI - 1) / C::BI, 1);
  hipLaunchKernelGGL((wino_kernel<C, EP, NBUF, ABL>), grid, dim3(C::NT), 0, st, U, ldu, urows, urow0, uoff, X, g, ep, Mi, K,
                     tile_map(grid));
  return hipGetLastError();
}

// Column tiles (BJ tiles each) of a Winograd launch: the row count of the
// per-(step, column tile) gate-bias partials its BPTT epilogue writes.
template <class C>
inline int wino_col_tiles(const WinoGeo& g) { return (g.ntiles + C::BJ - 1) / C::BJ; }

}  // namespace aaa
