// Generic MFMA tiled GEMM / implicit-GEMM convolution for gfx950.
//
//   D[i][j] = sum_k A(i,k) * B(j,k)          i in [0,Mi), j in [0,Nj), k in [0,K)
//
// A and B are produced by "loaders" that stage a BI x BK (resp. BJ x BK) tile
// into LDS, either k-contiguous (KC: rows of k) or row-contiguous (RC: rows of
// i/j for a fixed k).  The loaders are where the convolution lives: LdIm2col
// gathers NHWC pixels for a (tap, channel) k index (forward conv, or the
// transposed-conv gather used for dgrad), LdIm2colT does the same with the
// roles of rows and k swapped (weight gradients, where k runs over pixels).
//
// Fragment mapping (32x32 MFMA, both dtypes): lane l = r + 32h holds, for one
// 16-deep k step, the 8 consecutive k values [8h, 8h+8) of row r of A (and of
// row r of B).  f32: eight v_mfma_f32_32x32x2_f32 (kk = 0..7 feeds k pair
// {kk, 8+kk}); bf16: one v_mfma_f32_32x32x16_bf16.  D layout: column j =
// lane&31, rows 8g+4h+e in registers 4g+e, so every lane owns FOUR consecutive
// rows of one column -- with gate-interleaved row packing (row = 4*ch + gate)
// that is exactly the four LSTM gates of one (pixel, channel), which is what
// lets the gate math run in the GEMM epilogue.
#pragma once
#include <type_traits>
#include "common.h"

namespace aaa {

// Row-contiguous bf16 tiles are read with ds_read_b64_tr_b16 (frag_bf16): a
// 32-lane half reads 4 k-rows x 64 B, so the row pitch is padded to 16 dwords
// mod 64 banks (+32 elements) to keep those reads conflict-free.
template <typename T, int R, int BK, bool KC>
struct Tile {
  static constexpr int PAD = (!KC && sizeof(T) == 2) ? 32 : 16 / (int)sizeof(T);
  static constexpr int LD = KC ? (BK + PAD) : (R + PAD);
  static constexpr int ELEMS = (KC ? R : BK) * LD;
  __device__ static __forceinline__ int off(int r, int k) { return KC ? r * LD + k : k * LD + r; }
};

// ---------------------------------------------------------------- loaders --
// Plain rows: element (row, k) at src[row*ld + k].  K % VG == 0, ld % VG == 0.
template <typename G, typename T, int R, int BK, int NT>
struct LdRows {
  static constexpr bool KC = true;
  static constexpr int VG = 16 / (int)sizeof(G);
  static constexpr int CPR = BK / VG;
  static constexpr int NCH = R * CPR;
  static constexpr int PER = (NCH + NT - 1) / NT;
  struct Params { const G* src; int ld; int nrows; };
  const G* rowp[PER];
  int kc[PER], lr[PER];
  bool ok[PER], act[PER];
  using Regs = u32x4[PER];
  __device__ __forceinline__ LdRows(const Params& p, int row0) {
#pragma unroll
    for (int c = 0; c < PER; ++c) {
      int ch = threadIdx.x + c * NT;
      act[c] = ch < NCH;
      lr[c] = ch / CPR;
      kc[c] = (ch % CPR) * VG;
      int row = row0 + lr[c];
      ok[c] = act[c] && row < p.nrows;
      rowp[c] = p.src + (size_t)(ok[c] ? row : 0) * p.ld;
    }
  }
  __device__ __forceinline__ void fetch(int k0, int kend, Regs& buf) const {
#pragma unroll
    for (int c = 0; c < PER; ++c) {
      int k = k0 + kc[c];
      if (ok[c] && k < kend) buf[c] = *reinterpret_cast<const u32x4*>(rowp[c] + k);
      else buf[c] = u32x4{0, 0, 0, 0};
    }
  }
  __device__ __forceinline__ void commit(T* lds, const Regs& buf) const {
#pragma unroll
    for (int c = 0; c < PER; ++c)
      if (NCH % NT == 0 || act[c]) lds_store_chunk<G, T>(lds + Tile<T, R, BK, true>::off(lr[c], kc[c]), buf[c]);
  }
};

// Transposed rows: element (row, k) at src[k*ld + row]; staged row-contiguous.
template <typename G, typename T, int R, int BK, int NT>
struct LdRowsT {
  static constexpr bool KC = false;
  static constexpr int VG = 16 / (int)sizeof(G);
  static constexpr int CPK = R / VG;
  static constexpr int NCH = BK * CPK;
  static constexpr int PER = (NCH + NT - 1) / NT;
  struct Params { const G* src; int ld; int nrows; };
  const G* src;
  int ld, nrows;
  int kr[PER], rc[PER], row[PER];
  bool act[PER];
  using Regs = u32x4[PER];
  __device__ __forceinline__ LdRowsT(const Params& p, int row0) : src(p.src), ld(p.ld), nrows(p.nrows) {
#pragma unroll
    for (int c = 0; c < PER; ++c) {
      int ch = threadIdx.x + c * NT;
      act[c] = ch < NCH;
      kr[c] = ch / CPK;
      rc[c] = (ch % CPK) * VG;
      row[c] = row0 + rc[c];
    }
  }
  __device__ __forceinline__ void fetch(int k0, int kend, Regs& buf) const {
#pragma unroll
    for (int c = 0; c < PER; ++c) {
      int k = k0 + kr[c];
      u32x4 v = u32x4{0, 0, 0, 0};
      if (act[c] && k < kend) {
        const G* p = src + (size_t)k * ld + row[c];
        if (row[c] + VG <= nrows) {
          v = *reinterpret_cast<const u32x4*>(p);
        } else {
          G tmp[VG];
#pragma unroll
          for (int e = 0; e < VG; ++e) tmp[e] = (row[c] + e < nrows) ? p[e] : (G)0.0f;
          v = __builtin_bit_cast(u32x4, tmp);
        }
      }
      buf[c] = v;
    }
  }
  __device__ __forceinline__ void commit(T* lds, const Regs& buf) const {
#pragma unroll
    for (int c = 0; c < PER; ++c)
      if (NCH % NT == 0 || act[c]) lds_store_chunk<G, T>(lds + Tile<T, R, BK, false>::off(rc[c], kr[c]), buf[c]);
  }
};

// Convolution geometry shared by the im2col loaders.  NHWC input with pixel
// stride ``cs`` elements and channel offset ``coff``; k = (ky*KW + kx)*Cin + ci.
struct ConvGeo {
  int Cin, cs, coff;
  int Hin, Win, Hout, Wout;
  int KW, stride, pad;
  int transposed;  // 0: forward gather, 1: dgrad (transposed-conv) gather
  // K order: 0 = tap-major (k = tap * Cin + ci); cmaj = BK > 0: channel-chunk-major,
  // k = (ci / BK) * taps * BK + tap * BK + ci % BK -- the taps of one channel chunk
  // adjacent in K, so a tile's 3x3 re-reads of the same rows hit in L2 (glds.h
  // GIm2colB only; the A operand must be packed in the same order, reorder_cmaj)
  int cmaj;
  FastDiv dCin, dKW, dWout, dHW, dTaps;  // filled by prep()
  ConvGeo prep() const {
    ConvGeo g = *this;
    g.dCin = FastDiv((uint32_t)Cin);
    g.dKW = FastDiv((uint32_t)KW);
    g.dWout = FastDiv((uint32_t)Wout);
    g.dHW = FastDiv((uint32_t)(Hout * Wout));
    g.dTaps = FastDiv((uint32_t)(KW * KW));
    return g;
  }
};

__device__ __forceinline__ bool conv_src(const ConvGeo& g, int oy, int ox, int ky, int kx, int& iy, int& ix) {
  if (!g.transposed) {
    iy = oy * g.stride + ky - g.pad;
    ix = ox * g.stride + kx - g.pad;
    return iy >= 0 && iy < g.Hin && ix >= 0 && ix < g.Win;
  }
  int ty = oy + g.pad - ky, tx = ox + g.pad - kx;
  if (ty < 0 || tx < 0) return false;
  if (g.stride == 1) { iy = ty; ix = tx; }
  else if (g.stride == 2) {
    if ((ty | tx) & 1) return false;
    iy = ty >> 1; ix = tx >> 1;
  } else {
    if ((ty % g.stride) | (tx % g.stride)) return false;
    iy = ty / g.stride; ix = tx / g.stride;
  }
  return iy < g.Hin && ix < g.Win;
}

// Rows = output pixels (frame-major), k = (tap, ci).  VEC requires Cin % VG == 0.
template <typename G, typename T, int R, int BK, int NT, bool VEC>
struct LdIm2col {
  static constexpr bool KC = true;
  static constexpr int VG = 16 / (int)sizeof(G);
  static constexpr int CPR = BK / VG;
  static constexpr int NCH = R * CPR;
  static constexpr int PER = (NCH + NT - 1) / NT;
  struct Params { const G* src; ConvGeo g; int nrows; };
  ConvGeo g;
  const G* fbase[PER];
  int oy[PER], ox[PER], kc[PER], lr[PER];
  bool ok[PER], act[PER];
  using Regs = u32x4[PER];
  __device__ __forceinline__ LdIm2col(const Params& p, int row0) : g(p.g) {
    const int hw = g.Hout * g.Wout;
#pragma unroll
    for (int c = 0; c < PER; ++c) {
      int ch = threadIdx.x + c * NT;
      act[c] = ch < NCH;
      lr[c] = ch / CPR;
      kc[c] = (ch % CPR) * VG;
      int m = row0 + lr[c];
      ok[c] = act[c] && m < p.nrows;
      int mm = ok[c] ? m : 0;
      int f = (int)g.dHW.div(mm), pix = mm - f * hw;
      oy[c] = (int)g.dWout.div(pix);
      ox[c] = pix - oy[c] * g.Wout;
      fbase[c] = p.src + (size_t)f * g.Hin * g.Win * g.cs + g.coff;
    }
  }
  __device__ __forceinline__ void fetch(int k0, int kend, Regs& buf) const {
#pragma unroll
    for (int c = 0; c < PER; ++c) {
      u32x4 v = u32x4{0, 0, 0, 0};
      int k = k0 + kc[c];
      if constexpr (VEC) {
        if (ok[c] && k < kend) {
          int tap = (int)g.dCin.div(k), ci = k - tap * g.Cin;
          int ky = (int)g.dKW.div(tap), kx = tap - ky * g.KW, iy, ix;
          if (conv_src(g, oy[c], ox[c], ky, kx, iy, ix))
            v = *reinterpret_cast<const u32x4*>(fbase[c] + (size_t)(iy * g.Win + ix) * g.cs + ci);
        }
      } else {
        static_assert(sizeof(G) == 4, "scalar im2col path expects fp32 global data");
        float tmp[4] = {0.f, 0.f, 0.f, 0.f};
        if (ok[c]) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            int ke = k + e;
            if (ke < kend) {
              int tap = (int)g.dCin.div(ke), ci = ke - tap * g.Cin;
              int ky = (int)g.dKW.div(tap), kx = tap - ky * g.KW, iy, ix;
              if (conv_src(g, oy[c], ox[c], ky, kx, iy, ix))
                tmp[e] = (float)fbase[c][(size_t)(iy * g.Win + ix) * g.cs + ci];
            }
          }
        }
        v = __builtin_bit_cast(u32x4, tmp);
      }
      buf[c] = v;
    }
  }
  __device__ __forceinline__ void commit(T* lds, const Regs& buf) const {
#pragma unroll
    for (int c = 0; c < PER; ++c)
      if (NCH % NT == 0 || act[c]) lds_store_chunk<G, T>(lds + Tile<T, R, BK, true>::off(lr[c], kc[c]), buf[c]);
  }
};

// Rows = k' = (tap, ci) of a convolution, k = output pixel m (weight gradient).
// Staged row-contiguous.  VEC requires Cin % VG == 0 (a chunk never crosses a tap).
template <typename G, typename T, int R, int BK, int NT, bool VEC>
struct LdIm2colT {
  static constexpr bool KC = false;
  static constexpr int VG = 16 / (int)sizeof(G);
  static constexpr int CPK = R / VG;
  static constexpr int NCH = BK * CPK;
  static constexpr int PER = (NCH + NT - 1) / NT;
  struct Params { const G* src; ConvGeo g; int nrows; };  // nrows = KH*KW*Cin
  ConvGeo g;
  const G* src;
  int kr[PER], rc[PER];
  int ky[PER][VEC ? 1 : 4], kx[PER][VEC ? 1 : 4], ci[PER][VEC ? 1 : 4];
  bool act[PER], rok[PER][VEC ? 1 : 4];
  using Regs = u32x4[PER];
  __device__ __forceinline__ LdIm2colT(const Params& p, int row0) : g(p.g), src(p.src) {
#pragma unroll
    for (int c = 0; c < PER; ++c) {
      int ch = threadIdx.x + c * NT;
      act[c] = ch < NCH;
      kr[c] = ch / CPK;
      rc[c] = (ch % CPK) * VG;
      constexpr int NE = VEC ? 1 : 4;
#pragma unroll
      for (int e = 0; e < NE; ++e) {
        int kp = row0 + rc[c] + e;
        rok[c][e] = act[c] && kp < p.nrows;
        int kq = rok[c][e] ? kp : 0;
        int tap = (int)g.dCin.div(kq);
        ci[c][e] = kq - tap * g.Cin;
        ky[c][e] = (int)g.dKW.div(tap);
        kx[c][e] = tap - ky[c][e] * g.KW;
      }
    }
  }
  __device__ __forceinline__ void fetch(int k0, int kend, Regs& buf) const {
    const int hw = g.Hout * g.Wout;
#pragma unroll
    for (int c = 0; c < PER; ++c) {
      u32x4 v = u32x4{0, 0, 0, 0};
      int m = k0 + kr[c];
      if (act[c] && m < kend) {
        int f = (int)g.dHW.div(m), pix = m - f * hw;
        int oy = (int)g.dWout.div(pix), ox = pix - oy * g.Wout;
        const G* fb = src + (size_t)f * g.Hin * g.Win * g.cs + g.coff;
        if constexpr (VEC) {
          int iy, ix;
          if (rok[c][0] && conv_src(g, oy, ox, ky[c][0], kx[c][0], iy, ix))
            v = *reinterpret_cast<const u32x4*>(fb + (size_t)(iy * g.Win + ix) * g.cs + ci[c][0]);
        } else {
          static_assert(sizeof(G) == 4, "scalar im2col path expects fp32 global data");
          float tmp[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            int iy, ix;
            if (rok[c][e] && conv_src(g, oy, ox, ky[c][e], kx[c][e], iy, ix))
              tmp[e] = (float)fb[(size_t)(iy * g.Win + ix) * g.cs + ci[c][e]];
          }
          v = __builtin_bit_cast(u32x4, tmp);
        }
      }
      buf[c] = v;
    }
  }
  __device__ __forceinline__ void commit(T* lds, const Regs& buf) const {
#pragma unroll
    for (int c = 0; c < PER; ++c)
      if (NCH % NT == 0 || act[c]) lds_store_chunk<G, T>(lds + Tile<T, R, BK, false>::off(rc[c], kr[c]), buf[c]);
  }
};

// ----------------------------------------------------------- fragments ----
template <typename TL>
__device__ __forceinline__ void frag_f32(const float* t, int r, int k, float (&a)[8]) {
  if constexpr (TL::KC_) {
    const f32x4* p = reinterpret_cast<const f32x4*>(t + r * TL::LD + k);
    f32x4 x = p[0], y = p[1];
    a[0] = x[0]; a[1] = x[1]; a[2] = x[2]; a[3] = x[3];
    a[4] = y[0]; a[5] = y[1]; a[6] = y[2]; a[7] = y[3];
  } else {
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) a[kk] = t[(k + kk) * TL::LD + r];
  }
}

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

template <typename TL>
__device__ __forceinline__ bf16x8 frag_bf16(const __bf16* t, int r, int k) {
  if constexpr (TL::KC_) {
    return *reinterpret_cast<const bf16x8*>(t + r * TL::LD + k);
  } else {
    // [k][r] image: two hardware transpose reads.  In each 16-lane group (one
    // h, rows c0..c0+15) lane 4q+p addresses k-row k+q, columns c0+4p..+3 and
    // receives column c0 + (lane & 15) of the 4 k-rows.
    const int li = (int)(threadIdx.x & 15), q = li >> 2, p = li & 3;
    const __bf16* a0 = t + (k + q) * TL::LD + (r - li) + 4 * p;
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(const_cast<__bf16*>(a0)));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(const_cast<__bf16*>(a0 + 4 * TL::LD)));
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
  }
}

// Output tile (row block ti, column block tj, K slice tz) of this workgroup.
// remap != 0: bijective XCD remap -- dispatch places linear block id b on XCD
// b % 8, so logical tile t = that XCD's running index; t runs over the row
// blocks of a column block first, then column blocks, then K slices.  One
// XCD's L2 then holds a contiguous slice of the gathered operand (and, for
// split-K weight gradients, one K window shared by all its tiles).
struct TileMap {
  int remap;
  FastDiv ny, nxy;   // row blocks, row blocks x column blocks (host-computed magics: no divisions on device)
};
__device__ __forceinline__ void tile_of(const TileMap& m, int& ti, int& tj, int& tz) {
  if (!m.remap) { ti = blockIdx.y; tj = blockIdx.x; tz = blockIdx.z; return; }
  const int ny = (int)m.ny.d, nxy = (int)m.nxy.d, n = nxy * gridDim.z;
  const int b = (blockIdx.z * ny + blockIdx.y) * gridDim.x + blockIdx.x;
  const int q = n >> 3, r = n & 7, x = b & 7;
  const int t = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3);
  tz = (int)m.nxy.div((uint32_t)t);
  const int u = t - tz * nxy;
  tj = (int)m.ny.div((uint32_t)u);
  ti = u - tj * ny;
}
inline int xcd_remap_enabled() {   // A/B (AAA_XCD_REMAP) in ablation builds only
#ifdef AAA_ABLATION
  const char* e = getenv("AAA_XCD_REMAP");
  return e ? atoi(e) != 0 : 1;
#else
  return 1;
#endif
}
inline TileMap tile_map(dim3 grid) {
  TileMap m;
  m.remap = xcd_remap_enabled();
  m.ny = FastDiv(grid.y);
  m.nxy = FastDiv(grid.x * grid.y);
  return m;
}

template <typename T, int R, int BK, bool KC>
struct TileK : Tile<T, R, BK, KC> { static constexpr bool KC_ = KC; };

// ------------------------------------------------------------- kernel -----
// WI x WJ waves tile the output; WK > 1 additionally splits every BK slab
// among WK wave groups (intra-workgroup split-K), whose partial accumulators
// are summed through LDS before the epilogue.  That multiplies the number of
// waves for GEMMs whose output has fewer 32x32 tiles than the chip has SIMDs
// (the per-step ConvLSTM kernels at small batch).
template <typename T, int BI_, int BJ_, int BK_, int WI_, int WJ_, int WK_ = 1>
struct GemmCfg {
  using type = T;
  static constexpr int BI = BI_, BJ = BJ_, BK = BK_, WI = WI_, WJ = WJ_, WK = WK_;
  static constexpr int NT = WI * WJ * WK * 64;
};

// fp32 operands on the bf16 MFMA (configs with SPLIT3): each fp32 fragment
// value x = hi + lo, hi = bf16(x), lo = bf16(x - hi), and a.b is accumulated as
// hi.hi + hi.lo + lo.hi (the dropped lo.lo is ~2^-16 of the product) -- three
// 32x32x16 bf16 MFMAs per 16-k step instead of eight 32x32x2 fp32 ones.  Used for
// the fp32 tail GEMMs of the bf16 path (rt.h head_gemm).
template <class C, class = void> struct split3_of : std::false_type {};
template <class C> struct split3_of<C, std::enable_if_t<C::SPLIT3>> : std::true_type {};
template <int BI_, int BJ_, int BK_, int WI_, int WJ_, int WK_ = 1>
struct GemmCfgS3 : GemmCfg<float, BI_, BJ_, BK_, WI_, WJ_, WK_> {
  static constexpr bool SPLIT3 = true;
};
// fp32 operands at fp32 accuracy on the bf16 MFMA (configs with SPLIT6): x =
// hi + mid + lo, each bf16 (8 + 8 + 8 mantissa bits cover fp32's 24), and a.b
// accumulated as the six products with i + j <= 2 (hh, hm, mh, hl, lh, mm) --
// the dropped ml, lm, ll are ~2^-24 of the product, the size of an fp32
// rounding.  Six 32x32x16 bf16 MFMAs (6 x 32 cycles) per 16-k step instead of
// eight 32x32x2 fp32 ones (8 x 64): the fp32 path's large GEMMs
// (tests/test_gpu_parity.py test_f32_split6_accuracy: the error against the
// fp64 evaluation stays that of the fp32 MFMA).
template <class C, class = void> struct split6_of : std::false_type {};
template <class C> struct split6_of<C, std::enable_if_t<C::SPLIT6>> : std::true_type {};
template <int BI_, int BJ_, int BK_, int WI_, int WJ_, int WK_ = 1>
struct GemmCfgS6 : GemmCfg<float, BI_, BJ_, BK_, WI_, WJ_, WK_> {
  static constexpr bool SPLIT3 = true, SPLIT6 = true;
};
// The same products with each operand split ONCE per workgroup, where its staged fp32
// chunk is committed to LDS (lds_store_split3), instead of once per wave per fragment
// read: the LDS stages hold the three bf16 part tiles of each operand and the K loop
// reads bf16 fragments only (gemm_kernel_s6l; the register-staged TB loaders).
template <class C, class = void> struct split6l_of : std::false_type {};
template <class C> struct split6l_of<C, std::enable_if_t<C::SPLIT6L>> : std::true_type {};
template <int BI_, int BJ_, int BK_, int WI_, int WJ_, int FD_ = 1>
struct GemmCfgS6L : GemmCfg<float, BI_, BJ_, BK_, WI_, WJ_, 1> {
  static constexpr bool SPLIT3 = true, SPLIT6 = true, SPLIT6L = true;
  static constexpr int FD = FD_;   // K tiles of global loads in flight (register stages)
};
// The bf16 path's tail precision (SPLIT3: hi + lo parts, three products) split at commit the same
// way (gemm_kernel_s6l with two part tiles per operand): bit-identical to gemm_kernel's SPLIT3 path.
template <int BI_, int BJ_, int BK_, int WI_, int WJ_, int FD_ = 2>
struct GemmCfgS3L : GemmCfg<float, BI_, BJ_, BK_, WI_, WJ_, 1> {
  static constexpr bool SPLIT3 = true, SPLIT6L = true, TWO_PARTS = true;
  static constexpr int FD = FD_;
};
template <class C, class = void> struct two_parts_of : std::false_type {};
template <class C> struct two_parts_of<C, std::enable_if_t<C::TWO_PARTS>> : std::true_type {};
// 4 fp32 of a staged chunk -> hi, lo bf16 parts (split_bf16), 8 B each, ``plane`` elements apart
__device__ __forceinline__ void lds_store_split2(__bf16* dst, int plane, const u32x4& raw) {
  const f32x4 f = __builtin_bit_cast(f32x4, raw);
  bf16x4 hi, lo;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    hi[e] = (__bf16)f[e];
    lo[e] = (__bf16)(f[e] - (float)hi[e]);
  }
  *reinterpret_cast<bf16x4*>(dst) = hi;
  *reinterpret_cast<bf16x4*>(dst + plane) = lo;
}
// B operand exact in bf16 (configs with BEXACT: conv1's operand when the frames are uint8 -- integers
// 0..255 are bf16 values): its mid and lo parts are zero, so of the six split products only lo.hi,
// mid.hi and hi.hi are issued (in the SPLIT6 order; the three skipped ones add exact zeros -- the same
// sums) and B is converted, not split.
template <class C, class = void> struct bexact_of : std::false_type {};
template <class C> struct bexact_of<C, std::enable_if_t<C::BEXACT>> : std::true_type {};
template <int BI_, int BJ_, int BK_, int WI_, int WJ_, int WK_ = 1>
struct GemmCfgS6BX : GemmCfgS6<BI_, BJ_, BK_, WI_, WJ_, WK_> {
  static constexpr bool BEXACT = true;
};
template <int BI_, int BJ_, int BK_, int WI_, int WJ_, int FD_ = 1>
struct GemmCfgS6LBX : GemmCfgS6L<BI_, BJ_, BK_, WI_, WJ_, FD_> {
  static constexpr bool BEXACT = true;
};
__device__ __forceinline__ bf16x8 to_bf16x8(const float (&x)[8]) {
  bf16x8 r;
#pragma unroll
  for (int e = 0; e < 8; ++e) r[e] = (__bf16)x[e];
  return r;
}
__device__ __forceinline__ void split3_bf16(const float (&x)[8], bf16x8& hi, bf16x8& mid, bf16x8& lo) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    hi[e] = (__bf16)x[e];
    const float r = x[e] - (float)hi[e];
    mid[e] = (__bf16)r;
    lo[e] = (__bf16)(r - (float)mid[e]);
  }
}

// Split-at-commit (GemmCfgS6L): 4 fp32 of a staged chunk -> their three bf16 parts, 8 B
// each, into the three part tiles of one operand stage (``plane`` elements apart).
__device__ __forceinline__ void lds_store_split3(__bf16* dst, int plane, const u32x4& raw) {
  const f32x4 f = __builtin_bit_cast(f32x4, raw);
  bf16x4 hi, mid, lo;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    hi[e] = (__bf16)f[e];
    const float r = f[e] - (float)hi[e];
    mid[e] = (__bf16)r;
    lo[e] = (__bf16)(r - (float)mid[e]);
  }
  *reinterpret_cast<bf16x4*>(dst) = hi;
  *reinterpret_cast<bf16x4*>(dst + plane) = mid;
  *reinterpret_cast<bf16x4*>(dst + 2 * plane) = lo;
}

__device__ __forceinline__ void split_bf16(const float (&x)[8], bf16x8& hi, bf16x8& lo) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    hi[e] = (__bf16)x[e];
    lo[e] = (__bf16)(x[e] - (float)hi[e]);
  }
}

// One K tile of the register-staged GEMMs from the LDS tiles Ac / Bc into the wave's accumulators
// (gemm_kernel, gemm_kernel_deep): BK / 16 / WK k steps of 16 per wave, the fp32 paths split into bf16
// parts (SPLIT3 / SPLIT6) or on the fp32 MFMA.
template <class C, class TA, class TB, int MI, int MJ>
__device__ __forceinline__ void gemm_mma_tile(const typename C::type* Ac, const typename C::type* Bc,
                                              f32x16 (&acc)[MI][MJ], int wi, int wj, int wk, int r32, int h) {
  using T = typename C::type;
  constexpr int BK = C::BK, WK = C::WK, WTI = C::BI / C::WI, WTJ = C::BJ / C::WJ;
#pragma unroll
  for (int s2 = 0; s2 < BK / 16 / WK; ++s2) {
    const int kofs = 16 * (s2 * WK + wk) + 8 * h;
    if constexpr (is_f32<T>::value) {
      float af[MI][8], bfr[MJ][8];
#pragma unroll
      for (int a = 0; a < MI; ++a) frag_f32<TA>(Ac, wi * WTI + a * 32 + r32, kofs, af[a]);
#pragma unroll
      for (int b = 0; b < MJ; ++b) frag_f32<TB>(Bc, wj * WTJ + b * 32 + r32, kofs, bfr[b]);
      if constexpr (split6_of<C>::value) {
        // as SPLIT3 below, with a three-way split; smallest products first
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
      } else if constexpr (split3_of<C>::value) {
        // the 8 k of a lane's fp32 fragment are the 8 k of the bf16 operand layout
        // (lane (r32, h): k 8h .. 8h+7 of the 16-k step)
        bf16x8 ah[MI], al[MI], bh[MJ], bl[MJ];
#pragma unroll
        for (int a = 0; a < MI; ++a) split_bf16(af[a], ah[a], al[a]);
#pragma unroll
        for (int b = 0; b < MJ; ++b) split_bf16(bfr[b], bh[b], bl[b]);
#pragma unroll
        for (int a = 0; a < MI; ++a)
#pragma unroll
          for (int b = 0; b < MJ; ++b) {
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[a], bh[b], acc[a][b], 0, 0, 0);
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[a], bl[b], acc[a][b], 0, 0, 0);
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
      for (int a = 0; a < MI; ++a) af[a] = frag_bf16<TA>(Ac, wi * WTI + a * 32 + r32, kofs);
#pragma unroll
      for (int b = 0; b < MJ; ++b) bfr[b] = frag_bf16<TB>(Bc, wj * WTJ + b * 32 + r32, kofs);
#pragma unroll
      for (int a = 0; a < MI; ++a)
#pragma unroll
        for (int b = 0; b < MJ; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[a], bfr[b], acc[a][b], 0, 0, 0);
    }
  }
}

template <class C, class LA, class LB, class EP>
__global__ void __launch_bounds__(C::NT)
gemm_kernel(typename LA::Params pa, typename LB::Params pb, EP ep, int K, int kchunk, TileMap tm) {
  using T = typename C::type;
  constexpr int BI = C::BI, BJ = C::BJ, BK = C::BK, WI = C::WI, WJ = C::WJ, WK = C::WK;
  constexpr int WTI = BI / WI, WTJ = BJ / WJ, MI = WTI / 32, MJ = WTJ / 32;
  static_assert(MI >= 1 && MJ >= 1 && BK % (16 * WK) == 0, "tile shape");
  using TA = TileK<T, BI, BK, LA::KC>;
  using TB = TileK<T, BJ, BK, LB::KC>;
  __shared__ __attribute__((aligned(16))) T smem[2 * (TA::ELEMS + TB::ELEMS)];
  T* const As0 = smem;
  T* const As1 = smem + TA::ELEMS;
  T* const Bs0 = smem + 2 * TA::ELEMS;
  T* const Bs1 = Bs0 + TB::ELEMS;

  int ti, tj, tz;
  tile_of(tm, ti, tj, tz);
  const int i0 = ti * BI, j0 = tj * BJ;
  const int kb = tz * kchunk;
  const int ke = min(K, kb + kchunk);
  if (kb >= ke) return;

  LA la(pa, i0);
  LB lb(pb, j0);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wk = wave / (WI * WJ), wr = wave - wk * (WI * WJ);
  const int wi = wr / WJ, wj = wr - (wr / WJ) * WJ;
  const int r32 = lane & 31, h = lane >> 5;

  f32x16 acc[MI][MJ];
#pragma unroll
  for (int a = 0; a < MI; ++a)
#pragma unroll
    for (int b = 0; b < MJ; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.f;

  const int nk = (ke - kb + BK - 1) / BK;
  // One register stage + two LDS buffers: the global loads of tile k+1 are in
  // flight under the MFMAs of tile k; one barrier per K tile.
  typename LA::Regs ra;
  typename LB::Regs rb;
  la.fetch(kb, ke, ra);
  lb.fetch(kb, ke, rb);
  la.commit(As0, ra);
  lb.commit(Bs0, rb);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const bool odd = kt & 1;
    const T* Ac = odd ? As1 : As0;
    const T* Bc = odd ? Bs1 : Bs0;
    const bool more = kt + 1 < nk;
    if (more) {
      la.fetch(kb + (kt + 1) * BK, ke, ra);
      lb.fetch(kb + (kt + 1) * BK, ke, rb);
    }
    gemm_mma_tile<C, TA, TB, MI, MJ>(Ac, Bc, acc, wi, wj, wk, r32, h);
    if (more) {
      la.commit(odd ? As0 : As1, ra);
      lb.commit(odd ? Bs0 : Bs1, rb);
    }
    __syncthreads();
  }

  if constexpr (WK > 1) {
    // sum the WK partial accumulators through LDS (the staging buffers are free now)
    constexpr int RED = (WK - 1) * WI * WJ * MI * MJ * 16 * 64;
    static_assert(RED * sizeof(float) <= sizeof(smem), "split-K reduction does not fit in LDS");
    float* red = reinterpret_cast<float*>(smem);
    if (wk > 0) {
#pragma unroll
      for (int a = 0; a < MI; ++a)
#pragma unroll
        for (int b = 0; b < MJ; ++b)
#pragma unroll
          for (int e = 0; e < 16; ++e)
            red[((((wk - 1) * WI * WJ + wr) * MI * MJ + a * MJ + b) * 16 + e) * 64 + lane] = acc[a][b][e];
    }
    __syncthreads();
    if (wk > 0) return;
#pragma unroll
    for (int w = 1; w < WK; ++w)
#pragma unroll
      for (int a = 0; a < MI; ++a)
#pragma unroll
        for (int b = 0; b < MJ; ++b)
#pragma unroll
          for (int e = 0; e < 16; ++e)
            acc[a][b][e] += red[((((w - 1) * WI * WJ + wr) * MI * MJ + a * MJ + b) * 16 + e) * 64 + lane];
  }
#pragma unroll
  for (int a = 0; a < MI; ++a)
#pragma unroll
    for (int b = 0; b < MJ; ++b)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int i = i0 + wi * WTI + a * 32 + 8 * g + 4 * h;
        const int j = j0 + wj * WTJ + b * 32 + r32;
        ep(i, j, acc[a][b][4 * g], acc[a][b][4 * g + 1], acc[a][b][4 * g + 2], acc[a][b][4 * g + 3]);
      }
}

// Split-at-commit split6 GEMM (GemmCfgS6L): the register-staged double buffer of
// gemm_kernel, with each stage holding the hi / mid / lo bf16 tiles of both operands
// (the loaders' commit3).  Per 16-k step a wave reads 3 (MI + MJ) bf16 fragments and
// issues 6 MI MJ MFMAs; no VALU split in the loop.  Same products, same order, same
// parts as the SPLIT6 path of gemm_kernel: bit-identical results.
template <class C, class LA, class LB, class EP>
__global__ void __launch_bounds__(C::NT)
gemm_kernel_s6l(typename LA::Params pa, typename LB::Params pb, EP ep, int K, int kchunk, TileMap tm) {
  constexpr int BI = C::BI, BJ = C::BJ, BK = C::BK, WI = C::WI, WJ = C::WJ;
  constexpr int WTI = BI / WI, WTJ = BJ / WJ, MI = WTI / 32, MJ = WTJ / 32;
  static_assert(C::WK == 1 && MI >= 1 && MJ >= 1 && BK % 16 == 0, "tile shape");
  using TA = TileK<__bf16, BI, BK, LA::KC>;
  using TB = TileK<__bf16, BJ, BK, LB::KC>;
  constexpr bool TWO = two_parts_of<C>::value;   // SPLIT3 (hi, lo) instead of SPLIT6 (hi, mid, lo)
  constexpr int NPT = TWO ? 2 : 3;               // part tiles per operand
  constexpr int PA = TA::ELEMS, PB = TB::ELEMS, STG = NPT * (PA + PB);
  constexpr bool BX = bexact_of<C>::value;   // B's hi part only (commit1), three products
  static_assert(!(TWO && BX), "exact B: three-part configs only");
  __shared__ __attribute__((aligned(16))) __bf16 smem[2 * STG];

  int ti, tj, tz;
  tile_of(tm, ti, tj, tz);
  const int i0 = ti * BI, j0 = tj * BJ;
  const int kb = tz * kchunk;
  const int ke = min(K, kb + kchunk);
  if (kb >= ke) return;

  LA la(pa, i0);
  LB lb(pb, j0);
  auto commit_a = [&](__bf16* dst, const typename LA::Regs& r) {
    if constexpr (TWO) la.commit2(dst, PA, r);
    else la.commit3(dst, PA, r);
  };
  auto commit_b = [&](__bf16* dst, const typename LB::Regs& r) {
    if constexpr (BX) lb.commit1(dst, r);
    else if constexpr (TWO) lb.commit2(dst, PB, r);
    else lb.commit3(dst, PB, r);
  };
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wi = wave / WJ, wj = wave - (wave / WJ) * WJ;
  const int r32 = lane & 31, h = lane >> 5;

  f32x16 acc[MI][MJ];
#pragma unroll
  for (int a = 0; a < MI; ++a)
#pragma unroll
    for (int b = 0; b < MJ; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.f;

  const int nk = (ke - kb + BK - 1) / BK;
  // FD = 2: the loads of tile k+2 are in flight while tile k+1 is committed and tile k
  // multiplied (two register stages), so a load has two K steps of MFMAs to land
  constexpr int FD = C::FD;
  typename LA::Regs ra[FD];
  typename LB::Regs rb[FD];
  la.fetch(kb, ke, ra[0]);
  lb.fetch(kb, ke, rb[0]);
  if constexpr (FD == 2) {
    if (nk > 1) {
      la.fetch(kb + BK, ke, ra[1]);
      lb.fetch(kb + BK, ke, rb[1]);
    }
  }
  commit_a(smem, ra[0]);
  commit_b(smem + NPT * PA, rb[0]);
  __syncthreads();

  // one K step; E = kt & 1 (compile-time, so the register stages stay in registers)
  auto step = [&](int kt, auto E) {
    constexpr int e = decltype(E)::value;
    const __bf16* cur = smem + e * STG;
    __bf16* nxt = smem + (e ^ 1) * STG;
    const bool more = kt + 1 < nk;
    if constexpr (FD == 2) {   // tile kt+2 into register stage e (tile kt's, committed a step ago)
      // unconditional: a tile past the slice is fetched and never committed (the TB loaders read it in
      // range or as zeros); guarded by kt + 2 < nk, the compiler waited for tile kt+1 at the top of the
      // step instead of keeping it in flight to the commit (C2 wgrad 641-646 -> 632-647 us,
      // profiles/r06/ab/s6l_prio/)
      la.fetch(kb + (kt + 2) * BK, ke, ra[e]);
      lb.fetch(kb + (kt + 2) * BK, ke, rb[e]);
    } else if (more) {
      la.fetch(kb + (kt + 1) * BK, ke, ra[0]);
      lb.fetch(kb + (kt + 1) * BK, ke, rb[0]);
    }
#pragma unroll
    for (int s2 = 0; s2 < BK / 16; ++s2) {
      const int kofs = 16 * s2 + 8 * h;
      bf16x8 af[MI][3], bfr[MJ][3];
#pragma unroll
      for (int a = 0; a < MI; ++a)
#pragma unroll
        for (int p = 0; p < NPT; ++p) af[a][p] = frag_bf16<TA>(cur + p * PA, wi * WTI + a * 32 + r32, kofs);
#pragma unroll
      for (int b = 0; b < MJ; ++b)
#pragma unroll
        for (int p = 0; p < (BX ? 1 : NPT); ++p)
          bfr[b][p] = frag_bf16<TB>(cur + NPT * PA + p * PB, wj * WTJ + b * 32 + r32, kofs);
      if constexpr (TWO) {   // as gemm_kernel's SPLIT3: lo.hi, hi.lo, hi.hi
#pragma unroll
        for (int a = 0; a < MI; ++a)
#pragma unroll
          for (int b = 0; b < MJ; ++b) {
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[a][1], bfr[b][0], acc[a][b], 0, 0, 0);
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[a][0], bfr[b][1], acc[a][b], 0, 0, 0);
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[a][0], bfr[b][0], acc[a][b], 0, 0, 0);
          }
      } else
#pragma unroll
      for (int a = 0; a < MI; ++a)
#pragma unroll
        for (int b = 0; b < MJ; ++b) {   // smallest products first, as gemm_kernel's SPLIT6
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[a][2], bfr[b][0], acc[a][b], 0, 0, 0);
          if constexpr (!BX) {
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[a][0], bfr[b][2], acc[a][b], 0, 0, 0);
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[a][1], bfr[b][1], acc[a][b], 0, 0, 0);
          }
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[a][1], bfr[b][0], acc[a][b], 0, 0, 0);
          if constexpr (!BX) acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[a][0], bfr[b][1], acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[a][0], bfr[b][0], acc[a][b], 0, 0, 0);
        }
    }
    if (more) {   // tile kt+1: register stage e ^ 1 (FD 2) or 0
      constexpr int rs1 = FD == 2 ? (e ^ 1) : 0;
      commit_a(nxt, ra[rs1]);
      commit_b(nxt + NPT * PA, rb[rs1]);
    }
    __syncthreads();
  };
  for (int kt = 0; kt < nk; kt += 2) {
    step(kt, std::integral_constant<int, 0>{});
    if (kt + 1 < nk) step(kt + 1, std::integral_constant<int, 1>{});
  }
#pragma unroll
  for (int a = 0; a < MI; ++a)
#pragma unroll
    for (int b = 0; b < MJ; ++b)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int i = i0 + wi * WTI + a * 32 + 8 * g + 4 * h;
        const int j = j0 + wj * WTJ + b * 32 + r32;
        ep(i, j, acc[a][b][4 * g], acc[a][b][4 * g + 1], acc[a][b][4 * g + 2], acc[a][b][4 * g + 3]);
      }
}

// Host-side launcher.  Mi/Nj are the D extents, K the reduction length,
// nsplit the number of K slices (epilogue must accumulate when nsplit > 1).
template <class C, class LA, class LB, class EP>
inline hipError_t launch_gemm(const typename LA::Params& pa, const typename LB::Params& pb, const EP& ep,
                              int Mi, int Nj, int K, int nsplit, hipStream_t st) {
  if (Mi <= 0 || Nj <= 0 || K <= 0) return hipSuccess;
  if (nsplit < 1) nsplit = 1;
  int kchunk = (K + nsplit - 1) / nsplit;
  kchunk = (kchunk + C::BK - 1) / C::BK * C::BK;
  nsplit = (K + kchunk - 1) / kchunk;
  dim3 grid((Nj + C::BJ - 1) / C::BJ, (Mi + C::BI - 1) / C::BI, nsplit);
  if constexpr (split6l_of<C>::value)
    hipLaunchKernelGGL((gemm_kernel_s6l<C, LA, LB, EP>), grid, dim3(C::NT), 0, st, pa, pb, ep, K, kchunk,
                       tile_map(grid));
  else
    hipLaunchKernelGGL((gemm_kernel<C, LA, LB, EP>), grid, dim3(C::NT), 0, st, pa, pb, ep, K, kchunk,
                       tile_map(grid));
  return hipGetLastError();
}

}  // namespace aaa
