// Buffer-descriptor loaders for the convolution GEMMs (the hot path).
//
// Same interface as the generic loaders in gemm.h, but built for a low VALU
// count per MFMA: every per-thread quantity that does not change along K
// (row base offsets, which taps of a pixel are inside the image) is computed
// once in the constructor, the per-K-tile part is wave-uniform (scalar), and
// out-of-range / padding lanes are handled by the buffer descriptor's range
// check (offset >= num_records returns 0) instead of branches.
//
// Preconditions (checked by the host launcher): the source tensor is < 2 GiB;
// LdRowsB: K % BK == 0 (no partial k tiles); LdIm2colB: Cin % BK == 0 (a K
// tile never crosses a tap) and stride 1 for the transposed gather;
// LdRowsTB / LdIm2colTB: nrows % VG == 0 / Cin % VG == 0.
#pragma once
#include "gemm.h"

namespace aaa {

constexpr uint32_t kOOB = 0x80000000u;  // >= num_records of every buffer we build

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)bytes, 0x00020000);
}
// The same from a base address and size the compiler cannot prove wave-uniform although they are
// (e.g. derived through a lambda's captures): readfirstlane'd, so the descriptor sits in SGPRs -- an
// inline-asm "s" operand (dma16a) otherwise receives VGPRs and does not assemble.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc_u(const void* p, uint32_t bytes) {
  const uint64_t a = (uint64_t)(size_t)p;
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)a);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32));
  const uint32_t n = (uint32_t)__builtin_amdgcn_readfirstlane((int)bytes);
  return make_rsrc(reinterpret_cast<const void*>((size_t)lo | ((size_t)hi << 32)), n);
}
__device__ __forceinline__ u32x4 bload(__amdgpu_buffer_rsrc_t r, uint32_t voff) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, (int)voff, 0, 0);
}

// Plain rows (weights): element (row, k) at src[row*ld + k], K % BK == 0.
template <typename G, typename T, int R, int BK, int NT>
struct LdRowsB {
  static constexpr bool KC = true;
  static constexpr int VG = 16 / (int)sizeof(G);
  static constexpr int CPR = BK / VG;
  static constexpr int NCH = R * CPR;
  static constexpr int PER = (NCH + NT - 1) / NT;
  using Regs = u32x4[PER];
  struct Params { const G* src; int ld; int nrows; };
  __amdgpu_buffer_rsrc_t rs;
  uint32_t voff[PER];
  int ldo[PER];
  bool act[PER];
  __device__ __forceinline__ LdRowsB(const Params& p, int row0) {
    rs = make_rsrc(p.src, (uint32_t)((size_t)p.nrows * p.ld * sizeof(G)));
#pragma unroll
    for (int c = 0; c < PER; ++c) {
      const int ch = threadIdx.x + c * NT;
      act[c] = ch < NCH;
      const int lr = ch / CPR, kc = (ch % CPR) * VG, row = row0 + lr;
      voff[c] = (act[c] && row < p.nrows) ? (uint32_t)((row * p.ld + kc) * (int)sizeof(G)) : kOOB;
      ldo[c] = Tile<T, R, BK, true>::off(lr, kc);
    }
  }
  __device__ __forceinline__ void fetch(int k0, int, Regs& buf) const {
    const uint32_t ko = (uint32_t)(k0 * (int)sizeof(G));
#pragma unroll
    for (int c = 0; c < PER; ++c) buf[c] = bload(rs, voff[c] + ko);
  }
  __device__ __forceinline__ void commit(T* lds, const Regs& buf) const {
#pragma unroll
    for (int c = 0; c < PER; ++c)
      if (NCH % NT == 0 || act[c]) lds_store_chunk<G, T>(lds + ldo[c], buf[c]);
  }
};

// Transposed rows: element (row, k) at src[k*ld + row] (activation grads for
// weight gradients, k = pixel).  ktotal = rows of src; nrows % VG == 0.
template <typename G, typename T, int R, int BK, int NT>
struct LdRowsTB {
  static constexpr bool KC = false;
  static constexpr int VG = 16 / (int)sizeof(G);
  static constexpr int CPK = R / VG;
  static constexpr int NCH = BK * CPK;
  static constexpr int PER = (NCH + NT - 1) / NT;
  using Regs = u32x4[PER];
  struct Params { const G* src; int ld; int nrows; int ktotal; };
  __amdgpu_buffer_rsrc_t rs;
  uint32_t voff[PER];
  int ldo[PER];
  int rowbytes;
  bool act[PER];
  // split-at-commit GEMMs (gemm.h GemmCfgS6L): the chunk's place in the bf16 part tiles
  __device__ __forceinline__ static int off16(int ch) { return Tile<__bf16, R, BK, false>::off((ch % CPK) * VG, ch / CPK); }
  __device__ __forceinline__ LdRowsTB(const Params& p, int row0) {
    rs = make_rsrc(p.src, (uint32_t)((size_t)p.ktotal * p.ld * sizeof(G)));
    rowbytes = p.ld * (int)sizeof(G);
#pragma unroll
    for (int c = 0; c < PER; ++c) {
      const int ch = threadIdx.x + c * NT;
      act[c] = ch < NCH;
      const int kr = ch / CPK, rc = (ch % CPK) * VG, row = row0 + rc;
      voff[c] = (act[c] && row < p.nrows) ? (uint32_t)((kr * p.ld + row) * (int)sizeof(G)) : kOOB;
      ldo[c] = Tile<T, R, BK, false>::off(rc, kr);
    }
  }
  __device__ __forceinline__ void fetch(int k0, int, Regs& buf) const {
    const uint32_t ko = (uint32_t)(k0 * rowbytes);
#pragma unroll
    for (int c = 0; c < PER; ++c) buf[c] = bload(rs, voff[c] + ko);
  }
  __device__ __forceinline__ void commit(T* lds, const Regs& buf) const {
#pragma unroll
    for (int c = 0; c < PER; ++c)
      if (NCH % NT == 0 || act[c]) lds_store_chunk<G, T>(lds + ldo[c], buf[c]);
  }
  __device__ __forceinline__ void commit3(__bf16* lds, int plane, const Regs& buf) const {
#pragma unroll
    for (int c = 0; c < PER; ++c)
      if (NCH % NT == 0 || act[c]) lds_store_split3(lds + off16(threadIdx.x + c * NT), plane, buf[c]);
  }
  __device__ __forceinline__ void commit2(__bf16* lds, int plane, const Regs& buf) const {
#pragma unroll
    for (int c = 0; c < PER; ++c)
      if (NCH % NT == 0 || act[c]) lds_store_split2(lds + off16(threadIdx.x + c * NT), plane, buf[c]);
  }
};

// Per-(pixel row m, chunk column kc) constants of the implicit-GEMM gather:
// the element offset of the chunk's source at the K tile's first tap (base),
// the chunk's tap relative to that first tap (dt; BK % Cin == 0 tiles), and
// the pixel's valid-tap bitmask (validity is separable: tap (ky,kx) is inside
// iff row ky and column kx are).  ok = false gives an all-invalid mask.
__device__ __forceinline__ void im2col_setup(const ConvGeo& g, int BK, bool ok, int m, int kc, int& base, int& dt,
                                             uint64_t& vmask) {
  const int hw = g.Hout * g.Wout;
  const int KH = g.KW;  // square kernels
  const int sgn = g.transposed ? -1 : 1;
  const int mm = ok ? m : 0;
  const int f = (int)g.dHW.div(mm), pix = mm - f * hw;
  const int oy = (int)g.dWout.div(pix), ox = pix - oy * g.Wout;
  // transposed gathers here are stride 1 (host-checked), so no divisibility test
  uint32_t rowm = 0, colm = 0;
  uint64_t msk = 0;
  const int ty0 = g.transposed ? oy + g.pad : oy * g.stride - g.pad;   // row of tap 0; tap k at ty0 -/+ k
  const int tx0 = g.transposed ? ox + g.pad : ox * g.stride - g.pad;
  const int sg = g.transposed ? -1 : 1;
  if (KH == 3) {   // the ConvLSTM steps: straight-line
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      if (ok && (unsigned)(ty0 + sg * k) < (unsigned)g.Hin) rowm |= 1u << k;
      if ((unsigned)(tx0 + sg * k) < (unsigned)g.Win) colm |= 1u << k;
    }
#pragma unroll
    for (int k = 0; k < 3; ++k)
      if ((rowm >> k) & 1u) msk |= (uint64_t)colm << (3 * k);
  } else {
#pragma clang loop vectorize(disable)
    for (int k = 0; k < KH; ++k) {
      if (ok && (unsigned)(ty0 + sg * k) < (unsigned)g.Hin) rowm |= 1u << k;
      if ((unsigned)(tx0 + sg * k) < (unsigned)g.Win) colm |= 1u << k;
    }
#pragma clang loop vectorize(disable)
    for (int k = 0; k < KH; ++k)
      if ((rowm >> k) & 1u) msk |= (uint64_t)colm << (k * g.KW);
  }
  vmask = msk;
  const int d = g.Cin >= BK ? 0 : (int)g.dCin.div((uint32_t)kc);   // taps inside the tile before this chunk
  const int ci = kc - d * g.Cin;
  dt = d;
  const int dky = (int)g.dKW.div((uint32_t)d), dkx = d - dky * g.KW;
  base = ((f * g.Hin + ty0) * g.Win + tx0) * g.cs + g.coff + ci + sgn * (dky * g.Win + dkx) * g.cs;
}

// Implicit-GEMM gather, rows = output pixels, k = (tap, ci).  Either Cin % BK
// == 0 (a K tile lies inside one tap: the tap is wave-uniform) or BK % Cin == 0
// with the tile's BK/Cin taps forming whole kernel rows or part of one row (the
// per-chunk tap offset is then a per-thread constant).  Per chunk a fetch is
// one bit test of the pixel's precomputed valid-tap mask and one add.
template <typename G, typename T, int R, int BK, int NT>
struct LdIm2colB {
  static constexpr bool KC = true;
  static constexpr int VG = 16 / (int)sizeof(G);
  static constexpr int CPR = BK / VG;
  static constexpr int NCH = R * CPR;
  static constexpr int PER = (NCH + NT - 1) / NT;
  using Regs = u32x4[PER];
  struct Params { const G* src; ConvGeo g; int nrows; uint32_t src_bytes; };
  __amdgpu_buffer_rsrc_t rs;
  ConvGeo g;
  int base[PER];            // element offset of the chunk's source at the tile's first tap
  int dt[PER];              // tap of this chunk relative to the tile's first tap
  uint64_t vmask[PER];      // bit tap = that tap reads inside the input
  int ldo[PER];
  bool act[PER];
  __device__ static bool ok_shape(const ConvGeo& g) {
    if (g.Cin % BK == 0) return true;
    if (BK % g.Cin) return false;
    const int tpt = BK / g.Cin;
    return tpt % g.KW == 0 || g.KW % tpt == 0;
  }
  __device__ __forceinline__ LdIm2colB(const Params& p, int row0) : g(p.g) {
    rs = make_rsrc(p.src, p.src_bytes);
#pragma unroll
    for (int c = 0; c < PER; ++c) {
      const int ch = threadIdx.x + c * NT;
      act[c] = ch < NCH;
      const int lr = ch / CPR, kc = (ch % CPR) * VG, m = row0 + lr;
      im2col_setup(g, BK, act[c] && m < p.nrows, m, kc, base[c], dt[c], vmask[c]);
      ldo[c] = Tile<T, R, BK, true>::off(lr, kc);
    }
  }
  __device__ __forceinline__ void fetch(int k0, int, Regs& buf) const {
    const int tap = __builtin_amdgcn_readfirstlane((int)g.dCin.div(k0));
    const int ci0 = k0 - tap * g.Cin;
    const int ky = __builtin_amdgcn_readfirstlane((int)g.dKW.div(tap));
    const int kx = tap - ky * g.KW;
    const int toff = (g.transposed ? -(ky * g.Win + kx) : (ky * g.Win + kx)) * g.cs + ci0;
#pragma unroll
    for (int c = 0; c < PER; ++c) {
      const bool v = (vmask[c] >> (tap + dt[c])) & 1ull;
      buf[c] = bload(rs, v ? (uint32_t)((base[c] + toff) * (int)sizeof(G)) : kOOB);
    }
  }
  __device__ __forceinline__ void commit(T* lds, const Regs& buf) const {
#pragma unroll
    for (int c = 0; c < PER; ++c)
      if (NCH % NT == 0 || act[c]) lds_store_chunk<G, T>(lds + ldo[c], buf[c]);
  }
};

// Weight-gradient gather: rows = k' = (tap, ci) fixed per thread, k = output
// pixel m (forward geometry).  Cin % VG == 0, or (conv1's bordered bf16 RGBx
// image) a chunk spanning adjacent taps of one kernel row that are all in bounds.
template <typename G, typename T, int R, int BK, int NT>
struct LdIm2colTB {
  static constexpr bool KC = false;
  static constexpr int VG = 16 / (int)sizeof(G);
  static constexpr int CPK = R / VG;
  static constexpr int NCH = BK * CPK;
  static constexpr int PER = (NCH + NT - 1) / NT;
  using Regs = u32x4[PER];
  struct Params { const G* src; ConvGeo g; int nrows; uint32_t src_bytes; };
  __amdgpu_buffer_rsrc_t rs;
  ConvGeo g;
  int kr[PER], ky[PER], kx[PER], toff[PER];
  int ldo[PER];
  bool act[PER];
  __device__ __forceinline__ static int off16(int ch) { return Tile<__bf16, R, BK, false>::off((ch % CPK) * VG, ch / CPK); }
  __device__ __forceinline__ LdIm2colTB(const Params& p, int row0) : g(p.g) {
    rs = make_rsrc(p.src, p.src_bytes);
#pragma unroll
    for (int c = 0; c < PER; ++c) {
      const int ch = threadIdx.x + c * NT;
      const int rc = (ch % CPK) * VG, kp = row0 + rc;
      act[c] = ch < NCH;
      kr[c] = ch / CPK;
      const bool ok = act[c] && kp < p.nrows;
      const int kq = ok ? kp : 0;
      const int tap = (int)g.dCin.div(kq), ci = kq - tap * g.Cin;
      ky[c] = ok ? (int)g.dKW.div(tap) : -100000;  // invalid rows never pass the bounds test
      kx[c] = tap - (int)g.dKW.div(tap) * g.KW;
      toff[c] = (ky[c] * g.Win + kx[c]) * g.cs + ci + g.coff;
      ldo[c] = Tile<T, R, BK, false>::off(rc, kr[c]);
    }
  }
  __device__ __forceinline__ void fetch(int k0, int kend, Regs& buf) const {
    const int hw = g.Hout * g.Wout;
#pragma unroll
    for (int c = 0; c < PER; ++c) {
      const int m = k0 + kr[c];
      const int f = (int)g.dHW.div(m), pix = m - f * hw;
      const int oy = (int)g.dWout.div(pix), ox = pix - oy * g.Wout;
      const int iy0 = oy * g.stride - g.pad, ix0 = ox * g.stride - g.pad;
      const int iy = iy0 + ky[c], ix = ix0 + kx[c];
      const bool v = m < kend && (unsigned)iy < (unsigned)g.Hin && (unsigned)ix < (unsigned)g.Win;
      const int off = ((f * g.Hin + iy0) * g.Win + ix0) * g.cs + toff[c];
      buf[c] = bload(rs, v ? (uint32_t)(off * (int)sizeof(G)) : kOOB);
    }
  }
  __device__ __forceinline__ void commit(T* lds, const Regs& buf) const {
#pragma unroll
    for (int c = 0; c < PER; ++c)
      if (NCH % NT == 0 || act[c]) lds_store_chunk<G, T>(lds + ldo[c], buf[c]);
  }
  __device__ __forceinline__ void commit3(__bf16* lds, int plane, const Regs& buf) const {
#pragma unroll
    for (int c = 0; c < PER; ++c)
      if (NCH % NT == 0 || act[c]) lds_store_split3(lds + off16(threadIdx.x + c * NT), plane, buf[c]);
  }
  // the hi part only, for a source exact in bf16 (GemmCfgS6LBX)
  __device__ __forceinline__ void commit1(__bf16* lds, const Regs& buf) const {
#pragma unroll
    for (int c = 0; c < PER; ++c)
      if (NCH % NT == 0 || act[c]) lds_store_chunk<G, __bf16>(lds + off16(threadIdx.x + c * NT), buf[c]);
  }
};

}  // namespace aaa
