// Tail GEMMs (answer MLP, LSTMCell, policy / value heads: attention.py:339-366 and
// their backward) with a deep register pipeline.
//
// These GEMMs have few tiles (F = T*B rows) and a long serial K loop, and the
// register-staged gemm_kernel keeps one K tile of global loads in flight: each K
// tile then waits one full memory latency (C2: 16 tiles of the answer MLP's K =
// 1026 -> 17 us for 0.7 GFLOP).  gemm_kernel_deep issues NS tiles ahead into NS
// register stages; the loaders are branch-free (buffer loads, out-of-range
// offsets for rows past the matrix and k past the slice: the hardware returns
// zeros) so the compiler counts its vmcnt waits instead of draining them -- a
// guarded load whose other path zero-fills the same registers forces vmcnt(0)
// (recur_bwd.h load_in).  Same LDS tiles, fragments and MFMA sequence as
// gemm_kernel (gemm_mma_tile): bit-identical results.
#pragma once
#include "glds.h"

namespace aaa {

// Plain rows (LdRows' layout and LDS tile), element (row, k) at src[row*ld + k]; K % VG == 0.
template <typename G, typename T, int R, int BK, int NT>
struct LdRowsN {
  static constexpr bool KC = true;
  static constexpr int VG = 16 / (int)sizeof(G);
  static constexpr int CPR = BK / VG;
  static constexpr int NCH = R * CPR;
  static constexpr int PER = (NCH + NT - 1) / NT;
  struct Params { const G* src; int ld; int nrows; };
  __amdgpu_buffer_rsrc_t rs;
  int roff[PER], kc[PER], lr[PER];
  bool ok[PER], act[PER];
  using Regs = u32x4[PER];
  __device__ __forceinline__ LdRowsN(const Params& p, int row0) {
    rs = make_rsrc(p.src, (uint32_t)((size_t)p.nrows * p.ld * sizeof(G)));
#pragma unroll
    for (int c = 0; c < PER; ++c) {
      const int ch = threadIdx.x + c * NT;
      act[c] = ch < NCH;
      lr[c] = ch / CPR;
      kc[c] = (ch % CPR) * VG;
      const int row = row0 + lr[c];
      ok[c] = act[c] && row < p.nrows;
      roff[c] = (ok[c] ? row : 0) * p.ld;
    }
  }
  __device__ __forceinline__ void fetch(int k0, int kend, Regs& buf) const {
#pragma unroll
    for (int c = 0; c < PER; ++c) {
      const int k = k0 + kc[c];
      buf[c] = __builtin_amdgcn_raw_buffer_load_b128(
          rs, ok[c] && k < kend ? (uint32_t)((roff[c] + k) * (int)sizeof(G)) : kOOB, 0, 0);
    }
  }
  __device__ __forceinline__ void commit(T* lds, const Regs& buf) const {
#pragma unroll
    for (int c = 0; c < PER; ++c)
      if (NCH % NT == 0 || act[c]) lds_store_chunk<G, T>(lds + Tile<T, R, BK, true>::off(lr[c], kc[c]), buf[c]);
  }
  // split-at-commit part tiles (gemm_kernel_s6l): bf16 tiles of the same shape, ``plane`` elements apart
  __device__ __forceinline__ void commit3(__bf16* lds, int plane, const Regs& buf) const {
#pragma unroll
    for (int c = 0; c < PER; ++c)
      if (NCH % NT == 0 || act[c]) lds_store_split3(lds + Tile<__bf16, R, BK, true>::off(lr[c], kc[c]), plane, buf[c]);
  }
  __device__ __forceinline__ void commit2(__bf16* lds, int plane, const Regs& buf) const {
#pragma unroll
    for (int c = 0; c < PER; ++c)
      if (NCH % NT == 0 || act[c]) lds_store_split2(lds + Tile<__bf16, R, BK, true>::off(lr[c], kc[c]), plane, buf[c]);
  }
};

// Transposed rows (LdRowsT's layout), element (row, k) at src[k*ld + row]; nrows % VG == 0 (the host
// checks: a chunk is all in or all out), k bounded by the slice end only.
template <typename G, typename T, int R, int BK, int NT>
struct LdRowsTN {
  static constexpr bool KC = false;
  static constexpr int VG = 16 / (int)sizeof(G);
  static constexpr int CPK = R / VG;
  static constexpr int NCH = BK * CPK;
  static constexpr int PER = (NCH + NT - 1) / NT;
  struct Params { const G* src; int ld; int nrows; };
  __amdgpu_buffer_rsrc_t rs;
  int ld;
  int kr[PER], rc[PER], lc[PER];   // k row, absolute first row, tile-relative first row of the lane's chunk
  bool ok[PER], act[PER];
  using Regs = u32x4[PER];
  __device__ __forceinline__ LdRowsTN(const Params& p, int row0) : ld(p.ld) {
    rs = make_rsrc(p.src, 0x7fffffffu);   // k extent unknown here: rows and k are bounded per lane
#pragma unroll
    for (int c = 0; c < PER; ++c) {
      const int ch = threadIdx.x + c * NT;
      act[c] = ch < NCH;
      kr[c] = ch / CPK;
      lc[c] = (ch % CPK) * VG;
      rc[c] = row0 + lc[c];
      ok[c] = act[c] && rc[c] + VG <= p.nrows;
    }
  }
  __device__ __forceinline__ void fetch(int k0, int kend, Regs& buf) const {
#pragma unroll
    for (int c = 0; c < PER; ++c) {
      const int k = k0 + kr[c];
      buf[c] = __builtin_amdgcn_raw_buffer_load_b128(
          rs, ok[c] && k < kend ? (uint32_t)(((size_t)k * ld + rc[c]) * sizeof(G)) : kOOB, 0, 0);
    }
  }
  __device__ __forceinline__ void commit(T* lds, const Regs& buf) const {
#pragma unroll
    for (int c = 0; c < PER; ++c)
      if (NCH % NT == 0 || act[c]) lds_store_chunk<G, T>(lds + Tile<T, R, BK, false>::off(lc[c], kr[c]), buf[c]);
  }
  __device__ __forceinline__ void commit3(__bf16* lds, int plane, const Regs& buf) const {
#pragma unroll
    for (int c = 0; c < PER; ++c)
      if (NCH % NT == 0 || act[c]) lds_store_split3(lds + Tile<__bf16, R, BK, false>::off(lc[c], kr[c]), plane, buf[c]);
  }
  __device__ __forceinline__ void commit2(__bf16* lds, int plane, const Regs& buf) const {
#pragma unroll
    for (int c = 0; c < PER; ++c)
      if (NCH % NT == 0 || act[c]) lds_store_split2(lds + Tile<__bf16, R, BK, false>::off(lc[c], kr[c]), plane, buf[c]);
  }
};

// gemm_kernel with NS register stages of global loads in flight (NS even: the LDS double buffer's
// parity is then the stage's).  Per K tile kt: refill the stage tile kt came from with tile kt + NS,
// the MFMAs of tile kt from LDS, tile kt + 1 committed from its stage, one barrier (LDS counter only:
// the stages' loads stay in flight across it).
template <class C, class LA, class LB, class EP, int NS>
__global__ void __launch_bounds__(C::NT)
gemm_kernel_deep(typename LA::Params pa, typename LB::Params pb, EP ep, int K, int kchunk, TileMap tm) {
  static_assert(NS >= 2 && NS % 2 == 0, "stages");
  using T = typename C::type;
  constexpr int BI = C::BI, BJ = C::BJ, BK = C::BK, WI = C::WI, WJ = C::WJ, WK = C::WK;
  constexpr int WTI = BI / WI, WTJ = BJ / WJ, MI = WTI / 32, MJ = WTJ / 32;
  using TA = TileK<T, BI, BK, LA::KC>;
  using TB = TileK<T, BJ, BK, LB::KC>;
  __shared__ __attribute__((aligned(16))) T smem[2 * (TA::ELEMS + TB::ELEMS)];
  T* const As[2] = {smem, smem + TA::ELEMS};
  T* const Bs[2] = {smem + 2 * TA::ELEMS, smem + 2 * TA::ELEMS + TB::ELEMS};

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
  typename LA::Regs ra[NS];
  typename LB::Regs rb[NS];
  // every fetch and commit unconditional (tiles past the slice load zeros: k >= kend is out of range):
  // a uniform branch around them made the compiler drain vmcnt at its merge points
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    la.fetch(kb + s * BK, ke, ra[s]);
    lb.fetch(kb + s * BK, ke, rb[s]);
  }
  la.commit(As[0], ra[0]);
  lb.commit(Bs[0], rb[0]);
  barrier_lds();
  for (int kt0 = 0; kt0 < nk; kt0 += NS) {
#pragma unroll
    for (int j = 0; j < NS; ++j) {
      const int kt = kt0 + j;
      if (kt >= nk) break;
      la.fetch(kb + (kt + NS) * BK, ke, ra[j]);   // stage j held tile kt, committed one barrier ago
      lb.fetch(kb + (kt + NS) * BK, ke, rb[j]);
      gemm_mma_tile<C, TA, TB, MI, MJ>(As[j & 1], Bs[j & 1], acc, wi, wj, wk, r32, h);
      la.commit(As[(j + 1) & 1], ra[(j + 1) % NS]);   // (past the last tile: zeros nobody reads)
      lb.commit(Bs[(j + 1) & 1], rb[(j + 1) % NS]);
      barrier_lds();
    }
  }

  if constexpr (WK > 1) {   // sum the WK partial accumulators through LDS (as gemm_kernel)
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

template <class C, class LA, class LB, class EP, int NS>
inline hipError_t launch_gemm_deep(const typename LA::Params& pa, const typename LB::Params& pb, const EP& ep, int Mi,
                                   int Nj, int K, int nsplit, hipStream_t st) {
  if (Mi <= 0 || Nj <= 0 || K <= 0) return hipSuccess;
  if (nsplit < 1) nsplit = 1;
  int kchunk = (K + nsplit - 1) / nsplit;
  kchunk = (kchunk + C::BK - 1) / C::BK * C::BK;
  nsplit = (K + kchunk - 1) / kchunk;
  dim3 grid((Nj + C::BJ - 1) / C::BJ, (Mi + C::BI - 1) / C::BI, nsplit);
  hipLaunchKernelGGL((gemm_kernel_deep<C, LA, LB, EP, NS>), grid, dim3(C::NT), 0, st, pa, pb, ep, K, kchunk,
                     tile_map(grid));
  return hipGetLastError();
}

}  // namespace aaa
