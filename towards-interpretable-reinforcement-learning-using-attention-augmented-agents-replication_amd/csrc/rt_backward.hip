// Backward of the unroll (what autograd runs for main_mp.py:77): the batched
// tail backward, the ConvLSTM BPTT (frame-resident / frame-group / per-step),
// the conv / ConvLSTM weight gradients and the vision encoder backward.
#include "rt.h"

namespace aaa {


// conv2 dgrad (stride 2, k4, pad 2) as four parity-class 2x2 convs over dY2:
// output pixel (2a+py, 2b+px) only receives taps ky = py + 2(1-ty), kx = px + 2(1-tx).
template <typename T>
static int conv2_dgrad(const Layout& L, const char* pk, const T* dy2, T* dy1, int frames, float* gbias,
                       hipStream_t s) {
  {
    // small grids: the four classes share one gather (output (a, b) reads dY2
    // (a + ty, b + tx)), so one 128-row tile (class-major rows, [cls][32][256]
    // = k_WdT2) per frame reads the frame's dY2 once as a zero-bordered LDS
    // image (halo.h, KS = 2) -- one launch instead of four 32-row GEMMs whose
    // K = 256 loops were pure latency (4 x 65 us at C3, 0.06 of bf16 peak)
    constexpr int CKd = std::is_same<T, float>::value ? 32 : 64;
    const int Ha = (L.H1 + 1) / 2, Wa = (L.W1 + 1) / 2;
    auto halo4 = [&](auto cfg, auto nbuf) -> int {
      using HC = decltype(cfg);
      EpiStoreParity4<T> ep(dy1, frames * Ha * Wa, Ha, Wa, L.H1, L.W1, gbias);
      const HaloParams hp{pk + L.k_WdT2, 256, 128, dy2, 64, 0, 64, (uint32_t)((size_t)frames * L.P * 64 * L.esz),
                          L.h, L.w, frames, 0, Ha, Wa};
      HIPCHK((launch_halo<HC, EpiStoreParity4<T>, 2, decltype(nbuf)::value>(hp, ep, s)));
      return AAA_OK;
    };
    using NB3 = std::integral_constant<int, 3>;
    auto fits = [&](int fr, int bj, int hmax) {
      return fr * Ha * Wa <= bj && fr * (L.h + 2) * (L.w + 2) + 1 <= hmax && Ha <= L.h && Wa <= L.w;
    };
    // bf16: FR = 2 frames per tile -- the 64 KB weight tile streamed once per two frames and twice the
    // MFMA work per DMA round trip (C3 4.97 -> 4.94 ms); fp32 keeps FR = 1 (C2 4.306 vs 4.341 ms)
    // (profiles/r02/ab/dgrad_fr.txt; AAA_DGRAD2_FR overrides)
    const int fr = ab_int("AAA_DGRAD2_FR", std::is_same<T, float>::value ? 1 : 2);
    if (ab_int("AAA_DGRAD2_HALO", 1)) {
      if (fr == 2 && fits(2, 256, 352)) return halo4(HaloCfg<T, 128, 256, CKd, 2, 2, 2, 352>{}, NB3{});
      if constexpr (std::is_same<T, float>::value) {   // fp32 accuracy on the bf16 MFMA (gemm.h SPLIT6)
        // AAA_DGRAD2_NBUF=2 (A/B): a 2-stage weight ring, 80 KB of LDS -> two workgroups per CU
        if (f32_split6() && fits(1, 128, 192)) {
          if (ab_int("AAA_DGRAD2_NBUF", 3) == 2)
            return halo4(HaloCfgS6<128, 128, CKd, 2, 2, 1, 192>{}, std::integral_constant<int, 2>{});
          return halo4(HaloCfgS6<128, 128, CKd, 2, 2, 1, 192>{}, NB3{});
        }
      }
      if (fits(1, 128, 192)) return halo4(HaloCfg<T, 128, 128, CKd, 2, 2, 1, 192>{}, NB3{});
      // bf16, grids up to 21x21 (168x168 frames, C5): one frame per 512-column tile of 8 waves,
      // 32-channel chunks (two LDS images of 23x23 pixels), the epilogue in two column chunks
      if constexpr (!std::is_same<T, float>::value)
        if (fits(1, 512, 640) && ab_int("AAA_DGRAD2_WIDE", 1)) return halo4(HaloCfg<T, 128, 512, 32, 2, 4, 1, 640>{}, NB3{});
    }
  }
  if (ab_int("AAA_CONV2_DGRAD_RING", 1)) {
    // the LDS-DMA ring (dY2 is already in T), dY1 stored in T, conv1's bias
    // gradient summed from the fp32 values in the epilogue (no column-sum pass)
    constexpr int BKd = std::is_same<T, float>::value ? 32 : 64;
    auto classes = [&](auto cfg) -> int {
      using CP = decltype(cfg);
      using PA = GRowsB<T, CP::BI, CP::BK, CP::NT>;
      using PB = GIm2colB<T, CP::BJ, CP::BK, CP::NT>;
      for (int cls = 0; cls < 4; ++cls) {
        const int py = cls >> 1, px = cls & 1;
        const int Ha = (L.H1 - py + 1) / 2, Wa = (L.W1 - px + 1) / 2;
        if (Ha <= 0 || Wa <= 0) continue;
        const int rows = frames * Ha * Wa;
        EpiStoreParityBias<T> ep{dy1, 32, rows, Ha, Wa, L.H1, L.W1, py, px, gbias};
        HIPCHK((launch_pipe<CP, PA, PB, EpiStoreParityBias<T>, 2>(
            typename PA::Params{(const T*)(pk + L.k_WdT2) + (size_t)cls * 32 * 256, 256, 32},
            typename PB::Params{dy2, ConvGeo{64, 64, 0, L.h, L.w, Ha, Wa, 2, 1, 0, 0}.prep(), rows,
                                (uint32_t)((size_t)frames * L.P * 64 * L.esz)},
            ep, 32, rows, 256, 1, s)));
      }
      return AAA_OK;
    };
    // K = 256: four BK steps per tile, so 256 columns per workgroup (twice the MFMA work per DMA round
    // trip of 32x128): C5 14.945 -> 14.74 ms per iteration (profiles/r02/ab/vision_tiles.txt); AAA_DGRAD2_TILE=0 the old tile
    return ab_int("AAA_DGRAD2_TILE", 1) == 1 ? classes(GemmCfg<T, 32, 256, BKd, 1, 4>{})
                                             : classes(GemmCfg<T, 32, 128, BKd, 1, 4>{});
  }
  // register-staged fallback (fp32 only: dY2's loader converts from fp32)
  if constexpr (!std::is_same<T, float>::value) return fail(AAA_E_ARG, "AAA_CONV2_DGRAD_RING=0 needs fp32");
  using C3 = Cfg32For<T>;
  using LA = LdRowsB<T, T, C3::BI, C3::BK, C3::NT>;
  using LB = LdIm2colB<float, T, C3::BJ, C3::BK, C3::NT>;
  for (int cls = 0; cls < 4; ++cls) {
    const int py = cls >> 1, px = cls & 1;
    const int Ha = (L.H1 - py + 1) / 2, Wa = (L.W1 - px + 1) / 2;
    if (Ha <= 0 || Wa <= 0) continue;
    const int rows = frames * Ha * Wa;
    typename LA::Params pa{(const T*)(pk + L.k_WdT2) + (size_t)cls * 32 * 256, 256, 32};
    typename LB::Params pb{(const float*)dy2, ConvGeo{64, 64, 0, L.h, L.w, Ha, Wa, 2, 1, 0, 0}.prep(), rows,
                           (uint32_t)((size_t)frames * L.P * 64 * 4)};
    EpiStoreParity ep{(float*)dy1, 32, rows, Ha, Wa, L.H1, L.W1, py, px, FastDiv((uint32_t)(Ha * Wa)),
                      FastDiv((uint32_t)Wa)};
    HIPCHK((launch_gemm<C3, LA, LB>(pa, pb, ep, 32, rows, 256, 1, s)));
  }
  return AAA_OK;
}

// conv2 weight gradient over ``frames`` frames: gW[64][(ky*4+kx)*32 + ci] +=
// dY2^T x im2col(Y1) (k = output pixel), split-K atomics into a zeroed gW.
template <typename T>
static int conv2_wgrad(const Layout& L, const T* dy2, const T* y1, int frames, float* gW, hipStream_t s) {
  using C = CfgFor<T>;
  using LA = LdRowsTB<T, T, C::BI, C::BK, C::NT>;
  using LB = LdIm2colTB<T, T, C::BJ, C::BK, C::NT>;
  const int rows = frames * L.P;
  if constexpr (!std::is_same<T, float>::value) {
    // bf16 (AAA_CONV2_WGRAD_PIPE): the LDS-DMA ring of the ConvLSTM weight gradient, 64x256
    // tiles of 4 waves, split-K over about one wave of workgroups, atomics from the accumulators
    // default 1 (C3 1.063M -> 1.075M frames/s, C5 277.4k -> 279.0k vs the register-staged GEMM;
    // 2 = the read-ahead ring, slower here: profiles/r03/ab/convwgrad/); 0 = register-staged
    const int pipe = ab_int("AAA_CONV2_WGRAD_PIPE", 1);
    if (rows % 32 == 0 && pipe) {
      using CW = GemmCfg<T, 64, 256, 32, 1, 4>;
      using PA = GRowsT<T, CW::BI, CW::BK, CW::NT>;
      using PB = GIm2colT<T, CW::BJ, CW::BK, CW::NT>;
      typename PA::Params pa{dy2, 64, 64, rows};
      typename PB::Params pb{y1, ConvGeo{32, 32, 0, L.H1, L.W1, L.h, L.w, 4, 2, 2, 0}.prep(), 512,
                             (uint32_t)((size_t)frames * L.P1 * 32 * L.esz)};
      EpiAtomicD ep{{gW, 512, 64, 512}};
      const int ns = std::max(1, std::min(ab_int("AAA_CONV2_WGRAD_WGS", 256) / 2, rows / (8 * CW::BK)));
      if (pipe == 2) HIPCHK((launch_pipe_ra<CW, PA, PB, EpiAtomicD, 4>(pa, pb, ep, 64, 512, rows, ns, s)));
      else HIPCHK((launch_pipe<CW, PA, PB, EpiAtomicD, 4, 2>(pa, pb, ep, 64, 512, rows, ns, s)));
      return AAA_OK;
    }
  }
  typename LA::Params pa{dy2, 64, 64, rows};
  typename LB::Params pb{y1, ConvGeo{32, 32, 0, L.H1, L.W1, L.h, L.w, 4, 2, 2, 0}.prep(), 512,
                         (uint32_t)((size_t)frames * L.P1 * 32 * L.esz)};
  EpiStore<true> ep{gW, 512, 64, 512};
  const int tiles = cdiv(64, C::BI) * cdiv(512, C::BJ);
  if constexpr (std::is_same<T, float>::value) {
    if (f32_split6()) {   // the same tile at fp32 accuracy on the bf16 MFMA (gemm.h SPLIT6)
      // A/B (AAA_CONV2_WGRAD_S6L, ablation builds): split-at-commit tiles -- slower here (C2 59.4 ->
      // 67.9 us for 64x256, profiles/r05/ab/conv_wgrad_s6l/)
      auto s6l = [&](auto cfg, int ns) -> int {
        using CW = decltype(cfg);
        using LA6 = LdRowsTB<T, T, CW::BI, CW::BK, CW::NT>;
        using LB6 = LdIm2colTB<T, T, CW::BJ, CW::BK, CW::NT>;
        typename LA6::Params pa6{dy2, 64, 64, rows};
        typename LB6::Params pb6{y1, ConvGeo{32, 32, 0, L.H1, L.W1, L.h, L.w, 4, 2, 2, 0}.prep(), 512,
                                 (uint32_t)((size_t)frames * L.P1 * 32 * L.esz)};
        HIPCHK((launch_gemm<CW, LA6, LB6>(pa6, pb6, ep, 64, 512, rows, std::max(1, std::min(ns, rows / 128)), s)));
        return AAA_OK;
      };
#ifdef AAA_ABLATION
      const int c2s = ab_int("AAA_CONV2_WGRAD_S6L", 0);
      if (c2s == 1) return s6l(GemmCfgS6L<64, 256, 16, 1, 4, 2>{}, 256);
      if (c2s == 2) return s6l(GemmCfgS6L<64, 256, 16, 2, 4, 2>{}, 128);
      if (c2s == 3) return s6l(GemmCfgS6L<64, 128, 16, 1, 2, 2>{}, 256);
#else
      (void)s6l;
#endif
      HIPCHK((launch_gemm<typename S6Of<C>::type, LA, LB>(pa, pb, ep, 64, 512, rows, wgrad_splits(tiles, rows, C::BK), s)));
      return AAA_OK;
    }
  }
  HIPCHK((launch_gemm<C, LA, LB>(pa, pb, ep, 64, 512, rows, wgrad_splits(tiles, rows, C::BK), s)));
  return AAA_OK;
}

// conv1 weight gradient over RGBx frames (Cin 4; the 4th channel's grad is dropped on unpack)
template <typename T>
static int conv1_wgrad(const Layout& L, const T* dy1, const T* xp, int frames, float* gW, hipStream_t s) {
  const int rows1 = frames * L.P1;
  auto run = [&](auto cfg) -> int {
    using C3 = decltype(cfg);
    using LA = LdRowsTB<T, T, C3::BI, C3::BK, C3::NT>;
    using LB = LdIm2colTB<T, T, C3::BJ, C3::BK, C3::NT>;   // bf16 chunks = 2 taps x 4 ch, in-bounds (bordered image)
    typename LA::Params pa{dy1, 32, 32, rows1};
    typename LB::Params pb{xp, ConvGeo{4, 4, 0, L.H + 2, L.W + 2, L.H1, L.W1, 8, 4, 0, 0}.prep(), 256,
                           (uint32_t)((size_t)frames * (L.H + 2) * (L.W + 2) * 4 * L.esz)};
    EpiStore<true> ep{gW, 256, 32, 256};
    const int tiles = cdiv(32, C3::BI) * cdiv(256, C3::BJ);
    if constexpr (std::is_same<T, float>::value) {
      if (f32_split6()) {   // fp32 accuracy on the bf16 MFMA (gemm.h SPLIT6)
        HIPCHK((launch_gemm<typename S6Of<C3>::type, LA, LB>(pa, pb, ep, 32, 256, rows1,
                                                            wgrad_splits(tiles, rows1, C3::BK), s)));
        return AAA_OK;
      }
    }
    HIPCHK((launch_gemm<C3, LA, LB>(pa, pb, ep, 32, 256, rows1, wgrad_splits(tiles, rows1, C3::BK), s)));
    return AAA_OK;
  };
  if constexpr (!std::is_same<T, float>::value) {
    // bf16 on the LDS-DMA rings (AAA_CONV1_WGRAD_PIPE 1: pipe, 2: read-ahead): one 32x256 tile of 4
    // waves over all (tap, channel) columns, BK = 64 pixels; a 16-B piece = 2 taps x 4 channels,
    // contiguous in the bordered RGBx image (KW = 8 even, pad 0: every piece in bounds)
    // default 1 (C3 +0.5 %, C5 +0.8 % vs the register-staged GEMM: profiles/r03/ab/convwgrad/)
    const int pipe = ab_int("AAA_CONV1_WGRAD_PIPE", 1);
    if (rows1 % 64 == 0 && pipe) {
      using CW = GemmCfg<T, 32, 256, 64, 1, 4>;
      using PA = GRowsT<T, CW::BI, CW::BK, CW::NT>;
      using PB = GIm2colT<T, CW::BJ, CW::BK, CW::NT>;
      typename PA::Params pa{dy1, 32, 32, rows1};
      typename PB::Params pb{xp, ConvGeo{4, 4, 0, L.H + 2, L.W + 2, L.H1, L.W1, 8, 4, 0, 0}.prep(), 256,
                             (uint32_t)((size_t)frames * (L.H + 2) * (L.W + 2) * 4 * L.esz)};
      EpiAtomicD ep{{gW, 256, 32, 256}};
      const int ns = std::max(1, std::min(ab_int("AAA_CONV1_WGRAD_WGS", 256), rows1 / (8 * CW::BK)));
      if (pipe == 2) HIPCHK((launch_pipe_ra<CW, PA, PB, EpiAtomicD, 4>(pa, pb, ep, 32, 256, rows1, ns, s)));
      else HIPCHK((launch_pipe<CW, PA, PB, EpiAtomicD, 4, 2>(pa, pb, ep, 32, 256, rows1, ns, s)));
      return AAA_OK;
    }
  }
  if constexpr (std::is_same<T, float>::value) {
    // split-at-commit tile over all 256 (tap, channel) columns (GemmCfgS6L: each operand split once
    // at its LDS commit, two K tiles of loads in flight), 512-way split-K: C2 76.9 -> 66.9 us against
    // the 32x64 split6 tile (AAA_CONV1_WGRAD_S6L=0 in ablation builds; 2, 3: other tiles / splits,
    // slower: profiles/r05/ab/conv_wgrad_s6l/)
    const int c1s = f32_split6() ? ab_int("AAA_CONV1_WGRAD_S6L", 1) : 0;
    auto s6l = [&](auto cfg, int ns) -> int {
      using CW = decltype(cfg);
      using LA6 = LdRowsTB<T, T, CW::BI, CW::BK, CW::NT>;
      using LB6 = LdIm2colTB<T, T, CW::BJ, CW::BK, CW::NT>;
      typename LA6::Params pa6{dy1, 32, 32, rows1};
      typename LB6::Params pb6{xp, ConvGeo{4, 4, 0, L.H + 2, L.W + 2, L.H1, L.W1, 8, 4, 0, 0}.prep(), 256,
                               (uint32_t)((size_t)frames * (L.H + 2) * (L.W + 2) * 4 * L.esz)};
      EpiStore<true> ep6{gW, 256, 32, 256};
      HIPCHK((launch_gemm<CW, LA6, LB6>(pa6, pb6, ep6, 32, 256, rows1, std::max(1, std::min(ns, rows1 / 128)), s)));
      return AAA_OK;
    };
    if (c1s == 1)   // uint8 frames: the RGBx operand exact in bf16 (GemmCfgS6LBX: three of the six products)
      return L.fu8 && ab_int("AAA_CONV1_BEXACT", 1) ? s6l(GemmCfgS6LBX<32, 256, 16, 1, 4, 2>{}, 512)
                                                     : s6l(GemmCfgS6L<32, 256, 16, 1, 4, 2>{}, 512);
#ifdef AAA_ABLATION
    if (c1s == 2) return s6l(GemmCfgS6L<32, 256, 16, 1, 4, 2>{}, 256);
    if (c1s == 3) return s6l(GemmCfgS6L<32, 128, 16, 1, 2, 2>{}, 512);
#endif
  }
  // AAA_CONV1_WGRAD_TILE=1 (A/B): one 32x256 tile covering every (tap, channel) column, so each
  // pixel's 8x8 window is gathered once instead of by four 64-column tiles
  if (ab_int("AAA_CONV1_WGRAD_TILE", 0) == 1) return run(GemmCfg<T, 32, 256, Cfg32For<T>::BK, 1, 4>{});
  return run(Cfg32For<T>{});
}

// All 8 ConvLSTM weight gradients of ``rows`` pixels at once (attention.py:39-102
// as used at :119-122): gW[512 = 4ch+gate][1728 = tap*192 + c'] += dZ^T x
// im2col(XH) with k = pixel, accumulated (split-K atomics) into a zeroed gW.
// ``aux``: issued on the low-priority overlap stream.
template <typename T>
int lstm_wgrad(const T* dz, const T* xh, int rows, int h, int w, float* gW, hipStream_t s, bool aux) {
  const uint32_t xh_bytes = (uint32_t)((size_t)rows * 192 * sizeof(T));
  auto wgrad_lstm = [&](auto cfg) -> int {   // all 8 ConvLSTM weight grads: D[512][1728] += dZ^T * im2col(XH)
    using CW = decltype(cfg);
    using LA = LdRowsTB<T, T, CW::BI, CW::BK, CW::NT>;
    using LB = LdIm2colTB<T, T, CW::BJ, CW::BK, CW::NT>;
    typename LA::Params pa{dz, 512, 512, rows};
    typename LB::Params pb{xh, ConvGeo{192, 192, 0, h, w, h, w, 3, 1, 1, 0}.prep(),
                           1728, xh_bytes};
    EpiStore<true> ep{gW, 1728, 512, 1728};
    const int tiles = cdiv(512, CW::BI) * cdiv(1728, CW::BJ);
    // about two workgroups per CU of splits (both fit a CU; the 1024-WG rule of
    // the other weight gradients doubled the output atomics for the same time:
    // profiles/r02/ab/wgrad_split.txt)
    // (split-at-commit tiles hold 110 KB of LDS: one workgroup per CU, so one split per CU:
    // C2 655 us at 18-way against 679 at 36 and 845 at 27, profiles/r05/ab/wgrad_s6l/)
    const int per_cu = split6l_of<CW>::value ? device_cus() : 512;
    const int ns = std::max(1, std::min(ab_int("AAA_WGRAD_SPLIT", std::max(1, per_cu / tiles)), rows / CW::BK));
    TimerScope tim(AAA_TIMER_CORE_WGRAD, s, 2.0 * 512 * 1728 * rows,
                   strf("register-staged %dx%d BK%d%s, %d-way split-K atomics [kernel: gemm_kernel+%d, %d, %d, +LdIm2colTB]",
                        CW::BI, CW::BJ, CW::BK, split6_of<CW>::value ? " (fp32 as bf16x6 split products)" : "", ns,
                        CW::BI, CW::BJ, CW::BK));
    HIPCHK((launch_gemm<CW, LA, LB>(pa, pb, ep, 512, 1728, rows, ns, s)));
    return AAA_OK;
  };
  // LDS-DMA ring with transposed fragment reads for both operands (k = pixel)
  // and the split-K atomics straight from the accumulators
  auto wgrad_lstm_pipe = [&](auto cfg, auto nbuf, auto ilv) -> int {
    using CW = decltype(cfg);
    constexpr int NB = decltype(nbuf)::value, IL = decltype(ilv)::value;
    using LA = GRowsT<T, CW::BI, CW::BK, CW::NT>;
    using LB = GIm2colT<T, CW::BJ, CW::BK, CW::NT>;
    typename LA::Params pa{dz, 512, 512, rows};
    typename LB::Params pb{xh, ConvGeo{192, 192, 0, h, w, h, w, 3, 1, 1, 0}.prep(),
                           1728, xh_bytes};
    EpiAtomicD ep{{gW, 1728, 512, 1728}};
    const int tiles = cdiv(512, CW::BI) * cdiv(1728, CW::BJ);
    TimerScope tim(AAA_TIMER_CORE_WGRAD, s, 2.0 * 512 * 1728 * rows, strf("LDS-DMA ring %dx%d BK%d, %d-deep [kernel: gemm_pipe_kernel+GIm2colT]", CW::BI, CW::BJ, CW::BK, NB));
    // split-K over pixels: about one resident wave of workgroups (fewer
    // passes of the output's atomics than the register path's ~1024)
    const int wgs = ab_int("AAA_WGRAD_WGS", 256);
    const int ns = std::max(1, std::min(wgs / tiles, rows / (8 * CW::BK)));
    HIPCHK((launch_pipe<CW, LA, LB, EpiAtomicD, NB, IL>(pa, pb, ep, 512, 1728, rows, ns, s)));
    return AAA_OK;
  };
  // read-ahead ring (glds.h gemm_pipe_ra_kernel): fragments of tile kt+1 read during the MFMAs of tile kt
  auto wgrad_lstm_ra = [&](auto cfg, auto nbuf) -> int {
    using CW = decltype(cfg);
    constexpr int NB = decltype(nbuf)::value;
    using LA = GRowsT<T, CW::BI, CW::BK, CW::NT>;
    using LB = GIm2colT<T, CW::BJ, CW::BK, CW::NT>;
    typename LA::Params pa{dz, 512, 512, rows};
    typename LB::Params pb{xh, ConvGeo{192, 192, 0, h, w, h, w, 3, 1, 1, 0}.prep(), 1728, xh_bytes};
    EpiAtomicD ep{{gW, 1728, 512, 1728}};
    const int tiles = cdiv(512, CW::BI) * cdiv(1728, CW::BJ);
    TimerScope tim(AAA_TIMER_CORE_WGRAD, s, 2.0 * 512 * 1728 * rows,
                   strf("LDS-DMA read-ahead ring %dx%d BK%d, %d-deep [kernel: gemm_pipe_ra_kernel+GIm2colT]", CW::BI, CW::BJ, CW::BK, NB));
    const int wgs = ab_int("AAA_WGRAD_WGS", 256);
    const int ns = std::max(1, std::min(wgs / tiles, rows / (8 * CW::BK)));
    HIPCHK((launch_pipe_ra<CW, LA, LB, EpiAtomicD, NB>(pa, pb, ep, 512, 1728, rows, ns, s)));
    return AAA_OK;
  };
  // bf16 default (9): 256x256 (8 waves of 128x64), BK=32 in a 4-deep read-ahead
  // ring (C3 941 vs 988 us for the same tile with the reads behind each barrier
  // (6), C4 516 vs 531, C5 2206 vs 2235: profiles/r03/ab/wgrad_ra_*.json; round 2:
  // 6 at 1163 us vs 1296 for BK=64 in a 2-deep ring and 1400 register-staged)
  constexpr int WBK = std::is_same<T, float>::value ? 32 : 64;
  // (not on the aux stream: its 128 KB of LDS would keep the chain's step kernels off the CU)
  const int wpipe = rows % WBK == 0 ? env_int("AAA_WGRAD_PIPE", std::is_same<T, float>::value || aux ? 0 : 9) : 0;
  if (wpipe) {
    using I0 = std::integral_constant<int, 0>;
    using I2 = std::integral_constant<int, 2>;
    using I3 = std::integral_constant<int, 3>;
    int rc;
    switch (wpipe) {
      case 2: rc = wgrad_lstm_pipe(GemmCfg<T, 256, 128, WBK, 2, 2>{}, I2{}, I0{}); break;
      case 3:   // 8 waves of 128x64 (fp32: spills, so 256x128)
        if constexpr (std::is_same<T, float>::value) rc = wgrad_lstm_pipe(GemmCfg<T, 256, 128, WBK, 2, 2>{}, I2{}, I0{});
        else rc = wgrad_lstm_pipe(GemmCfg<T, 256, 256, WBK, 2, 4>{}, I2{}, I0{});
        break;
      case 4: rc = wgrad_lstm_pipe(GemmCfg<T, 128, 256, WBK, 2, 2>{}, I2{}, I0{}); break;
      case 5: rc = wgrad_lstm_pipe(GemmCfg<T, 256, 128, WBK, 2, 2>{}, I3{}, I0{}); break;
      case 6:   // bf16: 8 waves, BK=32, 4-deep ring, spread DMA issue
      case 7:   // bf16: the same in a 3-deep ring
        if constexpr (std::is_same<T, float>::value)
          rc = wgrad_lstm_pipe(GemmCfg<T, 128, 128, WBK, 2, 2>{}, I3{}, I2{});
        else if (wpipe == 6)
          rc = wgrad_lstm_pipe(GemmCfg<T, 256, 256, 32, 2, 4>{}, std::integral_constant<int, 4>{}, I2{});
        else
          rc = wgrad_lstm_pipe(GemmCfg<T, 256, 256, 32, 2, 4>{}, I3{}, I2{});
        break;
      case 8:   // bf16: 4 waves of 128x128 (half the LDS fragment reads per MFMA of the 8-wave tile), 4-deep ring:
                // measured slower (C3 1367 vs 1079 us, C4 691 vs 561 us: one wave per SIMD hides less)
        if constexpr (std::is_same<T, float>::value)
          rc = wgrad_lstm_pipe(GemmCfg<T, 128, 128, WBK, 2, 2>{}, I3{}, I2{});
        else
          rc = wgrad_lstm_pipe(GemmCfg<T, 256, 256, 32, 2, 2>{}, std::integral_constant<int, 4>{}, I2{});
        break;
      case 9:   // bf16: read-ahead ring, 8 waves, BK=32, 4-deep
        if constexpr (std::is_same<T, float>::value)
          rc = wgrad_lstm_pipe(GemmCfg<T, 128, 128, WBK, 2, 2>{}, I3{}, I2{});
        else
          rc = wgrad_lstm_ra(GemmCfg<T, 256, 256, 32, 2, 4>{}, std::integral_constant<int, 4>{});
        break;
      default: rc = wgrad_lstm_pipe(GemmCfg<T, 128, 128, WBK, 2, 2>{}, I2{}, I0{}); break;
    }
    if (rc) return rc;
  } else if (std::is_same<T, float>::value && f32_split6()) {
    // fp32: the register-staged 128x128 tile on the bf16 MFMA with three-way split operands (gemm.h SPLIT6)
    // AAA_WGRAD_S6_TILE (A/B): 0 = 128x128, 1 = 128x256, 2 = 256x128 (4 waves: fewer operand splits per
    // MFMA), 3 = 256x256 (8 waves of 128x64), the default: C2 842 / 936 / 832 / 729 us
    // (profiles/r04/ab/split6_tiles_c2_*.json)
    auto s6 = [&](auto cfg) {
      using CS6 = std::conditional_t<std::is_same<T, float>::value, decltype(cfg), CfgWFor<T>>;
      return wgrad_lstm(CS6{});
    };
    // 4 = 256x256 with each operand split once where it is committed to LDS (GemmCfgS6L, BK16,
    // two stages of bf16 part tiles); 5 = its 256x128 4-wave form; 6 (default) = 4 with two K
    // tiles of loads in flight: C2 633 vs 646 us (4) vs 776 (3) (profiles/r05/ab/wgrad_s6l/)
    // (tiles 0-5: ablation builds only)
#ifdef AAA_ABLATION
    const int tile6 = ab_int("AAA_WGRAD_S6_TILE", 6);
    const int rc = tile6 == 1   ? s6(GemmCfgS6<128, 256, 32, 2, 2>{})
                   : tile6 == 2 ? s6(GemmCfgS6<256, 128, 32, 2, 2>{})
                   : tile6 == 3 ? s6(GemmCfgS6<256, 256, 32, 2, 4>{})
                   : tile6 == 4 ? s6(GemmCfgS6L<256, 256, 16, 2, 4>{})
                   : tile6 == 5 ? s6(GemmCfgS6L<256, 128, 16, 2, 2>{})
                   : tile6 == 6 ? s6(GemmCfgS6L<256, 256, 16, 2, 4, 2>{})
                   : tile6 == 7 ? s6(GemmCfgS6L<256, 192, 16, 4, 2, 2>{})
                                : s6(GemmCfgS6<128, 128, 32, 2, 2>{});
#else
    const int rc = s6(GemmCfgS6L<256, 256, 16, 2, 4, 2>{});
#endif
    if (rc) return rc;
  } else {
    // on the aux stream a small-footprint tile lets the chain's step kernels co-reside on a CU
    const int wide = ab_int("AAA_AUX_WIDE", aux ? 0 : 1);
#ifdef AAA_ABLATION   // AAA_WGRAD_TILE=1: 128x192 tiles, 1728 = 9 x 192 columns without the half-empty last tile
    const int rc = !wide ? wgrad_lstm(CfgFor<T>{})
                   : ab_int("AAA_WGRAD_TILE", 0) == 1 ? wgrad_lstm(GemmCfg<T, 128, 192, 32, 2, 2>{})
                                                       : wgrad_lstm(CfgWFor<T>{});
#else
    const int rc = !wide ? wgrad_lstm(CfgFor<T>{}) : wgrad_lstm(CfgWFor<T>{});
#endif
    if (rc) return rc;
  }
  return AAA_OK;
}

// conv1 weight gradient over n frames whose bordered RGBx image (Xp) is
// rebuilt from the observation in chunks of L.xpc frames into the chunk
// buffer xpbuf: the forward keeps no Xp, and each chunk is written and read
// back while it sits in the memory-side cache (256 MB) instead of all F
// frames' images round-tripping through HBM between the two passes.
template <typename T>
static int conv1_wgrad_frames(const Layout& L, const T* dy1, const void* frames, int n, T* xpbuf, float* gW,
                              hipStream_t s) {
  const size_t fb = (size_t)L.H * L.W * 3 * (L.fu8 ? 1 : 4);
  for (int s0 = 0; s0 < n; s0 += L.xpc) {
    const int m = std::min(L.xpc, n - s0);
    const char* fr = (const char*)frames + (size_t)s0 * fb;
    if (L.fu8) HIPCHK((frames_rgbx<T, uint8_t>(m, L.H, L.W, (const uint8_t*)fr, xpbuf, s)));
    else HIPCHK((frames_rgbx<T, float>(m, L.H, L.W, (const float*)fr, xpbuf, s)));
    const int rc = conv1_wgrad<T>(L, dy1 + (size_t)s0 * L.P1 * 32, xpbuf, m, gW, s);
    if (rc) return rc;
  }
  return AAA_OK;
}

// Vision encoder backward over F frames in descriptor-sized chunks: conv2
// weight grad (gW2 +=), conv2 dgrad -> dY1 with conv1's bias grad (gb1 +=),
// conv1 weight grad (gW1 +=); accumulators zeroed by the caller.  frames:
// xp is the L.xpc-frame chunk buffer rebuilt from them (conv1_wgrad_frames);
// null: xp holds all F frames' images (the component entries).
template <typename T>
int vision_bwd(const Layout& L, const char* pk, const T* dy2, const T* y1, T* xp, T* dy1, int F,
                      float* gW2, float* gW1, float* gb1, hipStream_t s, const void* frames) {
  const size_t fb = (size_t)L.H * L.W * 3 * (L.fu8 ? 1 : 4);
  for (int f0 = 0; f0 < F; f0 += L.fchunk) {
    const int n = std::min(L.fchunk, F - f0);
    const T* d2 = dy2 + (size_t)f0 * L.P * 64;
    T* d1 = dy1 + (size_t)f0 * L.P1 * 32;
    int rc = conv2_wgrad<T>(L, d2, y1 + (size_t)f0 * L.P1 * 32, n, gW2, s);
    if (!rc) rc = conv2_dgrad<T>(L, pk, d2, d1, n, gb1, s);
    if (!rc && frames) rc = conv1_wgrad_frames<T>(L, d1, (const char*)frames + (size_t)f0 * fb, n, xp, gW1, s);
    else if (!rc) rc = conv1_wgrad<T>(L, d1, xp + (size_t)f0 * (L.H + 2) * (L.W + 2) * 4, n, gW1, s);
    if (rc) return rc;
  }
  return AAA_OK;
}

// The frame-resident vision backward (vision_bwd.h): bf16, uint8 observations (the environment's
// dtype: fp32 frames keep the layered launches), the frame-resident encoder's geometry, and F
// frames' dY1 buffer large enough for the workgroups' partials (AAA_VIS_BWD_FRAMES=0: the three
// layered launches above; AAA_VBWD_MINF: a frames-per-CU floor, 0 by default -- with the partial
// sums reduced 4 waves per 64 columns the fused kernel's fixed cost is ~30 us, below the layered
// launches' own: C3 (20 frames per CU) 281 vs 358 us, C4 (10) 155 vs 199 us).
template <typename T>
static bool vbwd_on(const Layout& L, int F) {
  if constexpr (!std::is_same<T, __bf16>::value) {
    (void)L; (void)F;
    return false;
  } else {
    return L.fu8 && vbwd_fits(L.H, L.W, L.H1, L.W1, L.h, L.w) && env_int("AAA_VIS_FRAMES", 1) &&
           env_int("AAA_VIS_BWD_FRAMES", 1) && F >= env_int("AAA_VBWD_MINF", 0) * device_cus() &&
           (size_t)vbwd_groups(F, device_cus()) * kVbPart * 4 <= (size_t)F * L.P1 * 32 * L.esz;
  }
}
// F frames from ``f0``: conv2 wgrad (gW2 +=), conv2 dgrad + conv1 wgrad (gW1 +=, conv1 bias gb1 +=),
// the partials in the frames' dY1 region (unused on this path)
template <typename T>
static int vbwd_run(const Layout& L, const char* pk, const void* frames, int f0, int F, const T* dy2, const T* y1,
                    T* dy1, float* gW2, float* gW1, float* gb1, hipStream_t s) {
  if constexpr (!std::is_same<T, __bf16>::value) {
    return fail(AAA_E_ARG, "the frame-resident vision backward is bf16 only");
  } else {
    VisBwdParams vp{(const char*)frames + (size_t)f0 * L.H * L.W * 3 * (L.fu8 ? 1 : 4), dy2, y1,
                    (const __bf16*)(pk + L.k_WdT2), (float*)dy1, F, L.H, L.W, L.H1, L.W1, L.h, L.w};
    HIPCHK(vision_bwd_frames(vp, device_cus(), gW2, gW1, gb1, s));
    return AAA_OK;
  }
}

// ------------------------------------------------------------ backward ----
// Stateful policy core, backward of the tail (phase HEAD): the dgrad chain runs
// step by step from t = T-1 (the carries dh, dc of the core state flow through
// the LSTMCell's W_hh and the query MLP into step t-1); every weight gradient
// is then one batched GEMM over all frames from the saved per-step operands.
static int head_backward_stateful(const Layout& L, const aaa_io* io, hipStream_t st) {
  constexpr int NTF = CF::NT;
  char* ws = (char*)io->workspace;
  const char* pk = (const char*)io->packed;
  const float* prm = io->params;
  float* grads = io->grads;
  auto Wf = [&](size_t off) { return (float*)(ws + off); };
  const int F = L.F, P = L.P, B = L.B, qd = L.qd, da = L.da;
  using LRfj = LdRows<float, float, CF::BJ, CF::BK, NTF>;
  using LTf = LdRowsT<float, float, CF::BI, CF::BK, NTF>;
  using LTfj = LdRowsT<float, float, CF::BJ, CF::BK, NTF>;
  float *CH = Wf(L.CH), *CC = Wf(L.CC), *AOX = Wf(L.AOX), *dAOX = Wf(L.dAOX), *dhc = Wf(L.dhc), *dcc = Wf(L.dcc);
  const size_t sB = (size_t)B * 256 * 4;
  if (io->dcore_hT) HIPCHK(hipMemcpyAsync(dhc, io->dcore_hT, sB, hipMemcpyDeviceToDevice, st));
  else HIPCHK(hipMemsetAsync(dhc, 0, sB, st));
  if (io->dcore_cT) HIPCHK(hipMemcpyAsync(dcc, io->dcore_cT, sB, hipMemcpyDeviceToDevice, st));
  else HIPCHK(hipMemsetAsync(dcc, 0, sB, st));
  for (int t = L.T - 1; t >= 0; --t) {
    const size_t f0 = (size_t)t * B;
    {  // heads dgrad + dh carry -> LSTMCell backward from (c_{t-1}, c_t), dc carry
      LTf::Params pa{(const float*)(pk + L.k_Whd), 256, 256};
      LRfj::Params pb{Wf(L.dY) + f0 * L.ldy, L.ldy, B};
      EpiLstmCellBwdS ep{Wf(L.LG) + f0 * 1024, CC + f0 * 256, CC + (f0 + B) * 256, dhc, dcc, Wf(L.dLG) + f0 * 1024, B};
      HIPCHK((head_gemm<LdRowsT, LdRows>(pa, pb, ep, 256, B, L.ldy, 1, st)));
    }
    {  // [d answer | d h_{t-1} (recurrent part)] = [W_ih | W_hh]^T dgates
      LTf::Params pa{(const float*)(pk + L.k_Wihhp), 512, 512};
      LRfj::Params pb{Wf(L.dLG) + f0 * 1024, 1024, B};
      EpiStoreT<float> ep{dAOX + f0 * 512, 512, 512, B, nullptr, 0};
      HIPCHK((head_gemm<LdRowsT, LdRows>(pa, pb, ep, 512, B, 1024, 1, st)));
    }
    {  // answer_processor.2 dgrad fused with the ReLU backward
      LTf::Params pa{prm + L.poff[A2W], 512, 512};
      LRfj::Params pb{dAOX + f0 * 512, 512, B};
      EpiReluBwdT ep{Wf(L.dH1) + f0 * 512, Wf(L.hid1) + f0 * 512, 512, 512, 512, B};
      HIPCHK((head_gemm<LdRowsT, LdRows>(pa, pb, ep, 512, B, 256, 1, st)));
    }
    {  // answer_processor.0 dgrad: readout and query columns of the answer row
      LTf::Params pa{(const float*)(pk + L.k_W1p), L.ans_ld, da};
      LRfj::Params pb{Wf(L.dH1) + f0 * 512, 512, B};
      EpiStoreT<float> ep{Wf(L.dAns) + f0 * da, da, da, B, nullptr, 0};
      HIPCHK((head_gemm<LdRowsT, LdRows>(pa, pb, ep, da, B, 512, 1, st)));
    }
    // readout / softmax / logits backward with this step's queries; dQ gets
    // the logits path plus the answer row's copy of Q
    {
      TimerScope tim(AAA_TIMER_ATTN_BWD, st, (double)B * attn_bwd_bytes(P, L.nq, L.esz), "k_attn_bwd, per-frame query (stateful core)");
      HIPCHK(attn_bwd(readout_h(L, ws).frame(f0, P), io->basis, Wf(L.Qf) + f0 * qd, Wf(L.Am) + f0 * P * L.nq,
                      Wf(L.dAns) + f0 * da, da, B, P, L.nq, Wf(L.dO) + f0 * P * 128, Wf(L.dQf) + f0 * qd, st, qd, 1, (cqm_layout(L) & kCqmDO) != 0));
    }
    {  // query MLP backward to its input h_{t-1}
      LTf::Params pa{prm + L.poff[Q4W], qd, qd};
      LRfj::Params pb{Wf(L.dQf) + f0 * qd, qd, B};
      EpiReluBwdT ep{Wf(L.dq2s) + f0 * qd, Wf(L.q2s) + f0 * qd, qd, qd, qd, B};
      HIPCHK((head_gemm<LdRowsT, LdRows>(pa, pb, ep, qd, B, qd, 1, st)));
    }
    {
      LTf::Params pa{prm + L.poff[Q2W], 128, 128};
      LRfj::Params pb{Wf(L.dq2s) + f0 * qd, qd, B};
      EpiReluBwdT ep{Wf(L.dq1s) + f0 * 128, Wf(L.q1s) + f0 * 128, 128, 128, 128, B};
      HIPCHK((head_gemm<LdRowsT, LdRows>(pa, pb, ep, 128, B, qd, 1, st)));
    }
    {  // dh_{t-1} = W0^T dq1 (query path) + W_hh^T dgates (recurrent path)
      LTf::Params pa{prm + L.poff[Q0W], 256, 256};
      LRfj::Params pb{Wf(L.dq1s) + f0 * 128, 128, B};
      EpiStoreAddT ep{dhc, dAOX + f0 * 512 + 256, 256, 512, 256, B};
      HIPCHK((head_gemm<LdRowsT, LdRows>(pa, pb, ep, 256, B, 128, 1, st)));
    }
  }
  if (io->dcore_h0) HIPCHK(hipMemcpyAsync(io->dcore_h0, dhc, sB, hipMemcpyDeviceToDevice, st));
  if (io->dcore_c0) HIPCHK(hipMemcpyAsync(io->dcore_c0, dcc, sB, hipMemcpyDeviceToDevice, st));
  // weight gradients, batched over all T*B frames
  auto wgrad = [&](const float* dA, int lda, int Mi, const float* X, int ldx, int Nj, float* out, int ldo) -> int {
    LTf::Params pa{dA, lda, Mi};
    LTfj::Params pb{X, ldx, Nj};
    EpiStore<true> ep{out, ldo, Mi, Nj};
    HIPCHK((head_gemm<LdRowsT, LdRowsT>(pa, pb, ep, Mi, Nj, F, wgrad_splits(cdiv(Mi, 64) * cdiv(Nj, 64), F, CF::BK),
                                        st)));
    return AAA_OK;
  };
  int rc;
  if ((rc = wgrad(Wf(L.dY), L.ldy, L.ldy, CH + (size_t)B * 256, 256, 256, Wf(L.gWhd), 256))) return rc;
  HIPCHK(colsum(Wf(L.dY), L.ldy, F, L.ldy, Wf(L.gbhd), st));
  if ((rc = wgrad(Wf(L.dLG), 1024, 1024, AOX, 512, 512, Wf(L.gWihhp), 512))) return rc;
  HIPCHK(colsum(Wf(L.dLG), 1024, F, 1024, Wf(L.gblc), st));
  if ((rc = wgrad(dAOX, 512, 256, Wf(L.hid1), 512, 512, grads + L.poff[A2W], 512))) return rc;
  HIPCHK(colsum(dAOX, 512, F, 256, grads + L.poff[A2B], st));
  if ((rc = wgrad(Wf(L.dH1), 512, 512, Wf(L.ans), L.ans_ld, L.ans_ld, Wf(L.gW1p), L.ans_ld))) return rc;
  HIPCHK(colsum(Wf(L.dH1), 512, F, 512, grads + L.poff[A0B], st));
  if ((rc = wgrad(Wf(L.dQf), qd, qd, Wf(L.q2s), qd, qd, grads + L.poff[Q4W], qd))) return rc;
  HIPCHK(colsum(Wf(L.dQf), qd, F, qd, grads + L.poff[Q4B], st));
  if ((rc = wgrad(Wf(L.dq2s), qd, qd, Wf(L.q1s), 128, 128, grads + L.poff[Q2W], 128))) return rc;
  HIPCHK(colsum(Wf(L.dq2s), qd, F, qd, grads + L.poff[Q2B], st));
  if ((rc = wgrad(Wf(L.dq1s), 128, 128, CH, 256, 256, grads + L.poff[Q0W], 256))) return rc;
  HIPCHK(colsum(Wf(L.dq1s), 128, F, 128, grads + L.poff[Q0B], st));
  F32Unpack up;
  up.gW1p = Wf(L.gW1p); up.gWihp = Wf(L.gWihp); up.gblc = Wf(L.gblc); up.gWhd = Wf(L.gWhd); up.gbhd = Wf(L.gbhd);
  up.a0w = grads + L.poff[A0W]; up.wih = grads + L.poff[WIH]; up.bih = grads + L.poff[BIH];
  up.bhh = grads + L.poff[BHH]; up.pw = grads + L.poff[PW]; up.vw = grads + L.poff[VW];
  up.pb = grads + L.poff[PB]; up.vb = grads + L.poff[VB];
  up.ans_in = L.ans_in; up.ans_ld = L.ans_ld; up.A = L.A;
  up.gWihhp = Wf(L.gWihhp); up.whh = grads + L.poff[WHH];
  HIPCHK(unpack_f32(up, st));
  return AAA_OK;
}

template <typename T>
int backward_impl(const Layout& L, const aaa_io* io, int phases, hipStream_t st) {
  using C = CfgFor<T>;
  // bf16 path: the fp32 tail GEMMs on the bf16 MFMA with split operands (AAA_TAIL_SPLIT3=0: fp32 MFMA)
  TailPrecision tail_prec(std::is_same<T, __bf16>::value && env_int("AAA_TAIL_SPLIT3", 1),
                          std::is_same<T, float>::value && f32_split6());
  constexpr int NTF = CF::NT;
  char* ws = (char*)io->workspace;
  const char* pk = (const char*)io->packed;
  const float* prm = io->params;
  float* grads = io->grads;
  auto Wf = [&](size_t off) { return (float*)(ws + off); };
  auto Wt = [&](size_t off) { return (T*)(ws + off); };
  const int F = L.F, P = L.P, M = L.B * L.P;
  using LRfj = LdRows<float, float, CF::BJ, CF::BK, NTF>;
  using LTf = LdRowsT<float, float, CF::BI, CF::BK, NTF>;
  using LTfj = LdRowsT<float, float, CF::BJ, CF::BK, NTF>;
  LstmGrads core_unpack{};   // the ConvLSTM grads' reference tensors, unpacked with the vision grads when both run here

  if (phases & AAA_BWD_HEAD) {
    {
      TimerScope tim(AAA_TIMER_MISC, st, 0.0, "grad/accumulator memsets, cotangent concat");
      ZeroRanges z{};   // the grads, the atomic accumulators and the cotangent concat: one launch
      z.add(grads, (long)L.ptotal);
      z.add(Wf(L.dQs), (long)((L.ws - L.dQs) / 4));
      HIPCHK(prologue<T>(z, 0, nullptr, (T*)nullptr, F, L.A, L.ldy, io->dlogits, io->dvalues, Wf(L.dY), st));
    }
    if (L.sc) {
      const int rc = head_backward_stateful(L, io, st);
      if (rc) return rc;
    } else {
    std::unique_ptr<TimerScope> tail(new TimerScope(AAA_TIMER_TAIL_BWD, st, 2.0 * F * (tail_fwd_flop(L) + 2.0 * 256 * L.ldy),
                                                    "heads + LSTMCell + answer MLP backward (fp32 GEMMs)"));
    // The dgrad chain (heads -> LSTMCell -> answer MLP -> readout) on st; each layer's weight gradient
    // on the side stream once the chain has produced its input gradient (few-tile GEMMs: the two
    // streams fill CUs the other leaves idle); joined before the gradients are unpacked.
    // Below ~2048 frames the GEMMs are too short for the overlap to pay for the second queue's dispatch
    // cost on the rest of the step (C2, 640 frames: tail bwd -20 us but the step +10-15 us;
    // profiles/r06/ab/side/): one stream there.
    hipStream_t ss = F >= 2048 ? side_stream() : nullptr;
    hipStream_t ws_ = ss ? ss : st;   // the weight gradients' stream
    if (ss) HIPCHK(stream_order(st, ss));   // the zeroed accumulators, the cotangent concat
    {  // heads wgrad (dY from the prologue)
      LTf::Params pa{Wf(L.dY), L.ldy, L.ldy};
      LTfj::Params pb{Wf(L.LH), 256, 256};
      EpiStore<true> ep{Wf(L.gWhd), 256, L.ldy, 256};
      HIPCHK((head_gemm<LdRowsT, LdRowsT>(pa, pb, ep, L.ldy, 256, F, wgrad_splits(cdiv(L.ldy, 64) * 4, F, CF::BK), ws_)));
    }
    {  // heads dgrad fused with the zero-state LSTMCell backward
      LTf::Params pa{(const float*)(pk + L.k_Whd), 256, 256};
      LRfj::Params pb{Wf(L.dY), L.ldy, F};
      EpiLstmCellBwd ep{Wf(L.LG), Wf(L.LC), Wf(L.dLG), F};
      HIPCHK((head_gemm<LdRowsT, LdRows>(pa, pb, ep, 256, F, L.ldy, 1, st)));
    }
    if (ss) HIPCHK(stream_order(st, ss));   // dLG
    {  // LSTMCell weight_ih grad (weight_hh grad is exactly zero: h0 = 0, Q1)
      LTf::Params pa{Wf(L.dLG), 1024, 1024};
      LTfj::Params pb{Wf(L.AO), 256, 256};
      EpiStore<true> ep{Wf(L.gWihp), 256, 1024, 256};
      HIPCHK((head_gemm<LdRowsT, LdRowsT>(pa, pb, ep, 1024, 256, F, wgrad_splits(16 * 4, F, CF::BK), ws_)));
    }
    {  // LSTMCell input dgrad
      LTf::Params pa{(const float*)(pk + L.k_Wihp), 256, 256};
      LRfj::Params pb{Wf(L.dLG), 1024, F};
      EpiStoreT<float> ep{Wf(L.dAO), 256, 256, F, nullptr, 0};
      HIPCHK((head_gemm<LdRowsT, LdRows>(pa, pb, ep, 256, F, 1024, 1, st)));
    }
    if (ss) HIPCHK(stream_order(st, ss));   // dAO
    {  // answer_processor.2 wgrad / bias
      LTf::Params pa{Wf(L.dAO), 256, 256};
      LTfj::Params pb{Wf(L.hid1), 512, 512};
      EpiStore<true> ep{grads + L.poff[A2W], 512, 256, 512};
      HIPCHK((head_gemm<LdRowsT, LdRowsT>(pa, pb, ep, 256, 512, F, wgrad_splits(4 * 8, F, CF::BK), ws_)));
    }
    {  // answer_processor.2 dgrad fused with ReLU backward
      LTf::Params pa{prm + L.poff[A2W], 512, 512};
      LRfj::Params pb{Wf(L.dAO), 256, F};
      EpiReluBwdT ep{Wf(L.dH1), Wf(L.hid1), 512, 512, 512, F};
      HIPCHK((head_gemm<LdRowsT, LdRows>(pa, pb, ep, 512, F, 256, 1, st)));
    }
    if (ss) HIPCHK(stream_order(st, ss));   // dH1
    {  // answer_processor.0 wgrad / bias
      LTf::Params pa{Wf(L.dH1), 512, 512};
      LTfj::Params pb{Wf(L.ans), L.ans_ld, L.ans_ld};
      EpiStore<true> ep{Wf(L.gW1p), L.ans_ld, 512, L.ans_ld};
      HIPCHK((head_gemm<LdRowsT, LdRowsT>(pa, pb, ep, 512, L.ans_ld, F,
                                        wgrad_splits(8 * cdiv(L.ans_ld, 64), F, CF::BK), ws_)));
    }
    {  // answer_processor.0 dgrad (readout columns only)
      LTf::Params pa{(const float*)(pk + L.k_W1p), L.ans_ld, L.da};
      LRfj::Params pb{Wf(L.dH1), 512, F};
      EpiStoreT<float> ep{Wf(L.dAns), L.da, L.da, F, nullptr, 0};
      HIPCHK((head_gemm<LdRowsT, LdRows>(pa, pb, ep, L.da, F, 512, 1, st)));
    }
    tail.reset();
    // attention readout / softmax / logits backward, then the query MLP
    {
      TimerScope tim(AAA_TIMER_ATTN_BWD, st, (double)F * attn_bwd_bytes(P, L.nq, L.esz), "k_attn_bwd, 1 WG per frame");
      HIPCHK(attn_bwd(readout_h(L, ws), io->basis, (const float*)(pk + L.k_Q), Wf(L.Am), Wf(L.dAns), L.da, F, P, L.nq,
                      Wf(L.dO), Wf(L.dQp), st, 0, 0, (cqm_layout(L) & kCqmDO) != 0));
    }
    tail.reset(new TimerScope(AAA_TIMER_TAIL_BWD, st, 0.0, "bias column sums, query MLP backward, grad unpack"));
    {  // the bias grads of the heads, the LSTMCell and both answer layers, and dQ summed over frames: one launch
      ColSums cs;
      cs.add(Wf(L.dY), L.ldy, L.ldy, Wf(L.gbhd));
      cs.add(Wf(L.dLG), 1024, 1024, Wf(L.gblc));
      cs.add(Wf(L.dAO), 256, 256, grads + L.poff[A2B]);
      cs.add(Wf(L.dH1), 512, 512, grads + L.poff[A0B]);
      cs.add(Wf(L.dQp), L.qd, L.qd, Wf(L.dQs));
      HIPCHK(colsum_multi(cs, F, st));
    }
    HIPCHK(query_bwd(Wf(L.dQs), grads + L.poff[A0B], prm + L.poff[A0W], L.ans_in, L.nq, prm + L.poff[Q2W],
                     prm + L.poff[Q4W], (const float*)(pk + L.k_q1), (const float*)(pk + L.k_q2), grads + L.poff[Q4W],
                     grads + L.poff[Q4B],
                     grads + L.poff[Q2W], grads + L.poff[Q2B], grads + L.poff[Q0B], st));
    if (ss) HIPCHK(stream_order(ss, st));   // join: the weight gradients
    F32Unpack up;
    up.gW1p = Wf(L.gW1p); up.gWihp = Wf(L.gWihp); up.gblc = Wf(L.gblc); up.gWhd = Wf(L.gWhd); up.gbhd = Wf(L.gbhd);
    up.a0w = grads + L.poff[A0W]; up.wih = grads + L.poff[WIH]; up.bih = grads + L.poff[BIH];
    up.bhh = grads + L.poff[BHH]; up.pw = grads + L.poff[PW]; up.vw = grads + L.poff[VW];
    up.pb = grads + L.poff[PB]; up.vb = grads + L.poff[VB];
    up.ans_in = L.ans_in; up.ans_ld = L.ans_ld; up.A = L.A;
    HIPCHK(unpack_f32(up, st));
    }
  }

  // Off-chain backward work for the steps [lo, hi): weight/bias grads of the
  // ConvLSTM, dx (conv2 output grad) and -- when VISION runs in the same call
  // -- the conv2/conv1 backward of those frames.  Every gradient accumulates
  // atomically into zeroed buffers, so chunks may run in any order.
  const bool vision_here = (phases & AAA_BWD_VISION) && (phases & AAA_BWD_CORE);
  bool dx_fused = false;   // the frame-resident BPTT computed dx (dY2) and conv2's bias gradient itself
  auto core_chunk = [&](int lo, int hi, hipStream_t s) -> int {
    const int rows = (hi - lo) * M;                       // pixels of these frames
    const int F1 = (hi - lo) * L.B;                       // frames
    const T* dz = Wt(L.dZ) + (size_t)lo * M * 512;
    // conv2 / conv1 backward of these frames (needs dY2 only)
    auto vision = [&](hipStream_t vs) -> int {
      const T* dy2 = Wt(L.dY2) + (size_t)lo * M * 64;
      T* dy1 = Wt(L.dY1) + (size_t)lo * L.B * L.P1 * 32;
      if (vbwd_on<T>(L, F1)) {   // one frame-resident launch (+ its partials' sum)
        TimerScope tim(AAA_TIMER_VISION_BWD, vs, (double)F1 * vision_bwd_flop(L),
                       "frame-resident conv2 wgrad + dgrad + conv1 wgrad [kernel: k_vision_bwd_frames]");
        return vbwd_run<T>(L, pk, io->frames, lo * L.B, F1, dy2, Wt(L.Y1) + (size_t)lo * L.B * L.P1 * 32, dy1,
                           Wf(L.gWp2), Wf(L.gWp1), grads + L.poff[C0B], vs);
      }
      TimerScope tim(AAA_TIMER_VISION_BWD, vs, (double)F1 * vision_bwd_flop(L), "conv2 wgrad + dgrad, conv1 wgrad");
      const int rows1 = F1 * L.P1;
      constexpr bool f32 = std::is_same<T, float>::value;   // fp32 with AAA_CONV2_DGRAD_RING=0: conv1 bias by a column sum
      {  // conv2 wgrad
        const int rc = conv2_wgrad<T>(L, dy2, Wt(L.Y1) + (size_t)lo * L.B * L.P1 * 32, F1, Wf(L.gWp2), vs);
        if (rc) return rc;
      }
      {  // conv2 dgrad (4 parity classes) -> dY1, then conv1 wgrad / bias
        int rc = conv2_dgrad<T>(L, pk, dy2, dy1, F1, grads + L.poff[C0B], vs);
        if (!rc && L.xpc < L.F)   // Xp chunk buffer: rebuilt from the observation
          rc = conv1_wgrad_frames<T>(L, dy1, (const char*)io->frames + (size_t)lo * L.B * L.H * L.W * 3 * (L.fu8 ? 1 : 4),
                                     F1, Wt(L.Xp), Wf(L.gWp1), vs);
        else if (!rc)
          rc = conv1_wgrad<T>(L, dy1, Wt(L.Xp) + (size_t)lo * L.B * (L.H + 2) * (L.W + 2) * 4, F1, Wf(L.gWp1), vs);
        if (rc) return rc;
        if (f32 && !ab_int("AAA_CONV2_DGRAD_RING", 1)) HIPCHK(colsum(dy1, 32, rows1, 32, grads + L.poff[C0B], vs));
      }
      return AAA_OK;
    };
    // (the layered vision backward on the side stream beside the ConvLSTM weight gradient, ablation
    // builds with AAA_VIS_SIDE=1: C2 232.0k -> 228.6-229.2k, C5 within noise -- the two contend for
    // the CUs; profiles/r06/ab/side/)
    hipStream_t vside = vision_here && dx_fused && !vbwd_on<T>(L, F1) && ab_int("AAA_VIS_SIDE", 0) ? side_stream()
                                                                                                 : nullptr;
    if (vside) {
      HIPCHK(stream_order(s, vside));
      const int rc = vision(vside);
      if (rc) return rc;
    }
    {
      const int rc = lstm_wgrad<T>(dz, Wt(L.XH) + (size_t)lo * M * 192, rows, L.h, L.w, Wf(L.gWpl), s, s != st);
      if (rc) return rc;
    }
    if (!dx_fused) {  // dx_t for these steps: D[64][rows] = WdT[0:64] * gather(dZ)
      TimerScope tim(AAA_TIMER_CORE_DX, s, 2.0 * rows * 64 * 4608, "batched dx (conv2-output grad), K=4608 [kernel: EpiStoreBiasT]");
      const ConvGeo g = ConvGeo{512, 512, 0, L.h, L.w, L.h, L.w, 3, 1, 1, 1}.prep();
      const T* WdT = (const T*)(pk + L.k_WdTl);
      const uint32_t zb = (uint32_t)((size_t)rows * 512 * L.esz);
      if constexpr (std::is_same<T, float>::value) {
        // 64x64 tiles (64x128 measured slower: occupancy); conv2's bias
        // gradient summed from the tile in the epilogue (no column-sum pass)
        EpiStoreBiasT<float> ep{Wf(L.dY2) + (size_t)lo * M * 64, 64, 64, rows, grads + L.poff[C1B]};
        using ED = EpiStoreBiasT<float>;
        const int dx6 = f32_split6() ? ab_int("AAA_DX_S6_TILE", 4) : -1;
        if (dx6 == 4) {   // the ring tile on the bf16 MFMA with three-way split operands (gemm.h SPLIT6):
          // 64x128 with the weights pre-split (k_WdT6 planes), only dZ split in the loop
          // (C2 340 vs 357 us for the in-loop split of both, profiles/r04/ab/README.md)
          using C6 = GemmCfgS6<64, 128, 32, 2, 2>;
          using LA3 = GRows3B<64, 32, C6::NT>;
          using LBx = GIm2colB<float, 128, 32, C6::NT>;
          HIPCHK((launch_pipe<C6, LA3, LBx, ED, 2>(
              typename LA3::Params{(const __bf16*)(pk + L.k_WdT6), 4608, 64, (size_t)64 * 4608},
              typename LBx::Params{dz, g, rows, zb}, ep, 64, rows, 4608, 1, s)));
        } else if (dx6 < 0) {   // exact fp32 MFMA (AAA_F32_SPLIT6=0)
          if (pipe_batched())
            HIPCHK((step_gemm<CfgFor<T>, true, T, T, ED>(WdT, 4608, 64, dz, g, rows, zb, ep, 64, 4608, s)));
          else
            HIPCHK((step_gemm<CfgFor<T>, false, T, T, ED>(WdT, 4608, 64, dz, g, rows, zb, ep, 64, 4608, s)));
        } else {
#ifdef AAA_ABLATION
          // the measured-slower variants (ablation builds): 0 = 64x64, 1 = 64x128 in-loop split
          // (C2 355 / 344 us), 2 = 64x64 BK64, 3 = 64x128 channel-chunk-major K order (ConvGeo::cmaj;
          // 365 vs 353 us), 5 = tile 4 with dZ pre-split too (GIm2colB3 over split_planes: 467-473 vs
          // 337 us), 6 = the halo-staged conv on split operands (C2 478 vs 370 us,
          // profiles/r04/ab/halo_dx_f32_c2_*.json)
          using HF6 = HaloCfgS6<64, 128, 32, 1, 2, 1, 176>;   // one 11x11 frame per tile, its dZ image in LDS
          switch (dx6) {
            case 6: {
              if (!halo_fits<HF6>(L.h, L.w, 512)) return fail(AAA_E_ARG, "AAA_DX_S6_TILE=6: grid too large");
              const HaloParams hp{WdT, 4608, 64, dz, 512, 0, 512, zb, L.h, L.w, (hi - lo) * L.B, 1};
              HIPCHK((launch_halo<HF6>(hp, ep, s)));
              break;
            }
            case 3: {
              HIPCHK(reorder_cmaj(WdT, 64, 512, 9, 32, (float*)(pk + L.k_WdTc), s));   // its weights, re-laid here
              ConvGeo gc = g;
              gc.cmaj = 32;
              HIPCHK((step_gemm<GemmCfgS6<64, 128, 32, 2, 2>, true, T, T, ED>((const T*)(pk + L.k_WdTc), 4608, 64, dz, gc,
                                                                             rows, zb, ep, 64, 4608, s)));
              break;
            }
            case 1:
              HIPCHK((step_gemm<GemmCfgS6<64, 128, 32, 2, 2>, true, T, T, ED>(WdT, 4608, 64, dz, g, rows, zb, ep, 64, 4608, s)));
              break;
            case 5: {
              if (!L.dZ6) return fail(AAA_E_ARG, "AAA_DX_S6_TILE=5 set after the workspace was laid out");
              using C6 = GemmCfgS6<64, 128, 32, 2, 2>;
              using LA3 = GRows3B<64, 32, C6::NT>;
              using LB3 = GIm2colB3<128, 32, C6::NT>;
              __bf16* z6 = (__bf16*)Wf(L.dZ6);
              HIPCHK(split_planes(dz, (long)rows * 512, z6, s));
              HIPCHK((launch_pipe<C6, LA3, LB3, ED, 2>(
                  typename LA3::Params{(const __bf16*)(pk + L.k_WdT6), 4608, 64, (size_t)64 * 4608},
                  typename LB3::Params{z6, g, rows, zb / 2, (size_t)rows * 512}, ep, 64, rows, 4608, 1, s)));
              break;
            }
            case 2:
              HIPCHK((step_gemm<GemmCfgS6<64, 64, 64, 2, 2>, true, T, T, ED>(WdT, 4608, 64, dz, g, rows, zb, ep, 64, 4608, s)));
              break;
            default:
              HIPCHK((step_gemm<GemmCfgS6<64, 64, 32, 2, 2>, true, T, T, ED>(WdT, 4608, 64, dz, g, rows, zb, ep, 64, 4608, s)));
          }
#else
          return fail(AAA_E_ARG, "AAA_DX_S6_TILE %d: ablation builds only", dx6);
#endif
        }
      } else {
        // bf16: dY2 stored bf16 (its readers round it to bf16 anyway), conv2's
        // bias gradient summed from the fp32 values in the epilogue
        EpiStoreBiasT<T> ep{Wt(L.dY2) + (size_t)lo * M * 64, 64, 64, rows, grads + L.poff[C1B]};
        // small grids: halo-staged conv, one frame per 64x128 tile
        // (tools/ubench/halo_tiles: 658 vs 771 us for the ring at C3)
        using HD = HaloCfg<__bf16, 64, 128, 64, 1, 2, 1, 176>;
        // 21x21 grids (168x168 frames): one frame per 512-column tile of 4 waves, 32-channel chunks
        using HW = HaloCfg<__bf16, 64, 512, 32, 1, 4, 1, 576>;
        if (halo_fits<HD>(L.h, L.w, 512) && ab_int("AAA_HALO_DX", 1)) {
          const HaloParams hp{WdT, 4608, 64, dz, 512, 0, 512, zb, L.h, L.w, (hi - lo) * L.B, 1};
          HIPCHK((launch_halo<HD>(hp, ep, s)));
        } else if (halo_fits<HW>(L.h, L.w, 512) && ab_int("AAA_HALO_DX", 1)) {
          const HaloParams hp{WdT, 4608, 64, dz, 512, 0, 512, zb, L.h, L.w, (hi - lo) * L.B, 1};
          HIPCHK((launch_halo<HW>(hp, ep, s)));
        } else {
          // larger grids (21x21 at 168x168): 64x128 on a 3-stage ring (bf16_tiles at C3: 643 vs 716 us for 64x64)
          HIPCHK((step_gemm<GemmCfg<T, 64, 128, 64, 2, 2>, true, T, T, EpiStoreBiasT<T>, 3>(WdT, 4608, 64, dz, g, rows,
                                                                                            zb, ep, 64, 4608, s)));
        }
      }
    }
    if (!vision_here) return AAA_OK;
    if (vside) return stream_order(vside, s) == hipSuccess ? AAA_OK : fail(AAA_E_LAUNCH, "side-stream join");
    return vision(s);
  };

  if (phases & AAA_BWD_CORE) {
    hipStream_t ax = aux_stream();
    hipStream_t os = ax ? ax : st;     // stream for the off-chain chunks
    const int cs = chunk_steps(L);
    std::unique_ptr<TimerScope> misc(new TimerScope(AAA_TIMER_MISC, st, 0.0, "BPTT state in, last-step gate backward"));
    // ConvLSTM BPTT, t = T-1 .. 0
    {   // dc_T = 0 (or the carried grad), and the frame kernels' hand-off flags and dx bias partials: one launch
      ZeroRanges z{};
      if (!io->dcT) z.add(Wf(L.dC), (long)M * 128);
      z.add(Wf(L.rflags), (long)8 * L.B);
      z.add(Wf(L.dxb), (long)L.B * 64);
      HIPCHK(prologue<T>(z, 0, nullptr, (T*)nullptr, 0, 0, 1, nullptr, nullptr, nullptr, st));
      if (io->dcT) HIPCHK(hipMemcpyAsync(Wf(L.dC), io->dcT, (size_t)M * 128 * 4, hipMemcpyDeviceToDevice, st));
    }
    const int t1 = L.T - 1;
    // Sequential part: only the h rows (dh_{t-1}, fused with the gate backward
    // of step t-1); everything else runs in chunks off the chain.
    const int bwd_tile = step_tile((long)(128 / 32) * cdiv(M, 32), "AAA_BPTT_TILE", true, L.dt == AAA_BF16);
    // pipe (glds.h) tiles reduce the gate-bias partials in their epilogue;
    // the register-staged ones leave the bias to a column sum over dZ
    // (split-K tiles 30/31: the gate backward kernel's pixel tile, kSplitBj -- finer than the GEMM's, so
    // that kernel spreads over the chip)
    const int bj = bwd_tile >= 30 && bwd_tile <= 33 ? kSplitBj : (bwd_tile == 7 || bwd_tile == 19 || bwd_tile == 20 ? 128 : (bwd_tile == 21 || bwd_tile == 22 || bwd_tile == 23 ? 64 : (bwd_tile >= 9 && bwd_tile != 14 ? 32 : 64)));
    const bool pipe = (bwd_tile == 4 && pipe_even<CfgK4BFor<T>>()) || (bwd_tile == 5 && pipe_even<CfgK4For<T>>()) ||
                      (bwd_tile == 6 && pipe_even<C>()) || bwd_tile == 7 || bwd_tile == 8 || bwd_tile >= 19 ||
                      (bwd_tile == 9 && pipe_even<GemmCfg<T, 64, 32, 128, 2, 1, 4>>()) ||
                      (bwd_tile == 10 && pipe_even<GemmCfg<T, 32, 32, 128, 1, 1, 4>>()) ||
                      ((bwd_tile == 11 || bwd_tile == 12 || bwd_tile == 16) && pipe_even<GemmCfg<T, 32, 32, 64, 1, 1, 4>>()) ||
                      (bwd_tile == 13 && pipe_even<GemmCfg<T, 32, 32, 128, 1, 1, 8>>()) ||
                      (bwd_tile == 15 && pipe_even<GemmCfg<T, 64, 32, 64, 2, 1, 4>>()) ||
                      (bwd_tile >= 27 && bwd_tile <= 31);   // fp32 split-product tiles (ring only)
    const bool fixk = bwd_tile == 32 || bwd_tile == 33;   // split-K finished in the GEMM: bias from dZ's column sum
    if (fixk && L.dhs)   // the fixup counters (self-resetting; zeroed per call in case a launch was abandoned)
      HIPCHK(hipMemsetAsync(ws + L.dhs + (size_t)std::max(kBpttSplitMax * 128, 4 * 512) * M * 4, 0, 4096, st));
    const int ntj = cdiv(M, bj);
    float* part = pipe && !fixk ? Wf(L.dZp) : nullptr;
    const bool g16 = gates_f16(L.dt, M);
    const int fb = frames_bwd(L, g16);   // the whole chain in one frame-resident launch (workgroups per frame)
    // fp32: the frame-group BPTT (recur_bwd_f32.h, G = 8) behind the forward's frame-group kernel
    const bool fb32 = std::is_same<T, float>::value && f32_frames(L) == 8 && env_int("AAA_F32_FRAMES_BWD", 1);
    if (fb32) part = nullptr;   // the kernel writes per-(step, frame) bias partials, step T-1's included
    if (fb) {
    } else if (g16)
      HIPCHK((gate_bwd_last<T, _Float16>(M, bj, Wf(L.dO) + (size_t)t1 * M * 128, io->dhT,
                                         (const _Float16*)(ws + L.Gt) + (size_t)t1 * M * 512,
                                         Wf(L.Cst) + (size_t)t1 * M * 128, Wf(L.Cst) + (size_t)(t1 + 1) * M * 128,
                                         Wf(L.dC), Wt(L.dZ) + (size_t)t1 * M * 512,
                                         part ? part + (size_t)t1 * ntj * 512 : nullptr, st)));
    else
      HIPCHK((gate_bwd_last<T, float>(M, bj, Wf(L.dO) + (size_t)t1 * M * 128, io->dhT, Wf(L.Gt) + (size_t)t1 * M * 512,
                                      Wf(L.Cst) + (size_t)t1 * M * 128, Wf(L.Cst) + (size_t)(t1 + 1) * M * 128,
                                      Wf(L.dC), Wt(L.dZ) + (size_t)t1 * M * 512,
                                      part ? part + (size_t)t1 * ntj * 512 : nullptr, st)));
    misc.reset();
    const uint32_t dz_bytes = (uint32_t)((size_t)M * 512 * L.esz);  // one step slice of dZ
    const T* WdTh = (const T*)(pk + L.k_WdTl) + (size_t)64 * 4608;
    int done_hi = L.T;   // chunks [lo, done_hi) not yet issued
    auto flush = [&](int ready_lo) -> int {   // dz of steps >= ready_lo are final
      while (done_hi - ready_lo >= cs || (ready_lo == 0 && done_hi > 0)) {
        const int lo = std::max(ready_lo, done_hi - cs);
        if (ax) HIPCHK(stream_order(st, ax));
        int rc = core_chunk(lo, done_hi, os);
        if (rc) return rc;
        done_hi = lo;
      }
      return AAA_OK;
    };
    if (fb) {
      if constexpr (!std::is_same<T, float>::value) {
        RecBwdParams rp{(const __bf16*)(pk + L.k_Wbf), Wf(L.dO), (const _Float16*)(ws + L.Gt), Wf(L.Cst), io->dhT,
                        Wf(L.dC), Wt(L.dZ), Wf(L.dZp), io->dh0, Wt(L.dY2), Wf(L.dxb), (int*)(ws + L.rflags),
                        L.T, L.B, L.h, L.w, L.P, nullptr, pair_budget(L.T), rec_stagger("AAA_REC_STAGGER_BWD"),
                        cqm_layout(L)};
        // single-workgroup and paired kernels: row-padded images (recur_bwd.h kBwIBP) where they fit
        // (C3 LDS bank conflicts 52.8 -> 10.0 %: profiles/r04/ab/rowpad_c3/); AAA_BW_ROWPAD=0 (A/B): 272-B rows only
        rp.rowpad = fb <= 2 && ab_int("AAA_BW_ROWPAD", 1) ? bw_rowpad(L.h, L.w) : 0;
        rp.sc1_all = ab_int("AAA_BW_SC1_ALL", 0);   // band kernel (A/B): sc1 for every dZ row, as in round 4
        // single-workgroup kernel: the epilogue's inputs by LDS-DMA into a counted ring (recur_bwd.h RING)
        rp.ring = fb == 1 && ab_int("AAA_BW_RING", 0);   // measured slower: ablation builds only
        if (fb >= 2) {   // paired or band mode: hand-off flags [B][fb]
          int dev = 0;
          HIPCHK(hipGetDevice(&dev));
          if (!(rp.report = pair_report(dev))) return fail(AAA_E_LAUNCH, "cannot map the paired-kernel report word");
        }
        {
          // work: the h rows over T-1 steps (+ dh0) and the dx rows over all T (the batched dx it replaces)
          TimerScope tim(AAA_TIMER_BPTT_STEP, st, 2.0 * M * 4608 * (128.0 * (L.T - 1 + (io->dh0 ? 1 : 0)) + 64.0 * L.T),
                         fb == kRecBands && !rec_fits(L.h, L.w)
                             ? strf("bf16 band-mode frame-resident BPTT + dx, %d steps per launch, %d bands per frame, "
                                    "fp16 gates [kernel: k_convlstm_bwd_frames<0, true]", L.T, fb)
                             : strf("bf16 frame-resident BPTT + dx, %d steps per launch, %d WG per frame, fp16 gates "
                                    "[kernel: %s]", L.T, fb, fb == 2 ? "k_convlstm_bwd_pairs" : (rp.ring ? "k_convlstm_bwd_frames<ring>" : "k_convlstm_bwd_frames<0, false")));
          HIPCHK(fb == 2 ? convlstm_bwd_pairs(rp, st) : (fb == 1 ? convlstm_bwd_frames(rp, st) : convlstm_bwd_band(rp, st)));
        }
        HIPCHK(colsum<float>(Wf(L.dxb), 64, L.B, 64, grads + L.poff[C1B], st));
        dx_fused = true;
      }
    }
    if (fb32) {
      if constexpr (std::is_same<T, float>::value) {
        int dev = 0;
        HIPCHK(hipGetDevice(&dev));
        int* rep = pair_report(dev);
        if (!rep) return fail(AAA_E_LAUNCH, "cannot map the frame-group report word");
        RecBwdF32Params rp{(const float*)(pk + L.k_Wb32), Wf(L.dO), Wf(L.Gt), Wf(L.Cst), Wf(L.dC), Wf(L.dZ),
                           Wf(L.dZp), io->dh0, Wf(L.xpart), (int*)(ws + L.rflags), rep, pair_budget(L.T),
                           L.T, L.B, L.h, L.w, L.P, {}};
        const bool s6 = f32_split6();
        rp.Wb6 = (const u32x2*)(pk + L.k_Wb6);
        if (s6) {   // dx fused (DX): conv2's output gradient and its bias partials from the same K loop
          rp.Wx6 = (const u32x2*)(pk + L.k_Wx6);
          rp.Wb6p = (const u32x4*)(pk + L.k_Wb6p);
          rp.Wx6p = (const u32x4*)(pk + L.k_Wx6p);
          rp.dx = Wf(L.dY2);
          rp.dxb = Wf(L.dxb);
        }
        {
          // work: the dh rows over T-1 steps (+ dh0), and with dx fused the dx rows over all T steps (the
          // batched dx it replaces) plus the dh rows of step 0 that the extra iteration computes
          const double dh_steps = L.T - 1 + ((io->dh0 || s6) ? 1 : 0);
          TimerScope tim(AAA_TIMER_BPTT_STEP, st, 2.0 * M * 4608 * (128.0 * dh_steps + (s6 ? 64.0 * L.T : 0.0)),
                         s6 ? strf("fp32 frame-group BPTT + dx (bf16x6 split products), %d steps per launch, 8 WG "
                                   "per frame [kernel: k_convlstm_bwd_f32]", L.T)
                            : strf("fp32 frame-group BPTT (dh rows), %d steps per launch, 8 WG per frame "
                                   "[kernel: k_convlstm_bwd_f32]", L.T));
          HIPCHK(convlstm_bwd_f32(rp, st, s6));
        }
        if (s6) {
          HIPCHK(colsum<float>(Wf(L.dxb), 64, L.B, 64, grads + L.poff[C1B], st));
          dx_fused = true;
        }
      }
    }
    for (int t = (fb || fb32) ? -1 : t1; t >= 0; --t) {
      const int rc0 = flush(t);   // dz_t .. dz_{T-1} are final here
      if (rc0) return rc0;
      const bool prev = t > 0;
      if (!prev && !io->dh0) break;
      const ConvGeo g = ConvGeo{512, 512, 0, L.h, L.w, L.h, L.w, 3, 1, 1, 1}.prep();
      const T* dzt = Wt(L.dZ) + (size_t)t * M * 512;
      TimerScope tim(AAA_TIMER_BPTT_STEP, st, 2.0 * M * 128 * 4608, strf("%s dh dgrad + fused gate bwd, K=4608, AAA_BPTT_TILE %d%s", std::is_same<T, float>::value ? "fp32" : "bf16", bwd_tile, g16 ? ", fp16 gates [kernel: EpiConvLstmBwd]" : " [kernel: EpiConvLstmBwd]"));
      if constexpr (std::is_same<T, float>::value) {
        if (fixk && prev) {   // split-K, the last slice of each tile runs the gate backward (EpiSliceFix)
          if (!L.dhs) return fail(AAA_E_ARG, "AAA_BPTT_TILE %d: split-K needs B*P < 8192 (got %d)", bwd_tile, M);
          const int bk = bwd_tile == 32 ? 64 : 128;
          const int ns = splitk_slices(4608, bk, bptt_splitk());
          float* dhp = Wf(L.dhs);
          int* cnt = (int*)(ws + L.dhs + (size_t)std::max(kBpttSplitMax * 128, 4 * 512) * M * 4);
          using EB = EpiConvLstmBwd<T, float>;
          const EB eb{nullptr, (const float*)(ws + L.Gt) + (size_t)(t - 1) * M * 512, Wf(L.Cst) + (size_t)(t - 1) * M * 128,
                      Wf(L.Cst) + (size_t)t * M * 128, Wf(L.dO) + (size_t)(t - 1) * M * 128, Wf(L.dC),
                      Wt(L.dZ) + (size_t)(t - 1) * M * 512, nullptr, 1, M, 64, nullptr};
          const EpiSliceFix<EB> ef{dhp, 128, 128, M, (size_t)M * 128, ns, cdiv(M, 32), cnt, eb};
          if (bwd_tile == 32)
            HIPCHK((step_gemm_splitk<GemmCfgS6<32, 32, 64, 1, 1, 4>>(WdTh, 4608, 128, dzt, g, M, dz_bytes, ef, 128,
                                                                     4608, st, ns)));
          else
            HIPCHK((step_gemm_splitk<GemmCfgS6<32, 32, 128, 1, 1, 8>>(WdTh, 4608, 128, dzt, g, M, dz_bytes, ef, 128,
                                                                      4608, st, ns, true)));
          continue;
        }
        if ((bwd_tile == 30 || bwd_tile == 31) && prev) {   // split-K: K-slice partials, then the gate backward
          if (!L.dhs) return fail(AAA_E_ARG, "AAA_BPTT_TILE %d: split-K needs B*P < 8192 (got %d)", bwd_tile, M);
          const int bk = bwd_tile == 30 ? 64 : 128;
          const int ns = splitk_slices(4608, bk, bptt_splitk());   // as launch_pipe rounds it
          float* dhp = Wf(L.dhs);
          const EpiSliceT es{dhp, 128, 128, M, (size_t)M * 128};
          if (bwd_tile == 30)   // tile 27's shape
            HIPCHK((step_gemm_splitk<GemmCfgS6<32, 32, 64, 1, 1, 4>>(WdTh, 4608, 128, dzt, g, M, dz_bytes, es, 128,
                                                                     4608, st, ns)));
          else                  // tile 28's shape (interleaved DMA)
            HIPCHK((step_gemm_splitk<GemmCfgS6<32, 32, 128, 1, 1, 8>>(WdTh, 4608, 128, dzt, g, M, dz_bytes, es, 128,
                                                                      4608, st, ns, true)));
          HIPCHK((gate_bwd_last<T, float>(M, bj, Wf(L.dO) + (size_t)(t - 1) * M * 128, dhp,
                                          Wf(L.Gt) + (size_t)(t - 1) * M * 512, Wf(L.Cst) + (size_t)(t - 1) * M * 128,
                                          Wf(L.Cst) + (size_t)t * M * 128, Wf(L.dC), Wt(L.dZ) + (size_t)(t - 1) * M * 512,
                                          part ? part + (size_t)(t - 1) * ntj * 512 : nullptr, st, ns,
                                          (size_t)M * 128)));
          continue;
        }
      }
      auto step = [&](auto gtag) -> hipError_t {
        using GT = decltype(gtag);
        using EB = EpiConvLstmBwd<T, GT>;
        EB ep{nullptr,
              prev ? (const GT*)(ws + L.Gt) + (size_t)(t - 1) * M * 512 : nullptr,
              prev ? Wf(L.Cst) + (size_t)(t - 1) * M * 128 : nullptr,
              Wf(L.Cst) + (size_t)t * M * 128,
              prev ? Wf(L.dO) + (size_t)(t - 1) * M * 128 : nullptr,
              Wf(L.dC),
              prev ? Wt(L.dZ) + (size_t)(t - 1) * M * 512 : nullptr,
              prev ? nullptr : io->dh0, prev ? 1 : 0, M, 64,
              part && prev ? part + (size_t)(t - 1) * ntj * 512 : nullptr};
        if constexpr (!std::is_same<GT, float>::value) {   // fp16 gates: the bf16 tiles only (gates_f16)
          if constexpr (std::is_same<T, float>::value) return hipErrorInvalidValue;
          else if (bwd_tile == 7)
            return step_gemm<GemmCfg<T, 128, 128, 128, 2, 2, 2>, true>(WdTh, 4608, 128, dzt, g, M, dz_bytes, ep, 128,
                                                                        4608, st);
          else if (bwd_tile == 19)   // 128x128, 4 waves of 64x64, BK64
            return step_gemm<GemmCfg<T, 128, 128, 64, 2, 2>, true>(WdTh, 4608, 128, dzt, g, M, dz_bytes, ep, 128, 4608,
                                                                    st);
          else if (bwd_tile == 20)   // the same on a 3-stage ring
            return step_gemm<GemmCfg<T, 128, 128, 64, 2, 2>, true, T, T, EB, 3, true>(WdTh, 4608, 128, dzt, g, M,
                                                                                      dz_bytes, ep, 128, 4608, st);
          else if (bwd_tile == 22)   // 128x64, BK128, 4-way in-WG split-K (8 waves)
            return step_gemm<GemmCfg<T, 128, 64, 128, 2, 1, 4>, true>(WdTh, 4608, 128, dzt, g, M, dz_bytes, ep, 128,
                                                                       4608, st);
          else if (bwd_tile == 23)   // 64x64, BK128, 2-way in-WG split-K (8 waves)
            return step_gemm<GemmCfg<T, 64, 64, 128, 2, 2, 2>, true>(WdTh, 4608, 128, dzt, g, M, dz_bytes, ep, 128,
                                                                      4608, st);
          else if (bwd_tile == 24)   // 64x32, BK128, 4-way in-WG split-K (8 waves)
            return step_gemm<GemmCfg<T, 64, 32, 128, 2, 1, 4>, true>(WdTh, 4608, 128, dzt, g, M, dz_bytes, ep, 128,
                                                                      4608, st);
          else if (bwd_tile == 21)   // 128x64, 4 waves of 64x32, BK64
            return step_gemm<GemmCfg<T, 128, 64, 64, 2, 2>, true>(WdTh, 4608, 128, dzt, g, M, dz_bytes, ep, 128, 4608,
                                                                   st);
          else
            return step_gemm<GemmCfg<T, 128, 64, 128, 2, 1, 2>, true>(WdTh, 4608, 128, dzt, g, M, dz_bytes, ep, 128,
                                                                       4608, st);
        } else {
          // tiles 19-24 other than 22 exist for fp16 gate storage only: fail loudly, never fall back
          if (bwd_tile >= 19 && bwd_tile <= 24 && bwd_tile != 22) return hipErrorInvalidValue;
          switch (bwd_tile) {
            case 1: return step_gemm<CfgKFor<T>, false>(WdTh, 4608, 128, dzt, g, M, dz_bytes, ep, 128, 4608, st);
            case 2: return step_gemm<CfgK4For<T>, false>(WdTh, 4608, 128, dzt, g, M, dz_bytes, ep, 128, 4608, st);
            case 3: return step_gemm<CfgK4BFor<T>, false>(WdTh, 4608, 128, dzt, g, M, dz_bytes, ep, 128, 4608, st);
            case 4:   // 3-stage ring, DMA interleaved with the MFMAs (tools/ubench/step_ablate: 57.9 vs 59.4 us)
              return step_gemm<CfgK4BFor<T>, true, T, T, EB, 3, true>(WdTh, 4608, 128, dzt, g, M, dz_bytes, ep, 128,
                                                                       4608, st);
            case 5: return step_gemm<CfgK4For<T>, true>(WdTh, 4608, 128, dzt, g, M, dz_bytes, ep, 128, 4608, st);
            case 6: return step_gemm<C, true>(WdTh, 4608, 128, dzt, g, M, dz_bytes, ep, 128, 4608, st);
            case 7:   // bf16: 128x128, BK128, 2-way in-WG split-K (tools/ubench/bf16_tiles: 48 vs 53-60 us at C3)
              if constexpr (std::is_same<T, float>::value) return hipErrorInvalidValue;
              else return step_gemm<GemmCfg<T, 128, 128, 128, 2, 2, 2>, true>(WdTh, 4608, 128, dzt, g, M, dz_bytes, ep,
                                                                              128, 4608, st);
            case 8:   // bf16: 128x64, BK128, 2-way in-WG split-K, 4 waves (small batches)
              if constexpr (std::is_same<T, float>::value) return hipErrorInvalidValue;
              else return step_gemm<GemmCfg<T, 128, 64, 128, 2, 1, 2>, true>(WdTh, 4608, 128, dzt, g, M, dz_bytes, ep,
                                                                             128, 4608, st);
            case 22:   // bf16 with fp32 gate storage (AAA_FUSED_X=0 / AAA_GATES_F16=0): the default small-batch tile
              if constexpr (std::is_same<T, float>::value) return hipErrorInvalidValue;
              else return step_gemm<GemmCfg<T, 128, 64, 128, 2, 1, 4>, true>(WdTh, 4608, 128, dzt, g, M, dz_bytes, ep,
                                                                             128, 4608, st);
            case 9:   // 64x32, BK128, 4-way in-WG split-K, 3-stage ring, interleaved DMA
              return step_gemm<GemmCfg<T, 64, 32, 128, 2, 1, 4>, true, T, T, EB, 3, true>(WdTh, 4608, 128, dzt, g, M,
                                                                                          dz_bytes, ep, 128, 4608, st);
            case 10:   // 32x32, BK128, 4-way in-WG split-K, 2-stage ring (2 WGs per CU, desynchronised barriers)
              return step_gemm<GemmCfg<T, 32, 32, 128, 1, 1, 4>, true, T, T, EB, 2, true>(WdTh, 4608, 128, dzt, g, M,
                                                                                         dz_bytes, ep, 128, 4608, st);
            case 11:   // 32x32, BK64, 4-way in-WG split-K, 3-stage ring
              return step_gemm<GemmCfg<T, 32, 32, 64, 1, 1, 4>, true, T, T, EB, 3, true>(WdTh, 4608, 128, dzt, g, M,
                                                                                        dz_bytes, ep, 128, 4608, st);
            case 12:   // 32x32, BK64, 4-way in-WG split-K, 4-stage ring
              return step_gemm<GemmCfg<T, 32, 32, 64, 1, 1, 4>, true, T, T, EB, 4, true>(WdTh, 4608, 128, dzt, g, M,
                                                                                        dz_bytes, ep, 128, 4608, st);
            case 13:   // 32x32, BK128, 8-way in-WG split-K (8 waves), 2-stage ring
              return step_gemm<GemmCfg<T, 32, 32, 128, 1, 1, 8>, true, T, T, EB, 2, true>(WdTh, 4608, 128, dzt, g, M,
                                                                                         dz_bytes, ep, 128, 4608, st);
            case 15:   // 64x32, BK64, 4-way in-WG split-K, 3-stage ring
              return step_gemm<GemmCfg<T, 64, 32, 64, 2, 1, 4>, true, T, T, EB, 3, true>(WdTh, 4608, 128, dzt, g, M,
                                                                                        dz_bytes, ep, 128, 4608, st);
            case 16:   // 32x32, BK64, 4-way in-WG split-K, 3-stage ring, DMA issued before the MFMAs
              return step_gemm<GemmCfg<T, 32, 32, 64, 1, 1, 4>, true, T, T, EB, 3, false>(WdTh, 4608, 128, dzt, g, M,
                                                                                         dz_bytes, ep, 128, 4608, st);
            // 27-29: fp32 as bf16x6 split products (gemm.h SPLIT6) on the small-batch shapes
            case 27:   // tile 16's shape
              if constexpr (!std::is_same<T, float>::value) return hipErrorInvalidValue;
              else return step_gemm<GemmCfgS6<32, 32, 64, 1, 1, 4>, true, T, T, EB, 3, false>(WdTh, 4608, 128, dzt, g,
                                                                                              M, dz_bytes, ep, 128,
                                                                                              4608, st);
            case 28:   // 32x32, BK128, 8-way in-WG split-K (8 waves), 2-stage ring
              if constexpr (!std::is_same<T, float>::value) return hipErrorInvalidValue;
              else return step_gemm<GemmCfgS6<32, 32, 128, 1, 1, 8>, true, T, T, EB, 2, true>(WdTh, 4608, 128, dzt, g,
                                                                                              M, dz_bytes, ep, 128,
                                                                                              4608, st);
            case 30:   // split-K tiles: t = 0 (dh0) takes tile 27
            case 31:
            case 32:
            case 33:
              if constexpr (!std::is_same<T, float>::value) return hipErrorInvalidValue;
              else return step_gemm<GemmCfgS6<32, 32, 64, 1, 1, 4>, true, T, T, EB, 3, false>(WdTh, 4608, 128, dzt, g,
                                                                                              M, dz_bytes, ep, 128,
                                                                                              4608, st);
            case 29:   // 64x32, BK128, 4-way in-WG split-K, 3-stage ring
              if constexpr (!std::is_same<T, float>::value) return hipErrorInvalidValue;
              else return step_gemm<GemmCfgS6<64, 32, 128, 2, 1, 4>, true, T, T, EB, 3, true>(WdTh, 4608, 128, dzt, g,
                                                                                              M, dz_bytes, ep, 128,
                                                                                              4608, st);
            default: return step_gemm<C, false>(WdTh, 4608, 128, dzt, g, M, dz_bytes, ep, 128, 4608, st);
          }
        }
      };
      const hipError_t e = g16 ? step(_Float16{}) : step(float{});
      HIPCHK(e);
    }
    { const int rc0 = flush(0); if (rc0) return rc0; }
    misc.reset(new TimerScope(AAA_TIMER_MISC, st, 0.0, "gate-bias column sums, state grads out, grad unpack"));
    // gate-bias gradient: column sum of the per-(step, tile) partials, or of dZ itself
    if (fb)   // per (step, frame[, pixel half]) partials
      HIPCHK(colsum<float>(Wf(L.dZp), 512, L.T * L.B * fb, 512, Wf(L.gbl), st));
    else if (fb32)   // per (step, frame) partials
      HIPCHK(colsum<float>(Wf(L.dZp), 512, L.T * L.B, 512, Wf(L.gbl), st));
    else if (part) HIPCHK(colsum<float>(part, 512, L.T * ntj, 512, Wf(L.gbl), st));
    else HIPCHK(colsum<T>(Wt(L.dZ), 512, F * P, 512, Wf(L.gbl), st));
    if (io->dc0) HIPCHK(hipMemcpyAsync(io->dc0, Wf(L.dC), (size_t)M * 128 * 4, hipMemcpyDeviceToDevice, st));
    if (ax) HIPCHK(stream_order(ax, st));   // join
    LstmGrads lg;
    for (int g = 0; g < 4; ++g) {
      lg.wx[g] = grads + L.poff[XI_W + 3 * g];
      lg.bx[g] = grads + L.poff[XI_B + 3 * g];
      lg.wh[g] = grads + L.poff[HI_W + 3 * g];
    }
    // with VISION in this call the ConvLSTM grads unpack in the vision phase's launch
    if (!(phases & AAA_BWD_VISION)) HIPCHK(unpack_lstm(Wf(L.gWpl), Wf(L.gbl), lg, st));
    else core_unpack = lg;
  }

  if (phases & AAA_BWD_VISION) {
    TimerScope tim(AAA_TIMER_VISION_BWD, st, vision_here ? 0.0 : (double)F * vision_bwd_flop(L),
                   vbwd_on<T>(L, F) ? "frame-resident conv2 wgrad + dgrad + conv1 wgrad [kernel: k_vision_bwd_frames], "
                                      "grad unpack"
                                    : "conv2 wgrad + dgrad, conv1 wgrad, grad unpack");
    if (!vision_here && vbwd_on<T>(L, F)) {   // VISION alone, frame-resident
      const int rc = vbwd_run<T>(L, pk, io->frames, 0, F, Wt(L.dY2), Wt(L.Y1), Wt(L.dY1), Wf(L.gWp2), Wf(L.gWp1),
                                 grads + L.poff[C0B], st);
      if (rc) return rc;
    } else if (!vision_here) {   // VISION alone: its chunk work over all frames, here
      const int rows1 = F * L.P1;
      constexpr bool f32 = std::is_same<T, float>::value;
      {
        const int rc = vision_bwd<T>(L, pk, Wt(L.dY2), Wt(L.Y1), Wt(L.Xp), Wt(L.dY1), F, Wf(L.gWp2), Wf(L.gWp1),
                                     grads + L.poff[C0B], st, L.xpc < L.F ? io->frames : nullptr);
        if (rc) return rc;
        if (f32 && !ab_int("AAA_CONV2_DGRAD_RING", 1)) HIPCHK(colsum(Wt(L.dY1), 32, rows1, 32, grads + L.poff[C0B], st));
      }
    }
    HIPCHK(unpack_cv((phases & AAA_BWD_CORE) ? Wf(L.gWpl) : nullptr, Wf(L.gbl), core_unpack, Wf(L.gWp2),
                     grads + L.poff[C1W], Wf(L.gWp1), grads + L.poff[C0W], st));
  }
  return AAA_OK;
}


template int lstm_wgrad<float>(const float*, const float*, int, int, int, float*, hipStream_t, bool);
template int lstm_wgrad<__bf16>(const __bf16*, const __bf16*, int, int, int, float*, hipStream_t, bool);
template int vision_bwd<float>(const Layout&, const char*, const float*, const float*, float*, float*, int,
                               float*, float*, float*, hipStream_t, const void*);
template int vision_bwd<__bf16>(const Layout&, const char*, const __bf16*, const __bf16*, __bf16*, __bf16*, int,
                                float*, float*, float*, hipStream_t, const void*);
template int backward_impl<float>(const Layout&, const aaa_io*, int, hipStream_t);
template int backward_impl<__bf16>(const Layout&, const aaa_io*, int, hipStream_t);

}  // namespace aaa
