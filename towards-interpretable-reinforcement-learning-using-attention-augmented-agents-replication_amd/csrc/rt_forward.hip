// Forward of the unroll (attention.py:298-368 over T steps): weight packing,
// the vision encoder, the ConvLSTM recurrence (frame-resident / frame-group /
// per-step kernels) and the batched attention / answer / policy-core / heads tail.
#include "rt.h"

namespace aaa {

// ------------------------------------------------------------- packing ----
template <typename T>
int pack_impl(const Layout& L, const float* prm, char* pk, hipStream_t st) {
  PackAll<T> a;
  a.c1w = prm + L.poff[C0W];
  a.c2w = prm + L.poff[C1W];
  a.Wp1 = (T*)(pk + L.k_Wp1); a.Wp2 = (T*)(pk + L.k_Wp2); a.WdT2 = (T*)(pk + L.k_WdT2);
  for (int g = 0; g < 4; ++g) {
    a.lstm.wx[g] = prm + L.poff[XI_W + 3 * g];
    a.lstm.bx[g] = prm + L.poff[XI_B + 3 * g];
    a.lstm.wh[g] = prm + L.poff[HI_W + 3 * g];
  }
  a.WpX = (T*)(pk + L.k_WpX); a.WpH = (T*)(pk + L.k_WpH); a.WdT = (T*)(pk + L.k_WdTl);
  a.WpXH = (T*)(pk + L.k_WpXH); a.bl = (float*)(pk + L.k_bl);
  F32Pack& fp = a.f32;
  fp.a0w = prm + L.poff[A0W]; fp.wih = prm + L.poff[WIH]; fp.bih = prm + L.poff[BIH]; fp.bhh = prm + L.poff[BHH];
  fp.pw = prm + L.poff[PW]; fp.vw = prm + L.poff[VW]; fp.pb = prm + L.poff[PB]; fp.vb = prm + L.poff[VB];
  fp.W1p = (float*)(pk + L.k_W1p); fp.Wihp = (float*)(pk + L.k_Wihp); fp.blc = (float*)(pk + L.k_blc);
  fp.Whd = (float*)(pk + L.k_Whd); fp.bhd = (float*)(pk + L.k_bhd);
  fp.ans_in = L.ans_in; fp.ans_ld = L.ans_ld; fp.A = L.A; fp.ldy = L.ldy;
  if (L.sc) {
    fp.whh = prm + L.poff[WHH];
    fp.Wihhp = (float*)(pk + L.k_Wihhp);
  }
  HIPCHK(pack_all<T>(a, st));   // conv1, conv2, conv2 dgrad classes, ConvLSTM layouts, fp32 tail: one launch
  if constexpr (!std::is_same<T, float>::value) {   // fragment orders of the frame-resident kernels (read WpXH / WdT)
    HIPCHK(pack_wfrag((const __bf16*)(pk + L.k_WpXH), (__bf16*)(pk + L.k_Wfr), st));
    HIPCHK(pack_wbfrag((const __bf16*)(pk + L.k_WdTl), (__bf16*)(pk + L.k_Wbf), st));
  } else {   // the fp32 frame-group recurrence's fragment order (recur_f32.h)
    // (pack_all wrote WpXH / WdT first: same stream)
    HIPCHK(pack_frag_f32(FragPack{(const float*)(pk + L.k_WpXH), (const float*)(pk + L.k_WdTl), (float*)(pk + L.k_Wf32),
                                  (u32x2*)(pk + L.k_Wf6), (u32x4*)(pk + L.k_Wf6p), (float*)(pk + L.k_Wb32),
                                  (u32x2*)(pk + L.k_Wb6), (u32x2*)(pk + L.k_Wx6), (u32x4*)(pk + L.k_Wb6p),
                                  (u32x4*)(pk + L.k_Wx6p), (__bf16*)(pk + L.k_WdT6)},
                         st));
  }
  HIPCHK(query_pack(prm + L.poff[Q0B], prm + L.poff[Q2W], prm + L.poff[Q2B], prm + L.poff[Q4W], prm + L.poff[Q4B], L.nq,
                    (float*)(pk + L.k_q1), (float*)(pk + L.k_q2), (float*)(pk + L.k_Q), st));
  return AAA_OK;
}

// Vision encoder over F frames (VisionNetwork.vision_cnn, attention.py:155-170,
// on X.transpose(1,3), :179 -- Q3): frames (F,H,W,3) -> zero-bordered RGBx
// image Xp -> conv 8/4/1 -> Y1 (F,H1,W1,32) -> conv 4/2/2 -> out (F,h,w,64) at
// row pitch out_ld (the ConvLSTM operand slots, or a plain output), no
// activation in between.  Packed conv weights at L.k_Wp1 / L.k_Wp2, biases
// from the flat params (state_dict order: the vision tensors come first).
template <typename T, typename OT>
static int vision_fwd_chunk(const Layout& L, int F, const char* pk, const float* prm, const void* frames, T* Xp, T* Y1,
                      OT* out, int out_ld, hipStream_t st, bool xp_full) {
  using C = CfgFor<T>;
  constexpr int NT = C::NT;
  const int P = L.P;
  bool banded = false;   // bf16 frames too large for the frame-resident encoder: the banded conv1 (vision.h)
  if constexpr (std::is_same<T, __bf16>::value) {
    if (band_fits(L.H, L.W, L.H1, L.W1) && ab_int("AAA_VIS_BAND", 1)) {
      const VisBandParams bp{frames, (const __bf16*)(pk + L.k_Wp1), prm + L.poff[C0B], xp_full ? Xp : nullptr, Y1, F,
                             L.H, L.W, L.H1, L.W1};
      HIPCHK(L.fu8 ? vision_conv1_band<uint8_t>(bp, st) : vision_conv1_band<float>(bp, st));
      banded = true;
    }
  }
  if (!banded) {  // conv1 (attention.py:156-162): frames -> zero-bordered RGBx (Cin 4, pad 1 stored) -> Y1
    // xp_full: Xp holds all F frames (the component entries keep it for their backward);
    // else Xp is the chunk buffer of L.xpc frames, rebuilt per chunk right before conv1 reads it
    const size_t fb = (size_t)L.H * L.W * 3 * (L.fu8 ? 1 : 4), xb = (size_t)(L.H + 2) * (L.W + 2) * 4;
    const int step = xp_full ? F : L.xpc;
    for (int s0 = 0; s0 < F; s0 += step) {
      const int n = std::min(step, F - s0);
      const char* fr = (const char*)frames + (size_t)s0 * fb;
      T* xp = xp_full ? Xp + (size_t)s0 * xb : Xp;
      if (L.fu8) HIPCHK((frames_rgbx<T, uint8_t>(n, L.H, L.W, (const uint8_t*)fr, xp, st)));
      else HIPCHK((frames_rgbx<T, float>(n, L.H, L.W, (const float*)fr, xp, st)));
      // LDS-DMA ring, 32x128 tile over 4 waves (tools/ubench/conv_cfg: 62 vs 90 us register-staged)
      constexpr int BKc = std::is_same<T, float>::value ? 32 : 64;
      EpiStoreT<T> ep{Y1 + (size_t)s0 * L.P1 * 32, 32, 32, n * L.P1, prm + L.poff[C0B], 0};
      auto conv1 = [&](auto cfg) -> int {
        using CP = decltype(cfg);
        using PA = GRowsB<T, CP::BI, CP::BK, CP::NT>;
        using PB = GIm2colB<T, CP::BJ, CP::BK, CP::NT>;
        HIPCHK((launch_pipe<CP, PA, PB, EpiStoreT<T>, 2>(
            typename PA::Params{(const T*)(pk + L.k_Wp1), 256, 32},
            typename PB::Params{xp, ConvGeo{4, 4, 0, L.H + 2, L.W + 2, L.H1, L.W1, 8, 4, 0, 0}.prep(), n * L.P1,
                                (uint32_t)((size_t)n * xb * L.esz)},
            ep, 32, n * L.P1, 256, 1, st)));
        return AAA_OK;
      };
      // K = 256 is four BK steps: a wider column tile does more MFMA work per DMA round trip (A/B: AAA_CONV1_TILE)
      const int c1t = ab_int("AAA_CONV1_TILE", 0);
      int rc;
      if constexpr (std::is_same<T, float>::value) {   // fp32 accuracy on the bf16 MFMA (gemm.h SPLIT6)
        // uint8 frames: the RGBx operand is exact in bf16 (three of the six split products, GemmCfgS6BX)
        if (f32_split6()) rc = L.fu8 && ab_int("AAA_CONV1_BEXACT", 1) ? conv1(GemmCfgS6BX<32, 128, BKc, 1, 4>{})
                                                                      : conv1(GemmCfgS6<32, 128, BKc, 1, 4>{});
        else rc = c1t == 1 ? conv1(GemmCfg<T, 32, 256, BKc, 1, 4>{}) : conv1(GemmCfg<T, 32, 128, BKc, 1, 4>{});
      } else {
        rc = c1t == 1 ? conv1(GemmCfg<T, 32, 256, BKc, 1, 4>{}) : conv1(GemmCfg<T, 32, 128, BKc, 1, 4>{});
      }
      if (rc) return rc;
    }
  }
  if constexpr (std::is_same<T, __bf16>::value && std::is_same<OT, __bf16>::value) {
    // after the banded conv1: the banded conv2 (vision.h), Y1 rows staged in LDS per band
    if (banded && band2_fits(L.H1, L.W1, L.h, L.w) && ab_int("AAA_VIS_BAND2", 1)) {
      const VisBand2Params bp{Y1, (const __bf16*)(pk + L.k_Wp2), prm + L.poff[C1B], out, out_ld, F, L.H1, L.W1, L.h, L.w};
      HIPCHK(vision_conv2_band(bp, st));
      return AAA_OK;
    }
  }
  {  // conv2 (attention.py:163-169): Y1 -> out
    using LA = LdRowsB<T, T, C::BI, C::BK, NT>;
    typename LA::Params pa{(const T*)(pk + L.k_Wp2), 512, 64};
    const ConvGeo g = ConvGeo{32, 32, 0, L.H1, L.W1, L.h, L.w, 4, 2, 2, 0}.prep();
    EpiStoreT<OT> ep{out, out_ld, 64, F * P, prm + L.poff[C1B], 0};
    const uint32_t y1b = (uint32_t)((size_t)F * L.P1 * 32 * L.esz);
    if constexpr (32 % C::BK == 0) {   // LDS-DMA ring (tools/ubench/conv_cfg: 62 vs 67 us)
      if (std::is_same<T, float>::value && f32_split6())   // fp32 accuracy on the bf16 MFMA (gemm.h SPLIT6)
        HIPCHK((step_gemm<std::conditional_t<std::is_same<T, float>::value, typename S6Of<C>::type, C>, true>(
            (const T*)(pk + L.k_Wp2), 512, 64, (const T*)Y1, g, F * P, y1b, ep, 64, 512, st)));
      else
        HIPCHK((step_gemm<C, true>((const T*)(pk + L.k_Wp2), 512, 64, (const T*)Y1, g, F * P, y1b, ep, 64, 512, st)));
    } else if (pipe_batched()) {   // bf16: a BK=32 ring, one 4x4 tap row's 32 channels per K tile
      HIPCHK((step_gemm<GemmCfg<T, 64, 128, 32, 2, 2>, true>((const T*)(pk + L.k_Wp2), 512, 64, (const T*)Y1, g,
                                                           F * P, y1b, ep, 64, 512, st)));
    } else {
      using LB = LdIm2col<T, T, C::BJ, C::BK, NT, true>;
      HIPCHK((launch_gemm<C, LA, LB>(pa, typename LB::Params{Y1, g, F * P}, ep, 64, F * P, 512, 1, st)));
    }
  }
  return AAA_OK;
}


template <typename T, typename OT>
int vision_fwd(const Layout& L, int F, const char* pk, const float* prm, const void* frames, T* Xp, T* Y1,
                      OT* out, int out_ld, hipStream_t st, bool xp_full) {
  if constexpr (std::is_same<T, __bf16>::value && std::is_same<OT, __bf16>::value) {
    // bf16: the frame-resident encoder (vision.h), one launch; AAA_VIS_FRAMES=0 -> the layered kernels
    if (vis_fits(L.H, L.W, L.H1, L.W1, L.h, L.w) && env_int("AAA_VIS_FRAMES", 1)) {
      VisFwdParams vp{frames, (const __bf16*)(pk + L.k_Wp1), prm + L.poff[C0B], (const __bf16*)(pk + L.k_Wp2),
                      prm + L.poff[C1B], xp_full ? Xp : nullptr, Y1, out, out_ld, F, L.H, L.W, L.H1, L.W1, L.h, L.w};
      HIPCHK(L.fu8 ? vision_fwd_frames<uint8_t>(vp, device_cus(), st) : vision_fwd_frames<float>(vp, device_cus(), st));
      return AAA_OK;
    }
  }
  for (int f0 = 0; f0 < F; f0 += L.fchunk) {   // descriptor-sized frame chunks (check_ranges)
    const int n = std::min(L.fchunk, F - f0);
    const int rc = vision_fwd_chunk<T, OT>(L, n, pk, prm,
                                           (const char*)frames + (size_t)f0 * L.H * L.W * 3 * (L.fu8 ? 1 : 4),
                                           xp_full ? Xp + (size_t)f0 * (L.H + 2) * (L.W + 2) * 4 : Xp,
                                           Y1 + (size_t)f0 * L.P1 * 32, out + (size_t)f0 * L.P * out_ld, out_ld, st,
                                           xp_full);
    if (rc) return rc;
  }
  return AAA_OK;
}

template <typename T>
static int forward_tail(const Layout& L, const aaa_io* io, hipStream_t st);

template <typename T>
int forward_impl(const Layout& L, const aaa_io* io, hipStream_t st, int phases) {
  using C = CfgFor<T>;
  // bf16 path: the fp32 tail GEMMs on the bf16 MFMA with split operands (AAA_TAIL_SPLIT3=0: fp32 MFMA)
  TailPrecision tail_prec(std::is_same<T, __bf16>::value && env_int("AAA_TAIL_SPLIT3", 1),
                          std::is_same<T, float>::value && f32_split6());
  char* ws = (char*)io->workspace;
  const char* pk = (const char*)io->packed;
  const float* prm = io->params;
  auto Wf = [&](size_t off) { return (float*)(ws + off); };
  auto Wt = [&](size_t off) { return (T*)(ws + off); };
  const int F = L.F, M = L.B * L.P;
  // fp32 h_t slices for the readout: fp32 path only (bf16 reads XH, readout_h)
  auto hs_out = [&](int t) { return L.esz == 4 ? Wf(L.Hs) + (size_t)t * M * 128 : (float*)nullptr; };

  {  // conv1 + conv2 over all T*B frames -> XH[:, :, 0:64] of every slot
    TimerScope tim(AAA_TIMER_VISION_FWD, st, (double)F * vision_fwd_flop(L), "conv1 + conv2 (vision encoder)");
    const int rc = vision_fwd<T, T>(L, F, pk, prm, io->frames, Wt(L.Xp), Wt(L.Y1), Wt(L.XH), 192, st, L.xpc >= F);
    if (rc) return rc;
  }
  {  // initial state (reset(): zeros, attention.py:142-149) or carried state
    TimerScope tim(AAA_TIMER_MISC, st, 0.0, "state in/out copies, memsets, bias column sums");
    // one launch: h_0 into XH slot 0, c_0 = 0 (reset) and the hand-off flags of this forward's
    // multi-workgroup recurrence launch (zeroed here for every kernel choice)
    ZeroRanges z{};
    if (!io->c0) z.add(Wf(L.Cst), (long)M * 128);
    if (phases & AAA_FWD_CORE) z.add(Wf(L.rflags), (long)8 * L.B);
    HIPCHK(prologue<T>(z, M, io->h0, Wt(L.XH), 0, 0, 1, nullptr, nullptr, nullptr, st));
    if (io->c0 && (cqm_layout(L) & kCqmC)) HIPCHK(cqm_convert(io->c0, Wf(L.Cst), L.B, L.P, 1, st));
    else if (io->c0) HIPCHK(hipMemcpyAsync(Wf(L.Cst), io->c0, (size_t)M * 128 * 4, hipMemcpyDeviceToDevice, st));
  }
  // no CORE (aaa_forward_phases, fp32): the recurrence's products are already in
  // Gt / Cst / Hs / XH (aaa_core_import)
  if (!(phases & AAA_FWD_CORE)) return forward_tail<T>(L, io, st);
  if constexpr (std::is_same<T, float>::value) {
    if (const int G = f32_frames(L)) {   // one frame-group launch for all T steps, x-part included (recur_f32.h)
      int dev = 0;
      HIPCHK(hipGetDevice(&dev));
      int* rep = pair_report(dev);
      if (!rep) return fail(AAA_E_LAUNCH, "cannot map the frame-group report word");
      RecF32Params rp{(const float*)(pk + L.k_Wf32), (const float*)(pk + L.k_bl), Wf(L.XH), Wf(L.Cst), Wf(L.Hs),
                      Wf(L.Gt), (int*)(ws + L.rflags), rep, pair_budget(L.T), L.T, L.B, L.h, L.w, L.P,
                      io->h0 ? 0 : 1, {}};
      {
        const bool s6 = f32_split6();
        rp.Wf6 = (const u32x2*)(pk + L.k_Wf6);
        rp.Wf6p = (const u32x4*)(pk + L.k_Wf6p);
        TimerScope tim(AAA_TIMER_FWD_STEP, st, 2.0 * M * 512 * (576.0 * L.T + 1152.0 * (L.T - (io->h0 ? 0 : 1))),
                       strf("fp32 frame-group [x|h] recurrence%s, %d steps per launch, %d WG per frame [kernel: %s]",
                            s6 ? " (bf16x6 split products)" : "", L.T, G,
                            f32_fwd_presplit(s6, G, L.P) ? "k_convlstm_fwd_f32ps" : "k_convlstm_fwd_f32<"));
        HIPCHK(convlstm_fwd_f32(rp, G, st, s6));
      }
      return forward_tail<T>(L, io, st);
    }
  }
  // bf16: the x-part rides in each step's GEMM (K over the whole XH slot,
  // [x_t | h_{t-1}], bias in the epilogue): no batched x-part GEMM and no
  // fp32 x-part round trip through HBM (tools/ubench/bf16_tiles: the step's
  // epilogue traffic, not its MFMAs, is half its time).  AAA_FUSED_X=0/1 overrides.
  if (fused_x(L.dt, M)) {
    const T* WpXH = (const T*)(pk + L.k_WpXH);
    // bf16: 128x128 tiles of 4 waves (64x64 per wave: twice the MFMA work per
    // fragment read of the 128x64 8-wave tile) -- C3 94.7 -> 81-83 us, C4 51.5 ->
    // 44.6 us, C5 90.7 -> 78.6-79.5 us per step (tools/ab_fused.sh); fp32 (only
    // small M, e.g. the B=1 actor, fuses the x-part): 128x64 8 waves.
    auto steps = [&](auto gtag) -> int {
      using GT = decltype(gtag);
      if constexpr (!std::is_same<T, float>::value) {
        if (const int NBd = frames_band(L)) {   // one band-mode launch for all T steps (recur.h BAND)
          int dev = 0;
          HIPCHK(hipGetDevice(&dev));
          int* rep = pair_report(dev);
          if (!rep) return fail(AAA_E_LAUNCH, "cannot map the band-mode report word");
          RecFwdParams<GT> rp{(const __bf16*)(pk + L.k_Wfr), (const float*)(pk + L.k_bl), Wt(L.XH), Wf(L.Cst),
                              nullptr, (GT*)(ws + L.Gt), (int*)(ws + L.rflags), L.T, L.B, L.h, L.w, L.P,
                              rep, pair_budget(L.T), rec_stagger("AAA_REC_STAGGER_FWD")};
          rp.cqm = cqm_layout(L);
          TimerScope tim(AAA_TIMER_FWD_STEP, st, 2.0 * M * 512 * 1728 * L.T,
                         strf("bf16 band-mode frame-resident [x|h] recurrence, %d steps per launch, %d bands per frame "
                              "[kernel: k_convlstm_fwd_frames+Lb1E]", L.T, NBd));
          HIPCHK(convlstm_fwd_frames_band<GT>(rp, st));
          return AAA_OK;
        }
        if (const int G = frames_fwd(L)) {   // one frame-resident launch for all T steps (recur.h)
          int* rep = nullptr;
          if (G == 2) {
            int dev = 0;
            HIPCHK(hipGetDevice(&dev));
            if (!(rep = pair_report(dev))) return fail(AAA_E_LAUNCH, "cannot map the paired-kernel report word");
          }
          RecFwdParams<GT> rp{(const __bf16*)(pk + L.k_Wfr), (const float*)(pk + L.k_bl), Wt(L.XH), Wf(L.Cst),
                              nullptr, (GT*)(ws + L.Gt), (int*)(ws + L.rflags), L.T, L.B, L.h, L.w, L.P,
                              rep, pair_budget(L.T), rec_stagger("AAA_REC_STAGGER_FWD")};
          rp.cqm = cqm_layout(L);
          // row-padded h image (recur.h rec_rowpad): measured neutral to 1 % slower (C3 forward 1234-1242 vs
          // 1247-1269 us, profiles/r06/ab/rowpad_fwd/), so an A/B option (AAA_REC_ROWPAD=1, ablation builds)
          rp.rowpad = ab_int("AAA_REC_ROWPAD", 0) ? rec_rowpad(L.h, L.w) : 0;
          TimerScope tim(AAA_TIMER_FWD_STEP, st, 2.0 * M * 512 * 1728 * L.T,
                         strf("bf16 frame-resident [x|h] recurrence, %d steps per launch, %d WG per frame%s [kernel: k_convlstm_fwd_frames+Lb0E]",
                              L.T, G, rp.rowpad ? ", row-padded h image" : ""));
          HIPCHK(convlstm_fwd_frames<GT>(rp, G, st));
          return AAA_OK;
        }
      }
      for (int t = 0; t < L.T; ++t) {   // ConvLSTM (attention.py:110-126), x- and h-part together
        EpiConvLstmFwd<T, GT> ep{Wf(L.Cst) + (size_t)t * M * 128, Wf(L.Cst) + (size_t)(t + 1) * M * 128,
                                 hs_out(t), Wt(L.XH) + (size_t)(t + 1) * M * 192,
                                 (GT*)(ws + L.Gt) + (size_t)t * M * 512, M, (const float*)(pk + L.k_bl)};
        const int rc = fused_step<T, GT>(WpXH, Wt(L.XH) + (size_t)t * M * 192, L.h, L.w, M, ep, st,
                                         L.dhs ? Wf(L.dhs) : nullptr);
        if (rc) return rc;
      }
      return AAA_OK;
    };
    const int rc = gates_f16(L.dt, M) ? steps(_Float16{}) : steps(float{});
    if (rc) return rc;
    return forward_tail<T>(L, io, st);
  }
  // x-part of the ConvLSTM steps (not recurrent): Gt <- Wx * x_t + b, in
  // chunks of ``cs`` steps on the aux stream; step t waits only for its chunk.
  hipStream_t ax = aux_stream();
  const int cs = chunk_steps(L);
  hipStream_t xs = ax ? ax : st;
  if (ax) HIPCHK(stream_order(st, ax));
  auto xpart = [&](int lo, int hi) -> int {
    // 64x64 tiles (128x128 measured slower: K is only 576)
    const ConvGeo g = ConvGeo{64, 192, 0, L.h, L.w, L.h, L.w, 3, 1, 1, 0}.prep();
    const int rows = (hi - lo) * M;
    EpiStoreT<float> ep{Wf(L.Gt) + (size_t)lo * M * 512, 512, 512, rows, (const float*)(pk + L.k_bl), 0};
    const T* WpX = (const T*)(pk + L.k_WpX);
    const T* xs0 = Wt(L.XH) + (size_t)lo * M * 192;
    const uint32_t xb = (uint32_t)((size_t)(hi - lo) * M * 192 * L.esz);
    switch (pipe_batched() ? ab_int("AAA_XPART_TILE", 0) : -1) {   // A/B: tools/ab_batched.sh
      case -1: HIPCHK((step_gemm<CfgFor<T>, false>(WpX, 576, 512, xs0, g, rows, xb, ep, 512, 576, xs))); break;
#ifdef AAA_ABLATION   // the measured-slower x-part tiles
      using EX = EpiStoreT<float>;
      case 1: HIPCHK((step_gemm<Cfg64For<T>, true>(WpX, 576, 512, xs0, g, rows, xb, ep, 512, 576, xs))); break;
      case 2: HIPCHK((step_gemm<CfgFor<T>, true, T, T, EX, 3, true>(WpX, 576, 512, xs0, g, rows, xb, ep, 512, 576, xs))); break;
      case 3: HIPCHK((step_gemm<CfgJFor<T>, true>(WpX, 576, 512, xs0, g, rows, xb, ep, 512, 576, xs))); break;
      case 4: HIPCHK((step_gemm<CfgSFor<T>, true>(WpX, 576, 512, xs0, g, rows, xb, ep, 512, 576, xs))); break;
      case 5:
        HIPCHK((step_gemm<GemmCfg<T, 128, 128, 32, 2, 2>, true>(WpX, 576, 512, xs0, g, rows, xb, ep, 512, 576, xs)));
        break;
#endif
      default: HIPCHK((step_gemm<CfgFor<T>, true>(WpX, 576, 512, xs0, g, rows, xb, ep, 512, 576, xs))); break;
    }
    return AAA_OK;
  };
  hipEvent_t xev[64];
  const int nchunks = (L.T + cs - 1) / cs;
  if (ax && nchunks > 48) return fail(AAA_E_ARG, "too many overlap chunks (T=%d, AAA_CHUNK=%d)", L.T, cs);
  for (int k = 0; k < nchunks; ++k) {
    int rc = xpart(k * cs, std::min(L.T, (k + 1) * cs));
    if (rc) return rc;
    if (ax) HIPCHK(record_event(ax, &xev[k]));
  }
  const int fwd_tile = step_tile((long)(512 / 32) * cdiv(M, 32), "AAA_STEP_TILE", false);
  const uint32_t xh_bytes = (uint32_t)((size_t)M * 192 * L.esz);  // one step slice of XH
  for (int t = 0; t < L.T; ++t) {  // ConvLSTM recurrence (attention.py:110-126): h-part only
    if (ax && t % cs == 0) HIPCHK(hipStreamWaitEvent(st, xev[t / cs], 0));   // x-part of steps [t, t+cs) done
    if (t == 0 && !io->h0) {       // zero state: gates come from the x-part alone
      HIPCHK(gate_fwd_zx<T>(M, Wf(L.Cst), Wf(L.Gt), Wf(L.Cst) + (size_t)M * 128, hs_out(0), Wt(L.XH) + (size_t)M * 192,
                            st));
      continue;
    }
    EpiConvLstmFwd<T> ep{Wf(L.Cst) + (size_t)t * M * 128, Wf(L.Cst) + (size_t)(t + 1) * M * 128,
                         hs_out(t), Wt(L.XH) + (size_t)(t + 1) * M * 192,
                         Wf(L.Gt) + (size_t)t * M * 512, M};
    const ConvGeo g = ConvGeo{128, 192, 64, L.h, L.w, L.h, L.w, 3, 1, 1, 0}.prep();
    TimerScope tim(AAA_TIMER_FWD_STEP, st, 2.0 * M * 512 * 1152, strf("%s h-part step (x-part batched), K=1152, tile %d [kernel: EpiConvLstmFwd]", std::is_same<T, float>::value ? "fp32" : "bf16", fwd_tile));
    const T* WpH = (const T*)(pk + L.k_WpH);
    const T* xh = Wt(L.XH) + (size_t)t * M * 192;
    hipError_t e;
    switch (fwd_tile) {
      case 1: case 2: e = step_gemm<CfgKFor<T>, false>(WpH, 1152, 512, xh, g, M, xh_bytes, ep, 512, 1152, st); break;
      case 3: e = step_gemm<Cfg64For<T>, false>(WpH, 1152, 512, xh, g, M, xh_bytes, ep, 512, 1152, st); break;
      case 4:   // 128x64, 8 waves
        e = step_gemm<CfgSFor<T>, true>(WpH, 1152, 512, xh, g, M, xh_bytes, ep, 512, 1152, st);
        break;
      case 7: e = step_gemm<C, true>(WpH, 1152, 512, xh, g, M, xh_bytes, ep, 512, 1152, st); break;
      case 5: e = step_gemm<CfgKFor<T>, true>(WpH, 1152, 512, xh, g, M, xh_bytes, ep, 512, 1152, st); break;
      case 6: e = step_gemm<Cfg64For<T>, true>(WpH, 1152, 512, xh, g, M, xh_bytes, ep, 512, 1152, st); break;
      case 12:   // 32x64 BK64, 2-way in-WG split-K, 3-stage ring
        e = step_gemm<CfgKFor<T>, true, T, T, EpiConvLstmFwd<T>, 3, true>(WpH, 1152, 512, xh, g, M, xh_bytes, ep, 512,
                                                                          1152, st);
        break;
      case 14:   // 32x32 BK64, 4-way in-WG split-K, 3-stage ring
        e = step_gemm<GemmCfg<T, 32, 32, 64, 1, 1, 4>, true, T, T, EpiConvLstmFwd<T>, 3, true>(WpH, 1152, 512, xh, g, M,
                                                                                              xh_bytes, ep, 512, 1152, st);
        break;
      case 17:   // 64x32 BK64, 2-way in-WG split-K, 3-stage ring
        e = step_gemm<GemmCfg<T, 64, 32, 64, 2, 1, 2>, true, T, T, EpiConvLstmFwd<T>, 3, true>(WpH, 1152, 512, xh, g, M,
                                                                                              xh_bytes, ep, 512, 1152, st);
        break;
      case 25:   // 64x64 BK64, 2-way in-WG split-K (8 waves), 2-stage ring
        e = step_gemm<GemmCfg<T, 64, 64, 64, 2, 2, 2>, true>(WpH, 1152, 512, xh, g, M, xh_bytes, ep, 512, 1152, st);
        break;
      case 26:   // 64x64 BK128, 2-way in-WG split-K (8 waves), 2-stage ring
        e = step_gemm<GemmCfg<T, 64, 64, 128, 2, 2, 2>, true>(WpH, 1152, 512, xh, g, M, xh_bytes, ep, 512, 1152, st);
        break;
      case 18:   // 64x64 BK64, 2x2 waves, 3-stage ring
        e = step_gemm<Cfg64For<T>, true, T, T, EpiConvLstmFwd<T>, 3, true>(WpH, 1152, 512, xh, g, M, xh_bytes, ep, 512,
                                                                           1152, st);
        break;
      default: e = step_gemm<C, false>(WpH, 1152, 512, xh, g, M, xh_bytes, ep, 512, 1152, st); break;
    }
    HIPCHK(e);
  }
  return forward_tail<T>(L, io, st);
}

// Stateful policy core (AAA_FLAG_STATEFUL_CORE; the reference's else branch,
// attention.py:324-331, 356-358): per step t, over the B frames of that step,
//   Q_t = QueryNetwork(h_{t-1}) -> attention readout with the per-frame Q_t ->
//   answer MLP -> LSTMCell([answer | h_{t-1}], c_{t-1}) -> (h_t, c_t).
// State slots CH/CC[t] hold (h, c) entering step t (slot 0 = io->core_*0 or
// zeros); the LSTMCell epilogue also writes h_t into step t+1's [answer | h]
// GEMM row, so each step is five small GEMMs and one attention launch.  The
// heads then run batched over all frames on CH[1..T].
static int forward_tail_stateful(const Layout& L, const aaa_io* io, hipStream_t st) {
  constexpr int NTF = CF::NT;
  char* ws = (char*)io->workspace;
  const char* pk = (const char*)io->packed;
  const float* prm = io->params;
  auto Wf = [&](size_t off) { return (float*)(ws + off); };
  const int B = L.B, P = L.P, qd = L.qd;
  const size_t sB = (size_t)B * 256 * 4;
  float *CH = Wf(L.CH), *CC = Wf(L.CC), *AOX = Wf(L.AOX);
  if (io->core_h0) HIPCHK(hipMemcpyAsync(CH, io->core_h0, sB, hipMemcpyDeviceToDevice, st));
  else HIPCHK(hipMemsetAsync(CH, 0, sB, st));
  if (io->core_c0) HIPCHK(hipMemcpyAsync(CC, io->core_c0, sB, hipMemcpyDeviceToDevice, st));
  else HIPCHK(hipMemsetAsync(CC, 0, sB, st));
  HIPCHK(hipMemcpy2DAsync(AOX + 256, 512 * 4, CH, 256 * 4, 256 * 4, B, hipMemcpyDeviceToDevice, st));
  using LRf = LdRows<float, float, CF::BI, CF::BK, NTF>;
  using LRfj = LdRows<float, float, CF::BJ, CF::BK, NTF>;
  for (int t = 0; t < L.T; ++t) {
    const size_t f0 = (size_t)t * B;
    float* q1 = Wf(L.q1s) + f0 * 128;
    float* q2 = Wf(L.q2s) + f0 * qd;
    float* Qt = Wf(L.Qf) + f0 * qd;
    {  // QueryNetwork(prev_output = h_{t-1}) (attention.py:184-198, 331)
      LRf::Params pa{prm + L.poff[Q0W], 256, 128};
      LRfj::Params pb{CH + f0 * 256, 256, B};
      EpiStoreT<float> ep{q1, 128, 128, B, prm + L.poff[Q0B], 1};
      HIPCHK((tail_gemm(pa, pb, ep, 128, B, 256, st)));
    }
    {
      LRf::Params pa{prm + L.poff[Q2W], 128, qd};
      LRfj::Params pb{q1, 128, B};
      EpiStoreT<float> ep{q2, qd, qd, B, prm + L.poff[Q2B], 1};
      HIPCHK((tail_gemm(pa, pb, ep, qd, B, 128, st)));
    }
    {
      LRf::Params pa{prm + L.poff[Q4W], qd, qd};
      LRfj::Params pb{q2, qd, B};
      EpiStoreT<float> ep{Qt, qd, qd, B, prm + L.poff[Q4B], 0};
      HIPCHK((tail_gemm(pa, pb, ep, qd, B, qd, st)));
    }
    // attention readout with this step's per-frame queries (basis logits in-kernel)
    {
      TimerScope tim(AAA_TIMER_ATTN_FWD, st, (double)B * attn_fwd_bytes(P, L.nq, L.ans_ld, L.esz), L.esz == 2 ? "k_attn_fwd_mfma, per-frame query (stateful core)" : "k_attn_fwd, per-frame query (stateful core)");
      HIPCHK(attn_fwd(readout_h(L, ws).frame(f0, P), io->basis, Qt, nullptr, io->prev_reward ? io->prev_reward + f0 : nullptr,
                      io->prev_action ? io->prev_action + f0 : nullptr, B, P, L.nq, Wf(L.Am) + f0 * P * L.nq,
                      Wf(L.ans) + f0 * L.ans_ld, L.ans_ld, st, qd));
    }
    {  // answer_processor.0 + ReLU
      LRf::Params pa{(const float*)(pk + L.k_W1p), L.ans_ld, 512};
      LRfj::Params pb{Wf(L.ans) + f0 * L.ans_ld, L.ans_ld, B};
      EpiStoreT<float> ep{Wf(L.hid1) + f0 * 512, 512, 512, B, prm + L.poff[A0B], 1};
      HIPCHK((tail_gemm(pa, pb, ep, 512, B, L.ans_ld, st)));
    }
    {  // answer_processor.2 -> the answer half of this step's [answer | h_{t-1}] rows
      LRf::Params pa{prm + L.poff[A2W], 512, 256};
      LRfj::Params pb{Wf(L.hid1) + f0 * 512, 512, B};
      EpiStoreT<float> ep{AOX + f0 * 512, 512, 256, B, prm + L.poff[A2B], 0};
      HIPCHK((tail_gemm(pa, pb, ep, 256, B, 512, st)));
    }
    {  // policy_core LSTMCell from (h_{t-1}, c_{t-1}) (attention.py:356-358)
      LRf::Params pa{(const float*)(pk + L.k_Wihhp), 512, 1024};
      LRfj::Params pb{AOX + f0 * 512, 512, B};
      EpiLstmCellFwdS ep{(const float*)(pk + L.k_blc), Wf(L.LG) + f0 * 1024, CC + f0 * 256, CC + (f0 + B) * 256,
                         CH + (f0 + B) * 256, t + 1 < L.T ? AOX + (f0 + B) * 512 + 256 : nullptr, B};
      HIPCHK((tail_gemm(pa, pb, ep, 1024, B, 512, st)));
    }
  }
  if (io->attn)
    HIPCHK(hipMemcpyAsync(io->attn, Wf(L.Am), (size_t)L.F * P * L.nq * 4, hipMemcpyDeviceToDevice, st));
  return AAA_OK;
}

// Everything after the ConvLSTM: query, attention readout, answer MLP,
// LSTMCell, heads (all batched over the T*B frames, Q1) and state outputs.
template <typename T>
static int forward_tail(const Layout& L, const aaa_io* io, hipStream_t st) {
  constexpr int NTF = CF::NT;
  char* ws = (char*)io->workspace;
  const char* pk = (const char*)io->packed;
  const float* prm = io->params;
  auto Wf = [&](size_t off) { return (float*)(ws + off); };
  const int F = L.F, P = L.P, M = L.B * L.P;
  if (L.sc) {   // stateful core: the tail runs step by step
    const int rc = forward_tail_stateful(L, io, st);
    if (rc) return rc;
  } else {
  // constant query (Q1) + fused attention readout over all T*B frames
  const float* Qc = (const float*)(pk + L.k_Q);
  {
    TimerScope tim(AAA_TIMER_TAIL_FWD, st, 0.0, "query basis logits");
    HIPCHK(query_sq(io->basis, Qc, P, L.nq, Wf(L.SQ), st));
  }
  {
    TimerScope tim(AAA_TIMER_ATTN_FWD, st, (double)F * attn_fwd_bytes(P, L.nq, L.ans_ld, L.esz), L.esz == 2 ? "k_attn_fwd_mfma (readout on the MFMA, map and basis in bf16 parts), 1 WG per frame" : "k_attn_fwd (VALU), 1 WG per frame");
    HIPCHK(attn_fwd(readout_h(L, ws), io->basis, Qc, Wf(L.SQ), io->prev_reward, io->prev_action, F, P, L.nq, Wf(L.Am),
                    Wf(L.ans), L.ans_ld, st));
  }
  TimerScope tim(AAA_TIMER_TAIL_FWD, st, (double)F * tail_fwd_flop(L), "answer MLP + LSTMCell + heads (fp32 GEMMs)");
  if (io->attn) HIPCHK(hipMemcpyAsync(io->attn, Wf(L.Am), (size_t)F * P * L.nq * 4, hipMemcpyDeviceToDevice, st));
  using LRf = LdRows<float, float, CF::BI, CF::BK, NTF>;
  using LRfj = LdRows<float, float, CF::BJ, CF::BK, NTF>;
  {  // answer_processor.0 + ReLU (attention.py:277-282, 350)
    LRf::Params pa{(const float*)(pk + L.k_W1p), L.ans_ld, 512};
    LRfj::Params pb{Wf(L.ans), L.ans_ld, F};
    EpiStoreT<float> ep{Wf(L.hid1), 512, 512, F, prm + L.poff[A0B], 1};
    HIPCHK((tail_gemm(pa, pb, ep, 512, F, L.ans_ld, st)));
  }
  {  // answer_processor.2
    LRf::Params pa{prm + L.poff[A2W], 512, 256};
    LRfj::Params pb{Wf(L.hid1), 512, F};
    EpiStoreT<float> ep{Wf(L.AO), 256, 256, F, prm + L.poff[A2B], 0};
    HIPCHK((tail_gemm(pa, pb, ep, 256, F, 512, st)));
  }
  {  // policy_core LSTMCell from zero state (attention.py:354-355)
    LRf::Params pa{(const float*)(pk + L.k_Wihp), 256, 1024};
    LRfj::Params pb{Wf(L.AO), 256, F};
    EpiLstmCellFwd ep{(const float*)(pk + L.k_blc), Wf(L.LG), Wf(L.LC), Wf(L.LH), F};
    HIPCHK((tail_gemm(pa, pb, ep, 1024, F, 256, st)));
  }
  }
  TimerScope tim(AAA_TIMER_TAIL_FWD, st, L.sc ? 0.0 : 2.0 * F * 256 * 2 * L.A, "policy/value heads + state out");
  {  // policy / values heads (attention.py:365-367), batched over all frames
    using LRf = LdRows<float, float, CF::BI, CF::BK, NTF>;
    using LRfj = LdRows<float, float, CF::BJ, CF::BK, NTF>;
    LRf::Params pa{(const float*)(pk + L.k_Whd), 256, 2 * L.A};
    LRfj::Params pb{L.sc ? Wf(L.CH) + (size_t)L.B * 256 : Wf(L.LH), 256, F};
    EpiHeads ep{io->logits, io->values, (const float*)(pk + L.k_bhd), L.A, F};
    HIPCHK((tail_gemm(pa, pb, ep, 2 * L.A, F, 256, st)));
  }
  if (io->hT && L.esz == 2)   // h_{T-1} from XH slot T (the bf16 path keeps no fp32 h_t)
    HIPCHK(xh_to_state<__bf16>(M, (const __bf16*)(ws + L.XH) + (size_t)L.T * M * 192, io->hT, st));
  else if (io->hT)
    HIPCHK(hipMemcpyAsync(io->hT, Wf(L.Hs) + (size_t)(L.T - 1) * M * 128, (size_t)M * 128 * 4,
                          hipMemcpyDeviceToDevice, st));
  if (io->cT && (cqm_layout(L) & kCqmC)) HIPCHK(cqm_convert(Wf(L.Cst) + (size_t)L.T * M * 128, io->cT, L.B, P, 0, st));
  else if (io->cT)
    HIPCHK(hipMemcpyAsync(io->cT, Wf(L.Cst) + (size_t)L.T * M * 128, (size_t)M * 128 * 4, hipMemcpyDeviceToDevice, st));
  if (L.sc && io->core_hT)
    HIPCHK(hipMemcpyAsync(io->core_hT, Wf(L.CH) + (size_t)L.T * L.B * 256, (size_t)L.B * 256 * 4,
                          hipMemcpyDeviceToDevice, st));
  if (L.sc && io->core_cT)
    HIPCHK(hipMemcpyAsync(io->core_cT, Wf(L.CC) + (size_t)L.T * L.B * 256, (size_t)L.B * 256 * 4,
                          hipMemcpyDeviceToDevice, st));
  return AAA_OK;
}

template int pack_impl<float>(const Layout&, const float*, char*, hipStream_t);
template int pack_impl<__bf16>(const Layout&, const float*, char*, hipStream_t);
template int vision_fwd<float, float>(const Layout&, int, const char*, const float*, const void*, float*, float*,
                                      float*, int, hipStream_t, bool);
template int vision_fwd<__bf16, __bf16>(const Layout&, int, const char*, const float*, const void*, __bf16*, __bf16*,
                                        __bf16*, int, hipStream_t, bool);
template int vision_fwd<__bf16, float>(const Layout&, int, const char*, const float*, const void*, __bf16*, __bf16*,
                                       float*, int, hipStream_t, bool);
template int forward_impl<float>(const Layout&, const aaa_io*, hipStream_t, int);
template int forward_impl<__bf16>(const Layout&, const aaa_io*, hipStream_t, int);

}  // namespace aaa
