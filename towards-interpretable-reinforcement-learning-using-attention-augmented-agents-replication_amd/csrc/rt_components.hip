// Component entries (include/aaa.h): the ConvLSTM cell, the vision network,
// the attention readout and the small unit-test convs / linear, each one module
// of the reference (attention.py) behind its own C entry.
#include "rt.h"

namespace aaa {

// ------------------------------------------------------ component entries --
// One reference module per entry, on caller-owned buffers,
// through the same kernels aaa_forward / aaa_backward run for that module.

// ConvLSTMCell(64, 128, 3) at one step (attention.py:110-126): packed weights
// (the four ConvLSTM layouts of pack_lstm_all) and the workspace that carries
// the forward's saved activations to the backward.
struct CellLayout {
  int B, h, w, M, dt, esz;
  size_t k_WpX, k_WpH, k_WdTl, k_bl, k_WpXH, packed;
  size_t XH, Cst, Hs, Gt, dZ, dC, dO, dX, gW, gb, ws;
};

static int cell_layout(const aaa_cell_desc* d, CellLayout& C) {
  if (!d) return fail(AAA_E_ARG, "cell desc is NULL");
  if (d->B < 1 || d->h < 1 || d->w < 1) return fail(AAA_E_ARG, "cell: need B, h, w >= 1");
  if (d->dtype != AAA_F32 && d->dtype != AAA_BF16) return fail(AAA_E_ARG, "cell: bad dtype %d", d->dtype);
  const size_t M = (size_t)d->B * d->h * d->w, e = d->dtype == AAA_BF16 ? 2 : 4;
  if (M * 512 * 4 >= (size_t(1) << 31))   // dZ / gates: buffer descriptors and int indices
    return fail(AAA_E_ARG, "cell: B*h*w = %zu pixels is above the 2 GiB descriptor range; split the batch", M);
  C.B = d->B; C.h = d->h; C.w = d->w; C.M = (int)M; C.dt = d->dtype; C.esz = (int)e;
  size_t p = 0;
  auto take = [&](size_t bytes) { size_t r = p; p = al256(p + bytes); return r; };
  C.k_WpX = take(512 * 576 * e);
  C.k_WpH = take(512 * 1152 * e);
  C.k_WdTl = take(192 * 4608 * e);
  C.k_bl = take(512 * 4);
  C.k_WpXH = take(512 * 1728 * e);
  C.packed = p;
  p = 0;
  C.XH = take(2 * M * 192 * e);
  C.Cst = take(2 * M * 128 * 4);
  C.Hs = take(M * 128 * 4);
  C.Gt = take(M * 512 * 4);
  C.dZ = take(M * 512 * e);
  C.dC = take(M * 128 * 4);
  C.dO = take(M * 128 * 4);
  C.dX = take(M * 64 * 4);
  C.gW = take(512 * 1728 * 4);
  C.gb = take(512 * 4);
  C.ws = p;
  return AAA_OK;
}

// the cell's 12 state_dict tensors, concatenated in state_dict order
// (Wx{g}.weight (128,64,3,3), Wx{g}.bias (128), Wh{g}.weight (128,128,3,3) for g = i, f, c, o)
constexpr size_t kCellGate = 128 * 64 * 9 + 128 + 128 * 128 * 9;
template <typename P, typename Ptrs>
static void cell_ptrs(P* base, Ptrs& lp) {
  for (int g = 0; g < 4; ++g) {
    lp.wx[g] = base + g * kCellGate;
    lp.bx[g] = base + g * kCellGate + 128 * 64 * 9;
    lp.wh[g] = base + g * kCellGate + 128 * 64 * 9 + 128;
  }
}

template <typename T>
static int cell_fwd_impl(const CellLayout& C, const char* pk, const float* x, const float* h0, const float* c0,
                         float* h1, float* c1, char* ws, hipStream_t st) {
  const int M = C.M;
  T* xh = (T*)(ws + C.XH);
  float* cst = (float*)(ws + C.Cst);
  HIPCHK(cell_xh<T>(M, x, h0, xh, st));
  if (c0) HIPCHK(hipMemcpyAsync(cst, c0, (size_t)M * 128 * 4, hipMemcpyDeviceToDevice, st));
  else HIPCHK(hipMemsetAsync(cst, 0, (size_t)M * 128 * 4, st));
  auto run = [&](auto gtag) -> int {
    using GT = decltype(gtag);
    EpiConvLstmFwd<T, GT> ep{cst, cst + (size_t)M * 128, (float*)(ws + C.Hs), xh + (size_t)M * 192,
                             (GT*)(ws + C.Gt), M, (const float*)(pk + C.k_bl)};
    return fused_step<T, GT>((const T*)(pk + C.k_WpXH), xh, C.h, C.w, M, ep, st);
  };
  const int rc = gates_f16(C.dt, M) ? run(_Float16{}) : run(float{});
  if (rc) return rc;
  if (h1) HIPCHK(hipMemcpyAsync(h1, ws + C.Hs, (size_t)M * 128 * 4, hipMemcpyDeviceToDevice, st));
  if (c1) HIPCHK(hipMemcpyAsync(c1, cst + (size_t)M * 128, (size_t)M * 128 * 4, hipMemcpyDeviceToDevice, st));
  return AAA_OK;
}

template <typename T>
static int cell_bwd_impl(const CellLayout& C, const char* pk, const float* dh1, const float* dc1, float* dx,
                         float* dh0, float* dc0, float* grads, char* ws, hipStream_t st) {
  const int M = C.M;
  const T* xh = (const T*)(ws + C.XH);
  const float* cst = (const float*)(ws + C.Cst);
  float* dC = (float*)(ws + C.dC);
  T* dZ = (T*)(ws + C.dZ);
  if (dc1) HIPCHK(hipMemcpyAsync(dC, dc1, (size_t)M * 128 * 4, hipMemcpyDeviceToDevice, st));
  else HIPCHK(hipMemsetAsync(dC, 0, (size_t)M * 128 * 4, st));
  const float* dh = dh1;
  if (!dh) {
    HIPCHK(hipMemsetAsync(ws + C.dO, 0, (size_t)M * 128 * 4, st));
    dh = (const float*)(ws + C.dO);
  }
  auto run = [&](auto gtag) -> int {
    using GT = decltype(gtag);
    // gate backward (dz of the four gates, dc carry -> dc0)
    HIPCHK((gate_bwd_last<T, GT>(M, 64, dh, nullptr, (const GT*)(ws + C.Gt), cst, cst + (size_t)M * 128, dC, dZ,
                                 nullptr, st)));
    // [dx | dh0] = W^T dz: the dgrad of all eight gate convs into [x | h] in one GEMM
    EpiConvLstmBwd<T, GT> ep{dx ? dx : (float*)(ws + C.dX), nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                             dh0, 0, M, 0, nullptr};
    const ConvGeo g = ConvGeo{512, 512, 0, C.h, C.w, C.h, C.w, 3, 1, 1, 1}.prep();
    HIPCHK((step_gemm<CfgFor<T>, false>((const T*)(pk + C.k_WdTl), 4608, 192, (const T*)dZ, g, M,
                                         (uint32_t)((size_t)M * 512 * C.esz), ep, 192, 4608, st)));
    return AAA_OK;
  };
  int rc = gates_f16(C.dt, M) ? run(_Float16{}) : run(float{});
  if (rc) return rc;
  if (dc0) HIPCHK(hipMemcpyAsync(dc0, dC, (size_t)M * 128 * 4, hipMemcpyDeviceToDevice, st));
  if (grads) {   // weight grads (all 8 convs, one GEMM over the pixels) and the gate biases
    float* gW = (float*)(ws + C.gW);
    float* gb = (float*)(ws + C.gb);
    HIPCHK(hipMemsetAsync(gW, 0, (size_t)512 * 1728 * 4, st));
    HIPCHK(hipMemsetAsync(gb, 0, 512 * 4, st));
    if ((rc = lstm_wgrad<T>(dZ, xh, M, C.h, C.w, gW, st, false))) return rc;
    HIPCHK(colsum<T>(dZ, 512, M, 512, gb, st));
    LstmGrads lg;
    cell_ptrs(grads, lg);
    HIPCHK(unpack_lstm(gW, gb, lg, st));
  }
  return AAA_OK;
}

// VisionNetwork.vision_cnn over N frames: a Layout with B = N, T = 1 gives the
// geometry and the packed-weight offsets (the conv weights are the first three
// packed layouts, the vision params the first four state_dict tensors).
struct CnnLayout {
  Layout L;
  size_t Xp, Y1, dY2, dY1, gW1, gW2, ws;
};

static int cnn_layout(const aaa_cnn_desc* d, CnnLayout& C) {
  if (!d) return fail(AAA_E_ARG, "cnn desc is NULL");
  if (d->N < 1) return fail(AAA_E_ARG, "cnn: need N >= 1");
  const aaa_cfg cfg{d->N, 1, d->H, d->W, 4, 18, d->dtype, 0};
  int r = build_layout(&cfg, C.L, 1);
  if (r) return r;
  const Layout& L = C.L;
  const size_t F = L.F, e = L.esz;
  size_t p = 0;
  auto take = [&](size_t bytes) { size_t q = p; p = al256(p + bytes); return q; };
  C.Xp = take(F * (L.H + 2) * (L.W + 2) * 4 * e);
  C.Y1 = take(F * L.P1 * 32 * e);
  C.dY2 = take(F * L.P * 64 * e);
  C.dY1 = take(F * L.P1 * 32 * e);
  C.gW1 = take(32 * 256 * 4);
  C.gW2 = take(64 * 512 * 4);
  C.ws = p;
  return AAA_OK;
}

template <typename T>
static int cnn_pack_impl(const Layout& L, const float* prm, char* pk, hipStream_t st) {
  HIPCHK(pack_conv1_rgbx<T>(prm + L.poff[C0W], (T*)(pk + L.k_Wp1), st));
  HIPCHK(pack_conv<T>(prm + L.poff[C1W], 64, 32, 4, (T*)(pk + L.k_Wp2), st));
  HIPCHK(pack_conv2_classes<T>(prm + L.poff[C1W], (T*)(pk + L.k_WdT2), st));
  return AAA_OK;
}

template <typename T>
static int cnn_bwd_impl(const CnnLayout& CL, const char* pk, const float* dy2, float* dy1, float* grads, char* ws,
                        hipStream_t st) {
  const Layout& L = CL.L;
  const int N = L.F;
  const T* dy2t;
  if constexpr (std::is_same<T, float>::value) {
    dy2t = dy2;
  } else {
    HIPCHK((cast<float, T>((long)N * L.P * 64, dy2, (T*)(ws + CL.dY2), st)));
    dy2t = (const T*)(ws + CL.dY2);
  }
  float* gW1 = (float*)(ws + CL.gW1);
  float* gW2 = (float*)(ws + CL.gW2);
  T* dY1 = (T*)(ws + CL.dY1);
  HIPCHK(hipMemsetAsync(grads, 0, L.poff[XI_W] * 4, st));
  HIPCHK(hipMemsetAsync(gW1, 0, 32 * 256 * 4, st));
  HIPCHK(hipMemsetAsync(gW2, 0, 64 * 512 * 4, st));
  HIPCHK(colsum<float>(dy2, 64, N * L.P, 64, grads + L.poff[C1B], st));   // conv2 bias (fp32 grads)
  const int rc = vision_bwd<T>(L, pk, dy2t, (const T*)(ws + CL.Y1), (T*)(ws + CL.Xp), dY1, N, gW2, gW1,
                               grads + L.poff[C0B], st);
  if (rc) return rc;
  if (std::is_same<T, float>::value && !ab_int("AAA_CONV2_DGRAD_RING", 1))
    HIPCHK(colsum(dY1, 32, N * L.P1, 32, grads + L.poff[C0B], st));
  HIPCHK(unpack_conv(gW2, 64, 32, 4, grads + L.poff[C1W], st));
  HIPCHK(unpack_conv1_rgbx(gW1, grads + L.poff[C0W], st));
  if (dy1) HIPCHK((cast<T, float>((long)N * L.P1 * 32, dY1, dy1, st)));
  return AAA_OK;
}

// ----------------------------------------------------- unit-test entries --
template <typename T>
static int conv_nhwc_impl(const aaa_conv_desc* d, const float* x, const float* w, const float* bias, float* y,
                          hipStream_t st) {
  using C = CfgFor<T>;
  constexpr int NT = C::NT;
  const int K = d->KH * d->KW * d->Cin, M = d->N * d->Hout * d->Wout;
  using LA = LdRows<float, T, C::BI, C::BK, NT>;
  typename LA::Params pa{w, K, d->Cout};
  const ConvGeo g = ConvGeo{d->Cin, d->Cin, 0, d->Hin, d->Win, d->Hout, d->Wout, d->KW, d->stride, d->pad, 0}.prep();
  EpiStoreT<float> ep{y, d->Cout, d->Cout, M, bias, 0};
  const int tpt = C::BK / std::max(1, d->Cin);
  if (d->Cin % C::BK == 0 || (C::BK % d->Cin == 0 && (tpt % d->KW == 0 || d->KW % tpt == 0))) {   // hot-path loaders
    using LAB = LdRowsB<float, T, C::BI, C::BK, NT>;
    using LB = LdIm2colB<float, T, C::BJ, C::BK, NT>;
    const uint32_t xb = (uint32_t)((size_t)d->N * d->Hin * d->Win * d->Cin * 4);
    HIPCHK((launch_gemm<C, LAB, LB>(typename LAB::Params{w, K, d->Cout}, typename LB::Params{x, g, M, xb}, ep, d->Cout,
                                    M, K, 1, st)));
  } else if (d->Cin % 4 == 0) {
    using LB = LdIm2col<float, T, C::BJ, C::BK, NT, true>;
    HIPCHK((launch_gemm<C, LA, LB>(pa, typename LB::Params{x, g, M}, ep, d->Cout, M, K, 1, st)));
  } else {
    using LB = LdIm2col<float, T, C::BJ, C::BK, NT, false>;
    HIPCHK((launch_gemm<C, LA, LB>(pa, typename LB::Params{x, g, M}, ep, d->Cout, M, K, 1, st)));
  }
  return AAA_OK;
}

template <typename T>
static int dgrad_nhwc_impl(const aaa_conv_desc* d, const float* dy, const float* wT, float* dx, hipStream_t st) {
  using C = CfgFor<T>;
  constexpr int NT = C::NT;
  const int K = d->KH * d->KW * d->Cout, M = d->N * d->Hin * d->Win;
  using LA = LdRows<float, T, C::BI, C::BK, NT>;
  using LB = LdIm2col<float, T, C::BJ, C::BK, NT, true>;
  typename LA::Params pa{wT, K, d->Cin};
  const ConvGeo g = ConvGeo{d->Cout, d->Cout, 0, d->Hout, d->Wout, d->Hin, d->Win, d->KW, d->stride, d->pad, 1}.prep();
  EpiStoreT<float> ep{dx, d->Cin, d->Cin, M, nullptr, 0};
  if (d->stride == 1 && d->Cout % C::BK == 0) {
    using LAB = LdRowsB<float, T, C::BI, C::BK, NT>;
    using LBB = LdIm2colB<float, T, C::BJ, C::BK, NT>;
    const uint32_t yb = (uint32_t)((size_t)d->N * d->Hout * d->Wout * d->Cout * 4);
    HIPCHK((launch_gemm<C, LAB, LBB>(typename LAB::Params{wT, K, d->Cin}, typename LBB::Params{dy, g, M, yb}, ep,
                                     d->Cin, M, K, 1, st)));
    return AAA_OK;
  }
  HIPCHK((launch_gemm<C, LA, LB>(pa, typename LB::Params{dy, g, M}, ep, d->Cin, M, K, 1, st)));
  return AAA_OK;
}

template <typename T>
static int wgrad_nhwc_impl(const aaa_conv_desc* d, const float* x, const float* dy, float* dw, hipStream_t st) {
  using C = CfgFor<T>;
  constexpr int NT = C::NT;
  const int Kp = d->KH * d->KW * d->Cin, M = d->N * d->Hout * d->Wout;
  HIPCHK(hipMemsetAsync(dw, 0, (size_t)d->Cout * Kp * 4, st));
  using LA = LdRowsT<float, T, C::BI, C::BK, NT>;
  typename LA::Params pa{dy, d->Cout, d->Cout};
  const ConvGeo g = ConvGeo{d->Cin, d->Cin, 0, d->Hin, d->Win, d->Hout, d->Wout, d->KW, d->stride, d->pad, 0}.prep();
  EpiStore<true> ep{dw, Kp, d->Cout, Kp};
  const int tiles = cdiv(d->Cout, C::BI) * cdiv(Kp, C::BJ);
  const int ns = wgrad_splits(tiles, M, C::BK);
  if (d->Cin % 4 == 0 && d->Cout % 4 == 0) {   // hot-path loaders
    using LAB = LdRowsTB<float, T, C::BI, C::BK, NT>;
    using LB = LdIm2colTB<float, T, C::BJ, C::BK, NT>;
    const uint32_t xb = (uint32_t)((size_t)d->N * d->Hin * d->Win * d->Cin * 4);
    HIPCHK((launch_gemm<C, LAB, LB>(typename LAB::Params{dy, d->Cout, d->Cout, M}, typename LB::Params{x, g, Kp, xb},
                                    ep, d->Cout, Kp, M, ns, st)));
  } else if (d->Cin % 4 == 0) {
    using LB = LdIm2colT<float, T, C::BJ, C::BK, NT, true>;
    HIPCHK((launch_gemm<C, LA, LB>(pa, typename LB::Params{x, g, Kp}, ep, d->Cout, Kp, M, ns, st)));
  } else {
    using LB = LdIm2colT<float, T, C::BJ, C::BK, NT, false>;
    HIPCHK((launch_gemm<C, LA, LB>(pa, typename LB::Params{x, g, Kp}, ep, d->Cout, Kp, M, ns, st)));
  }
  return AAA_OK;
}


}  // namespace aaa

using namespace aaa;

extern "C" {

static int check_conv(const aaa_conv_desc* d) {
  if (!d) return fail(AAA_E_ARG, "NULL desc");
  if (d->N < 1 || d->Cin < 1 || d->Cout < 1 || d->KH != d->KW || d->stride < 1 || d->pad < 0)
    return fail(AAA_E_ARG, "bad conv desc");
  if (d->Hout != conv_out(d->Hin, d->KH, d->stride, d->pad) || d->Wout != conv_out(d->Win, d->KW, d->stride, d->pad))
    return fail(AAA_E_ARG, "Hout/Wout inconsistent with Hin/Win/K/stride/pad");
  if ((d->KH * d->KW * d->Cin) % 4 || d->Cout % 4) return fail(AAA_E_ARG, "KH*KW*Cin and Cout must be multiples of 4");
  // buffer descriptors span the whole input / output gradient (32-bit byte offsets, kOOB = 2^31)
  const size_t lim = size_t(1) << 31;
  if ((size_t)d->N * d->Hin * d->Win * d->Cin * 4 >= lim || (size_t)d->N * d->Hout * d->Wout * d->Cout * 4 >= lim)
    return fail(AAA_E_ARG, "conv tensors must stay below 2 GiB (split N)");
  return check_device();
}

int aaa_conv2d_nhwc(const aaa_conv_desc* d, const float* x, const float* w, const float* bias, float* y,
                    hipStream_t stream) {
  int r = check_conv(d);
  if (r) return r;
  return d->dtype == AAA_BF16 ? conv_nhwc_impl<__bf16>(d, x, w, bias, y, stream)
                              : conv_nhwc_impl<float>(d, x, w, bias, y, stream);
}

int aaa_conv2d_nhwc_dgrad(const aaa_conv_desc* d, const float* dy, const float* wT, float* dx, hipStream_t stream) {
  int r = check_conv(d);
  if (r) return r;
  if (d->Cout % 4) return fail(AAA_E_ARG, "Cout must be a multiple of 4");
  return d->dtype == AAA_BF16 ? dgrad_nhwc_impl<__bf16>(d, dy, wT, dx, stream)
                              : dgrad_nhwc_impl<float>(d, dy, wT, dx, stream);
}

int aaa_conv2d_nhwc_wgrad(const aaa_conv_desc* d, const float* x, const float* dy, float* dw, hipStream_t stream) {
  int r = check_conv(d);
  if (r) return r;
  return d->dtype == AAA_BF16 ? wgrad_nhwc_impl<__bf16>(d, x, dy, dw, stream)
                              : wgrad_nhwc_impl<float>(d, x, dy, dw, stream);
}

// ---- component entries (include/aaa.h) ----
size_t aaa_convlstm_packed_bytes(const aaa_cell_desc* d) {
  CellLayout C;
  return cell_layout(d, C) ? 0 : C.packed;
}

size_t aaa_convlstm_workspace_bytes(const aaa_cell_desc* d) {
  CellLayout C;
  return cell_layout(d, C) ? 0 : C.ws;
}

int aaa_convlstm_pack(const aaa_cell_desc* d, const float* cell_params, void* packed, hipStream_t stream) {
  CellLayout C;
  int r = cell_layout(d, C);
  if (r) return r;
  if ((r = check_device())) return r;
  if (!cell_params || !packed) return fail(AAA_E_ARG, "convlstm_pack: NULL argument");
  if (!aligned16(packed)) return fail(AAA_E_ALIGN, "packed must be 16-byte aligned");
  LstmPtrs lp;
  cell_ptrs(cell_params, lp);
  char* pk = (char*)packed;
  if (C.dt == AAA_BF16)
    HIPCHK(pack_lstm_all<__bf16>(lp, (__bf16*)(pk + C.k_WpX), (__bf16*)(pk + C.k_WpH), (__bf16*)(pk + C.k_WdTl),
                                 (float*)(pk + C.k_bl), (__bf16*)(pk + C.k_WpXH), stream));
  else
    HIPCHK(pack_lstm_all<float>(lp, (float*)(pk + C.k_WpX), (float*)(pk + C.k_WpH), (float*)(pk + C.k_WdTl),
                                (float*)(pk + C.k_bl), (float*)(pk + C.k_WpXH), stream));
  return AAA_OK;
}

int aaa_convlstm_cell_fwd(const aaa_cell_desc* d, const void* packed, const float* x, const float* h0,
                          const float* c0, float* h1, float* c1, void* workspace, hipStream_t stream) {
  CellLayout C;
  int r = cell_layout(d, C);
  if (r) return r;
  if ((r = check_device())) return r;
  if (!packed || !x || !workspace) return fail(AAA_E_ARG, "convlstm_cell_fwd: packed/x/workspace must be set");
  const void* ptrs[] = {packed, x, h0, c0, h1, c1, workspace};
  for (const void* p : ptrs)
    if (p && !aligned16(p)) return fail(AAA_E_ALIGN, "buffers must be 16-byte aligned");
  return C.dt == AAA_BF16 ? cell_fwd_impl<__bf16>(C, (const char*)packed, x, h0, c0, h1, c1, (char*)workspace, stream)
                          : cell_fwd_impl<float>(C, (const char*)packed, x, h0, c0, h1, c1, (char*)workspace, stream);
}

int aaa_convlstm_cell_bwd(const aaa_cell_desc* d, const void* packed, const float* dh1, const float* dc1, float* dx,
                          float* dh0, float* dc0, float* cell_grads, void* workspace, hipStream_t stream) {
  CellLayout C;
  int r = cell_layout(d, C);
  if (r) return r;
  if ((r = check_device())) return r;
  if (!packed || !workspace) return fail(AAA_E_ARG, "convlstm_cell_bwd: packed/workspace must be set");
  const void* ptrs[] = {packed, dh1, dc1, dx, dh0, dc0, cell_grads, workspace};
  for (const void* p : ptrs)
    if (p && !aligned16(p)) return fail(AAA_E_ALIGN, "buffers must be 16-byte aligned");
  return C.dt == AAA_BF16
             ? cell_bwd_impl<__bf16>(C, (const char*)packed, dh1, dc1, dx, dh0, dc0, cell_grads, (char*)workspace, stream)
             : cell_bwd_impl<float>(C, (const char*)packed, dh1, dc1, dx, dh0, dc0, cell_grads, (char*)workspace, stream);
}

size_t aaa_vision_cnn_packed_bytes(const aaa_cnn_desc* d) {
  CnnLayout C;
  return cnn_layout(d, C) ? 0 : C.L.k_WpX;   // the first three packed layouts
}

size_t aaa_vision_cnn_workspace_bytes(const aaa_cnn_desc* d) {
  CnnLayout C;
  return cnn_layout(d, C) ? 0 : C.ws;
}

int aaa_vision_cnn_pack(const aaa_cnn_desc* d, const float* cnn_params, void* packed, hipStream_t stream) {
  CnnLayout C;
  int r = cnn_layout(d, C);
  if (r) return r;
  if ((r = check_device())) return r;
  if (!cnn_params || !packed) return fail(AAA_E_ARG, "vision_cnn_pack: NULL argument");
  if (!aligned16(packed)) return fail(AAA_E_ALIGN, "packed must be 16-byte aligned");
  return C.L.dt == AAA_BF16 ? cnn_pack_impl<__bf16>(C.L, cnn_params, (char*)packed, stream)
                            : cnn_pack_impl<float>(C.L, cnn_params, (char*)packed, stream);
}

int aaa_vision_cnn_fwd(const aaa_cnn_desc* d, const float* cnn_params, const void* packed, const float* frames,
                       float* y1, float* y2, void* workspace, hipStream_t stream) {
  CnnLayout C;
  int r = cnn_layout(d, C);
  if (r) return r;
  if ((r = check_device())) return r;
  if (!cnn_params || !packed || !frames || !y2 || !workspace)
    return fail(AAA_E_ARG, "vision_cnn_fwd: cnn_params/packed/frames/y2/workspace must be set");
  const void* ptrs[] = {packed, frames, y1, y2, workspace};
  for (const void* p : ptrs)
    if (p && !aligned16(p)) return fail(AAA_E_ALIGN, "buffers must be 16-byte aligned");
  const Layout& L = C.L;
  char* ws = (char*)workspace;
  auto run = [&](auto tag) -> int {
    using T = decltype(tag);
    int rc = vision_fwd<T, float>(L, L.F, (const char*)packed, cnn_params, frames, (T*)(ws + C.Xp), (T*)(ws + C.Y1),
                                  y2, 64, stream);
    if (rc) return rc;
    if (y1) HIPCHK((cast<T, float>((long)L.F * L.P1 * 32, (const T*)(ws + C.Y1), y1, stream)));
    return AAA_OK;
  };
  return L.dt == AAA_BF16 ? run(__bf16{}) : run(float{});
}

int aaa_vision_cnn_bwd(const aaa_cnn_desc* d, const void* packed, const float* dy2, float* dy1, float* cnn_grads,
                       void* workspace, hipStream_t stream) {
  CnnLayout C;
  int r = cnn_layout(d, C);
  if (r) return r;
  if ((r = check_device())) return r;
  if (!packed || !dy2 || !cnn_grads || !workspace)
    return fail(AAA_E_ARG, "vision_cnn_bwd: packed/dy2/cnn_grads/workspace must be set");
  const void* ptrs[] = {packed, dy2, dy1, cnn_grads, workspace};
  for (const void* p : ptrs)
    if (p && !aligned16(p)) return fail(AAA_E_ALIGN, "buffers must be 16-byte aligned");
  return C.L.dt == AAA_BF16
             ? cnn_bwd_impl<__bf16>(C, (const char*)packed, dy2, dy1, cnn_grads, (char*)workspace, stream)
             : cnn_bwd_impl<float>(C, (const char*)packed, dy2, dy1, cnn_grads, (char*)workspace, stream);
}

static int check_attn(int F, int h, int w, int nq, int q_stride) {
  if (F < 1 || h < 1 || w < 1) return fail(AAA_E_ARG, "attn: need F, h, w >= 1");
  if (nq != 4 && nq != 8) return fail(AAA_E_ARG, "attn: nq must be 4 or 8 (got %d)", nq);
  if (q_stride != 0 && q_stride != nq * 72) return fail(AAA_E_ARG, "attn: q_stride must be 0 or nq*72");
  if ((size_t)F * h * w * 128 >= (size_t(1) << 31)) return fail(AAA_E_ARG, "attn: F*h*w too large; split F");
  return check_device();
}

int aaa_attn_fwd(int F, int h, int w, int nq, const float* O, const float* S, const float* Q, int q_stride,
                 const float* prev_reward, const float* prev_action, float* attn, float* answer, hipStream_t stream) {
  int r = check_attn(F, h, w, nq, q_stride);
  if (r) return r;
  if (!O || !S || !Q || !attn || !answer) return fail(AAA_E_ARG, "attn_fwd: O/S/Q/attn/answer must be set");
  if (!aligned16(O) || !aligned16(S)) return fail(AAA_E_ALIGN, "O and S must be 16-byte aligned");
  TimerScope tim(AAA_TIMER_ATTN_FWD, stream, (double)F * attn_fwd_bytes(h * w, nq, 256 * nq + 2), "k_attn_fwd (aaa_attn_fwd)");
  HIPCHK(attn_fwd(o_f32(O), S, Q, nullptr, prev_reward, prev_action, F, h * w, nq, attn, answer, 256 * nq + 2, stream,
                  q_stride));
  return AAA_OK;
}

int aaa_attn_bwd(int F, int h, int w, int nq, const float* O, const float* S, const float* Q, int q_stride,
                 const float* attn, const float* danswer, float* dO, float* dQ, hipStream_t stream) {
  int r = check_attn(F, h, w, nq, q_stride);
  if (r) return r;
  if (!O || !S || !Q || !attn || !danswer || !dO || !dQ)
    return fail(AAA_E_ARG, "attn_bwd: O/S/Q/attn/danswer/dO/dQ must be set");
  if (!aligned16(O) || !aligned16(S) || !aligned16(dO)) return fail(AAA_E_ALIGN, "O, S, dO must be 16-byte aligned");
  TimerScope tim(AAA_TIMER_ATTN_BWD, stream, (double)F * attn_bwd_bytes(h * w, nq), "k_attn_bwd (aaa_attn_bwd)");
  HIPCHK(attn_bwd(o_f32(O), S, Q, attn, danswer, 256 * nq + 2, F, h * w, nq, dO, dQ, stream, q_stride, 1));
  return AAA_OK;
}

int aaa_linear(int M, int N, int K, const float* x, const float* w, const float* bias, float* y,
               hipStream_t stream) {
  if (M < 1 || N < 1 || K < 1 || K % 4) return fail(AAA_E_ARG, "linear: need M,N,K >= 1 and K %% 4 == 0");
  int r = check_device();
  if (r) return r;
  using LA = LdRows<float, float, CF::BI, CF::BK, CF::NT>;
  using LB = LdRows<float, float, CF::BJ, CF::BK, CF::NT>;
  EpiStoreT<float> ep{y, N, N, M, bias, 0};
  HIPCHK((launch_gemm<CF, LA, LB>(LA::Params{w, K, N}, LB::Params{x, K, M}, ep, N, M, K, 1, stream)));
  return AAA_OK;
}

}  // extern "C"
