#pragma once
#include "common.h"
#include "epilogues.h"

namespace aaa {

struct LstmPtrs {
  const float* wx[4];  // Wx{i,f,c,o}.weight (128,64,3,3)
  const float* bx[4];  // Wx{i,f,c,o}.bias   (128)
  const float* wh[4];  // Wh{i,f,c,o}.weight (128,128,3,3)
};
struct LstmGrads {
  float* wx[4];
  float* bx[4];
  float* wh[4];
};
struct F32Pack {
  const float *a0w, *wih, *bih, *bhh, *pw, *vw, *pb, *vb;
  float *W1p, *Wihp, *blc, *Whd, *bhd;
  int ans_in, ans_ld, A, ldy;
  const float* whh = nullptr;   // stateful core: also pack [W_ih | W_hh] into Wihhp
  float* Wihhp = nullptr;
};
struct F32Unpack {
  const float *gW1p, *gWihp, *gblc, *gWhd, *gbhd;
  float *a0w, *wih, *bih, *bhh, *pw, *vw, *pb, *vb;
  int ans_in, ans_ld, A;
  const float* gWihhp = nullptr;   // stateful core: W_ih and W_hh grads from [1024][512]
  float* whh = nullptr;
};

// aaa_pack_weights' param-only layouts in one launch (misc.hip k_pack_all)
template <typename T>
struct PackAll {
  const float *c1w, *c2w;
  T *Wp1, *Wp2, *WdT2;
  LstmPtrs lstm;
  T *WpX, *WpH, *WdT, *WpXH;
  float* bl;
  F32Pack f32;
};
template <typename T> hipError_t pack_all(const PackAll<T>& a, hipStream_t st);

hipError_t query_pack(const float* b0, const float* W2, const float* b2, const float* W4, const float* b4, int nq,
                      float* q1, float* q2, float* Q, hipStream_t st);
hipError_t query_sq(const float* S, const float* Q, int P, int nq, float* SQ, hipStream_t st);
// qs: per-frame query stride in floats (0 = one query for all frames, Q1);
// SQ == NULL computes the basis half of the logits per frame.  addq adds the
// answer row's Q-column gradient (dAns[f][184*nq ...]) into dQp.
//
// OSrc: h_t (the readout's O, frame rows of P pixels) as the readout reads it:
// fp32 rows of 128 (Hs, the fp32 path) or the bf16 h half of the ConvLSTM's
// [x | h] operand rows (XH, row pitch 192: the bf16 path keeps no fp32 copy).
struct OSrc {
  const void* p;
  int bf16, ld;   // element type, row pitch in elements
  OSrc frame(size_t f, int P) const {   // frame f's rows
    return {(const char*)p + f * P * ld * (bf16 ? 2 : 4), bf16, ld};
  }
};
inline OSrc o_f32(const float* Hs) { return {Hs, 0, 128}; }
inline OSrc o_bf16(const __bf16* h, int ld) { return {h, 1, ld}; }
hipError_t attn_fwd(OSrc O, const float* S, const float* Q, const float* SQ, const float* pr,
                    const float* pa, int F, int P, int nq, float* Am, float* ans, int ans_ld, hipStream_t st,
                    int qs = 0);
// cqm: write dO in the channel-quad-major per-frame layout of the frame-resident BPTT (recur.h cqm4)
hipError_t attn_bwd(OSrc O, const float* S, const float* Q, const float* Am, const float* dAns,
                    int da_ld, int F, int P, int nq, float* dO, float* dQp, hipStream_t st, int qs = 0,
                    int addq = 0, int cqm = 0);
// (nf, P, 128) fp32 slices: row-major -> channel-quad-major (to_cqm) or back
hipError_t cqm_convert(const float* src, float* dst, int nf, int P, int to_cqm, hipStream_t st);
hipError_t query_bwd(const float* dQs, const float* gb1, const float* W1, int ans_in, int nq, const float* W2,
                     const float* W4, const float* q1, const float* q2, float* gW4, float* gb4, float* gW2,
                     float* gb2, float* gb0, hipStream_t st);
struct ColSumSeg {
  const float* X;
  int ld, N;
  float* out;   // out[n] += sum over the M rows of X[m*ld + n]
};
struct ColSums {
  ColSumSeg s[6];
  int n = 0;
  int cb[7];    // column-block prefix (filled by colsum_multi)
  void add(const float* X, int ld, int N, float* out) { s[n++] = ColSumSeg{X, ld, N, out}; }
};
hipError_t colsum_multi(ColSums c, int M, hipStream_t st);
template <typename TI> hipError_t colsum(const TI* X, int ld, int M, int N, float* out, hipStream_t st);
template <typename TZ, typename GT>
hipError_t gate_bwd_last(int M, int bj, const float* dO, const float* dhT, const GT* gates, const float* cprev,
                         const float* ccur, float* dC, TZ* dz, float* part, hipStream_t st, int nsl = 1,
                         size_t sls = 0);
hipError_t concat_dy(int F, int A, int ldy, const float* dl, const float* dv, float* dY, hipStream_t st);
// The tiny fills of a phase's start in ONE launch (each launch costs ~5 us on the stream however
// little it does): up to 4 zeroed fp32 ranges, then optionally XH slot 0's h channels <- h0 (or 0)
// (xh != nullptr) and the cotangent concat dY <- [dlogits | dvalues | 0] (dY != nullptr)
struct ZeroRanges {
  float* p[4];
  long n[4];   // floats
  int cnt;
  void add(float* q, long m) {
    if (q && m > 0) { p[cnt] = q; n[cnt] = m; ++cnt; }
  }
};
template <typename T>
hipError_t prologue(const ZeroRanges& z, int M, const float* h0, T* xh, int F, int A, int ldy, const float* dl,
                    const float* dv, float* dY, hipStream_t st);
template <typename T> hipError_t state_to_xh(int M, const float* h0, T* xh, hipStream_t st);
template <typename T> hipError_t xh_to_state(int M, const T* xh, float* h, hipStream_t st);
template <typename T> hipError_t cell_xh(int M, const float* x, const float* h, T* xh, hipStream_t st);
template <typename TI, typename TO> hipError_t cast(long n, const TI* src, TO* dst, hipStream_t st);
template <typename T> hipError_t pack_conv(const float* w, int Cout, int Cin, int K, T* dst, hipStream_t st);
template <typename T>
hipError_t pack_lstm_all(const LstmPtrs& L, T* WpX, T* WpH, T* WdT, float* bl, T* WpXH, hipStream_t st);
template <typename T>
hipError_t gate_fwd_zx(int M, const float* cprev, float* gates, float* cnext, float* hout, T* xhnext, hipStream_t st,
                       const float* zs = nullptr, int nsl = 0, size_t sls = 0, const float* bias = nullptr);
hipError_t pack_f32(const F32Pack& p, hipStream_t st);
// Channel-chunk-major copy of conv-GEMM rows (ConvGeo::cmaj): row r's K = taps x Cin
// (tap-major) -> dst[r][(c / BK) * taps * BK + tap * BK + c % BK]
hipError_t reorder_cmaj(const float* src, int rows, int Cin, int taps, int BK, float* dst, hipStream_t st);
// fp32 -> three bf16 planes (hi, mid, lo; gemm.h split3_bf16's split): dst[p * n + i]
hipError_t split_planes(const float* src, long n, __bf16* dst, hipStream_t st);
template <typename T, typename TI> hipError_t frames_rgbx(int F, int H, int W, const TI* x, T* y, hipStream_t st);
template <typename T> hipError_t pack_conv2_classes(const float* w2, T* dst, hipStream_t st);
template <typename T> hipError_t pack_conv1_rgbx(const float* w, T* dst, hipStream_t st);
hipError_t unpack_conv1_rgbx(const float* g, float* dst, hipStream_t st);
hipError_t unpack_conv(const float* g, int Cout, int Cin, int K, float* dst, hipStream_t st);
hipError_t unpack_lstm(const float* gW, const float* gb, const LstmGrads& L, hipStream_t st);
hipError_t unpack_f32(const F32Unpack& p, hipStream_t st);
// ConvLSTM grads (gW == null: none) + conv2 + conv1 weight grads, one launch
hipError_t unpack_cv(const float* gW, const float* gb, const LstmGrads& L, const float* g2, float* d2, const float* g1,
                     float* d1, hipStream_t st);

}  // namespace aaa
