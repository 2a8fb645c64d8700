// GEMM epilogues.  Each is called once per (4 consecutive rows i..i+3, column j)
// of the D tile with the fp32 accumulators; it owns its bounds checks.
#pragma once
#include <type_traits>
#include "common.h"

namespace aaa {

__device__ __forceinline__ void store4(float* p, float a, float b, float c, float d) {
  *reinterpret_cast<f32x4*>(p) = f32x4{a, b, c, d};
}
__device__ __forceinline__ void store4(__bf16* p, float a, float b, float c, float d) {
  *reinterpret_cast<bf16x4*>(p) = bf16x4{(__bf16)a, (__bf16)b, (__bf16)c, (__bf16)d};
}

// out[j*ld + i + e] = v[e] (+ bias[i+e]) (relu?)  -- D stored transposed, e.g.
// a conv output [pixel][channel] or a linear output [row][feature].
template <typename OT>
struct EpiStoreT {
  OT* out;
  int ld, Mi, Nj;
  const float* bias;
  int relu;
  __device__ __forceinline__ void operator()(int i, int j, float v0, float v1, float v2, float v3) const {
    if (j >= Nj || i >= Mi) return;
    float v[4] = {v0, v1, v2, v3};
    OT* o = out + (size_t)j * ld + i;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (i + e < Mi) {
        float x = v[e] + (bias ? bias[i + e] : 0.f);
        if (relu) x = fmaxf(x, 0.f);
        o[e] = (OT)x;
      }
    }
  }
};

// Split-K partial of a D^T store: K slice z of the launch writes
// out[z*sls + j*ld + i..i+3] (glds.h with_z calls set_z); a later kernel sums
// the slices in a fixed order (deterministic, unlike atomics).
struct EpiSliceT {
  float* out;
  int ld, Mi, Nj;
  size_t sls;
  __device__ __forceinline__ void set_z(int z) { out += (size_t)z * sls; }
  __device__ __forceinline__ void operator()(int i, int j, float v0, float v1, float v2, float v3) const {
    if (j >= Nj || i >= Mi) return;
    store4(out + (size_t)j * ld + i, v0, v1, v2, v3);
  }
};

// Stride-2 conv dgrad, one parity class (py, px): column j = (frame, a, b) of
// the class grid (Ha x Wa) lands at output pixel (2a+py, 2b+px) of H1 x W1.
struct EpiStoreParity {
  float* out;          // [F][H1][W1][C]
  int C, Nj, Ha, Wa, H1, W1, py, px;
  FastDiv dHW, dW;     // Ha*Wa and Wa
  __device__ __forceinline__ void operator()(int i, int j, float v0, float v1, float v2, float v3) const {
    if (j >= Nj || i >= C) return;
    const int f = (int)dHW.div((uint32_t)j), r = j - f * Ha * Wa;
    const int a = (int)dW.div((uint32_t)r), b = r - a * Wa;
    float* o = out + ((size_t)(f * H1 + 2 * a + py) * W1 + 2 * b + px) * C + i;
    *reinterpret_cast<f32x4*>(o) = f32x4{v0, v1, v2, v3};
  }
};

// Bias partials of a conv-input gradient for the LDS-staged epilogues
// (glds.h/halo.h: Pre/Acc/flush): every thread sums the fp32 values of its
// fixed 4-row group, the workgroup reduces them through LDS and adds one
// atomic per channel -- the bias gradient is the column sum of the fp32
// gradient (as the reference's autograd takes it) even where the gradient
// itself is stored rounded to the next GEMM's operand type.
struct BiasAcc {
  struct Pre {};
  struct Acc { float s[4]; };
  __device__ __forceinline__ Pre prefetch(int, int) const { return {}; }
  template <int G4, int NT>
  __device__ __forceinline__ void flush_to(const Acc& acc, float* red, int i0, int Mi, float* bg) const {
    static_assert(NT % G4 == 0, "fixed row group per thread");
    constexpr int NS = NT / G4;
    const int r4 = threadIdx.x % G4, sl = threadIdx.x / G4;
    *reinterpret_cast<f32x4*>(red + (sl * G4 + r4) * 4) = f32x4{acc.s[0], acc.s[1], acc.s[2], acc.s[3]};
    __syncthreads();
    for (int c = threadIdx.x; c < G4 * 4; c += NT) {
      float t = 0.f;
#pragma unroll 4
      for (int k = 0; k < NS; ++k) t += red[k * G4 * 4 + c];
      if (i0 + c < Mi) atomicAdd(bg + i0 + c, t);
    }
  }
};

// out[j*ld + i..i+3] = (OT)v (a conv-input gradient stored in the operand type
// of the GEMMs that read it) and bg[i] += sum_j v (its conv's bias gradient).
template <typename OT>
struct EpiStoreBiasT : BiasAcc {
  OT* out;
  int ld, Mi, Nj;
  float* bg;
  EpiStoreBiasT(OT* o, int l, int mi, int nj, float* b) : out(o), ld(l), Mi(mi), Nj(nj), bg(b) {}
  __device__ __forceinline__ void finish(int i, int j, float v0, float v1, float v2, float v3, const Pre&,
                                         Acc* acc = nullptr) const {
    if (j >= Nj || i >= Mi) return;
    store4(out + (size_t)j * ld + i, v0, v1, v2, v3);
    if (acc) { acc->s[0] += v0; acc->s[1] += v1; acc->s[2] += v2; acc->s[3] += v3; }
  }
  __device__ __forceinline__ void operator()(int i, int j, float v0, float v1, float v2, float v3) const {
    if (j >= Nj || i >= Mi) return;   // unstaged kernels: per-element bias atomics
    store4(out + (size_t)j * ld + i, v0, v1, v2, v3);
    atomicAdd(bg + i, v0); atomicAdd(bg + i + 1, v1); atomicAdd(bg + i + 2, v2); atomicAdd(bg + i + 3, v3);
  }
  template <int G4, int NT>
  __device__ __forceinline__ void flush(const Acc& acc, float* red, int i0, int) const {
    flush_to<G4, NT>(acc, red, i0, Mi, bg);
  }
};

// The stride-2 dgrad parity class of EpiStoreParity, stored in OT, with the
// bias partials of BiasAcc (conv1's bias gradient from dY1).
template <typename OT>
struct EpiStoreParityBias : BiasAcc {
  OT* out;             // [F][H1][W1][C]
  int C, Nj, Ha, Wa, H1, W1, py, px;
  FastDiv dHW, dW;
  float* bg;
  EpiStoreParityBias(OT* o, int c, int nj, int ha, int wa, int h1, int w1, int py_, int px_, float* b)
      : out(o), C(c), Nj(nj), Ha(ha), Wa(wa), H1(h1), W1(w1), py(py_), px(px_), dHW((uint32_t)(ha * wa)),
        dW((uint32_t)wa), bg(b) {}
  __device__ __forceinline__ OT* at(int i, int j) const {
    const int f = (int)dHW.div((uint32_t)j), r = j - f * Ha * Wa;
    const int a = (int)dW.div((uint32_t)r), b = r - a * Wa;
    return out + ((size_t)(f * H1 + 2 * a + py) * W1 + 2 * b + px) * C + i;
  }
  __device__ __forceinline__ void finish(int i, int j, float v0, float v1, float v2, float v3, const Pre&,
                                         Acc* acc = nullptr) const {
    if (j >= Nj || i >= C) return;
    store4(at(i, j), v0, v1, v2, v3);
    if (acc) { acc->s[0] += v0; acc->s[1] += v1; acc->s[2] += v2; acc->s[3] += v3; }
  }
  __device__ __forceinline__ void operator()(int i, int j, float v0, float v1, float v2, float v3) const {
    if (j >= Nj || i >= C) return;
    store4(at(i, j), v0, v1, v2, v3);
    atomicAdd(bg + i, v0); atomicAdd(bg + i + 1, v1); atomicAdd(bg + i + 2, v2); atomicAdd(bg + i + 3, v3);
  }
  template <int G4, int NT>
  __device__ __forceinline__ void flush(const Acc& acc, float* red, int i0, int) const {
    flush_to<G4, NT>(acc, red, i0, C, bg);
  }
};

// All four stride-2 dgrad parity classes of one tile (the KS = 2 halo conv,
// halo.h): row i = 32*cls + ci, class cls = (py, px) = (cls>>1, cls&1); column
// j = (frame, a, b) of the shared Ha x Wa class grid (Ha = ceil(H1/2)) lands at
// (2a+py, 2b+px) when that is inside H1 x W1 (odd H1: the py = 1 class is one
// row short).  The bias partials fold the four classes: bg[ci] += sum of the
// fp32 values of every valid output of channel ci.
template <typename OT>
struct EpiStoreParity4 : BiasAcc {
  OT* out;             // [F][H1][W1][32]
  int Nj, Wa, H1, W1;
  FastDiv dHW, dW;
  float* bg;
  EpiStoreParity4(OT* o, int nj, int ha, int wa, int h1, int w1, float* b)
      : out(o), Nj(nj), Wa(wa), H1(h1), W1(w1), dHW((uint32_t)(ha * wa)), dW((uint32_t)wa), bg(b) {}
  __device__ __forceinline__ void finish(int i, int j, float v0, float v1, float v2, float v3, const Pre&,
                                         Acc* acc = nullptr) const {
    if (j >= Nj || i >= 128) return;
    const int cls = i >> 5, ci = i & 31;
    const int f = (int)dHW.div((uint32_t)j), r = j - f * (int)dHW.d;
    const int a = (int)dW.div((uint32_t)r), b = r - a * Wa;
    const int oy = 2 * a + (cls >> 1), ox = 2 * b + (cls & 1);
    if (oy >= H1 || ox >= W1) return;
    store4(out + ((size_t)(f * H1 + oy) * W1 + ox) * 32 + ci, v0, v1, v2, v3);
    if (acc) { acc->s[0] += v0; acc->s[1] += v1; acc->s[2] += v2; acc->s[3] += v3; }
  }
  template <int G4, int NT>
  __device__ __forceinline__ void flush(const Acc& acc, float* red, int, int) const {
    static_assert(G4 == 32 && NT % G4 == 0, "one 128-row tile: 32 four-row groups");
    constexpr int NS = NT / G4;
    const int r4 = threadIdx.x % G4, sl = threadIdx.x / G4;
    *reinterpret_cast<f32x4*>(red + (sl * G4 + r4) * 4) = f32x4{acc.s[0], acc.s[1], acc.s[2], acc.s[3]};
    __syncthreads();
    for (int c = threadIdx.x; c < 32; c += NT) {   // channel c: rows c, 32+c, 64+c, 96+c
      float t = 0.f;
      for (int k = 0; k < NS; ++k)
#pragma unroll
        for (int cls = 0; cls < 4; ++cls) t += red[k * G4 * 4 + 32 * cls + c];
      atomicAdd(bg + c, t);
    }
  }
};

// dx[j*ld + i] = v * (mask[j*ldm + i] > 0)   (ReLU backward through a saved output)
struct EpiReluBwdT {
  float* out;
  const float* mask;
  int ld, ldm, Mi, Nj;
  __device__ __forceinline__ void operator()(int i, int j, float v0, float v1, float v2, float v3) const {
    if (j >= Nj || i >= Mi) return;
    float v[4] = {v0, v1, v2, v3};
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (i + e < Mi) out[(size_t)j * ld + i + e] = mask[(size_t)j * ldm + i + e] > 0.f ? v[e] : 0.f;
  }
};

// Row-major D: out[(i+e)*ld + j] (+)= v[e].  ATOMIC for split-K weight grads.
template <bool ATOMIC>
struct EpiStore {
  float* out;
  int ld, Mi, Nj;
  __device__ __forceinline__ void operator()(int i, int j, float v0, float v1, float v2, float v3) const {
    if (j >= Nj || i >= Mi) return;
    float v[4] = {v0, v1, v2, v3};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (i + e < Mi) {
        if constexpr (ATOMIC) atomicAdd(out + (size_t)(i + e) * ld + j, v[e]);
        else out[(size_t)(i + e) * ld + j] = v[e];
      }
    }
  }
};

// Split-K weight gradients on the LDS-DMA ring: atomics from the accumulators.
struct EpiAtomicD : EpiStore<true> {
  static constexpr bool kDirect = true;
};

// Policy / value heads: rows o < A -> logits, A <= o < 2A -> values (+bias).
struct EpiHeads {
  float* logits;
  float* values;
  const float* bias;  // [2A]
  int A, Nj;
  __device__ __forceinline__ void operator()(int i, int j, float v0, float v1, float v2, float v3) const {
    if (j >= Nj) return;
    float v[4] = {v0, v1, v2, v3};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      int o = i + e;
      if (o < A) logits[(size_t)j * A + o] = v[e] + bias[o];
      else if (o < 2 * A) values[(size_t)j * A + o - A] = v[e] + bias[o];
    }
  }
};

// ---------------------------------------------------------------- LSTMs ---
// Gate-interleaved rows: row 4*u + g, g = (i, f, c~, o).  Zero-peephole
// ConvLSTM cell (attention.py:119-123) / zero-state LSTMCell (Q1).
struct GateFwd {
  __device__ static __forceinline__ void run(float zi, float zf, float zc, float zo, float cprev,
                                             float& gi, float& gf, float& gc, float& go,
                                             float& c, float& h) {
    gi = sigm_acc(zi);
    gf = sigm_acc(zf);
    gc = tanhf(zc);
    c = gf * cprev + gi * gc;
    go = sigm_acc(zo);
    h = go * tanhf(c);
  }
};

// Backward of one cell given the incoming dh and the carried dc (from t+1).
// Returns dz (i,f,c~,o) and updates dc to the carry for t-1 (= dc_t * f_t).
__device__ __forceinline__ void gate_bwd(float dh, const f32x4& g, float cprev, float ccur, float& dc,
                                         float& di, float& df, float& dcg, float& dout) {
  const float gi = g[0], gf = g[1], gc = g[2], go = g[3];
  const float tc = tanhf(ccur);
  const float dcc = dc + dh * go * (1.f - tc * tc);
  dout = dh * tc * (1.f - go) * go;
  di = dcc * gc * (1.f - gi) * gi;
  df = dcc * cprev * (1.f - gf) * gf;
  dcg = dcc * gi * (1.f - gc * gc);
  dc = dcc * gf;
}

// Gate-activation storage: fp32, or fp16 on the bf16 path (values in (-1, 1),
// 2^-11 relative; the backward's only use of them), half the bytes of the
// step epilogues' largest stream.
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f32x4 load_gates(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
__device__ __forceinline__ f32x4 load_gates(const _Float16* p) {
  const f16x4 h = *reinterpret_cast<const f16x4*>(p);
  return f32x4{(float)h[0], (float)h[1], (float)h[2], (float)h[3]};
}
__device__ __forceinline__ void store_gates(float* p, const f32x4& v) { *reinterpret_cast<f32x4*>(p) = v; }
__device__ __forceinline__ void store_gates(_Float16* p, const f32x4& v) {
  *reinterpret_cast<f16x4*>(p) = f16x4{(_Float16)v[0], (_Float16)v[1], (_Float16)v[2], (_Float16)v[3]};
}

// ConvLSTM forward step epilogue: D[n = 4ch+g][m] = Wh*h_{t-1}; the x-part
// (Wx*x_t + b, batched over all frames beforehand) is read from ``gates``
// and overwritten in place with the activations.
template <typename T, typename GT = float>
struct EpiConvLstmFwd {
  const float* cprev;  // [M][128]  c_{t-1}
  float* cnext;        // [M][128]  c_t
  float* hout;         // [M][128]  h_t (fp32, the fp32 path's attention input), or null (bf16: readout_h reads XH)
  T* xhnext;           // [M][192]  slot t+1, channels 64..191 <- h_t (next step operand)
  GT* gates;           // [M][512]  in: Wx*x_t + b (fp32 only);  out: post-activation (i,f,c~,o)
  int Nj;              // M = B*P
  // Fused x-part (the GEMM's K covers [x_t | h_{t-1}]): the gate bias [512]
  // takes the place of the batched x-part, which ``gates`` then does not hold
  // (and must not: an fp16 gate buffer only ever holds activations).
  const float* bias = nullptr;
  // Inputs of one (4-row, column) group, loadable before the K loop (glds.h).
  struct Pre { f32x4 zx; float cp; };
  __device__ __forceinline__ Pre prefetch(int i, int j) const {
    Pre p{f32x4{0.f, 0.f, 0.f, 0.f}, 0.f};
    if (j < Nj && i < 512) {
      if constexpr (std::is_same<GT, float>::value)
        p.zx = bias ? *reinterpret_cast<const f32x4*>(bias + i)
                    : *reinterpret_cast<const f32x4*>(gates + (size_t)j * 512 + i);
      else
        p.zx = *reinterpret_cast<const f32x4*>(bias + i);
      p.cp = cprev[(size_t)j * 128 + (i >> 2)];
    }
    return p;
  }
  __device__ __forceinline__ void finish(int i, int j, float v0, float v1, float v2, float v3, const Pre& p) const {
    if (j >= Nj || i >= 512) return;
    const int ch = i >> 2;
    float gi, gf, gc, go, c, h;
    GateFwd::run(p.zx[0] + v0, p.zx[1] + v1, p.zx[2] + v2, p.zx[3] + v3, p.cp, gi, gf, gc, go, c, h);
    cnext[(size_t)j * 128 + ch] = c;
    if (hout) hout[(size_t)j * 128 + ch] = h;
    xhnext[(size_t)j * 192 + 64 + ch] = (T)h;
    store_gates(gates + (size_t)j * 512 + i, f32x4{gi, gf, gc, go});
  }
  __device__ __forceinline__ void operator()(int i, int j, float v0, float v1, float v2, float v3) const {
    finish(i, j, v0, v1, v2, v3, prefetch(i, j));
  }
};

// ConvLSTM backward step epilogue on D[c'][m] = dgrad of dz_t into [x_t | h_{t-1}]:
// rows c' < 64 -> dx_t (conv2 output grad); rows >= 64 -> dh_{t-1}, fused with
// the gate backward of step t-1 (writes dz_{t-1} as TZ -- the GEMM operand type
// of the later dgrad / wgrad passes -- and the dc carry), or dh0.
//
// Gate-bias gradient (sum of dz over pixels): with ``part`` set, every thread
// sums the fp32 dz it produces (Acc), and flush() reduces them over the
// workgroup's columns into one 4*BI-wide row part[tile_j][4*(row0-64) ...] --
// the bias gradient then needs only a column sum over T x (column tiles) rows
// instead of a pass over the whole dZ tensor, and it is taken before dz is
// rounded to TZ (the reference sums fp32 gradients).
template <typename TZ, typename GT = float>
struct EpiConvLstmBwd {
  float* dx;            // [M][64]  dY2 slot t
  const GT* gates;      // [M][512] slot t-1
  const float* cprev;   // [M][128] c_{t-2}
  const float* ccur;    // [M][128] c_{t-1}
  const float* dO;      // [M][128] attention-path grad of h_{t-1}
  float* dC;            // [M][128] dc carry (in/out)
  TZ* dz;               // [M][512] slot t-1
  float* dh0;           // [M][128] or null (only when t == 0)
  int has_prev, Nj;
  int ioff;             // 64 when the GEMM computes only the h rows (dx batched separately)
  float* part;          // [column tiles][512] bias partials of slot t-1, or null
  // Inputs of one (4-row, column) group of the fused gate backward, loadable
  // before the K loop (glds.h); only the has_prev h-row path has any.
  struct Pre { f32x4 g[4], dov, cp, cc, dcv; };
  struct Acc { f32x4 s[4]; };   // dz sums of the thread's 4 channels x 4 gates
  __device__ __forceinline__ Pre prefetch(int i, int j) const {
    Pre p;
    i += ioff;
    if (j >= Nj || i < 64 || i >= 192 || !has_prev) return p;
    const int ch = i - 64;
    p.dov = *reinterpret_cast<const f32x4*>(dO + (size_t)j * 128 + ch);
    p.cp = *reinterpret_cast<const f32x4*>(cprev + (size_t)j * 128 + ch);
    p.cc = *reinterpret_cast<const f32x4*>(ccur + (size_t)j * 128 + ch);
    p.dcv = *reinterpret_cast<const f32x4*>(dC + (size_t)j * 128 + ch);
#pragma unroll
    for (int e = 0; e < 4; ++e) p.g[e] = load_gates(gates + (size_t)j * 512 + 4 * (ch + e));
    return p;
  }
  __device__ __forceinline__ void finish(int i, int j, float v0, float v1, float v2, float v3, const Pre& p,
                                         Acc* acc = nullptr) const {
    i += ioff;
    if (j >= Nj || i >= 192) return;
    if (i < 64) {
      *reinterpret_cast<f32x4*>(dx + (size_t)j * 64 + i) = f32x4{v0, v1, v2, v3};
      return;
    }
    const int ch = i - 64;
    if (!has_prev) {
      if (dh0) *reinterpret_cast<f32x4*>(dh0 + (size_t)j * 128 + ch) = f32x4{v0, v1, v2, v3};
      return;
    }
    const float v[4] = {v0, v1, v2, v3};
    f32x4 dcv = p.dcv;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float dc = dcv[e], di, df, dcg, dout;
      gate_bwd(v[e] + p.dov[e], p.g[e], p.cp[e], p.cc[e], dc, di, df, dcg, dout);
      dcv[e] = dc;
      store4(dz + (size_t)j * 512 + 4 * (ch + e), di, df, dcg, dout);
      if (acc) {
        acc->s[e][0] += di; acc->s[e][1] += df; acc->s[e][2] += dcg; acc->s[e][3] += dout;
      }
    }
    *reinterpret_cast<f32x4*>(dC + (size_t)j * 128 + ch) = dcv;
  }
  __device__ __forceinline__ void operator()(int i, int j, float v0, float v1, float v2, float v3) const {
    finish(i, j, v0, v1, v2, v3, prefetch(i, j));
  }
  // Workgroup reduction of the Acc of threads that share a row group (r4 =
  // tid % G4: the pipe kernel's epilogue walks columns with a fixed row group
  // per thread when NT % G4 == 0), then one row of partials per column tile.
  template <int G4, int NT>
  __device__ __forceinline__ void flush(const Acc& acc, float* red, int i0, int tj) const {
    static_assert(NT % G4 == 0, "fixed row group per thread");
    constexpr int NS = NT / G4;            // threads per row group
    if (!part || !has_prev) return;
    const int r4 = threadIdx.x % G4, sl = threadIdx.x / G4;
#pragma unroll
    for (int e = 0; e < 4; ++e) *reinterpret_cast<f32x4*>(red + (sl * G4 + r4) * 16 + 4 * e) = acc.s[e];
    __syncthreads();
    const int row0 = i0 + ioff - 64;       // first dh channel of this tile
    for (int c = threadIdx.x; c < G4 * 16; c += NT) {
      float t = 0.f;
#pragma unroll 4
      for (int k = 0; k < NS; ++k) t += red[k * G4 * 16 + c];
      if (row0 >= 0 && row0 * 4 + c < 512) part[(size_t)tj * 512 + row0 * 4 + c] = t;
    }
  }
};

// LSTMCell(256,256) with zero state (attention.py:355, Q1), rows 4u+g.
struct EpiLstmCellFwd {
  const float* bias;  // [1024] interleaved b_ih + b_hh
  float* gates;       // [F][1024]
  float* cout;        // [F][256]
  float* hout;        // [F][256]
  int Nj;
  __device__ __forceinline__ void operator()(int i, int j, float v0, float v1, float v2, float v3) const {
    if (j >= Nj || i >= 1024) return;
    const int u = i >> 2;
    const f32x4 b = *reinterpret_cast<const f32x4*>(bias + i);
    const float gi = sigm_acc(v0 + b[0]), gf = sigm_acc(v1 + b[1]);
    const float gc = tanhf(v2 + b[2]), go = sigm_acc(v3 + b[3]);
    const float c = gf * 0.f + gi * gc;
    cout[(size_t)j * 256 + u] = c;
    hout[(size_t)j * 256 + u] = go * tanhf(c);
    *reinterpret_cast<f32x4*>(gates + (size_t)j * 1024 + i) = f32x4{gi, gf, gc, go};
  }
};

// Stateful policy core (the reference's else branch, attention.py:356-358):
// LSTMCell from (h_{t-1}, c_{t-1}), D = [W_ih | W_hh] x [answer | h_{t-1}].
// Writes the gate activations, c_t and h_t into the state slots and h_t into
// the next step's GEMM operand row (cols 256..511 of its [answer | h] row).
struct EpiLstmCellFwdS {
  const float* bias;   // [1024] interleaved b_ih + b_hh
  float* gates;        // [B][1024]
  const float* cprev;  // [B][256] c_{t-1}
  float* cout;         // [B][256] c_t
  float* hout;         // [B][256] h_t
  float* hnext;        // [B][512] next step's operand rows (+256 applied by the caller), or null
  int Nj;
  __device__ __forceinline__ void operator()(int i, int j, float v0, float v1, float v2, float v3) const {
    if (j >= Nj || i >= 1024) return;
    const int u = i >> 2;
    const f32x4 b = *reinterpret_cast<const f32x4*>(bias + i);
    const float gi = sigm_acc(v0 + b[0]), gf = sigm_acc(v1 + b[1]);
    const float gc = tanhf(v2 + b[2]), go = sigm_acc(v3 + b[3]);
    const float c = gf * cprev[(size_t)j * 256 + u] + gi * gc;
    const float h = go * tanhf(c);
    cout[(size_t)j * 256 + u] = c;
    hout[(size_t)j * 256 + u] = h;
    if (hnext) hnext[(size_t)j * 512 + u] = h;
    *reinterpret_cast<f32x4*>(gates + (size_t)j * 1024 + i) = f32x4{gi, gf, gc, go};
  }
};

// Its backward: dh = heads' dgrad (the GEMM, rows = units u..u+3) + the carry
// from step t+1 (dhc); the cell-state carry dcc is read and replaced by the
// carry for t-1.
struct EpiLstmCellBwdS {
  const float* gates;  // [B][1024]
  const float* cprev;  // [B][256] c_{t-1}
  const float* ccur;   // [B][256] c_t
  const float* dhc;    // [B][256] dh carried from t+1
  float* dcc;          // [B][256] dc carry (in/out)
  float* dgates;       // [B][1024]
  int Nj;
  __device__ __forceinline__ void operator()(int i, int j, float v0, float v1, float v2, float v3) const {
    if (j >= Nj || i >= 256) return;
    const float v[4] = {v0, v1, v2, v3};
    const f32x4 cv = *reinterpret_cast<const f32x4*>(ccur + (size_t)j * 256 + i);
    const f32x4 cp = *reinterpret_cast<const f32x4*>(cprev + (size_t)j * 256 + i);
    const f32x4 hc = *reinterpret_cast<const f32x4*>(dhc + (size_t)j * 256 + i);
    f32x4 dc = *reinterpret_cast<const f32x4*>(dcc + (size_t)j * 256 + i);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const f32x4 g = *reinterpret_cast<const f32x4*>(gates + (size_t)j * 1024 + 4 * (i + e));
      float d = dc[e], di, df, dcg, dout;
      gate_bwd(v[e] + hc[e], g, cp[e], cv[e], d, di, df, dcg, dout);
      dc[e] = d;
      *reinterpret_cast<f32x4*>(dgates + (size_t)j * 1024 + 4 * (i + e)) = f32x4{di, df, dcg, dout};
    }
    *reinterpret_cast<f32x4*>(dcc + (size_t)j * 256 + i) = dc;
  }
};

// out[j*ld + i] = v + add[j*ld_add + i]  (two gradient paths into one tensor)
struct EpiStoreAddT {
  float* out;
  const float* add;
  int ld, ld_add, Mi, Nj;
  __device__ __forceinline__ void operator()(int i, int j, float v0, float v1, float v2, float v3) const {
    if (j >= Nj || i >= Mi) return;
    const float v[4] = {v0, v1, v2, v3};
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (i + e < Mi) out[(size_t)j * ld + i + e] = v[e] + add[(size_t)j * ld_add + i + e];
  }
};

// dh from the heads' dgrad (rows = units u..u+3) -> d(gates) of the zero-state cell.
struct EpiLstmCellBwd {
  const float* gates;  // [F][1024]
  const float* cst;    // [F][256]
  float* dgates;       // [F][1024]
  int Nj;
  __device__ __forceinline__ void operator()(int i, int j, float v0, float v1, float v2, float v3) const {
    if (j >= Nj || i >= 256) return;
    const float v[4] = {v0, v1, v2, v3};
    const f32x4 cv = *reinterpret_cast<const f32x4*>(cst + (size_t)j * 256 + i);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const f32x4 g = *reinterpret_cast<const f32x4*>(gates + (size_t)j * 1024 + 4 * (i + e));
      float dc = 0.f, di, df, dcg, dout;
      gate_bwd(v[e], g, 0.f, cv[e], dc, di, df, dcg, dout);
      *reinterpret_cast<f32x4*>(dgates + (size_t)j * 1024 + 4 * (i + e)) = f32x4{di, df, dcg, dout};
    }
  }
};

}  // namespace aaa
