// Attention readout forward with the readout product on the MFMA, bf16 O (the h half of the XH rows)
// (attention.py:319-348 -- logits, spatial_softmax :235-254, readout, the answer row; the VALU kernel
// k_attn_fwd computes the same).  Included by misc.hip only (uses its wave_sum / wave_max / lds_barrier).
//
// One workgroup (4 waves) per frame.  After the logits and the softmax (as k_attn_fwd), the frame
// streams through LDS in chunks of 32 grid positions, each chunk one K step of
// v_mfma_f32_16x16x32_bf16:
//     a[q][c] = sum_p A[p][q] V[p][c],   V = [O[:, 0:128] | S]   (key channels 0..7 computed, dropped)
// with M = the V channels (16 per tile), N = the map rows, K = the positions.  The fp32 operands are
// split into hi + mid + lo bf16 parts -- the map A as the rows n = s*NQ + q of Wt[n][position] (zeros
// past the grid), the basis S as three more channel planes of the chunk image -- and every part
// product is summed in fp32: the value of fp32 FMAs up to summation order (O is bf16 already).  A wave
// owns every part of its channel blocks (O blocks w, w + 4, S block w), so the parts meet in registers.
// Chunk image: one row per position, [O | S hi | S mid | S lo] bf16, 16-B pieces XOR-keyed by row
// (am_key) so the A operand's transposed reads (ds_read_b64_tr_b16, rows 8g+tq and 8g+4+tq of 16-lane
// group g) hit 64 distinct banks per half-wave.  The logits L[q][p] live there before the first chunk.
// Chunks are register-staged two ahead by buffer loads (positions past the grid read as zeros: no
// branch, the waits stay counted) and committed -- S split -- once per chunk.
#pragma once
#include "loaders_b.h"

namespace aaa {

constexpr int kAmRB = 768;   // chunk image row bytes: 320 bf16 (40 pieces), padded to 48 pieces (the key XORs 4 bits)
__device__ __forceinline__ int am_key(int r) { return ((r & 3) << 2) | (((r >> 3) & 1) << 1); }
// byte offset of bf16 element e of image row r
__device__ __forceinline__ int am_off(int r, int e) {
  return r * kAmRB + (((e >> 3) ^ am_key(r)) << 4) + ((e & 7) << 1);
}
__device__ __forceinline__ bf16x8 am_tr(const unsigned char* lds, int o0, int o1) {
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(const_cast<unsigned char*>(lds + o0)));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(const_cast<unsigned char*>(lds + o1)));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}
__device__ __forceinline__ void am_split(float x, __bf16& hi, __bf16& mid, __bf16& lo) {
  hi = (__bf16)x;
  const float r = x - (float)hi;
  mid = (__bf16)r;
  lo = (__bf16)(r - (float)mid);
}
// 4 fp32 -> their three bf16 parts, 8 B each, at image elements e, e + 64, e + 128 of row r
__device__ __forceinline__ void am_store_split(unsigned char* im, int r, int e, const u32x4& raw) {
  const f32x4 f = __builtin_bit_cast(f32x4, raw);
  bf16x4 h, m, l;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    __bf16 a, b, c;
    am_split(f[i], a, b, c);
    h[i] = a;
    m[i] = b;
    l[i] = c;
  }
  *reinterpret_cast<bf16x4*>(im + am_off(r, e)) = h;
  *reinterpret_cast<bf16x4*>(im + am_off(r, e + 64)) = m;
  *reinterpret_cast<bf16x4*>(im + am_off(r, e + 128)) = l;
}

constexpr int kAmD = 2;   // chunks staged ahead
__host__ __device__ inline int attn_mfma_pp(int P) { return (P + 32 * kAmD - 1) / (32 * kAmD) * (32 * kAmD); }
__host__ __device__ inline int attn_mfma_img(int P, int nq) {   // chunk image / logits bytes
  return 32 * kAmRB > nq * P * 4 ? 32 * kAmRB : nq * P * 4;
}
inline size_t attn_mfma_lds(int P, int nq) {
  return (size_t)attn_mfma_img(P, nq) + (size_t)3 * nq * (2 * attn_mfma_pp(P) + 16) + (size_t)nq * 72 * 4;
}

// NTL_: the frame's O rows loaded non-temporal (nt: streamed past L2, keeping the basis resident there)
// SQP_: the basis half of the logits comes precomputed (SQ, a constant query); else computed here (per-frame query)
template <int NQ, bool NTL_, bool SQP_ = true>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(NQ == 8 ? 4 : 5)))
k_attn_fwd_mfma(const __bf16* __restrict__ Hs, int old, const float* __restrict__ S, const float* __restrict__ Q,
                int qs, const float* __restrict__ SQ, const float* __restrict__ pr, const float* __restrict__ pa, int P,
                float* __restrict__ Am, float* __restrict__ ans, int ans_ld) {
  constexpr int D = kAmD, NR = 3 * NQ, NTN = NQ == 8 ? 2 : 1;   // map-part rows, their 16-row tiles
  constexpr int NTL = 5;   // M tiles per wave: O blocks w, w + 4, S block w (3 parts)
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int Pp = attn_mfma_pp(P), WS = 2 * Pp + 16;
  unsigned char* const vim = reinterpret_cast<unsigned char*>(sm);   // chunk image; L[q][p] before the loop
  float* const L = sm;
  unsigned char* const wt = vim + attn_mfma_img(P, NQ);              // Wt[n][p], NR rows of WS bytes
  float* const Qs = reinterpret_cast<float*>(wt + NR * WS);           // NQ x 72
  const int f = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 15, g = lane >> 4;
  const __bf16* O = Hs + (size_t)f * P * old;
  const float* Qf = Q + (size_t)f * qs;
  const __amdgpu_buffer_rsrc_t ro = make_rsrc(O, (uint32_t)((size_t)P * old * 2));
  const __amdgpu_buffer_rsrc_t rsb = make_rsrc(S, (uint32_t)(P * 256));
  const __amdgpu_buffer_rsrc_t rsq = make_rsrc(SQ ? SQ : S, SQ ? (uint32_t)(P * NQ * 4) : 0u);
  auto oload = [&](uint32_t off) { return __builtin_amdgcn_raw_buffer_load_b128(ro, off, 0, NTL_ ? 2 : 0); };

  // ---- loads in the order they are used: queries, keys and basis logits of positions tid, tid + 256,
  // then the first D chunks (the waits for the first ones are then counted, not drained)
  constexpr int NQL = (NQ * 72 + 255) / 256;
  float qv[NQL];
#pragma unroll
  for (int j = 0; j < NQL; ++j) qv[j] = Qf[min(tid + 256 * j, NQ * 72 - 1)];
  u32x4 kr[2];
  f32x4 sq[2][NQ / 4];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int p = tid + 256 * i;
    kr[i] = oload(p < P ? (uint32_t)(p * old * 2) : kOOB);
    const uint32_t so = p < P ? (uint32_t)(p * NQ * 4) : kOOB;
#pragma unroll
    for (int j = 0; j < NQ / 4; ++j) sq[i][j] = __builtin_bit_cast(f32x4, bload(rsq, so + 16 * j));
  }
  // staged chunk: this thread's 16-B pieces i = tid + 256 j of the chunk's O rows (row i >> 4, piece
  // i & 15, 8 channels) and of its S rows (row i >> 4, 4 fp32 channels 4 (i & 15))
  u32x4 ost[D][2], sst[D][2];
  auto fetch = [&](int k, u32x4 (&o)[2], u32x4 (&s)[2]) {
    const int pb = 32 * k;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int i = tid + 256 * j, p = pb + (i >> 4);
      o[j] = oload(p < P ? (uint32_t)(p * old * 2 + 16 * (i & 15)) : kOOB);
      s[j] = bload(rsb, p < P ? (uint32_t)(p * 256 + 16 * (i & 15)) : kOOB);
    }
  };
  auto commit = [&](u32x4 (&o)[2], u32x4 (&s)[2]) {
    // pinned behind the previous barrier (volatile asm keeps its order): otherwise the scheduler
    // hoists the next chunk's split above this chunk's refill and waits for its loads there
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      asm volatile("" : "+v"(o[j]));
      asm volatile("" : "+v"(s[j]));
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int i = tid + 256 * j, r = i >> 4, c = i & 15;
      *reinterpret_cast<u32x4*>(vim + am_off(r, 8 * c)) = o[j];
      am_store_split(vim, r, 128 + 4 * c, s[j]);
    }
  };
#pragma unroll
  for (int d = 0; d < D; ++d) fetch(d, ost[d], sst[d]);

#pragma unroll
  for (int j = 0; j < NQL; ++j)
    if (tid + 256 * j < NQ * 72) Qs[tid + 256 * j] = qv[j];
  lds_barrier();   // (LDS only: the chunk loads stay in flight)

  // ---- logits L[q][p] = K[p].Q[q], K = [O[:8] | S] (the basis half precomputed in SQ for a constant query)
  auto logits = [&](int p, const u32x4& k, const f32x4 (&sqp)[NQ / 4]) {
    const f32x4 ka = bf4_f32(u32x2{k.x, k.y}), kb = bf4_f32(u32x2{k.z, k.w});
    float acc[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const float* qq = Qs + q * 72;
      acc[q] = ka[0] * qq[0] + ka[1] * qq[1] + ka[2] * qq[2] + ka[3] * qq[3] + kb[0] * qq[4] + kb[1] * qq[5] +
               kb[2] * qq[6] + kb[3] * qq[7];
    }
    if constexpr (SQP_) {
#pragma unroll
      for (int q = 0; q < NQ; ++q) acc[q] += sqp[q / 4][q % 4];
    } else {   // per-frame query: the basis half here
      const f32x4* s4 = reinterpret_cast<const f32x4*>(S + p * 64);
#pragma unroll 4
      for (int c = 0; c < 16; ++c) {
        const f32x4 v = s4[c];
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
          const float* qq = Qs + q * 72 + 8 + 4 * c;
          acc[q] += v[0] * qq[0] + v[1] * qq[1] + v[2] * qq[2] + v[3] * qq[3];
        }
      }
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q) L[q * P + p] = acc[q];
  };
#pragma unroll
  for (int i = 0; i < 2; ++i)
    if (tid + 256 * i < P) logits(tid + 256 * i, kr[i], sq[i]);
  for (int p = tid + 512; p < P; p += 256) {   // grids past 512 positions
    f32x4 s[NQ / 4];
#pragma unroll
    for (int j = 0; j < NQ / 4; ++j) s[j] = __builtin_bit_cast(f32x4, bload(rsq, (uint32_t)(p * NQ * 4 + 16 * j)));
    logits(p, bload(ro, (uint32_t)(p * old * 2)), s);
  }
  lds_barrier();

  // ---- spatial softmax over the P positions, one wave per query (k_attn_fwd's order of operations):
  // the map's three bf16 parts to Wt (zeros past the grid).  The map itself goes to HBM after the
  // readout, rebuilt from its parts (hi + mid + lo is the fp32 value exactly): a store here, among
  // the staged chunk loads, would make the compiler drain vmcnt at the first chunk (a counter with
  // both reads and writes pending is waited to zero)
  for (int q = wave; q < NQ; q += 4) {
    float* Lq = L + q * P;
    float m = -INFINITY;
    for (int p = lane; p < P; p += 64) m = fmaxf(m, Lq[p]);
    m = wave_max(m);
    float s = 0.f;
    for (int p = lane; p < P; p += 64) {
      const float e = expf(Lq[p] - m);
      Lq[p] = e;
      s += e;
    }
    s = wave_sum(s);
    const float inv = 1.f / s;
    for (int p = lane; p < Pp; p += 64) {
      const float a = p < P ? Lq[p] * inv : 0.f;
      __bf16 h, mi, lo;
      am_split(a, h, mi, lo);
      *reinterpret_cast<__bf16*>(wt + q * WS + 2 * p) = h;
      *reinterpret_cast<__bf16*>(wt + (NQ + q) * WS + 2 * p) = mi;
      *reinterpret_cast<__bf16*>(wt + (2 * NQ + q) * WS + 2 * p) = lo;
    }
  }
  lds_barrier();   // Wt complete; every wave is done with L (the chunk image may be overwritten)

  // ---- readout
  const int tq = li >> 2, tp = li & 3, r0 = 8 * g + tq;
  int ao0[NTL], ao1[NTL];   // transposed-read addresses (rows r0, r0 + 4) of the wave's tiles
#pragma unroll
  for (int t = 0; t < NTL; ++t) {
    const int e = t < 2 ? 16 * (wave + 4 * t) : 128 + 64 * (t - 2) + 16 * wave;   // O blocks, S parts
    ao0[t] = am_off(r0, e + 4 * tp);
    ao1[t] = am_off(r0 + 4, e + 4 * tp);
  }
  // map-part rows n = li (+16) of this lane, clamped into the image; rows past NR read as zeros
  const int n0 = li, n1 = 16 + li;
  const unsigned char* wb0 = wt + min(n0, NR - 1) * WS + 16 * g;
  const unsigned char* wb1 = wt + min(n1, NR - 1) * WS + 16 * g;
  f32x4 acc[3][NTN];   // O block w, O block w + 4, S block w (its three parts summed by the MFMA chain)
#pragma unroll
  for (int t = 0; t < 3; ++t)
#pragma unroll
    for (int n = 0; n < NTN; ++n) acc[t][n] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = Pp / 32;
  const bf16x8 zero8 = {};
  for (int k0 = 0; k0 < nk; k0 += D) {
#pragma unroll
    for (int j = 0; j < D; ++j) {
      const int k = k0 + j;
      commit(ost[j], sst[j]);
      fetch(k + D, ost[j], sst[j]);
      lds_barrier();   // chunk k in the image
      bf16x8 w[NTN];
      w[0] = *reinterpret_cast<const bf16x8*>(wb0 + 64 * k);
      if (n0 >= NR) w[0] = zero8;
      if constexpr (NTN == 2) {
        w[NTN - 1] = *reinterpret_cast<const bf16x8*>(wb1 + 64 * k);
        if (n1 >= NR) w[NTN - 1] = zero8;
      }
#pragma unroll
      for (int t = 0; t < NTL; ++t) {
        const bf16x8 a = am_tr(vim, ao0[t], ao1[t]);
        const int ti = t < 2 ? t : 2;
#pragma unroll
        for (int n = 0; n < NTN; ++n) acc[ti][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, w[n], acc[ti][n], 0, 0, 0);
      }
      lds_barrier();   // every wave is done with chunk k: the next commit may overwrite the image
    }
  }

  // ---- the answer row: lane (g, li) holds D[channel 4g + r][map row li (+16)] of its three blocks; the
  // parts of query q are map rows q, NQ + q, 2 NQ + q: lanes li + NQ, li + 2 NQ of the group, or tile 2
  float* arow = ans + (size_t)f * ans_ld;
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    f32x4 r;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float v0 = acc[t][0][e];
      if constexpr (NQ == 4) r[e] = v0 + __shfl_down(v0, 4, 64) + __shfl_down(v0, 8, 64);
      else r[e] = v0 + __shfl_down(v0, 8, 64) + acc[t][NTN - 1][e];
    }
    const int c = 16 * (t < 2 ? wave + 4 * t : wave) + 4 * g;   // O channel (0..7: the keys) or S channel
    const int oc = t < 2 ? c - 8 : 120 + c;
    if (li < NQ && (t == 2 || c >= 8)) {
      float* dst = arow + li * 184 + oc;
      *reinterpret_cast<float2*>(dst) = float2{r[0], r[1]};
      *reinterpret_cast<float2*>(dst + 2) = float2{r[2], r[3]};
    }
  }
  for (int i = tid; i < P * NQ; i += 256) {   // the map, coalesced: Am[f][p][q]
    const int p = i / NQ, q = i - p * NQ;
    const __bf16* w = reinterpret_cast<const __bf16*>(wt + q * WS) + p;
    Am[(size_t)f * P * NQ + i] = ((float)w[0] + (float)w[NQ * WS / 2]) + (float)w[NQ * WS];
  }
  for (int i = tid; i < NQ * 72; i += 256) arow[NQ * 184 + i] = Qs[i];
  for (int i = NQ * 256 + tid; i < ans_ld; i += 256) {
    float v = 0.f;
    if (i == NQ * 256) v = pr ? pr[f] : 0.f;
    else if (i == NQ * 256 + 1) v = pa ? pa[f] : 0.f;
    arow[i] = v;
  }
}

// Attention readout backward with the dA pass on the MFMA, bf16 O (attention.py:336-348, 235-254
// backward; the VALU kernel k_attn_bwd computes the same -- phases 2-4 below are its code).
//   dA[p][q] = sum_c V[p][c] da[q][c],  V = [O[:, 8:128] | S]
// as 16x16x32 bf16 MFMAs over 16-position blocks: M = positions, K = the channels of V' = [O[:, 0:128] |
// S hi | S mid | S lo] (the A operand straight from the O and S rows: 8 consecutive channels of one
// position per lane, S split on the fly), N = the rows n = s*NQ + q of Dp[n][k'], the answer gradient
// da split into bf16 parts (zero for O's key channels 0..7; its S columns repeated under each S part,
// so all nine S-part x da-part products are summed).  Exact to fp32 up to summation order.  Dp lives
// in the dQ reduction's LDS (red, used only after the pass).  The key channels for dQ are taken from
// the O fragments of channels 0..7.
template <int NQ>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4)))   // two frames per CU
k_attn_bwd_mfma(const __bf16* __restrict__ Hs, int old, const float* __restrict__ S, const float* __restrict__ Q,
                int qs, const float* __restrict__ Am, const float* __restrict__ dAns, int da_ld, int addq, int P,
                float* __restrict__ dO, float* __restrict__ dQp, int cqm) {
  constexpr int NT = 512, NW = NT / 64;
  constexpr int G = 7;                                  // position groups of the dQ reduction (7*72 <= NT)
  constexpr int NR = 3 * NQ, NTN = NQ == 8 ? 2 : 1;    // da-part rows, their 16-row tiles
  constexpr int DS = 320 * 2 + 16;                      // Dp row bytes: 320 bf16 (K of V') + pad
  static_assert(NR * DS <= G * NQ * 72 * 4, "Dp aliases the dQ reduction buffer");
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* A = sm;                 // P*NQ
  float* dA = A + P * NQ;        // P*NQ  (becomes dlogits)
  float* da = dA + P * NQ;       // NQ*184
  float* Qs = da + NQ * 184;     // NQ*72
  float* ss = Qs + NQ * 72;      // NQ (padded to 8)
  float* red = ss + 8;           // G*NQ*72; Dp during the dA pass
  float* Kc = red + G * NQ * 72; // P*8  key channels O[:8] as fp32
  unsigned char* const Dp = reinterpret_cast<unsigned char*>(red);
  const int f = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, g = lane >> 4;
  const __bf16* O = Hs + (size_t)f * P * old;
  const __amdgpu_buffer_rsrc_t ro = make_rsrc(O, (uint32_t)((size_t)P * old * 2));
  const __amdgpu_buffer_rsrc_t rsb = make_rsrc(S, (uint32_t)(P * 256));
  // a position block's A-operand loads of this lane: O channels 32 kk + 8g .. +7 (kk < 4) and S channels
  // 32 h + 8g .. +7 (h < 2, two 16-B pieces each) of position p0 + li (past the grid: zeros)
  struct Blk { u32x4 o[4], s[4]; };
  auto bfetch = [&](int p0, Blk& b) {
    const int p = p0 + li;
    const bool v = p < P;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) b.o[kk] = bload(ro, v ? (uint32_t)((p * old + 32 * kk + 8 * g) * 2) : kOOB);
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int e = 0; e < 2; ++e)
        b.s[2 * h + e] = bload(rsb, v ? (uint32_t)((p * 64 + 32 * h + 8 * g + 4 * e) * 4) : kOOB);
  };
  const int nb = (P + 15) / 16;
  Blk cur;
  bfetch(16 * wave, cur);   // (a block past the grid loads zeros and is never used)
  for (int i = tid; i < P * NQ; i += NT) A[i] = Am[(size_t)f * P * NQ + i];
  for (int i = tid; i < NQ * 184; i += NT) da[i] = dAns[(size_t)f * da_ld + i];
  for (int i = tid; i < NQ * 72; i += NT) Qs[i] = Q[(size_t)f * qs + i];
  __syncthreads();
  // Dp[n = s NQ + q][k'] = part s of: 0 (k' < 8), da[q][k' - 8] (k' < 128), da[q][120 + (k' - 128) % 64]
  for (int i = tid; i < NR * 80; i += NT) {
    const int n = i / 80, k = 4 * (i - n * 80), sp = n / NQ, q = n - sp * NQ;
    bf16x4 v;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int kk = k + e;
      const float x = kk < 8 ? 0.f : da[q * 184 + (kk < 128 ? kk - 8 : 120 + ((kk - 128) & 63))];
      __bf16 h, m, l;
      am_split(x, h, m, l);
      v[e] = sp == 0 ? h : sp == 1 ? m : l;
    }
    *reinterpret_cast<bf16x4*>(Dp + n * DS + 2 * k) = v;
  }
  __syncthreads();
  // ---- phase 1: dA on the MFMA, wave w takes blocks w, w + 8, ...
  {
    const int n0 = li, n1 = 16 + li;
    const unsigned char* db0 = Dp + min(n0, NR - 1) * DS + 16 * g;
    const unsigned char* db1 = Dp + min(n1, NR - 1) * DS + 16 * g;
    const bf16x8 zero8 = {};
    for (int b = wave; b < nb; b += NW) {
      Blk nxt;
      if (b + NW < nb) bfetch(16 * (b + NW), nxt);
      bf16x8 a[10];
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) a[kk] = __builtin_bit_cast(bf16x8, cur.o[kk]);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const f32x4 x0 = __builtin_bit_cast(f32x4, cur.s[2 * h]), x1 = __builtin_bit_cast(f32x4, cur.s[2 * h + 1]);
        bf16x8 hi, mi, lo;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          __bf16 th, tm, tl;
          am_split(e < 4 ? x0[e] : x1[e - 4], th, tm, tl);
          hi[e] = th;
          mi[e] = tm;
          lo[e] = tl;
        }
        a[4 + h] = hi;
        a[6 + h] = mi;
        a[8 + h] = lo;
      }
      f32x4 acc[NTN];
#pragma unroll
      for (int n = 0; n < NTN; ++n) acc[n] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 10; ++ks) {
        bf16x8 w0 = *reinterpret_cast<const bf16x8*>(db0 + 64 * ks);
        if (n0 >= NR) w0 = zero8;
        acc[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[ks], w0, acc[0], 0, 0, 0);
        if constexpr (NTN == 2) {
          bf16x8 w1 = *reinterpret_cast<const bf16x8*>(db1 + 64 * ks);
          if (n1 >= NR) w1 = zero8;
          acc[NTN - 1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[ks], w1, acc[NTN - 1], 0, 0, 0);
        }
      }
      // lane (g, li) holds D[position p0 + 4g + r][n = li (+16)]: the parts of q are n = q, NQ + q, 2 NQ + q
      const int p0 = 16 * b;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v0 = acc[0][r];
        float v;
        if constexpr (NQ == 4) v = v0 + __shfl_down(v0, 4, 64) + __shfl_down(v0, 8, 64);
        else v = v0 + __shfl_down(v0, 8, 64) + acc[NTN - 1][r];
        const int p = p0 + 4 * g + r;
        if (li < NQ && p < P) dA[p * NQ + li] = v;
      }
      if (g == 0 && p0 + li < P) {   // the key channels O[p][0..7] for dQ
        const u32x4 k = cur.o[0];
        *reinterpret_cast<f32x4*>(Kc + (p0 + li) * 8) = bf4_f32(u32x2{k.x, k.y});
        *reinterpret_cast<f32x4*>(Kc + (p0 + li) * 8 + 4) = bf4_f32(u32x2{k.z, k.w});
      }
      cur = nxt;
    }
  }
  __syncthreads();
  // ---- phases 2-4 as k_attn_bwd
  // softmax backward: dlogit = A (dA - sum_p A dA)
  for (int q = wave; q < NQ; q += NW) {
    float s = 0.f;
    for (int p = lane; p < P; p += 64) s += A[p * NQ + q] * dA[p * NQ + q];
    s = wave_sum(s);
    if (lane == 0) ss[q] = s;
  }
  __syncthreads();
  for (int i = tid; i < P * NQ; i += NT) {
    const int q = i - (i / NQ) * NQ;
    dA[i] = A[i] * (dA[i] - ss[q]);
  }
  __syncthreads();
  // dO[p][c4..c4+3] = sum_q w[p][q] coef[q][0..3]: key channels (c4 < 8) w = dlogit, coef = Q[q][c4..];
  // the rest w = A, coef = da[q][c4-8..]
  float* dOf = dO + (size_t)f * P * 128;
  auto dO_pos = [&](int p, const f32x4 (&coef)[NQ], const float* W) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < NQ / 4; ++j) {
      const f32x4 w = *reinterpret_cast<const f32x4*>(W + p * NQ + 4 * j);
#pragma unroll
      for (int i = 0; i < 4; ++i) acc += w[i] * coef[4 * j + i];
    }
    return acc;
  };
  if (cqm) {   // quad-major: a wave per channel quad, lanes along the positions (1-KB stores)
    for (int qd = wave; qd < 32; qd += NW) {
      const int c4 = qd * 4;
      f32x4 coef[NQ];
#pragma unroll
      for (int q = 0; q < NQ; ++q)
        coef[q] = *reinterpret_cast<const f32x4*>(c4 < 8 ? Qs + q * 72 + c4 : da + q * 184 + c4 - 8);
      const float* W = c4 < 8 ? dA : A;
      for (int p = lane; p < P; p += 64)
        *reinterpret_cast<f32x4*>(dOf + ((size_t)qd * P + p) * 4) = dO_pos(p, coef, W);
    }
  } else {     // row-major: lanes along a row's 32 quads, 16 positions per pass (512-B stores)
    const int qd = lane & 31, c4 = qd * 4;
    f32x4 coef[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const f32x4 cq = *reinterpret_cast<const f32x4*>(Qs + q * 72 + min(c4, 4));
      const f32x4 cd = *reinterpret_cast<const f32x4*>(da + q * 184 + max(c4 - 8, 0));
      coef[q] = c4 < 8 ? cq : cd;
    }
    for (int p = 2 * wave + (lane >> 5); p < P; p += 2 * NW) {
      const f32x4 a = dO_pos(p, coef, A), d = dO_pos(p, coef, dA);
      *reinterpret_cast<f32x4*>(dOf + (size_t)p * 128 + c4) = c4 < 8 ? d : a;
    }
  }
  // dQ[q][c] = sum_p dlogit[p][q] K[p][c], K = [O[:8] (Kc) | S]: G position groups, partials through LDS
  if (tid < G * 72) {
    const int gg = tid / 72, c = tid - gg * 72;
    float acc[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) acc[q] = 0.f;
    const float* ks = S + max(c - 8, 0);
    const float* kc = Kc + min(c, 7);
#pragma unroll 8
    for (int p = gg; p < P; p += G) {
      const float kS = ks[p * 64], kO = kc[p * 8];
      const float k = c < 8 ? kO : kS;
#pragma unroll
      for (int q = 0; q < NQ; ++q) acc[q] += dA[p * NQ + q] * k;
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q) red[(gg * NQ + q) * 72 + c] = acc[q];
  }
  __syncthreads();
  for (int i = tid; i < NQ * 72; i += NT) {
    float acc = 0.f;
#pragma unroll 4
    for (int gg = 0; gg < G; ++gg) acc += red[gg * NQ * 72 + i];
    if (addq) acc += dAns[(size_t)f * da_ld + NQ * 184 + i];   // the answer row's copy of Q (stateful core)
    dQp[(size_t)f * NQ * 72 + i] = acc;
  }
}

}  // namespace aaa
