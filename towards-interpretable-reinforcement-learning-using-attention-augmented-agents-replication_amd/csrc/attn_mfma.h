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
template <int NQ, bool NTL_>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(NQ == 8 ? 4 : 3)))
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
    if (SQ) {
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

}  // namespace aaa
