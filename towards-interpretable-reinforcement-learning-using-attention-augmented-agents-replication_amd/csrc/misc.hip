// Non-GEMM kernels of the attention-agent path: constant query MLP, fused
// spatial-softmax attention readout (fwd/bwd), column reductions, the last
// BPTT gate step, and parameter (un)packing.
#include <cstdlib>
#include <type_traits>

#include "misc.h"

namespace aaa {

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
// Workgroup barrier that drains only the LDS counter: global loads issued
// before it stay in flight (a __syncthreads fence would wait for them).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// y[k] += sum over this workgroup's rows o of W[o*ldw + k] x[o]  (multi-WG, atomics)
__global__ void k_gemv_cols_atomic(const float* __restrict__ W, int ldw, const float* __restrict__ x, int N, int K,
                                   int rows_per, float* y) {
  const int o0 = blockIdx.x * rows_per, o1 = min(N, o0 + rows_per);
  for (int k = threadIdx.x; k < K; k += blockDim.x) {
    float s = 0.f;
#pragma unroll 8
    for (int o = o0; o < o1; ++o) s += W[(size_t)o * ldw + k] * x[o];
    atomicAdd(y + k, s);
  }
}

// ---------------------------------------------------------------------------
// QueryNetwork on the always-zero prev_output (attention.py:184-198, 325-331;
// Q1): q1 = relu(b0), q2 = relu(W2 q1 + b2), Q = W4 q2 + b4.  Also the basis
// half of the attention logits, SQ[p][q] = sum_c S[p][c] * Q[q][8 + c].
// One wave per output row, 4 rows per workgroup, so the weight rows stream in
// from many CUs at once (a single workgroup was latency-bound at ~80 us):
// y[o] = act(sum_k W[o][k] act_in(x[k]) + b[o]).  xcopy (optional) <- act_in(x).
__global__ void __launch_bounds__(256)
k_query_layer(const float* __restrict__ W, int K, const float* __restrict__ x, int relu_in,
              const float* __restrict__ b, int relu_out, int N, float* __restrict__ y, float* __restrict__ xcopy) {
  const int lane = threadIdx.x & 63, o = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (xcopy && blockIdx.x == 0)
    for (int k = threadIdx.x; k < K; k += 256) xcopy[k] = relu_in ? fmaxf(x[k], 0.f) : x[k];
  if (o >= N) return;
  float s = 0.f;
  for (int k = lane; k < K; k += 64) {
    const float xk = relu_in ? fmaxf(x[k], 0.f) : x[k];
    s += W[(size_t)o * K + k] * xk;
  }
  s = wave_sum(s) + b[o];
  if (lane == 0) y[o] = relu_out ? fmaxf(s, 0.f) : s;
}

// Basis half of the attention logits, SQ[p][q] = sum_c S[p][c] * Q[q][8 + c]:
// one wave per grid position, lanes over the 64 basis channels.
__global__ void __launch_bounds__(256)
k_query_sq(const float* __restrict__ S, const float* __restrict__ Q, int P, int nq, float* __restrict__ SQ) {
  const int lane = threadIdx.x & 63, p = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (p >= P) return;
  const float sv = S[p * 64 + lane];
  for (int q = 0; q < nq; ++q) {
    const float acc = wave_sum(sv * Q[q * 72 + 8 + lane]);
    if (lane == 0) SQ[p * nq + q] = acc;
  }
}

// ---------------------------------------------------------------------------
// Fused attention readout, one workgroup per frame (attention.py:319-348):
// logits A[p][q] = K[p]·Q[q] with K = [O[:8] | S], softmax over the P grid
// positions (spatial_softmax), readout a[q] = sum_p A[p][q] [O[8:] | S][p],
// and the answer row [a_0..a_nq-1 | Q_0..Q_nq-1 | r | a_prev | 0-pad].
// HBM-bound: every load of the frame is issued before the first wait -- the
// key channels by the logit threads (one position each) and the first
// kAttnPre positions of each readout thread's V slice straight into
// registers -- so the frame's O rows stream in as one burst (no load phase
// behind the softmax).
//   fp32 O (TO = float, rows of 128): readout thread (g, sl) takes 4-column
// group g of the 184 V columns (46 groups, 16 B per lane, consecutive lanes
// along a row), position slice sl of SL; slices summed through LDS.
//   bf16 O (TO = __bf16, the h half of the XH rows, pitch ``old``): waves 0-3
// read O (30 groups of 4 channels, 8 B per lane), waves 4-7 read S (32 groups
// of 2 channels, 8 B per lane), kAttnSlicesBf slices each -- one load width
// for every lane (the prefetch is one straight-line burst) and the compute
// branch is wave-uniform.
constexpr int kAttnFwdThreads = 512;
constexpr int kAttnSlices = 11;         // default position slices of the readout (46 * 11 = 506 threads)
constexpr int kAttnSlicesBf = 8;        // bf16 O: 256 threads over 30 O groups / 32 S groups
template <int NQ, int PRE, int SL, typename TO>
__global__ void __launch_bounds__(kAttnFwdThreads) __attribute__((amdgpu_waves_per_eu(PRE > 0 || NQ > 4 ? 4 : 8)))
k_attn_fwd(const TO* __restrict__ Hs, int old, const float* __restrict__ S, const float* __restrict__ Q, int qs,
           const float* __restrict__ SQ, const float* __restrict__ pr, const float* __restrict__ pa,
           int P, float* __restrict__ Am, float* __restrict__ ans, int ans_ld) {
  constexpr bool BF = !std::is_same<TO, float>::value;
  constexpr int kAttnPre = PRE;   // V positions per readout thread loaded before the first wait
  constexpr int NSL = BF ? kAttnSlicesBf : SL;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* L = sm;                         // P*NQ
  float* Qs = L + P * NQ;                // NQ*72
  float* red = Qs + NQ * 72;             // NSL * NQ * 184
  const int f = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const TO* O = Hs + (size_t)f * P * old;
  const float* Qf = Q + (size_t)f * qs;   // qs = 0: one query for every frame (Q1)
  // the queries first (their LDS copy below then waits only for them), then
  // the first logit position's keys, then this thread's V slice head
  static_assert(NQ * 72 <= 2 * kAttnFwdThreads, "two query elements per thread");
  const int qi1 = min(tid + kAttnFwdThreads, NQ * 72 - 1);
  const float qv0 = Qf[min(tid, NQ * 72 - 1)], qv1 = Qf[qi1];
  // position tid's keys and (constant query) basis logits: unconditional
  // loads from a clamped valid position, used only when tid < P
  const int p0 = min(tid, P - 1);
  // key channels 0..7 of position p, raw (converted at their use, not here)
  auto key_raw = [&](int p) {
    if constexpr (BF) {
      return *reinterpret_cast<const u32x4*>(O + (size_t)p * old);
    } else {
      struct { f32x4 a, b; } k{*reinterpret_cast<const f32x4*>(O + (size_t)p * old),
                               *reinterpret_cast<const f32x4*>(O + (size_t)p * old + 4)};
      return k;
    }
  };
  const auto k0 = key_raw(p0);
  f32x4 sq[NQ / 4];
#pragma unroll
  for (int j = 0; j < NQ / 4; ++j)
    sq[j] = SQ ? *reinterpret_cast<const f32x4*>(SQ + p0 * NQ + 4 * j) : f32x4{0.f, 0.f, 0.f, 0.f};
  // readout slice of this thread: g = column group, sl = position slice
  bool isO, rd;
  int g, sl;
  const char* src;   // column group g of position 0
  size_t ldb;        // bytes per position
  if constexpr (BF) {
    isO = tid < 256;
    const int t2 = isO ? tid : tid - 256;
    g = isO ? t2 % 30 : t2 & 31;
    sl = isO ? t2 / 30 : t2 >> 5;
    rd = sl < NSL;
    src = isO ? (const char*)(O + 8 + 4 * g) : (const char*)(S + 2 * g);
    ldb = isO ? (size_t)old * 2 : 256;
  } else {
    isO = true;
    rd = tid < 46 * SL;
    g = tid % 46;
    sl = tid / 46;
    src = g < 30 ? (const char*)(O + 8 + 4 * g) : (const char*)(S + 4 * (g - 30));
    ldb = g < 30 ? (size_t)old * 4 : 256;
  }
  using VR = typename std::conditional<BF, u32x2, f32x4>::type;   // one position's load of this lane
  VR pre[kAttnPre > 0 ? kAttnPre : 1];
#pragma unroll
  for (int i = 0; i < kAttnPre; ++i) {
    // unconditional load from a valid address (a select on the loaded value
    // would wait for it here); positions past P are skipped at their use
    const int p = min(sl + i * NSL, P - 1);
    pre[i] = *reinterpret_cast<const VR*>(src + (size_t)p * ldb);
  }
  if (tid < NQ * 72) Qs[tid] = qv0;
  if (tid + kAttnFwdThreads < NQ * 72) Qs[tid + kAttnFwdThreads] = qv1;
  __syncthreads();
  // logits: one thread per position, all NQ queries (its 8 key channels read once)
  auto logits = [&](int p, const auto& kr, const f32x4* sqp) {
    f32x4 ka, kb;
    if constexpr (BF) {
      ka = bf4_f32(u32x2{kr.x, kr.y});
      kb = bf4_f32(u32x2{kr.z, kr.w});
    } else {
      ka = kr.a;
      kb = kr.b;
    }
    float acc[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const float* qq = Qs + q * 72;
      acc[q] = ka[0] * qq[0] + ka[1] * qq[1] + ka[2] * qq[2] + ka[3] * qq[3] +
               kb[0] * qq[4] + kb[1] * qq[5] + kb[2] * qq[6] + kb[3] * qq[7];
    }
    if (SQ) {
#pragma unroll
      for (int q = 0; q < NQ; ++q) acc[q] += sqp[q / 4][q % 4];
    } else {   // per-frame query: the basis half of the logit here
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
    for (int q = 0; q < NQ; ++q) L[p * NQ + q] = acc[q];
  };
  if (tid < P) logits(tid, k0, sq);
  for (int p = tid + kAttnFwdThreads; p < P; p += kAttnFwdThreads) {   // grids past 512 positions
    const auto kp = key_raw(p);
    f32x4 sp[NQ / 4];
#pragma unroll
    for (int j = 0; j < NQ / 4; ++j)
      sp[j] = SQ ? *reinterpret_cast<const f32x4*>(SQ + p * NQ + 4 * j) : f32x4{0.f, 0.f, 0.f, 0.f};
    logits(p, kp, sp);
  }
  __syncthreads();
  for (int q = wave; q < NQ; q += kAttnFwdThreads / 64) {
    float m = -INFINITY;
    for (int p = lane; p < P; p += 64) m = fmaxf(m, L[p * NQ + q]);
    m = wave_max(m);
    float s = 0.f;
    for (int p = lane; p < P; p += 64) { float e = expf(L[p * NQ + q] - m); L[p * NQ + q] = e; s += e; }
    s = wave_sum(s);
    const float inv = 1.f / s;
    for (int p = lane; p < P; p += 64) {
      const float a = L[p * NQ + q] * inv;
      L[p * NQ + q] = a;
      Am[((size_t)f * P + p) * NQ + q] = a;
    }
  }
  __syncthreads();
  // readout: the prefetched head of the slice, then the rest (large grids)
  // CW channels of this lane: 4 (fp32; bf16 O) or 2 (bf16 path's S lanes)
  auto readout = [&](auto cw) {
    constexpr int CW = decltype(cw)::value;
    auto cvt = [&](const VR& r) {
      if constexpr (!BF) return r;
      else if constexpr (CW == 4) return bf4_f32(r);
      else return f32x4{__uint_as_float(r.x), __uint_as_float(r.y), 0.f, 0.f};
    };
    float acc[NQ][CW];
#pragma unroll
    for (int q = 0; q < NQ; ++q)
#pragma unroll
      for (int k = 0; k < CW; ++k) acc[q][k] = 0.f;
    auto fma_pos = [&](int p, const f32x4& v) {
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const float a = L[p * NQ + q];
#pragma unroll
        for (int k = 0; k < CW; ++k) acc[q][k] += a * v[k];
      }
    };
#pragma unroll
    for (int i = 0; i < kAttnPre; ++i) {
      const int p = sl + i * NSL;
      if (p < P) fma_pos(p, cvt(pre[i]));
    }
    // (a ring refilling each prefetch slot as it is consumed -- kAttnPre loads in flight
    // through the whole slice -- measured slower: C5 203 vs 190 us, profiles/r05/ab/attn_fwd_ring/)
#pragma unroll 4
    for (int p = sl + kAttnPre * NSL; p < P; p += NSL)
      fma_pos(p, cvt(*reinterpret_cast<const VR*>(src + (size_t)p * ldb)));
    // column of this lane's first channel in the 184 V columns
    const int col = BF ? (isO ? 4 * g : 120 + 2 * g) : 4 * g;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      float* r = red + (sl * NQ + q) * 184 + col;
      if constexpr (CW == 4) *reinterpret_cast<f32x4*>(r) = f32x4{acc[q][0], acc[q][1], acc[q][2], acc[q][3]};
      else *reinterpret_cast<float2*>(r) = float2{acc[q][0], acc[q][1]};
    }
  };
  if (rd) {
    if (!BF || isO) readout(std::integral_constant<int, 4>{});   // wave-uniform (bf16: waves 0-3)
    else readout(std::integral_constant<int, 2>{});
  }
  __syncthreads();
  float* arow = ans + (size_t)f * ans_ld;
  for (int i = tid; i < NQ * 184; i += kAttnFwdThreads) {
    float v = 0.f;
#pragma unroll
    for (int s2 = 0; s2 < NSL; ++s2) v += red[s2 * NQ * 184 + i];
    arow[i] = v;
  }
  for (int i = tid; i < NQ * 72; i += kAttnFwdThreads) arow[NQ * 184 + i] = Qs[i];
  for (int i = NQ * 256 + tid; i < ans_ld; i += kAttnFwdThreads) {
    float v = 0.f;
    if (i == NQ * 256) v = pr ? pr[f] : 0.f;
    else if (i == NQ * 256 + 1) v = pa ? pa[f] : 0.f;
    arow[i] = v;
  }
}

}  // namespace aaa
#include "attn_mfma.h"
namespace aaa {

#ifdef AAA_STAMPS
// Diagnostic builds only (tools/ubench/attn_stamps): per-workgroup phase stamps (s_memrealtime, 100 MHz).
__device__ uint64_t aaa_attn_stamps[16384 * 8];
#define AAA_AT_STAMP(k)                                                                                      \
  do {                                                                                                       \
    if (threadIdx.x == 0 && blockIdx.x < 16384) aaa_attn_stamps[blockIdx.x * 8 + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define AAA_AT_STAMP(k) do {} while (0)
#endif

// Backward of the readout / softmax / logits for one frame: from da (the
// answer-gradient's readout part) to dO (grad of the ConvLSTM output h_t) and
// this frame's dQ (logits path, plus the answer row's Q columns when addq).
//
// Latency-bound per frame (a few hundred KB of traffic), so every phase keeps
// all 512 threads busy and issues its global loads up front:
//  1. dA[p][q] = sum_c da[q][c] V[p][c], V = [O[8:128] | S]: 8 lanes per
//     position, each streaming 16-B pieces of the V row straight from memory
//     (no LDS staging, no barrier in the loop) against da from LDS; the 8
//     partials meet in a 3-step transpose reduction (lane j ends with q = j).
//     The same lanes park the position's key channels O[:8] in LDS (Kc).
//  2. softmax backward: dlogit = A (dA - sum_p A dA).
//  3. dO (16 B per thread): each thread's channel quad fixed, its NQ
//     coefficients (da columns, or Q for the key channels) in registers, per
//     position only the NQ weights (A or dlogit) read from LDS; row-major
//     rows, or channel-quad-major slices (cqm, recur.h cqm4) in 1-KB runs.
//  4. dQ[q][c] = sum_p dlogit[p][q] K[p][c], K = [O[:8] (Kc) | S], G position
//     groups reduced through LDS.
// Pieces of a V row: O = 30 fp32 quads or 15 bf16 octets (one padding piece
// pads them to a multiple of 8 lanes), then S = 16 fp32 quads.
template <int NQ, typename TO, int PPL>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4)))   // two frames per CU
k_attn_bwd(const TO* __restrict__ Hs, int old, const float* __restrict__ S, const float* __restrict__ Q, int qs,
           const float* __restrict__ Am, const float* __restrict__ dAns, int da_ld, int addq, int P,
           float* __restrict__ dO, float* __restrict__ dQp, int cqm) {
  constexpr int NT = 512, NW = NT / 64;
  constexpr int G = 7;             // position groups of the dQ reduction (7*72 <= NT)
  constexpr bool BF = !std::is_same<TO, float>::value;
  constexpr int NOP = BF ? 15 : 30, NOPP = BF ? 16 : 32;   // O pieces, padded to 8 lanes
  constexpr int NK = (NOPP + 16) / 8, NKO = NOPP / 8;      // pieces per lane: all, O
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* A = sm;                 // P*NQ
  float* dA = A + P * NQ;        // P*NQ  (becomes dlogits)
  float* da = dA + P * NQ;       // NQ*184
  float* Qs = da + NQ * 184;     // NQ*72
  float* ss = Qs + NQ * 72;      // NQ (padded to 8)
  float* red = ss + 8;           // G*NQ*72
  float* Kc = red + G * NQ * 72; // P*8  key channels O[:8] as fp32
  const int f = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const TO* O = Hs + (size_t)f * P * old;
  AAA_AT_STAMP(0);
  // phase 1: 64 * PPL positions per pass, 8 lanes each; a lane takes PPL positions
  // (64 apart) with the same channel pieces, so each da read from LDS (the phase's
  // bound: NQ 16-B reads per piece) serves PPL positions
  const int part = tid & 7, pl = tid >> 3;
  constexpr int PPS = 64 * PPL;
  // the V pieces and key piece of position p: unconditional loads from valid
  // (clamped) addresses; a padding piece is zeroed at its use
  auto vload = [&](int p, u32x4 (&raw)[NK], u32x4& kraw) {
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      const int j = part + 8 * k;
      const void* src;
      if (k < NKO) src = O + (size_t)p * old + 8 + min(j, NOP - 1) * (BF ? 8 : 4);
      else src = S + p * 64 + 4 * (j - NOPP);
      raw[k] = *reinterpret_cast<const u32x4*>(src);
    }
    kraw = *reinterpret_cast<const u32x4*>(O + (size_t)p * old + (BF ? 0 : 4 * (part & 1)));
  };
  u32x4 raw[PPL][NK], kraw[PPL];
#pragma unroll
  for (int u = 0; u < PPL; ++u) vload(min(pl + 64 * u, P - 1), raw[u], kraw[u]);
  for (int i = tid; i < P * NQ; i += NT) A[i] = Am[(size_t)f * P * NQ + i];
  for (int i = tid; i < NQ * 184; i += NT) da[i] = dAns[(size_t)f * da_ld + i];
  for (int i = tid; i < NQ * 72; i += NT) Qs[i] = Q[(size_t)f * qs + i];
  __syncthreads();
  AAA_AT_STAMP(1);
  for (int p0 = 0; p0 < P; p0 += PPS) {
    // da's LDS reads stay inside the pass: hoisted out of the loop they would
    // hold NQ x 184 / 8 floats per lane in registers (spills)
    int opq = 0;
    asm volatile("" : "+v"(opq));
    const float* dap = da + opq;
    // packed accumulators: each pair of channels on one v_pk_fma_f32 (the pass is VALU-bound
    // once PPL positions share the da reads); the halves are summed after the last piece
    f32x2 acc2[PPL][NQ];
#pragma unroll
    for (int u = 0; u < PPL; ++u)
#pragma unroll
      for (int q = 0; q < NQ; ++q) acc2[u][q] = f32x2{0.f, 0.f};
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      const int j = part + 8 * k;
      if (k < NKO && BF) {   // 8 bf16 channels of O
        const float m = j < NOP ? 1.f : 0.f;
        f32x4 v0[PPL], v1[PPL];
#pragma unroll
        for (int u = 0; u < PPL; ++u) {
          v0[u] = bf4_f32(u32x2{raw[u][k].x, raw[u][k].y}) * m;
          v1[u] = bf4_f32(u32x2{raw[u][k].z, raw[u][k].w}) * m;
        }
        const int c0 = 8 * min(j, NOP - 1);
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
          const f32x4 d0 = *reinterpret_cast<const f32x4*>(dap + q * 184 + c0);
          const f32x4 d1 = *reinterpret_cast<const f32x4*>(dap + q * 184 + c0 + 4);
#pragma unroll
          for (int u = 0; u < PPL; ++u) {
            f32x2 a = acc2[u][q];
            a = __builtin_elementwise_fma(f32x2{v0[u][0], v0[u][1]}, f32x2{d0[0], d0[1]}, a);
            a = __builtin_elementwise_fma(f32x2{v0[u][2], v0[u][3]}, f32x2{d0[2], d0[3]}, a);
            a = __builtin_elementwise_fma(f32x2{v1[u][0], v1[u][1]}, f32x2{d1[0], d1[1]}, a);
            a = __builtin_elementwise_fma(f32x2{v1[u][2], v1[u][3]}, f32x2{d1[2], d1[3]}, a);
            acc2[u][q] = a;
          }
        }
      } else {               // 4 fp32 channels (O quads of the fp32 path, or S)
        const float m = k < NKO ? (j < NOP ? 1.f : 0.f) : 1.f;
        f32x4 v[PPL];
#pragma unroll
        for (int u = 0; u < PPL; ++u) v[u] = __builtin_bit_cast(f32x4, raw[u][k]) * m;
        const int c0 = k < NKO ? 4 * min(j, NOP - 1) : 120 + 4 * (j - NOPP);
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
          const f32x4 d = *reinterpret_cast<const f32x4*>(dap + q * 184 + c0);
#pragma unroll
          for (int u = 0; u < PPL; ++u) {
            f32x2 a = acc2[u][q];
            a = __builtin_elementwise_fma(f32x2{v[u][0], v[u][1]}, f32x2{d[0], d[1]}, a);
            a = __builtin_elementwise_fma(f32x2{v[u][2], v[u][3]}, f32x2{d[2], d[3]}, a);
            acc2[u][q] = a;
          }
        }
      }
      // one piece's da reads at a time: the next piece's addresses depend on
      // this piece's sums (scheduled all up front the reads need NK * NQ * 4
      // registers and spill)
#pragma unroll
      for (int u = 0; u < PPL; ++u)
#pragma unroll
        for (int q = 0; q < NQ; ++q) asm volatile("" : "+v"(acc2[u][q]));
      asm volatile("" : "+v"(opq));
      dap = da + opq;
    }
    float acc[PPL][NQ];
#pragma unroll
    for (int u = 0; u < PPL; ++u)
#pragma unroll
      for (int q = 0; q < NQ; ++q) acc[u][q] = acc2[u][q][0] + acc2[u][q][1];
    u32x4 kr[PPL];
#pragma unroll
    for (int u = 0; u < PPL; ++u) kr[u] = kraw[u];
    if (p0 + PPS < P) {   // the next pass's pieces in flight
#pragma unroll
      for (int u = 0; u < PPL; ++u) vload(min(p0 + PPS + pl + 64 * u, P - 1), raw[u], kraw[u]);
    }
#pragma unroll
    for (int u = 0; u < PPL; ++u) {
      const int p = p0 + pl + 64 * u;
      // 3-step transpose reduction over the 8 lanes of the position: lane part
      // ends with the total of q = part (NQ = 8) or part & 3 (NQ = 4)
      float v[NQ];
#pragma unroll
      for (int q = 0; q < NQ; ++q) v[q] = acc[u][q];
      if constexpr (NQ == 4) {
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] += __shfl_xor(v[q], 4, 64);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const bool up = part & 4;
          const float keep = up ? v[i + 4] : v[i], send = up ? v[i] : v[i + 4];
          v[i] = keep + __shfl_xor(send, 4, 64);
        }
      }
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const bool up = part & 2;
        const float keep = up ? v[i + 2] : v[i], send = up ? v[i] : v[i + 2];
        v[i] = keep + __shfl_xor(send, 2, 64);
      }
      {
        const bool up = part & 1;
        const float keep = up ? v[1] : v[0], send = up ? v[0] : v[1];
        v[0] = keep + __shfl_xor(send, 1, 64);
      }
      if (p < P) {
        if (part < NQ) dA[p * NQ + part] = v[0];
        if constexpr (BF) {
          if (part == 0) {
            *reinterpret_cast<f32x4*>(Kc + p * 8) = bf4_f32(u32x2{kr[u].x, kr[u].y});
            *reinterpret_cast<f32x4*>(Kc + p * 8 + 4) = bf4_f32(u32x2{kr[u].z, kr[u].w});
          }
        } else {
          if (part < 2) *reinterpret_cast<u32x4*>(Kc + p * 8 + 4 * part) = kr[u];
        }
      }
    }
  }
  __syncthreads();
  AAA_AT_STAMP(2);
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
  AAA_AT_STAMP(3);
  // dO[p][c4..c4+3] = sum_q w[p][q] coef[q][0..3]: key channels (c4 < 8) w =
  // dlogit, coef = Q[q][c4..]; the rest w = A, coef = da[q][c4-8..]
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
    for (int q = 0; q < NQ; ++q) {   // both candidates read, then selected (no divergent branch)
      const f32x4 cq = *reinterpret_cast<const f32x4*>(Qs + q * 72 + min(c4, 4));
      const f32x4 cd = *reinterpret_cast<const f32x4*>(da + q * 184 + max(c4 - 8, 0));
      coef[q] = c4 < 8 ? cq : cd;
    }
    for (int p = 2 * wave + (lane >> 5); p < P; p += 2 * NW) {
      const f32x4 a = dO_pos(p, coef, A), d = dO_pos(p, coef, dA);
      *reinterpret_cast<f32x4*>(dOf + (size_t)p * 128 + c4) = c4 < 8 ? d : a;
    }
  }
  AAA_AT_STAMP(4);
  // dQ[q][c] = sum_p dlogit[p][q] K[p][c], K = [O[:8] (Kc) | S]: G position
  // groups, every K element feeding all NQ heads, partials reduced through LDS
  if (tid < G * 72) {
    const int g = tid / 72, c = tid - g * 72;
    float acc[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) acc[q] = 0.f;
    const float* ks = S + max(c - 8, 0);
    const float* kc = Kc + min(c, 7);
#pragma unroll 8
    for (int p = g; p < P; p += G) {
      const float kS = ks[p * 64], kO = kc[p * 8];   // both read, then selected
      const float k = c < 8 ? kO : kS;
#pragma unroll
      for (int q = 0; q < NQ; ++q) acc[q] += dA[p * NQ + q] * k;
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q) red[(g * NQ + q) * 72 + c] = acc[q];
  }
  __syncthreads();
  AAA_AT_STAMP(5);
  for (int i = tid; i < NQ * 72; i += NT) {
    float acc = 0.f;
#pragma unroll 4
    for (int g = 0; g < G; ++g) acc += red[g * NQ * 72 + i];
    if (addq) acc += dAns[(size_t)f * da_ld + NQ * 184 + i];   // the answer row's copy of Q (stateful core)
    dQp[(size_t)f * NQ * 72 + i] = acc;
  }
  AAA_AT_STAMP(6);
}

// Backward of the query MLP (one workgroup of 1024 threads).  dQ = sum over
// frames of the logits-path grads + the answer-path grad, which summed over
// rows is W1[:, Q-cols]^T . db1.
// y[k] = (mask[k] > 0) * sum_o W[o][k] x[o]  for W [N][K]: lanes over 64
// columns, 16 waves split the rows, LDS reduce.  grid ceil(K/64), 1024 threads.
__global__ void __launch_bounds__(1024)
k_query_colgemv(const float* __restrict__ W, int N, int K, const float* __restrict__ x,
                const float* __restrict__ mask, float* __restrict__ y) {
  __shared__ float red[16][64];
  const int lane = threadIdx.x & 63, g = threadIdx.x >> 6, k = blockIdx.x * 64 + lane;
  float s = 0.f;
  if (k < K) {
#pragma unroll 4
    for (int o = g; o < N; o += 16) s += W[(size_t)o * K + k] * x[o];
  }
  red[g][lane] = s;
  __syncthreads();
  if (g == 0 && k < K) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < 16; ++w) t += red[w][lane];
    y[k] = mask[k] > 0.f ? t : 0.f;
  }
}

// k_query_colgemv (blocks [0, cgb)) and k_query_outer (the rest, 1024 threads each) in one
// launch: the two products of a query layer's backward that need the same input gradient
__global__ void __launch_bounds__(1024)
k_query_colgemv_outer(const float* __restrict__ W, int N, int K, const float* __restrict__ x,
                      const float* __restrict__ mask, float* __restrict__ y, int cgb, const float* __restrict__ a,
                      int Na, const float* __restrict__ bv, int Kb, float* __restrict__ out, float* acopy) {
  if ((int)blockIdx.x < cgb) {
    __shared__ float red[16][64];
    const int lane = threadIdx.x & 63, g = threadIdx.x >> 6, k = blockIdx.x * 64 + lane;
    float s = 0.f;
    if (k < K) {
#pragma unroll 4
      for (int o = g; o < N; o += 16) s += W[(size_t)o * K + k] * x[o];
    }
    red[g][lane] = s;
    __syncthreads();
    if (g == 0 && k < K) {
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < 16; ++w) t += red[w][lane];
      y[k] = mask[k] > 0.f ? t : 0.f;
    }
    return;
  }
  const int n = Na * Kb, ob = (int)gridDim.x - cgb;
  for (int i = ((int)blockIdx.x - cgb) * 1024 + (int)threadIdx.x; i < n; i += ob * 1024) {
    const int o = i / Kb;
    out[i] = a[o] * bv[i - o * Kb];
    if (acopy && i < Na) acopy[i] = a[i];
  }
}

// out[o][k] = a[o] * b[k] (weight grad of a rank-1 layer), acopy <- a (bias grad).
__global__ void k_query_outer(const float* __restrict__ a, int N, const float* __restrict__ b, int K,
                              float* __restrict__ out, float* acopy) {
  const int n = N * K;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int o = i / K;
    out[i] = a[o] * b[i - o * K];
    if (acopy && i < N) acopy[i] = a[i];
  }
}

// out[n] += sum_{m} X[m*ld + n]; grid (ceil(N/64), nsplit), 256 threads.
template <typename TI>
__global__ void k_colsum(const TI* __restrict__ X, int ld, int M, int N, int rows_per, float* out) {
  __shared__ float red[256];
  const int col = blockIdx.x * 64 + (threadIdx.x & 63);
  const int r0 = blockIdx.y * rows_per, r1 = min(M, r0 + rows_per);
  float s = 0.f;
  if (col < N) {
#pragma unroll 8
    for (int r = r0 + (threadIdx.x >> 6); r < r1; r += 4) s += (float)X[(size_t)r * ld + col];
  }
  red[threadIdx.x] = s;
  __syncthreads();
  if (threadIdx.x < 64 && col < N) {
    float t = red[threadIdx.x] + red[threadIdx.x + 64] + red[threadIdx.x + 128] + red[threadIdx.x + 192];
    atomicAdd(out + col, t);
  }
}

// Gate backward of the LAST step (t = T-1): dh = dO + dhT, dc = carry (dcT).
// One workgroup per tile of ``bj`` pixels (the BPTT GEMM's column tile), 128
// channels x 4 pixel lanes; dz is stored as TZ and, when ``part`` is set, the
// tile's fp32 gate-bias partials go to part[tile][512] (EpiConvLstmBwd::flush).
// nsl > 1: dhT holds nsl split-K partials (stride sls floats) of the BPTT dgrad
// (EpiSliceT), summed in slice order -- the gate backward of any step t-1 of a
// split-K BPTT chain (rt_backward.hip tiles 30/31).
template <typename TZ, typename GT>
__global__ void __launch_bounds__(512)
k_gate_bwd_last(int M, int bj, const float* __restrict__ dO, const float* __restrict__ dhT,
                const GT* __restrict__ gates, const float* __restrict__ cprev, const float* __restrict__ ccur,
                float* dC, TZ* dz, float* part, int nsl, size_t sls) {
  __shared__ f32x4 red[4][128];
  const int ch = threadIdx.x & 127, sl = threadIdx.x >> 7;
  const int m0 = blockIdx.x * bj, m1 = min(M, m0 + bj);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
  for (int m = m0 + sl; m < m1; m += 4) {
    const size_t idx = (size_t)m * 128 + ch;
    float dh = dO[idx];
#pragma unroll
    for (int k = 0; k < 8; ++k)   // <= kBpttSplitMax slices, summed in order
      if (k < nsl) dh += dhT[k * sls + idx];
    const f32x4 g = load_gates(gates + (size_t)m * 512 + 4 * ch);
    float dc = dC[idx], di, df, dcg, dout;
    gate_bwd(dh, g, cprev[idx], ccur[idx], dc, di, df, dcg, dout);
    dC[idx] = dc;
    store4(dz + (size_t)m * 512 + 4 * ch, di, df, dcg, dout);
    acc[0] += di; acc[1] += df; acc[2] += dcg; acc[3] += dout;
  }
  if (!part) return;
  red[sl][ch] = acc;
  __syncthreads();
  if (sl == 0) {
    f32x4 t = red[0][ch];
#pragma unroll
    for (int k = 1; k < 4; ++k) { t[0] += red[k][ch][0]; t[1] += red[k][ch][1]; t[2] += red[k][ch][2]; t[3] += red[k][ch][3]; }
    *reinterpret_cast<f32x4*>(part + (size_t)blockIdx.x * 512 + 4 * ch) = t;
  }
}

// dY[m][o] = [dlogits | dvalues | 0-pad], ld = ldy
__global__ void k_concat_dy(int F, int A, int ldy, const float* dl, const float* dv, float* dY) {
  const int n = F * ldy;
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < n; idx += gridDim.x * blockDim.x) {
    const int m = idx / ldy, o = idx - m * ldy;
    float v = 0.f;
    if (o < A) v = dl[(size_t)m * A + o];
    else if (o < 2 * A) v = dv ? dv[(size_t)m * A + o - A] : 0.f;
    dY[idx] = v;
  }
}

// Per-frame (P, 128) fp32 state slices between row-major (the C ABI's h/c
// tensors) and the channel-quad-major slices of the frame-resident kernels
// (recur.h cqm4): 16 B (one channel quad of one pixel) per thread, pixels
// fastest on the quad-major side.
__global__ void k_cqm_convert(const float* __restrict__ src, float* __restrict__ dst, int nf, int P, int to_cqm) {
  const long n = (long)nf * P * 32;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long f = i / ((long)P * 32);
    const int r = (int)(i - f * P * 32), q = r / P, pp = r - q * P;
    const size_t rm = (size_t)f * P * 128 + (size_t)pp * 128 + q * 4, cq = (size_t)f * P * 128 + (size_t)r * 4;
    *reinterpret_cast<f32x4*>(dst + (to_cqm ? cq : rm)) = *reinterpret_cast<const f32x4*>(src + (to_cqm ? rm : cq));
  }
}

// XH slot 0 channels 64..191 <- h0 (or zero)

template <typename T>
__global__ void k_state_to_xh(int M, const float* h0, T* xh) {
  const int n = M * 128;
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < n; idx += gridDim.x * blockDim.x) {
    const int m = idx >> 7, ch = idx & 127;
    xh[(size_t)m * 192 + 64 + ch] = (T)(h0 ? h0[idx] : 0.f);
  }
}

// Block roles: [0, zb) zero the ranges (16-B stores where a range is 16-B aligned), [zb, zb + xb)
// state_to_xh, the rest concat_dy -- each role grid-strides over its own blocks.
template <typename T>
__global__ void __launch_bounds__(256) k_prologue(ZeroRanges z, int zb, int M, const float* h0, T* xh, int xb, int F,
                                                  int A, int ldy, const float* dl, const float* dv, float* dY) {
  const int b = (int)blockIdx.x, tid = (int)threadIdx.x;
  if (b < zb) {
    const long st = (long)zb * 256, i0 = (long)b * 256 + tid;
    for (int r = 0; r < z.cnt; ++r) {
      float* p = z.p[r];
      const long n = z.n[r], n4 = ((uintptr_t)p & 15) == 0 ? n / 4 : 0;
      for (long i = i0; i < n4; i += st) reinterpret_cast<f32x4*>(p)[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      for (long i = 4 * n4 + i0; i < n; i += st) p[i] = 0.f;
    }
    return;
  }
  if (b < zb + xb) {
    const int n = M * 128;
    for (int idx = (b - zb) * 256 + tid; idx < n; idx += xb * 256) {
      const int m = idx >> 7, ch = idx & 127;
      xh[(size_t)m * 192 + 64 + ch] = (T)(h0 ? h0[idx] : 0.f);
    }
    return;
  }
  const int cb = (int)gridDim.x - zb - xb, n = F * ldy;
  for (int idx = (b - zb - xb) * 256 + tid; idx < n; idx += cb * 256) {
    const int m = idx / ldy, o = idx - m * ldy;
    float v = 0.f;
    if (o < A) v = dl[(size_t)m * A + o];
    else if (o < 2 * A) v = dv ? dv[(size_t)m * A + o - A] : 0.f;
    dY[idx] = v;
  }
}

// h_T (fp32 state out) <- the h half of XH slot T (the bf16 path's only copy of h_t)
template <typename T>
__global__ void k_xh_to_state(int M, const T* __restrict__ xh, float* __restrict__ h) {
  const int n = M * 128;
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < n; idx += gridDim.x * blockDim.x)
    h[idx] = (float)xh[(size_t)(idx >> 7) * 192 + 64 + (idx & 127)];
}

// XH slot <- [x (64) | h (128)] of the standalone ConvLSTM cell (h NULL: the
// zero state of init_hidden, attention.py:142-149).
template <typename T>
__global__ void k_cell_xh(int M, const float* __restrict__ x, const float* __restrict__ h, T* xh) {
  const int n = M * 192;
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < n; idx += gridDim.x * blockDim.x) {
    const int m = idx / 192, c = idx - m * 192;
    const float v = c < 64 ? x[(size_t)m * 64 + c] : (h ? h[(size_t)m * 128 + c - 64] : 0.f);
    xh[idx] = (T)v;
  }
}

// dst[i] = (TO) src[i]
template <typename TI, typename TO>
__global__ void k_cast(long n, const TI* __restrict__ src, TO* __restrict__ dst) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    dst[i] = (TO)(float)src[i];
}

// ------------------------------------------------------------- packing ----
// Conv weight in the reference's (Cout, Cin, kx, ky) orientation (Q3) ->
// [Cout][(ky*K + kx)*Cin + ci].
template <typename T>
__device__ __forceinline__ void pack_conv_el(int idx, const float* __restrict__ w, int Cin, int K, T* dst) {
  const int o = idx / (K * K * Cin), r = idx - o * (K * K * Cin);
  const int tap = r / Cin, ci = r - tap * Cin, ky = tap / K, kx = tap - ky * K;
  dst[idx] = (T)w[((size_t)(o * Cin + ci) * K + kx) * K + ky];
}
template <typename T>
__global__ void k_pack_conv(const float* __restrict__ w, int Cout, int Cin, int K, T* dst) {
  const int n = Cout * K * K * Cin;
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < n; idx += gridDim.x * blockDim.x)
    pack_conv_el(idx, w, Cin, K, dst);
}

// Frames (F,H,W,3) fp32 or uint8 (the environment's observation, cast here
// instead of on the host as main_mp.py:53 does) -> (F,H+2,W+2,4): a zero 4th channel (conv1's gather is
// 16-byte vectors instead of scalar loads) and conv1's one-pixel zero padding
// stored in the image, so every tap of the conv reads in-bounds memory -- a
// bf16 16-byte chunk (two adjacent taps x 4 channels) never straddles the
// image border.  Raw pixels 0..255 are exact in bf16; other values are
// rounded exactly where the bf16 oracle rounds conv1's input.
template <typename T, typename TI>
__global__ void k_frames_rgbx(int F, int H, int W, const TI* __restrict__ x, T* __restrict__ y) {
  const int Hp = H + 2, Wp = W + 2;
  const long n = (long)F * Hp * Wp;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int f = (int)(i / (Hp * Wp)), r = (int)(i - (long)f * Hp * Wp);
    const int py = r / Wp, px = r - py * Wp;
    const int iy = py - 1, ix = px - 1;
    float v0 = 0.f, v1 = 0.f, v2 = 0.f;
    if (iy >= 0 && iy < H && ix >= 0 && ix < W) {
      const TI* s = x + (((long)f * H + iy) * W + ix) * 3;
      v0 = (float)s[0]; v1 = (float)s[1]; v2 = (float)s[2];
    }
    store4(y + i * 4, v0, v1, v2, 0.f);
  }
}

// conv2 dgrad by parity class (py, px) of the output pixel: a 2x2, stride-1,
// pad-0 conv over dY2 with W_c[ci][(ty*2+tx)*64 + co] = W2[co][ci][kx][ky],
// ky = py + 2(1-ty), kx = px + 2(1-tx) (reference (Cout,Cin,kx,ky) layout, Q3).
template <typename T>
__device__ __forceinline__ void pack_conv2_classes_el(int idx, const float* __restrict__ w2, T* dst) {
  const int cls = idx >> 13, r = idx & 8191, ci = r >> 8, k = r & 255;
  const int t = k >> 6, co = k & 63, ty = t >> 1, tx = t & 1;
  const int py = cls >> 1, px = cls & 1;
  const int ky = py + 2 * (1 - ty), kx = px + 2 * (1 - tx);
  dst[idx] = (T)w2[((size_t)(co * 32 + ci) * 4 + kx) * 4 + ky];
}
template <typename T>
__global__ void k_pack_conv2_classes(const float* __restrict__ w2, T* dst) {
  const int n = 4 * 32 * 256;
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < n; idx += gridDim.x * blockDim.x)
    pack_conv2_classes_el(idx, w2, dst);
}

// conv1 weights with a zero 4th input channel: [32][(ky*8 + kx)*4 + ci]
template <typename T>
__device__ __forceinline__ void pack_conv1_rgbx_el(int idx, const float* __restrict__ w, T* dst) {
  const int o = idx >> 8, r = idx & 255, tap = r >> 2, ci = r & 3, ky = tap >> 3, kx = tap & 7;
  dst[idx] = ci < 3 ? (T)w[((size_t)(o * 3 + ci) * 8 + kx) * 8 + ky] : (T)0.f;
}
template <typename T>
__global__ void k_pack_conv1_rgbx(const float* __restrict__ w, T* dst) {
  const int n = 32 * 256;
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < n; idx += gridDim.x * blockDim.x)
    pack_conv1_rgbx_el(idx, w, dst);
}

__device__ __forceinline__ void unpack_conv1_rgbx_el(int idx, const float* __restrict__ g, float* dst) {
  int r = idx;
  const int ky = r % 8; r /= 8;
  const int kx = r % 8; r /= 8;
  const int ci = r % 3, o = r / 3;
  dst[idx] = g[o * 256 + (ky * 8 + kx) * 4 + ci];
}
__global__ void k_unpack_conv1_rgbx(const float* __restrict__ g, float* dst) {
  const int n = 32 * 3 * 64;
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < n; idx += gridDim.x * blockDim.x)
    unpack_conv1_rgbx_el(idx, g, dst);
}


// ConvLSTM weight (gate g, channel ch) for tap (ky,kx) and input channel ci of
// [x (64) | h (128)], in the reference's (Cout, Cin, kx, ky) orientation (Q3).
__device__ __forceinline__ float lstm_w(const LstmPtrs& L, int row, int ky, int kx, int ci) {
  const int ch = row >> 2, g = row & 3;
  return ci < 64 ? L.wx[g][((size_t)(ch * 64 + ci) * 3 + kx) * 3 + ky]
                 : L.wh[g][((size_t)(ch * 128 + ci - 64) * 3 + kx) * 3 + ky];
}

// All four ConvLSTM weight layouts in one launch, row n = 4*ch + gate (gate
// interleaved; biases the same way), one grid-stride pass over their
// concatenated index ranges:
//   x-part  WpX[n][tap*64 + ci]      (batched x-part GEMM over all frames)
//   h-part  WpH[n][tap*128 + ci]     (the recurrent step)
//   dgrad   WdT[c'][tap*512 + n]     (c' over [x | h]: dx and dh of the BPTT)
//   fused   WpXH[n][tap*192 + c']    (the step GEMM whose K covers the whole XH slot)
constexpr int kPackLstmN = 512 * 576 + 512 * 1152 + 192 * 4608 + 512 * 1728;
template <typename T>
__device__ __forceinline__ void pack_lstm_el(int idx, const LstmPtrs& L, T* WpX, T* WpH, float* bl, T* WdT, T* WpXH) {
  const int nx = 512 * 576, nh = 512 * 1152, nd = 192 * 4608;
  {
    int i = idx;
    if (i < nx) {
      const int row = i / 576, k = i - row * 576;
      const int tap = k / 64, ci = k - tap * 64, ky = tap / 3, kx = tap - ky * 3;
      WpX[i] = (T)lstm_w(L, row, ky, kx, ci);
      if (k == 0) bl[row] = L.bx[row & 3][row >> 2];
    } else if ((i -= nx) < nh) {
      const int row = i / 1152, k = i - row * 1152;
      const int tap = k / 128, ci = k - tap * 128, ky = tap / 3, kx = tap - ky * 3;
      WpH[i] = (T)lstm_w(L, row, ky, kx, 64 + ci);
    } else if ((i -= nh) < nd) {
      const int cp = i / 4608, r = i - cp * 4608;
      const int tap = r >> 9, row = r & 511, ky = tap / 3, kx = tap - ky * 3;
      WdT[i] = (T)lstm_w(L, row, ky, kx, cp);
    } else {
      i -= nd;
      const int row = i / 1728, k = i - row * 1728;
      const int tap = k / 192, cp = k - tap * 192, ky = tap / 3, kx = tap - ky * 3;
      WpXH[i] = (T)lstm_w(L, row, ky, kx, cp);
    }
  }
}
template <typename T>
__global__ void k_pack_lstm_all(LstmPtrs L, T* WpX, T* WpH, float* bl, T* WdT, T* WpXH) {
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < kPackLstmN; idx += gridDim.x * blockDim.x)
    pack_lstm_el(idx, L, WpX, WpH, bl, WdT, WpXH);
}

// Step 0 from a zero state: the gates come from the batched x-part alone.
// nsl > 0 (the split-K fused step, rt.h fused_step tiles 17/18): the gate
// pre-activations are bias + the nsl K-slice partials zs[k*sls + m*512 + ..]
// (EpiSliceT), summed in slice order, instead of ``gates``' contents.
template <typename T>
__global__ void k_gate_fwd_zx(int M, const float* __restrict__ cprev, float* gates, float* cnext, float* hout,
                              T* xhnext, const float* __restrict__ zs, int nsl, size_t sls,
                              const float* __restrict__ bias) {
  const int n = M * 128;
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < n; idx += gridDim.x * blockDim.x) {
    const int m = idx >> 7, ch = idx & 127;
    f32x4 z;
    if (nsl > 0) {
      z = *reinterpret_cast<const f32x4*>(bias + 4 * ch);
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (k < nsl) {
          const f32x4 u = *reinterpret_cast<const f32x4*>(zs + k * sls + (size_t)m * 512 + 4 * ch);
          z[0] += u[0]; z[1] += u[1]; z[2] += u[2]; z[3] += u[3];
        }
    } else {
      z = *reinterpret_cast<const f32x4*>(gates + (size_t)m * 512 + 4 * ch);
    }
    float gi, gf, gc, go, c, h;
    GateFwd::run(z[0], z[1], z[2], z[3], cprev[idx], gi, gf, gc, go, c, h);
    cnext[idx] = c;
    if (hout) hout[idx] = h;   // null on the bf16 path (the readout reads xhnext)
    xhnext[(size_t)m * 192 + 64 + ch] = (T)h;
    *reinterpret_cast<f32x4*>(gates + (size_t)m * 512 + 4 * ch) = f32x4{gi, gf, gc, go};
  }
}

__host__ __device__ inline int pack_f32_n(const F32Pack& p) {
  return 512 * p.ans_ld + 1024 * 256 + 1024 + p.ldy * 256 + p.ldy + (p.Wihhp ? 1024 * 512 : 0);
}
__device__ __forceinline__ void pack_f32_el(int idx, const F32Pack& p) {
  const int n1 = 512 * p.ans_ld, n2 = 1024 * 256, n3 = 1024, n4 = p.ldy * 256, n5 = p.ldy;
  int i = idx;
  if (i >= n1 + n2 + n3 + n4 + n5) {   // [W_ih | W_hh] rows 4u+g (stateful core)
    i -= n1 + n2 + n3 + n4 + n5;
    const int row = i >> 9, k = i & 511, u = row >> 2, g = row & 3;
    p.Wihhp[i] = k < 256 ? p.wih[(size_t)(g * 256 + u) * 256 + k] : p.whh[(size_t)(g * 256 + u) * 256 + k - 256];
    return;
  }
  if (i < n1) {
    const int o = i / p.ans_ld, k = i - o * p.ans_ld;
    p.W1p[i] = k < p.ans_in ? p.a0w[(size_t)o * p.ans_in + k] : 0.f;
    return;
  }
  i -= n1;
  if (i < n2) {
    const int row = i >> 8, k = i & 255, u = row >> 2, g = row & 3;
    p.Wihp[i] = p.wih[(size_t)(g * 256 + u) * 256 + k];
    return;
  }
  i -= n2;
  if (i < n3) {
    const int u = i >> 2, g = i & 3;
    p.blc[i] = p.bih[g * 256 + u] + p.bhh[g * 256 + u];
    return;
  }
  i -= n3;
  if (i < n4) {
    const int o = i >> 8, k = i & 255;
    float v = 0.f;
    if (o < p.A) v = p.pw[o * 256 + k];
    else if (o < 2 * p.A) v = p.vw[(o - p.A) * 256 + k];
    p.Whd[i] = v;
    return;
  }
  i -= n4;
  float v = 0.f;
  if (i < p.A) v = p.pb[i];
  else if (i < 2 * p.A) v = p.vb[i - p.A];
  p.bhd[i] = v;
}
__global__ void k_pack_f32(F32Pack p) {
  const int tot = pack_f32_n(p);
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < tot; idx += gridDim.x * blockDim.x) pack_f32_el(idx, p);
}

// Every weight layout of aaa_pack_weights that depends on the params alone, in
// one launch (each was its own ~5 us launch): conv1 RGBx, conv2, conv2's dgrad
// classes, the four ConvLSTM layouts and the fp32 tail layouts, one grid-stride
// pass over their concatenated index ranges.
template <typename T>
__global__ void k_pack_all(PackAll<T> a) {
  const int n1 = 32 * 256, n2 = n1 + 64 * 512, n3 = n2 + 4 * 32 * 256, n4 = n3 + kPackLstmN;
  const int tot = n4 + pack_f32_n(a.f32);
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < tot; idx += gridDim.x * blockDim.x) {
    if (idx < n1) pack_conv1_rgbx_el(idx, a.c1w, a.Wp1);
    else if (idx < n2) pack_conv_el(idx - n1, a.c2w, 32, 4, a.Wp2);
    else if (idx < n3) pack_conv2_classes_el(idx - n2, a.c2w, a.WdT2);
    else if (idx < n4) pack_lstm_el(idx - n3, a.lstm, a.WpX, a.WpH, a.bl, a.WdT, a.WpXH);
    else pack_f32_el(idx - n4, a.f32);
  }
}


// ------------------------------------------------------------ unpacking ---
__device__ __forceinline__ void unpack_conv_el(int idx, const float* __restrict__ g, int Cin, int K, float* dst) {
  int r = idx;
  const int ky = r % K; r /= K;
  const int kx = r % K; r /= K;
  const int ci = r % Cin, o = r / Cin;
  dst[idx] = g[(size_t)o * K * K * Cin + (ky * K + kx) * Cin + ci];
}
__global__ void k_unpack_conv(const float* __restrict__ g, int Cout, int Cin, int K, float* dst) {
  const int n = Cout * Cin * K * K;
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < n; idx += gridDim.x * blockDim.x)
    unpack_conv_el(idx, g, Cin, K, dst);
}

constexpr int kUnpackLstmN = 4 * (128 * 64 * 9 + 128 * 128 * 9 + 128);
__device__ __forceinline__ void unpack_lstm_el(int idx, const float* __restrict__ gW, const float* __restrict__ gb,
                                               const LstmGrads& L) {
  const int nx = 128 * 64 * 9, nh = 128 * 128 * 9;
  {
    const int per = nx + nh + 128;
    const int g = idx / per;
    int i = idx - g * per;
    if (i < nx) {
      int r = i;
      const int ky = r % 3; r /= 3;
      const int kx = r % 3; r /= 3;
      const int ci = r % 64, ch = r / 64;
      L.wx[g][i] = gW[(size_t)(4 * ch + g) * 1728 + (ky * 3 + kx) * 192 + ci];
    } else if ((i -= nx) < nh) {
      int r = i;
      const int ky = r % 3; r /= 3;
      const int kx = r % 3; r /= 3;
      const int ci = r % 128, ch = r / 128;
      L.wh[g][i] = gW[(size_t)(4 * ch + g) * 1728 + (ky * 3 + kx) * 192 + 64 + ci];
    } else {
      i -= nh;
      L.bx[g][i] = gb[4 * i + g];
    }
  }
}
__global__ void k_unpack_lstm(const float* __restrict__ gW, const float* __restrict__ gb, LstmGrads L) {
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < kUnpackLstmN; idx += gridDim.x * blockDim.x)
    unpack_lstm_el(idx, gW, gb, L);
}
// The ConvLSTM (optional: gW == null skips it) and both conv weight grads back
// into the reference layouts in one launch (the end of a CORE + VISION backward).
__global__ void k_unpack_cv(const float* __restrict__ gW, const float* __restrict__ gb, LstmGrads L,
                            const float* __restrict__ g2, float* d2, const float* __restrict__ g1, float* d1) {
  const int n0 = gW ? kUnpackLstmN : 0, n1 = n0 + 64 * 32 * 16, n2 = n1 + 32 * 3 * 64;
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < n2; idx += gridDim.x * blockDim.x) {
    if (idx < n0) unpack_lstm_el(idx, gW, gb, L);
    else if (idx < n1) unpack_conv_el(idx - n0, g2, 32, 4, d2);
    else unpack_conv1_rgbx_el(idx - n1, g1, d1);
  }
}

__global__ void k_unpack_f32(F32Unpack p) {
  const int n1 = 512 * p.ans_in, n2 = 1024 * 256, n3 = 1024, n4 = 2 * p.A * 256, n5 = 2 * p.A;
  const int tot = n1 + n2 + n3 + n4 + n5;
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < tot; idx += gridDim.x * blockDim.x) {
    int i = idx;
    if (i < n1) {
      const int o = i / p.ans_in, k = i - o * p.ans_in;
      p.a0w[i] = p.gW1p[(size_t)o * p.ans_ld + k];
      continue;
    }
    i -= n1;
    if (i < n2) {
      const int row = i >> 8, k = i & 255, g = row >> 8, u = row & 255;
      if (p.gWihhp) {   // stateful core: W_ih | W_hh from one [1024][512] gradient
        p.wih[i] = p.gWihhp[(size_t)(4 * u + g) * 512 + k];
        p.whh[i] = p.gWihhp[(size_t)(4 * u + g) * 512 + 256 + k];
      } else {
        p.wih[i] = p.gWihp[(size_t)(4 * u + g) * 256 + k];
      }
      continue;
    }
    i -= n2;
    if (i < n3) {
      const int g = i >> 8, u = i & 255;
      const float v = p.gblc[4 * u + g];
      p.bih[i] = v;
      p.bhh[i] = v;
      continue;
    }
    i -= n3;
    if (i < n4) {
      const int o = i >> 8, k = i & 255;
      if (o < p.A) p.pw[o * 256 + k] = p.gWhd[i];
      else p.vw[(o - p.A) * 256 + k] = p.gWhd[i];
      continue;
    }
    i -= n4;
    if (i < p.A) p.pb[i] = p.gbhd[i];
    else p.vb[i - p.A] = p.gbhd[i];
  }
}

// ---------------------------------------------------------- launchers -----
static inline int nblk(long n, int bs = 256) {
  long b = (n + bs - 1) / bs;
  return (int)(b < 4096 ? (b > 0 ? b : 1) : 4096);
}

hipError_t query_pack(const float* b0, const float* W2, const float* b2, const float* W4, const float* b4, int nq,
                      float* q1, float* q2, float* Q, hipStream_t st) {
  // QueryNetwork on the always-zero prev_output (attention.py:184-198, 325-331; Q1):
  // q1 = relu(b0), q2 = relu(W2 q1 + b2), Q = W4 q2 + b4 -- a function of the
  // weights alone, so it is computed when they are packed, not per forward.
  const int qd = 72 * nq;
  hipLaunchKernelGGL(k_query_layer, dim3((qd + 3) / 4), dim3(256), 0, st, W2, 128, b0, 1, b2, 1, qd, q2, q1);
  hipLaunchKernelGGL(k_query_layer, dim3((qd + 3) / 4), dim3(256), 0, st, W4, qd, q2, 0, b4, 0, qd, Q,
                     (float*)nullptr);
  return hipGetLastError();
}

hipError_t query_sq(const float* S, const float* Q, int P, int nq, float* SQ, hipStream_t st) {
  hipLaunchKernelGGL(k_query_sq, dim3((P + 3) / 4), dim3(256), 0, st, S, Q, P, nq, SQ);
  return hipGetLastError();
}

hipError_t attn_fwd(OSrc O, const float* S, const float* Q, const float* SQ, const float* pr,
                    const float* pa, int F, int P, int nq, float* Am, float* ans, int ans_ld, hipStream_t st,
                    int qs) {
  // register prefetch of the V slice only on large grids (many positions per
  // slice): at 84x84 (11 per slice) the registers cost more occupancy than the
  // early loads buy (C3: 118 vs 104 us; 168x168, C5: 217 vs 275 us)
#ifdef AAA_ABLATION   // A/B overrides (ablation builds)
  static const int pre_env = getenv("AAA_ATTN_PRE") ? atoi(getenv("AAA_ATTN_PRE")) : -1;
  static const int sl_env = getenv("AAA_ATTN_SLICES") ? atoi(getenv("AAA_ATTN_SLICES")) : -1;
#else
  constexpr int pre_env = -1, sl_env = -1;
#endif
  // the readout product on the MFMA for bf16 O (attn_mfma.h); AAA_ATTN_MFMA=0: the VALU kernel below
  static const int mfma_env = getenv("AAA_ATTN_MFMA") ? atoi(getenv("AAA_ATTN_MFMA")) : 1;
  if (mfma_env && O.bf16 && (nq == 4 || nq == 8)) {
    if (O.ld < 128 || O.ld % 8) return hipErrorInvalidValue;   // 16-B loads
    const size_t sh = attn_mfma_lds(P, nq);
    if (sh > 160 * 1024) return hipErrorInvalidValue;
#ifdef AAA_ABLATION   // O loaded non-temporal (A/B: the backward then reads those rows slower, profiles/r06/ab/attn_nt/)
    static const int nt_env = getenv("AAA_ATTN_NT") ? atoi(getenv("AAA_ATTN_NT")) : 0;
#else
    constexpr int nt_env = 0;
#endif
    auto kern = !SQ ? (nq == 4 ? k_attn_fwd_mfma<4, false, false> : k_attn_fwd_mfma<8, false, false>)
                : nt_env ? (nq == 4 ? k_attn_fwd_mfma<4, true> : k_attn_fwd_mfma<8, true>)
                         : (nq == 4 ? k_attn_fwd_mfma<4, false> : k_attn_fwd_mfma<8, false>);
    if (sh > 64 * 1024)
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)sh);
    hipLaunchKernelGGL(kern, dim3(F), dim3(256), sh, st, (const __bf16*)O.p, O.ld, S, Q, qs, SQ, pr, pa, P, Am, ans,
                       ans_ld);
    return hipGetLastError();
  }
  const bool pre = pre_env >= 0 ? pre_env != 0 : P > 2 * kAttnSlices * 11;
  const int sl = O.bf16 ? kAttnSlicesBf : sl_env > 0 ? sl_env : kAttnSlices;
  const size_t sh = (size_t)(P * nq + nq * 72 + sl * nq * 184) * sizeof(float);
  if (sh > 160 * 1024) return hipErrorInvalidValue;
  if (O.bf16 ? (O.ld < 136 || O.ld % 8) : O.ld < 128 || O.ld % 4) return hipErrorInvalidValue;   // 16-B key loads
  auto launch = [&](auto kern, auto* o) {
    if (sh > 64 * 1024)
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)sh);
    hipLaunchKernelGGL(kern, dim3(F), dim3(kAttnFwdThreads), sh, st, o, O.ld, S, Q, qs, SQ, pr, pa, P, Am, ans,
                       ans_ld);
  };
  auto go = [&](auto slc) {
    constexpr int SL = decltype(slc)::value;
    if (O.bf16) {
      const __bf16* o = (const __bf16*)O.p;
      if (nq == 4) pre ? launch(k_attn_fwd<4, 8, SL, __bf16>, o) : launch(k_attn_fwd<4, 0, SL, __bf16>, o);
      else if (nq == 8) pre ? launch(k_attn_fwd<8, 8, SL, __bf16>, o) : launch(k_attn_fwd<8, 0, SL, __bf16>, o);
      return;
    }
    const float* o = (const float*)O.p;
    if (nq == 4) pre ? launch(k_attn_fwd<4, 8, SL, float>, o) : launch(k_attn_fwd<4, 0, SL, float>, o);
    else if (nq == 8) pre ? launch(k_attn_fwd<8, 8, SL, float>, o) : launch(k_attn_fwd<8, 0, SL, float>, o);
  };
  if (nq != 4 && nq != 8) return hipErrorInvalidValue;
  if (O.bf16) go(std::integral_constant<int, 0>{});   // (SL unused: kAttnSlicesBf)
  else if (sl == kAttnSlices) go(std::integral_constant<int, kAttnSlices>{});
#ifdef AAA_ABLATION
  else if (sl == 8) go(std::integral_constant<int, 8>{});
  else if (sl == 5) go(std::integral_constant<int, 5>{});
#endif
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t cqm_convert(const float* src, float* dst, int nf, int P, int to_cqm, hipStream_t st) {
  hipLaunchKernelGGL(k_cqm_convert, dim3(nblk((long)nf * P * 32)), dim3(256), 0, st, src, dst, nf, P, to_cqm);
  return hipGetLastError();
}

hipError_t attn_bwd(OSrc O, const float* S, const float* Q, const float* Am, const float* dAns,
                    int da_ld, int F, int P, int nq, float* dO, float* dQp, hipStream_t st, int qs, int addq,
                    int cqm) {
  const int G = 7;   // k_attn_bwd's dQ position groups
  const size_t sh = (size_t)(2 * P * nq + nq * 184 + nq * 72 + 8 + G * nq * 72 + P * 8) * sizeof(float);
  if (sh > 160 * 1024) return hipErrorInvalidValue;
  if (O.bf16 ? (O.ld < 136 || O.ld % 4) : O.ld < 128 || O.ld % 4) return hipErrorInvalidValue;
  auto launch = [&](auto kern, auto* o) {
    if (sh > 64 * 1024)   // large grids (168x168: P = 441, nq = 8) use more than the default 64 KiB
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)sh);
    hipLaunchKernelGGL(kern, dim3(F), dim3(512), sh, st, o, O.ld, S, Q, qs, Am, dAns, da_ld, addq, P, dO, dQp, cqm);
  };
  if (nq != 4 && nq != 8) return hipErrorInvalidValue;
  // positions per lane in the dA pass: 2 on large grids halves its LDS reads of da (C5,
  // P = 441: 322 -> 296-311 us); at 84x84 (P = 121, two passes of 64 or one of 128) the
  // doubled per-lane chain costs more than the shared reads save (C3 113 vs 119-122 us)
  // (profiles/r05/ab/attn_bwd_ppl/)
#ifdef AAA_ABLATION
  static const int ppl_env = getenv("AAA_ATTN_BWD_PPL") ? atoi(getenv("AAA_ATTN_BWD_PPL")) : 0;
#else
  constexpr int ppl_env = 0;
#endif
  const int ppl = ppl_env ? ppl_env : P > 256 ? 2 : 1;
  if (ppl != 1 && ppl != 2) return hipErrorInvalidValue;
  // bf16 O on large grids: the dA pass on the MFMA (attn_mfma.h; C5, P = 441: 320 -> 290 us; at 84x84,
  // P = 121, the VALU pass is faster: 126 vs 139 us, profiles/r06/ab/attn_bwd_mfma/).  AAA_ATTN_BWD_MFMA=0:
  // the VALU kernel everywhere, 2: the MFMA pass everywhere
  static const int bm_env = getenv("AAA_ATTN_BWD_MFMA") ? atoi(getenv("AAA_ATTN_BWD_MFMA")) : 1;
  if (O.bf16 && (bm_env == 2 || (bm_env == 1 && P > 256))) {
    const __bf16* o = (const __bf16*)O.p;
    nq == 4 ? launch(k_attn_bwd_mfma<4>, o) : launch(k_attn_bwd_mfma<8>, o);
    return hipGetLastError();
  }
  if (O.bf16) {
    const __bf16* o = (const __bf16*)O.p;
    if (ppl == 2) nq == 4 ? launch(k_attn_bwd<4, __bf16, 2>, o) : launch(k_attn_bwd<8, __bf16, 2>, o);
    else nq == 4 ? launch(k_attn_bwd<4, __bf16, 1>, o) : launch(k_attn_bwd<8, __bf16, 1>, o);
  } else {
    const float* o = (const float*)O.p;
    if (ppl == 2) nq == 4 ? launch(k_attn_bwd<4, float, 2>, o) : launch(k_attn_bwd<8, float, 2>, o);
    else nq == 4 ? launch(k_attn_bwd<4, float, 1>, o) : launch(k_attn_bwd<8, float, 1>, o);
  }
  return hipGetLastError();
}

hipError_t query_bwd(const float* dQs, const float* gb1, const float* W1, int ans_in, int nq, const float* W2,
                     const float* W4, const float* q1, const float* q2, float* gW4, float* gb4, float* gW2,
                     float* gb2, float* gb0, hipStream_t st) {
  // dQ += W1[:, Q-cols]^T . db1 (the answer path summed over rows), 512 rows over 32 WGs
  hipLaunchKernelGGL(k_gemv_cols_atomic, dim3(32), dim3(256), 0, st, W1 + nq * 184, ans_in, gb1, 512, 72 * nq, 16,
                     const_cast<float*>(dQs));
  // Back through Q = W4 q2 + b4, q2 = relu(W2 q1 + b2), q1 = relu(b0).  The
  // pre-ReLU masks are q2 > 0 and q1 > 0; gb2 = dq2 and gb0 = dq1 are written
  // straight into the grad buffer (gb2 doubles as dq2 for the next layer).
  const int qd = 72 * nq;
  (void)W1; (void)ans_in;
  // each layer's two products from the same input gradient in one launch (colgemv blocks, then outer)
  const int cg4 = (qd + 63) / 64, ob4 = nblk((long)qd * qd, 1024), ob2 = nblk((long)qd * 128, 1024);
  hipLaunchKernelGGL(k_query_colgemv_outer, dim3(cg4 + ob4), dim3(1024), 0, st, W4, qd, qd, dQs, q2, gb2, cg4, dQs,
                     qd, q2, qd, gW4, gb4);
  hipLaunchKernelGGL(k_query_colgemv_outer, dim3(2 + ob2), dim3(1024), 0, st, W2, qd, 128, gb2, q1, gb0, 2, gb2, qd,
                     q1, 128, gW2, (float*)nullptr);
  return hipGetLastError();
}

template <typename TI>
hipError_t colsum(const TI* X, int ld, int M, int N, float* out, hipStream_t st) {
  if (M <= 0 || N <= 0) return hipSuccess;
  const int cols = (N + 63) / 64;
  int split = (1024 + cols - 1) / cols;
  int rows_per = (M + split - 1) / split;
  if (rows_per < 64) rows_per = 64;
  split = (M + rows_per - 1) / rows_per;
  hipLaunchKernelGGL(k_colsum<TI>, dim3(cols, split), dim3(256), 0, st, X, ld, M, N, rows_per, out);
  return hipGetLastError();
}

template <typename TZ, typename GT>
hipError_t gate_bwd_last(int M, int bj, const float* dO, const float* dhT, const GT* gates, const float* cprev,
                         const float* ccur, float* dC, TZ* dz, float* part, hipStream_t st, int nsl, size_t sls) {
  hipLaunchKernelGGL((k_gate_bwd_last<TZ, GT>), dim3((M + bj - 1) / bj), dim3(512), 0, st, M, bj, dO, dhT, gates,
                     cprev, ccur, dC, dz, part, dhT ? nsl : 0, sls);
  return hipGetLastError();
}

hipError_t concat_dy(int F, int A, int ldy, const float* dl, const float* dv, float* dY, hipStream_t st) {
  hipLaunchKernelGGL(k_concat_dy, dim3(nblk((long)F * ldy)), dim3(256), 0, st, F, A, ldy, dl, dv, dY);
  return hipGetLastError();
}

template <typename T>
hipError_t state_to_xh(int M, const float* h0, T* xh, hipStream_t st) {
  hipLaunchKernelGGL(k_state_to_xh<T>, dim3(nblk((long)M * 128)), dim3(256), 0, st, M, h0, xh);
  return hipGetLastError();
}

template <typename T>
hipError_t prologue(const ZeroRanges& z, int M, const float* h0, T* xh, int F, int A, int ldy, const float* dl,
                    const float* dv, float* dY, hipStream_t st) {
  if (z.cnt < 0 || z.cnt > 4) return hipErrorInvalidValue;
  long zn = 0;
  for (int r = 0; r < z.cnt; ++r) zn += z.n[r];
  const int zb = z.cnt ? std::min(nblk(zn / 4 + 1), 1024) : 0;
  const int xb = xh ? std::min(nblk((long)M * 128), 1024) : 0;
  const int cb = dY ? std::min(nblk((long)F * ldy), 1024) : 0;
  if (zb + xb + cb == 0) return hipSuccess;
  hipLaunchKernelGGL(k_prologue<T>, dim3(zb + xb + cb), dim3(256), 0, st, z, zb, M, h0, xh, xb, F, A, ldy, dl, dv, dY);
  return hipGetLastError();
}

template <typename T>
hipError_t xh_to_state(int M, const T* xh, float* h, hipStream_t st) {
  hipLaunchKernelGGL(k_xh_to_state<T>, dim3(nblk((long)M * 128)), dim3(256), 0, st, M, xh, h);
  return hipGetLastError();
}

template <typename T>
hipError_t cell_xh(int M, const float* x, const float* h, T* xh, hipStream_t st) {
  hipLaunchKernelGGL(k_cell_xh<T>, dim3(nblk((long)M * 192)), dim3(256), 0, st, M, x, h, xh);
  return hipGetLastError();
}

template <typename TI, typename TO>
hipError_t cast(long n, const TI* src, TO* dst, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL((k_cast<TI, TO>), dim3(nblk(n)), dim3(256), 0, st, n, src, dst);
  return hipGetLastError();
}

template <typename T>
hipError_t pack_conv(const float* w, int Cout, int Cin, int K, T* dst, hipStream_t st) {
  hipLaunchKernelGGL(k_pack_conv<T>, dim3(nblk((long)Cout * Cin * K * K)), dim3(256), 0, st, w, Cout, Cin, K, dst);
  return hipGetLastError();
}



template <typename T>
hipError_t pack_lstm_all(const LstmPtrs& L, T* WpX, T* WpH, T* WdT, float* bl, T* WpXH, hipStream_t st) {
  hipLaunchKernelGGL(k_pack_lstm_all<T>, dim3(nblk(512L * 576 + 512L * 1152 + 192L * 4608 + 512L * 1728)), dim3(256), 0,
                     st, L, WpX, WpH, bl, WdT, WpXH);
  return hipGetLastError();
}


template <typename T>
hipError_t gate_fwd_zx(int M, const float* cprev, float* gates, float* cnext, float* hout, T* xhnext,
                       hipStream_t st, const float* zs, int nsl, size_t sls, const float* bias) {
  if (nsl > 0 && (!zs || !bias || nsl > 8)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_gate_fwd_zx<T>, dim3(nblk((long)M * 128)), dim3(256), 0, st, M, cprev, gates, cnext, hout,
                     xhnext, zs, nsl, sls, bias);
  return hipGetLastError();
}

__global__ void k_reorder_cmaj(const float* __restrict__ src, int rows, int Cin, int taps, int BK,
                               float* __restrict__ dst) {
  const long K = (long)taps * Cin, n = (long)rows * K;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long r = i / K;
    const int k = (int)(i - r * K), tap = k / Cin, c = k - tap * Cin;
    dst[r * K + (long)(c / BK) * taps * BK + tap * BK + c % BK] = src[i];
  }
}

hipError_t reorder_cmaj(const float* src, int rows, int Cin, int taps, int BK, float* dst, hipStream_t st) {
  if (Cin % BK) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_reorder_cmaj, dim3(nblk((long)rows * taps * Cin)), dim3(256), 0, st, src, rows, Cin, taps, BK,
                     dst);
  return hipGetLastError();
}

__global__ void k_split_planes(const float* __restrict__ src, long n, __bf16* __restrict__ dst) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float x = src[i];
    const __bf16 hi = (__bf16)x;
    const float r = x - (float)hi;
    const __bf16 mid = (__bf16)r;
    dst[i] = hi;
    dst[n + i] = mid;
    dst[2 * n + i] = (__bf16)(r - (float)mid);
  }
}

hipError_t split_planes(const float* src, long n, __bf16* dst, hipStream_t st) {
  hipLaunchKernelGGL(k_split_planes, dim3(nblk(n)), dim3(256), 0, st, src, n, dst);
  return hipGetLastError();
}

hipError_t pack_f32(const F32Pack& p, hipStream_t st) {
  long n = 512L * p.ans_ld + 1024L * 256 + 1024 + (long)p.ldy * 256 + p.ldy + (p.Wihhp ? 1024L * 512 : 0);
  hipLaunchKernelGGL(k_pack_f32, dim3(nblk(n)), dim3(256), 0, st, p);
  return hipGetLastError();
}

hipError_t unpack_conv(const float* g, int Cout, int Cin, int K, float* dst, hipStream_t st) {
  hipLaunchKernelGGL(k_unpack_conv, dim3(nblk((long)Cout * Cin * K * K)), dim3(256), 0, st, g, Cout, Cin, K, dst);
  return hipGetLastError();
}

hipError_t unpack_lstm(const float* gW, const float* gb, const LstmGrads& L, hipStream_t st) {
  hipLaunchKernelGGL(k_unpack_lstm, dim3(nblk(4L * (128 * 64 * 9 + 128 * 128 * 9 + 128))), dim3(256), 0, st, gW,
                     gb, L);
  return hipGetLastError();
}

hipError_t unpack_f32(const F32Unpack& p, hipStream_t st) {
  long n = 512L * p.ans_in + 1024L * 256 + 1024 + 2L * p.A * 256 + 2 * p.A;
  hipLaunchKernelGGL(k_unpack_f32, dim3(nblk(n)), dim3(256), 0, st, p);
  return hipGetLastError();
}

template <typename T, typename TI>
hipError_t frames_rgbx(int F, int H, int W, const TI* x, T* y, hipStream_t st) {
  hipLaunchKernelGGL((k_frames_rgbx<T, TI>), dim3(nblk((long)F * (H + 2) * (W + 2))), dim3(256), 0, st, F, H, W, x, y);
  return hipGetLastError();
}
template <typename T>
hipError_t pack_conv2_classes(const float* w2, T* dst, hipStream_t st) {
  hipLaunchKernelGGL(k_pack_conv2_classes<T>, dim3(nblk(4 * 32 * 256)), dim3(256), 0, st, w2, dst);
  return hipGetLastError();
}
template <typename T>
hipError_t pack_conv1_rgbx(const float* w, T* dst, hipStream_t st) {
  hipLaunchKernelGGL(k_pack_conv1_rgbx<T>, dim3(nblk(32 * 256)), dim3(256), 0, st, w, dst);
  return hipGetLastError();
}
hipError_t unpack_conv1_rgbx(const float* g, float* dst, hipStream_t st) {
  hipLaunchKernelGGL(k_unpack_conv1_rgbx, dim3(nblk(32 * 3 * 64)), dim3(256), 0, st, g, dst);
  return hipGetLastError();
}
template hipError_t colsum<float>(const float*, int, int, int, float*, hipStream_t);
template hipError_t colsum<__bf16>(const __bf16*, int, int, int, float*, hipStream_t);
template hipError_t gate_bwd_last<float, float>(int, int, const float*, const float*, const float*, const float*,
                                                const float*, float*, float*, float*, hipStream_t, int, size_t);
template hipError_t gate_bwd_last<__bf16, float>(int, int, const float*, const float*, const float*, const float*,
                                                 const float*, float*, __bf16*, float*, hipStream_t, int, size_t);
template hipError_t gate_bwd_last<float, _Float16>(int, int, const float*, const float*, const _Float16*,
                                                   const float*, const float*, float*, float*, float*, hipStream_t, int, size_t);
template hipError_t gate_bwd_last<__bf16, _Float16>(int, int, const float*, const float*, const _Float16*,
                                                    const float*, const float*, float*, __bf16*, float*, hipStream_t, int, size_t);
template hipError_t frames_rgbx<float, float>(int, int, int, const float*, float*, hipStream_t);
template hipError_t frames_rgbx<__bf16, float>(int, int, int, const float*, __bf16*, hipStream_t);
template hipError_t frames_rgbx<float, uint8_t>(int, int, int, const uint8_t*, float*, hipStream_t);
template hipError_t frames_rgbx<__bf16, uint8_t>(int, int, int, const uint8_t*, __bf16*, hipStream_t);
template hipError_t pack_conv2_classes<float>(const float*, float*, hipStream_t);
template hipError_t pack_conv2_classes<__bf16>(const float*, __bf16*, hipStream_t);
template hipError_t pack_conv1_rgbx<float>(const float*, float*, hipStream_t);
template hipError_t pack_conv1_rgbx<__bf16>(const float*, __bf16*, hipStream_t);
template hipError_t cell_xh<float>(int, const float*, const float*, float*, hipStream_t);
template hipError_t cell_xh<__bf16>(int, const float*, const float*, __bf16*, hipStream_t);
template hipError_t cast<float, __bf16>(long, const float*, __bf16*, hipStream_t);
template hipError_t cast<__bf16, float>(long, const __bf16*, float*, hipStream_t);
template hipError_t cast<float, float>(long, const float*, float*, hipStream_t);
template hipError_t state_to_xh<float>(int, const float*, float*, hipStream_t);
template hipError_t state_to_xh<__bf16>(int, const float*, __bf16*, hipStream_t);
template hipError_t prologue<float>(const ZeroRanges&, int, const float*, float*, int, int, int, const float*,
                                    const float*, float*, hipStream_t);
template hipError_t prologue<__bf16>(const ZeroRanges&, int, const float*, __bf16*, int, int, int, const float*,
                                     const float*, float*, hipStream_t);
template hipError_t xh_to_state<__bf16>(int, const __bf16*, float*, hipStream_t);
template hipError_t pack_conv<float>(const float*, int, int, int, float*, hipStream_t);
template hipError_t pack_conv<__bf16>(const float*, int, int, int, __bf16*, hipStream_t);
template hipError_t pack_lstm_all<float>(const LstmPtrs&, float*, float*, float*, float*, float*, hipStream_t);
template hipError_t pack_lstm_all<__bf16>(const LstmPtrs&, __bf16*, __bf16*, __bf16*, float*, __bf16*, hipStream_t);
template hipError_t gate_fwd_zx<float>(int, const float*, float*, float*, float*, float*, hipStream_t, const float*, int, size_t,
                                         const float*);
template hipError_t gate_fwd_zx<__bf16>(int, const float*, float*, float*, float*, __bf16*, hipStream_t, const float*, int, size_t,
                                         const float*);

template <typename T>
hipError_t pack_all(const PackAll<T>& a, hipStream_t st) {
  const long n = 32L * 256 + 64 * 512 + 4 * 32 * 256 + kPackLstmN + pack_f32_n(a.f32);
  hipLaunchKernelGGL(k_pack_all<T>, dim3(nblk(n)), dim3(256), 0, st, a);
  return hipGetLastError();
}
template hipError_t pack_all<float>(const PackAll<float>&, hipStream_t);
template hipError_t pack_all<__bf16>(const PackAll<__bf16>&, hipStream_t);

hipError_t unpack_cv(const float* gW, const float* gb, const LstmGrads& L, const float* g2, float* d2, const float* g1,
                     float* d1, hipStream_t st) {
  const long n = (gW ? kUnpackLstmN : 0) + 64L * 32 * 16 + 32 * 3 * 64;
  hipLaunchKernelGGL(k_unpack_cv, dim3(nblk(n)), dim3(256), 0, st, gW, gb, L, g2, d2, g1, d1);
  return hipGetLastError();
}

// Several column sums over the same M rows in one launch (the heads / LSTMCell /
// answer-MLP bias grads and the query's dQ, each ~5 us as its own launch):
// block x runs column block (x - cb[k]) of segment k.
__global__ void k_colsum_multi(ColSums c, int M, int rows_per) {
  __shared__ float red[256];
  int k = 0;
  while (k + 1 < c.n && (int)blockIdx.x >= c.cb[k + 1]) ++k;
  const ColSumSeg s = c.s[k];
  const int col = ((int)blockIdx.x - c.cb[k]) * 64 + (threadIdx.x & 63);
  const int r0 = blockIdx.y * rows_per, r1 = min(M, r0 + rows_per);
  float acc = 0.f;
  if (col < s.N) {
#pragma unroll 8
    for (int r = r0 + (threadIdx.x >> 6); r < r1; r += 4) acc += s.X[(size_t)r * s.ld + col];
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  if (threadIdx.x < 64 && col < s.N)
    atomicAdd(s.out + col, red[threadIdx.x] + red[threadIdx.x + 64] + red[threadIdx.x + 128] + red[threadIdx.x + 192]);
}

hipError_t colsum_multi(ColSums c, int M, hipStream_t st) {
  if (M <= 0 || c.n <= 0) return hipSuccess;
  c.cb[0] = 0;
  for (int k = 0; k < c.n; ++k) c.cb[k + 1] = c.cb[k] + (c.s[k].N + 63) / 64;
  const int cols = c.cb[c.n];
  int split = (1024 + cols - 1) / cols;
  int rows_per = (M + split - 1) / split;
  if (rows_per < 64) rows_per = 64;
  split = (M + rows_per - 1) / rows_per;
  hipLaunchKernelGGL(k_colsum_multi, dim3(cols, split), dim3(256), 0, st, c, M, rows_per);
  return hipGetLastError();
}

}  // namespace aaa
