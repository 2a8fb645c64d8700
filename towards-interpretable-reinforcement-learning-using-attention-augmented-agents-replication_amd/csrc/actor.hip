// Actor step chain (aaa_actor_step): one environment step of the agent for a
// few rows -- the acting half of the reference's loop (Policy.forward,
// main_mp.py:49-59; test_model.py:42-73 rollouts): vision CNN -> ConvLSTM
// step with carried state -> constant-query attention readout -> answer MLP
// -> LSTMCell (zero state, Q1) -> policy/value heads -> action draw.
//
// The learner's kernels are whole-batch GEMMs; at B = 1 they run as ~25
// latency-bound launches (188-226 us graph-replayed, profiles/r01).  Here each
// stage is split across the chip by its OUTPUT (conv2 pixels, ConvLSTM
// tile x K-slice, readout position chunks, answer rows, LSTMCell units), and
// the chain is six launches.  Launches and not one persistent kernel: a
// seam inside one launch costs a grid barrier (~4-5 us, MI355X_MICROARCH.md
// 'barrier-xcd'), a kernel boundary ~1.2-1.5 us ('boundary'); the answer MLP /
// LSTMCell / heads seams are all-to-all.  The two reductions that are not
// (the ConvLSTM's K slices, the readout's position chunks) finish inside
// their launch: the last workgroup to arrive at a counter merges the partials.
//
// Numerics: fp32 throughout (the ConvLSTM and conv1 on exact-fp32
// v_mfma_f32_16x16x4_f32, the rest fp32 FMA); only the summation order
// differs from the learner path (tests/test_gpu_actor.py compares both at
// 1e-4).  The action draw is draw_row (sampling.h), bit-identical to
// aaa_sample_actions on the same logits, seed and counter.
#include "actor.h"
#include "epilogues.h"
#include "loaders_b.h"
#include "sampling.h"

namespace aaa {

namespace {

__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
__device__ __forceinline__ float dot4(const f32x4& a, const f32x4& b) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2] + a[3] * b[3];
}
__device__ __forceinline__ float wsum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wmax(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ f32x4 mfma4(float a, float b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// ------------------------------------------------------------ vision ------
// One workgroup per (conv2 output pixel, frame): VisionNetwork.vision_cnn
// (attention.py:155-170 on X.transpose(1,3), Q3: the packed weights carry
// the transposed kernel orientation).  conv2 (4x4, stride 2, pad 2) of pixel
// (oy, ox) reads the 4x4 window of conv1 outputs at rows 2oy-2.., which read
// frame rows 8oy-9 .. 8oy+10: that 20x20 RGB patch is staged in LDS once
// (conv1's zero padding included), conv1 runs on the window as a 32x16x256
// MFMA GEMM (rows = channels, columns = window pixels, K = 64 taps x RGBx;
// 4 waves split K), conv1 outputs outside the H1 x W1 map are conv2's zero
// padding, and conv2 is 64 dot products of length 512 (4 waves x 16
// channels, lanes along K).
constexpr int kPatchLd = 81;   // floats per patch row: 4*81 = 4 (mod 64) spreads the 4 window rows over banks

template <typename TI>
__global__ void __launch_bounds__(256) k_act_vision(ActorParams p) {
  __shared__ float patch[20 * kPatchLd];
  __shared__ __attribute__((aligned(16))) float red[4][2][64][4];
  __shared__ __attribute__((aligned(16))) float y1w[16 * 32];
  __shared__ float red2[4][16][65];
  const int pix = blockIdx.x, f = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int oy = pix / p.w, ox = pix - oy * p.w;
  if (pix == 0) {   // this step's ConvLSTM tile, readout and LSTMCell counters, before those launches
    const int nt = 8 * actor_pix_tiles(p.P);
    for (int i = tid; i < nt; i += 256) p.zcnt[f * nt + i] = 0;
    if (tid == 0) p.zcnt[p.B * nt + f] = 0;
    if (tid == 0 && f == 0) p.zcnt[p.B * nt + p.B] = 0;   // the LSTMCell's (one launch-wide counter)
  }
  // conv2 weights of this wave's 16 channels, lane's 8 K values: issued first
  f32x4 w2a[16], w2b[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const float* wr = p.Wp2 + (size_t)(wv * 16 + j) * 512 + 8 * lane;
    w2a[j] = ld4(wr);
    w2b[j] = ld4(wr + 4);
  }
  // conv1 weights: A[i = lane&15][k = lane>>4] of the wave's 16 taps, both row tiles
  const int r = lane & 15, q = lane >> 4;
  float w1a[16], w1b[16];
#pragma unroll
  for (int t = 0; t < 16; ++t) {
    const int tap = wv * 16 + t;
    w1a[t] = p.Wp1[r * 256 + tap * 4 + q];
    w1b[t] = p.Wp1[(16 + r) * 256 + tap * 4 + q];
  }
  {
    const int r0 = 8 * oy - 9, c0 = 8 * ox - 9;
    const TI* fr = (const TI*)p.frames + (size_t)f * p.H * p.W * 3;
    for (int i = tid; i < 400; i += 256) {
      const int pr = i / 20, pc = i - pr * 20, iy = r0 + pr, ix = c0 + pc;
      float v0 = 0.f, v1 = 0.f, v2 = 0.f;
      if (iy >= 0 && iy < p.H && ix >= 0 && ix < p.W) {
        const TI* s = fr + ((size_t)iy * p.W + ix) * 3;
        v0 = (float)s[0]; v1 = (float)s[1]; v2 = (float)s[2];
      }
      float* d = patch + pr * kPatchLd + pc * 4;
      d[0] = v0; d[1] = v1; d[2] = v2; d[3] = 0.f;
    }
  }
  __syncthreads();
  {
    const int a = r >> 2, b = r & 3;   // B operand: window pixel r = lane&15, channel q of the tap
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const int tap = wv * 16 + t, ky = tap >> 3, kx = tap & 7;
      const float bv = patch[(4 * a + ky) * kPatchLd + (4 * b + kx) * 4 + q];
      acc0 = mfma4(w1a[t], bv, acc0);
      acc1 = mfma4(w1b[t], bv, acc1);
    }
    *reinterpret_cast<f32x4*>(red[wv][0][lane]) = acc0;
    *reinterpret_cast<f32x4*>(red[wv][1][lane]) = acc1;
  }
  __syncthreads();
  if (tid < 128) {   // D[row 4(l>>4)+v][col l&15] of row tile ``tile``: sum the 4 K quarters, bias, padding
    const int tile = tid >> 6, l = tid & 63, wp = l & 15, o0 = tile * 16 + 4 * (l >> 4);
    f32x4 s = *reinterpret_cast<const f32x4*>(red[0][tile][l]);
#pragma unroll
    for (int k = 1; k < 4; ++k) s += *reinterpret_cast<const f32x4*>(red[k][tile][l]);
    const int iy = 2 * oy - 2 + (wp >> 2), ix = 2 * ox - 2 + (wp & 3);
    const bool ok = iy >= 0 && iy < p.H1 && ix >= 0 && ix < p.W1;
#pragma unroll
    for (int v = 0; v < 4; ++v) y1w[wp * 32 + o0 + v] = ok ? s[v] + p.b1[o0 + v] : 0.f;
  }
  __syncthreads();
  {   // conv2: y1w index (a*4 + b)*32 + ci is the packed K order (tap*32 + ci)
    const f32x4 ya = *reinterpret_cast<const f32x4*>(y1w + 8 * lane);
    const f32x4 yb = *reinterpret_cast<const f32x4*>(y1w + 8 * lane + 4);
#pragma unroll
    for (int j = 0; j < 16; ++j) red2[wv][j][lane] = dot4(w2a[j], ya) + dot4(w2b[j], yb);
  }
  __syncthreads();
  {
    const int j = lane >> 2, part = lane & 3;
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) s += red2[wv][j][part * 16 + i];
    s += __shfl_xor(s, 1, 64);
    s += __shfl_xor(s, 2, 64);
    const int o = wv * 16 + j;
    if (part == 0) p.X[((size_t)f * p.P + pix) * 64 + o] = s + p.b2[o];
  }
}

// ---------------------------------------------------------- ConvLSTM ------
// ConvLSTMCell step (attention.py:110-126, zero peepholes) as an implicit
// GEMM D[512 gate rows][P pixels] = W[.][1728] * [x | h_{t-1}] (3x3 taps) on
// exact-fp32 MFMA.  The chain's floor is the fp32 MFMA rate (1.27 GFLOP at
// 210x160 = 8 us chip-wide), so the tiling keeps the operand traffic far
// below what the chip can feed: 64 rows (16 channels x 4 gates,
// gate-interleaved) x 64 pixels per tile, each operand element read once per
// tile, and K cut into kActLstmKS slices so that B = 1 still fills the chip
// (8 x 9 tiles x 6 slices = 432 workgroups at 210x160).  Per K block of 16,
// half the workgroup stages the weight rows and half the pixels' im2col
// values (one float4 each, all of the slice's loads issued before the first
// MFMA) into a double-buffered LDS tile; each wave then runs a 16-row x
// 32-pixel block (one A read, two B reads, eight MFMAs).  The slices write
// their partial tiles to the workspace and the last to arrive (a per-tile
// counter the vision launch zeroed) sums them in slice order -- the same
// result whichever slice is last -- and runs the cell update.
// blockIdx -> tile is XCD-aware: row tile = blockIdx % 8, so an XCD's L2
// holds one 442 KB weight slab, and a tile's slices share that L2.
constexpr int kSC1 = 16;                      // buffer cache policy: sc1 (cross-workgroup hand-off)
constexpr int kLsPitch = 20;                  // floats per LDS row: 80 B puts 16 rows on disjoint banks
constexpr int kLsSteps = 108 / kActLstmKS;    // K blocks of 16 per slice

__global__ void __launch_bounds__(512) k_act_convlstm(ActorParams p, int npt) {
  __shared__ __attribute__((aligned(16))) float Wt[2][64 * kLsPitch];
  __shared__ __attribute__((aligned(16))) float Bt[2][64 * kLsPitch];
  __shared__ int is_last;
  const int f = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int rt = blockIdx.x & 7, slot = blockIdx.x >> 3;
  const int pt = slot / kActLstmKS, ks = slot - pt * kActLstmKS;
  const int tile = f * 8 * npt + pt * 8 + rt;
  // loader role: threads 0..255 the weight rows, 256..511 the pixels; 4 threads per row
  const bool isw = tid < 256;
  const int lr = (tid & 255) >> 2, qd = tid & 3;
  const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
  f32x4 g[kLsSteps];
  if (isw) {
    const float* src = p.WpXH + (size_t)(rt * 64 + lr) * 1728 + ks * kLsSteps * 16 + 4 * qd;
#pragma unroll
    for (int i = 0; i < kLsSteps; ++i) g[i] = ld4(src + 16 * i);
  } else {
    const int pix = pt * 64 + lr;
    const bool pin = pix < p.P;
    const int pc = pin ? pix : 0, y = pc / p.w, x = pc - y * p.w;
    const float* Xf = p.X + (size_t)f * p.P * 64;
    const float* Hf = p.hst + (size_t)f * p.P * 128;
#pragma unroll
    for (int i = 0; i < kLsSteps; ++i) {
      const int kb = ks * kLsSteps + i, tap = kb / 12, c0 = (kb - tap * 12) * 16 + 4 * qd;
      const int ky = tap / 3, kx = tap - ky * 3, ny = y + ky - 1, nx = x + kx - 1;
      const bool ok = pin && ny >= 0 && ny < p.h && nx >= 0 && nx < p.w;
      const int np = ok ? ny * p.w + nx : 0;
      const f32x4 v = c0 < 64 ? ld4(Xf + (size_t)np * 64 + c0) : ld4(Hf + (size_t)np * 128 + (c0 - 64));
      g[i] = ok ? v : zero;   // padding taps and the ragged last pixel tile
    }
  }
  const int st = lr * kLsPitch + 4 * qd;
  const int rb = wv >> 1, pb = (wv & 1) * 2, i16 = lane & 15, kq = lane >> 4;
  const int ra = (rb * 16 + i16) * kLsPitch + 4 * kq, rb0 = (pb * 16 + i16) * kLsPitch + 4 * kq;
  f32x4 acc0 = zero, acc1 = zero;
#pragma unroll
  for (int s = 0; s < kLsSteps; ++s) {
    *reinterpret_cast<f32x4*>((isw ? Wt[s & 1] : Bt[s & 1]) + st) = g[s];
    __syncthreads();   // double buffer: the buffer written here was last read before the previous barrier
    const f32x4 a = *reinterpret_cast<const f32x4*>(Wt[s & 1] + ra);
    const f32x4 b0 = *reinterpret_cast<const f32x4*>(Bt[s & 1] + rb0);
    const f32x4 b1 = *reinterpret_cast<const f32x4*>(Bt[s & 1] + rb0 + 16 * kLsPitch);
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      acc0 = mfma4(a[v], b0[v], acc0);
      acc1 = mfma4(a[v], b1[v], acc1);
    }
  }
  // partial tile (lane-native layout: 8 waves x 2 blocks x 64 lanes x 4) -> workspace.  Hand-off
  // without fences (an agent release writes back the whole L2): write-through (sc1) stores, every
  // wave's vmcnt(0), a barrier, one lane's agent-scope add; the last slice takes one agent acquire
  // (the partials are rewritten every step) and reads them with sc1 loads (glds.h EpiSliceFix)
  const __amdgpu_buffer_rsrc_t rs = make_rsrc(p.Zp + (size_t)tile * kActLstmKS * 4096, kActLstmKS * 4096 * 4);
  const uint32_t po = (uint32_t)((wv * 512 + 4 * lane) * 4);
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc0), rs, po + ks * 16384, 0, kSC1);
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc1), rs, po + ks * 16384 + 1024, 0, kSC1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const int old = __hip_atomic_fetch_add(p.zcnt + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old == kActLstmKS - 1) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    is_last = old == kActLstmKS - 1;
  }
  __syncthreads();
  if (!is_last) return;
  f32x4 z[2] = {zero, zero};
#pragma unroll
  for (int k = 0; k < kActLstmKS; ++k) {
    z[0] += __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, po + k * 16384, 0, kSC1));
    z[1] += __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, po + k * 16384 + 1024, 0, kSC1));
  }
  const int ch = rt * 16 + rb * 4 + kq;
  const f32x4 bias = ld4(p.bl + 4 * ch);
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const int pix = pt * 64 + (pb + e) * 16 + i16;
    if (pix >= p.P) continue;
    const size_t si = ((size_t)f * p.P + pix) * 128 + ch;
    float gi, gf, gc, go, c, h;
    GateFwd::run(z[e][0] + bias[0], z[e][1] + bias[1], z[e][2] + bias[2], z[e][3] + bias[3], p.cst[si], gi, gf,
                 gc, go, c, h);
    (p.cout ? p.cout : p.cst)[si] = c;
    p.Hs[si] = h;
    if (p.gates) *reinterpret_cast<f32x4*>(p.gates + ((size_t)f * p.P + pix) * 512 + 4 * ch) = f32x4{gi, gf, gc, go};
  }
}

// ----------------------------------------------------- attention readout --
// attention.py:319-348 with the constant query (Q1): logits K.Q with
// K = [O[:8] | S], spatial_softmax over the P positions (attention.py:235-241),
// readout of V = [O[8:] | S] (apply_alpha, :244-254).  One workgroup per chunk
// of kAttnChunk positions (34 at 210x160) reads only its positions' O and S
// rows: it stores its logits (for the map), its per-query max m_c and sum
// s_c of exp(l - m_c), and the partial readout sum_j exp(l_j - m_c) V_j.  The
// last chunk to arrive (the ConvLSTM's sc1 hand-off) merges them in chunk
// order -- weights exp(m_c - m) / sum_c exp(m_c - m) s_c, the same result
// whichever chunk is last -- into the answer row [a | Q | r | a_prev | 0-pad]
// and writes the attention map.  Each chunk also copies its share of h_t
// into the carried state (read by the next step's ConvLSTM launch).
template <int NQ>
__global__ void __launch_bounds__(256) k_act_attn(ActorParams p, int nch) {
  __shared__ float Qs[NQ * 72];
  __shared__ float E[kAttnChunk][NQ];
  __shared__ float Wc[kActMaxChunks][NQ];
  __shared__ float Mq[NQ], Tq[NQ];
  __shared__ int is_last;
  const int P = p.P, f = blockIdx.y, c = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const float* O = p.Hs + (size_t)f * P * 128;
  const float* S = p.basis;
  const int p0 = c * kAttnChunk, np = min(kAttnChunk, P - p0);
  for (int i = tid; i < NQ * 72; i += 256) Qs[i] = p.Q[i];
  {   // this chunk's share of h_t -> the carried state
    const int n4 = P * 32, per = (n4 + nch - 1) / nch;
    const f32x4* src = reinterpret_cast<const f32x4*>(O);
    f32x4* dst = reinterpret_cast<f32x4*>((p.hout ? p.hout : p.hst) + (size_t)f * P * 128);
    for (int i = c * per + tid; i < min(n4, (c + 1) * per); i += 256) dst[i] = src[i];
  }
  __syncthreads();
  const __amdgpu_buffer_rsrc_t rl = make_rsrc(p.Lg + (size_t)f * P * NQ, (uint32_t)(P * NQ * 4));
  if (tid < kAttnChunk * NQ) {   // logits: one thread per (position, query)
    const int j = tid / NQ, q = tid - j * NQ;
    float l = -INFINITY;
    if (j < np) {
      const int pp = p0 + j;
      const float* Qq = Qs + q * 72;
      f32x4 kv[18];
      kv[0] = ld4(O + (size_t)pp * 128);
      kv[1] = ld4(O + (size_t)pp * 128 + 4);
#pragma unroll
      for (int k = 0; k < 16; ++k) kv[2 + k] = ld4(S + (size_t)pp * 64 + 4 * k);
      __builtin_amdgcn_sched_barrier(0);   // all 18 loads in flight before the sums
      float acc = 0.f;
#pragma unroll
      for (int k = 0; k < 18; ++k)
        acc += kv[k][0] * Qq[4 * k] + kv[k][1] * Qq[4 * k + 1] + kv[k][2] * Qq[4 * k + 2] + kv[k][3] * Qq[4 * k + 3];
      l = acc;
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, l), rl, (uint32_t)((pp * NQ + q) * 4), 0,
                                            kSC1);
    }
    E[j][q] = l;
  }
  __syncthreads();
  for (int q = wv; q < NQ; q += 4) {   // the chunk's max and sum per query (lanes over positions)
    const float l = lane < kAttnChunk ? E[lane][q] : -INFINITY;
    const float m = wmax(l);
    const float e = lane < np ? expf(l - m) : 0.f;
    const float sm = wsum(e);
    if (lane < kAttnChunk) E[lane][q] = e;
    if (lane == 0) { Mq[q] = m; Tq[q] = sm; }
  }
  __syncthreads();
  float* part = p.Apart + (size_t)f * nch * NQ * kAttnPart;
  const __amdgpu_buffer_rsrc_t rp = make_rsrc(part, (uint32_t)(nch * NQ * kAttnPart * 4));
  for (int u = tid; u < 46 * NQ; u += 256) {   // partial readout: (column float4 g, query q)
    const int q = u / 46, g = u - q * 46;
    const float* src = g < 30 ? O + 8 + 4 * g : S + 4 * (g - 30);
    const int ld = g < 30 ? 128 : 64;
    f32x4 vv[kAttnChunk];
#pragma unroll
    for (int j = 0; j < kAttnChunk; ++j) vv[j] = ld4(src + (size_t)(p0 + min(j, np - 1)) * ld);   // clamped rows
    __builtin_amdgcn_sched_barrier(0);   // every load issued before the sums
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < kAttnChunk; ++j) acc += (j < np ? E[j][q] : 0.f) * vv[j];
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc), rp,
                                           (uint32_t)(((c * NQ + q) * kAttnPart + 4 * g) * 4), 0, kSC1);
  }
  if (tid < NQ) {
    const f32x4 ms = {Mq[tid], Tq[tid], 0.f, 0.f};
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, ms), rp,
                                           (uint32_t)(((c * NQ + tid) * kAttnPart + 184) * 4), 0, kSC1);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const int old = __hip_atomic_fetch_add(p.zcnt + p.B * 8 * actor_pix_tiles(P) + f, 1, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
    if (old == nch - 1) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    is_last = old == nch - 1;
  }
  __syncthreads();
  if (!is_last) return;
  for (int q = wv; q < NQ; q += 4) {   // merge weights: exp(m_c - m) / sum_c exp(m_c - m) s_c
    float mc[kActMaxChunks / 64], sc[kActMaxChunks / 64];
    float m = -INFINITY;
#pragma unroll
    for (int k = 0; k < kActMaxChunks / 64; ++k) {
      const int cc = lane + 64 * k;
      mc[k] = -INFINITY;
      sc[k] = 0.f;
      if (cc < nch) {
        const f32x4 v = __builtin_bit_cast(
            f32x4, __builtin_amdgcn_raw_buffer_load_b128(rp, (uint32_t)(((cc * NQ + q) * kAttnPart + 184) * 4), 0, kSC1));
        mc[k] = v[0];
        sc[k] = v[1];
      }
      m = fmaxf(m, mc[k]);
    }
    m = wmax(m);
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < kActMaxChunks / 64; ++k) {
      mc[k] = lane + 64 * k < nch ? expf(mc[k] - m) : 0.f;
      t += mc[k] * sc[k];
    }
    t = wsum(t);
    const float inv = 1.f / t;
#pragma unroll
    for (int k = 0; k < kActMaxChunks / 64; ++k)
      if (lane + 64 * k < nch) Wc[lane + 64 * k][q] = mc[k] * inv;
    if (lane == 0) { Mq[q] = m; Tq[q] = inv; }
  }
  __syncthreads();
  float* arow = p.arow + (size_t)f * p.ans_ld;
  for (int u = tid; u < 46 * NQ; u += 256) {   // answer row: the merged readouts
    const int q = u / 46, g = u - q * 46;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int c0 = 0; c0 < nch; c0 += 8) {   // 8 chunks' loads in flight (clamped, zero weights past nch)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int cc = min(c0 + k, nch - 1);
        const float w = c0 + k < nch ? Wc[cc][q] : 0.f;
        acc += w * __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                 rp, (uint32_t)(((cc * NQ + q) * kAttnPart + 4 * g) * 4), 0, kSC1));
      }
    }
    *reinterpret_cast<f32x4*>(arow + q * 184 + 4 * g) = acc;
  }
  for (int i = NQ * 184 + tid; i < p.ans_ld; i += 256) {   // [.. | Q | r | a_prev | 0-pad]
    float v = 0.f;
    if (i < NQ * 256) v = Qs[i - NQ * 184];
    else if (i == NQ * 256) v = p.prev_reward ? p.prev_reward[f] : 0.f;
    else if (i == NQ * 256 + 1) v = p.prev_action ? p.prev_action[f] : 0.f;
    arow[i] = v;
  }
  if (p.attn) {
    for (int i = tid; i < P * NQ; i += 256) {
      const int q = i % NQ;
      const float l = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rl, (uint32_t)(i * 4), 0, kSC1));
      p.attn[(size_t)f * P * NQ + i] = expf(l - Mq[q]) * Tq[q];
    }
  }
}

// ------------------------------------------------- answer layer 0 (ReLU) --
// answer_processor.0 + ReLU (attention.py:277-282, 350): one wave per row of
// the [512][ans_ld] weights, the answer row read from the readout's output.
template <int NQ>
__global__ void __launch_bounds__(256) k_act_ans0(ActorParams p) {
  constexpr int NIT = NQ == 4 ? 5 : 9;   // float4 slices per lane: 256 * NIT >= ans_ld
  const int f = blockIdx.y, lane = threadIdx.x & 63, row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const float* wr = p.W1p + (size_t)row * p.ans_ld;
  const float* x = p.arow + (size_t)f * p.ans_ld;
  f32x4 wv[NIT], xv[NIT];
#pragma unroll
  for (int i = 0; i < NIT; ++i) {   // clamped offsets: every load unconditional and in flight at once
    const int k = min(4 * lane + 256 * i, p.ans_ld - 4);
    wv[i] = ld4(wr + k);
    xv[i] = ld4(x + k);
  }
  __builtin_amdgcn_sched_barrier(0);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NIT; ++i)
    if (4 * lane + 256 * i < p.ans_ld) s += dot4(wv[i], xv[i]);
  s = wsum(s) + p.a0b[row];
  if (lane == 0) p.hid1[(size_t)f * 512 + row] = fmaxf(s, 0.f);
}

// ------------------------------------------- answer layer 2 (linear) -----
// answer_processor.2 (attention.py:277-282): AO = W2 hid1 + b2, one wave per
// output row (weights read once into registers), all B frames.
__global__ void __launch_bounds__(256) k_act_ans2(ActorParams p) {
  const int lane = threadIdx.x & 63, row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const float* wr = p.A2W + (size_t)row * 512 + 8 * lane;
  const f32x4 w0 = ld4(wr), w1 = ld4(wr + 4);
  for (int f = 0; f < p.B; ++f) {
    const float* x = p.hid1 + (size_t)f * 512 + 8 * lane;
    const float s = wsum(dot4(w0, ld4(x)) + dot4(w1, ld4(x + 4)));
    if (lane == 0) p.AO[(size_t)f * 256 + row] = s + p.a2b[row];
  }
}

// --------------------------------------------------- heads + action draw --
// policy_head / values_head (attention.py:365-367) and Policy.forward's draw
// (main_mp.py:54-58) in one workgroup: rows o < A -> logits, A <= o < 2A ->
// values, then one wave per frame runs draw_row on the logits it just wrote
// (the device counter is read by every wave before the single increment).
// LH comes from the other LSTMCell workgroups' sc1 stores: sc1 loads.
__device__ __forceinline__ void heads_draw(const ActorParams& p, float* lg) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, A = p.A, R = 2 * A;
  const __amdgpu_buffer_rsrc_t rh = make_rsrc(p.LH, (uint32_t)(p.B * 256 * 4));
  // rows in chunks of 8 per wave, each chunk's weight and state loads issued before its math
  for (int o0 = wv * 8; o0 < R; o0 += 32) {
    f32x4 w[8];
    float b[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int o = min(o0 + j, R - 1);
      w[j] = ld4(p.Whd + (size_t)o * 256 + 4 * lane);
      b[j] = p.bhd[o];
    }
    for (int f = 0; f < p.B; ++f) {
      const f32x4 x =
          __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rh, (uint32_t)((f * 256 + 4 * lane) * 4), 0, kSC1));
      float s[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] = dot4(w[j], x);
#pragma unroll
      for (int o = 32; o > 0; o >>= 1)
#pragma unroll
        for (int j = 0; j < 8; ++j) s[j] += __shfl_xor(s[j], o, 64);
      if (lane < 8 && o0 + lane < R) {   // lane j stores row o0 + j
        float v = s[0] + b[0];
#pragma unroll
        for (int j = 1; j < 8; ++j) v = lane == j ? s[j] + b[j] : v;
        const int o = o0 + lane;
        if (o < A) {
          p.logits[(size_t)f * A + o] = v;
          lg[f * A + o] = v;
        } else {
          p.values[(size_t)f * A + o - A] = v;
        }
      }
    }
  }
  if (!p.actions) return;
  __syncthreads();
  const uint64_t ctr = p.counter ? (uint64_t)*p.counter : 0ull;
  for (int f = wv; f < p.B; f += 4) draw_row(lg + f * A, A, p.seed, ctr, f, p.actions, p.logp, p.jac);
  __syncthreads();   // every wave has read the counter
  if (p.counter && tid == 0) *p.counter = ctr + 1ull;
}

// ------------------------------------------- LSTMCell (zero state) + heads --
// policy_core from zero state (attention.py:354-355, Q1): one wave per unit u,
// its four gate rows 4u..4u+3 of the interleaved [1024][256] weights;
// c = i*g~ (+ f*0), h = o*tanh(c) -- the learner's EpiLstmCellFwd.  The last
// workgroup to arrive (sc1 hand-off as the ConvLSTM's) runs the heads and the
// draw: one launch fewer than a separate heads kernel.
__global__ void __launch_bounds__(256) k_act_lstmcell(ActorParams p) {
  __shared__ float lg[16 * 256];
  __shared__ int is_last;
  const int tid = threadIdx.x, lane = tid & 63, u = blockIdx.x * 4 + (tid >> 6);
  f32x4 w[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) w[g] = ld4(p.Wihp + (size_t)(4 * u + g) * 256 + 4 * lane);
  const f32x4 b = ld4(p.blc + 4 * u);
  const __amdgpu_buffer_rsrc_t rh = make_rsrc(p.LH, (uint32_t)(p.B * 256 * 4));
  for (int f = 0; f < p.B; ++f) {
    const f32x4 x = ld4(p.AO + (size_t)f * 256 + 4 * lane);
    float z[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) z[g] = wsum(dot4(w[g], x));
    if (lane == 0) {
      const float gi = sigm_acc(z[0] + b[0]), gf = sigm_acc(z[1] + b[1]);
      const float gc = tanhf(z[2] + b[2]), go = sigm_acc(z[3] + b[3]);
      const float c = gf * 0.f + gi * gc;
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, go * tanhf(c)), rh,
                                            (uint32_t)((f * 256 + u) * 4), 0, kSC1);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const int old = __hip_atomic_fetch_add(p.zcnt + p.B * 8 * actor_pix_tiles(p.P) + p.B, 1, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
    if (old == (int)gridDim.x - 1) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    is_last = old == (int)gridDim.x - 1;
  }
  __syncthreads();
  if (is_last) heads_draw(p, lg);
}

}  // namespace

hipError_t actor_launch(const ActorParams& p, hipStream_t st) {
  if (p.B < 1 || p.B > 16 || (p.nq != 4 && p.nq != 8) || p.A < 1 || p.A > 256 || p.ans_ld % 4 ||
      p.ans_ld > 2304 || actor_chunks(p.P) > kActMaxChunks)
    return hipErrorInvalidValue;
  if (p.u8)
    hipLaunchKernelGGL(k_act_vision<uint8_t>, dim3(p.P, p.B), dim3(256), 0, st, p);
  else
    hipLaunchKernelGGL(k_act_vision<float>, dim3(p.P, p.B), dim3(256), 0, st, p);
  const int npt = actor_pix_tiles(p.P);
  hipLaunchKernelGGL(k_act_convlstm, dim3(8 * kActLstmKS * npt, p.B), dim3(512), 0, st, p, npt);
  const int nch = actor_chunks(p.P);
  if (p.nq == 4)
    hipLaunchKernelGGL(k_act_attn<4>, dim3(nch, p.B), dim3(256), 0, st, p, nch);
  else
    hipLaunchKernelGGL(k_act_attn<8>, dim3(nch, p.B), dim3(256), 0, st, p, nch);
  if (p.nq == 4)
    hipLaunchKernelGGL(k_act_ans0<4>, dim3(128, p.B), dim3(256), 0, st, p);
  else
    hipLaunchKernelGGL(k_act_ans0<8>, dim3(128, p.B), dim3(256), 0, st, p);
  hipLaunchKernelGGL(k_act_ans2, dim3(64), dim3(256), 0, st, p);
  hipLaunchKernelGGL(k_act_lstmcell, dim3(64), dim3(256), 0, st, p);
  return hipGetLastError();
}

}  // namespace aaa
