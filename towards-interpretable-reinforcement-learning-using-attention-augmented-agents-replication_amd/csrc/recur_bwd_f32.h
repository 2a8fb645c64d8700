// Frame-group-resident ConvLSTM BPTT, fp32 (exact v_mfma_f32_32x32x2_f32).
//
// The backward of the reference's recurrence (attention.py:117-125, autograd
// at main_mp.py:77): per step s = T-1 .. 1, dh_{s-1} = W_h^T (*) dZ_s (the
// transposed 3x3 gate convs) and the gate backward of step s-1, which turns
// dh_{s-1} + dO_{s-1} and the carried dc into dZ_{s-1}.  As in the forward
// (recur_f32.h), G = 8 workgroups own one frame for all steps (config 2:
// B = 32 -> 256 workgroups).  Workgroup kh owns the h channels
// [16 kh, 16 kh + 16): the 64 gate-interleaved dZ rows its gate backward
// produces, which stay in its LDS as the B operand of its next dgrad.  That
// dgrad is split over the workgroups by K: workgroup kh contracts only its own
// 64 dZ rows (9 taps x 64 = K 576) but for ALL 128 output channels, and the
// eight partial dh slices are exchanged -- each workgroup publishes the
// 7 x 16 channels that belong to the others (write-through stores, a flag) and
// sums the seven partials addressed to it with its own.  Per step a workgroup
// moves 2 x 54 KB through L2.  (The alternative, every workgroup re-reading
// the frame's whole dZ_s -- 248 KB per step by LDS-DMA -- was LDS-DMA bound:
// 1030 us at config 2 against 980 us for the per-step launches,
// profiles/r03/f32rec/bwd_dz_exchange.txt.)
//
// Workgroup: 4 waves; D[128 channels][128 pixel columns] as 4 x 4 tiles of
// 32 x 32; wave w owns row blocks 2 (w & 1) + {0, 1} and column blocks
// 2 (w >> 1) + {0, 1} (two phases of two column blocks each, the first
// half's partials travelling under the second half's MFMAs, measured slower:
// 961 vs 916 us, the 8-MFMA quads cost more than the exposed exchange saved).
// K order: 72 quads (9 taps x 8 groups of 8 dZ rows);
// lane (r32, hh) reads the 4 rows 8 q8 + 4 hh .. + 3 of its pixel with one
// ds_read_b128 (4 k-steps) and the matching 16 B of the fragment-order weights
// (k_pack_wb32).
// DX (the production S6 + PS kernel): the 64 dx rows (conv2's output gradient,
// rows 0..63 of W^T) ride in the same K loop on the same pre-split dZ image --
// a third 32-row block per wave (dx row block rw, its two column blocks), so
// dZ is split once, where the gate backward produces it, for both dgrads
// (the batched dx GEMM it replaces split each dZ element once per tap it
// gathered).  The dx partials travel with the dh partials: workgroup kh owns dx
// channels [8 kh, 8 kh + 8), sums the eight partials of its channels and
// writes them to dY2 (every step, s = T-1 .. 0), and keeps their pixel sums
// for conv2's bias gradient (dxb).
#pragma once
#include "common.h"
#include "epilogues.h"
#include "glds.h"
#include "recur.h"
#include "recur_f32.h"

namespace aaa {

constexpr int kB32Q = 72;                     // quads per step (9 taps x 8)
constexpr int kB32PD = 8;                     // A quads in flight (register slots): slot = q8
constexpr int kB32QP = kB32Q + kB32PD - 1;    // packed quads per workgroup slice (first PD-1 repeated)
constexpr int kB32PP = (kB32Q + kB32PD) / 2;   // packed quad PAIRS per workgroup slice (DX's paired streams)
constexpr int kB32IB = 44 * 1024;             // own dZ image: 169 pixels x 64 rows fp32 (256 B)
constexpr int kB32NBUF = 3;                   // partial-dh exchange buffers (step mod 3)

// Wb[(((kh * kB32QP + q) * 4 + rb) * 64 + lane) * 4 + j] =
//   WdT[64 + 32 rb + lane % 32][tap * 512 + 64 kh + 8 q8 + 4 (lane / 32) + j],  q % kB32Q = tap * 8 + q8
static __global__ void __launch_bounds__(256) k_pack_wb32(const float* __restrict__ WdT, float* __restrict__ Wb) {
  const int i = blockIdx.x * 256 + (int)threadIdx.x;   // one 16-B chunk
  if (i >= 8 * kB32QP * 4 * 64) return;
  const int lane = i & 63, rb = (i >> 6) & 3, kq = i >> 8, q = kq % kB32QP, kh = kq / kB32QP;
  const int qq = q % kB32Q, tap = qq >> 3, q8 = qq & 7;
  const int row = 64 + 32 * rb + (lane & 31), k = tap * 512 + 64 * kh + 8 * q8 + 4 * (lane >> 5);
  *reinterpret_cast<f32x4*>(Wb + (size_t)i * 4) = *reinterpret_cast<const f32x4*>(WdT + (size_t)row * 4608 + k);
}

inline hipError_t pack_wb32(const float* WdT, float* Wb, hipStream_t st) {
  hipLaunchKernelGGL(k_pack_wb32, dim3((8 * kB32QP * 4 * 64 + 255) / 256), dim3(256), 0, st, WdT, Wb);
  return hipGetLastError();
}

// Exchange buffer floats: [kB32NBUF][B][8 dst][8 src][128 px][kB32XC ch]: 16 dh channels, then
// (DX) the destination's 8 dx channels
constexpr int kB32XC = 24;
inline size_t b32_xpart_floats(int B) { return (size_t)kB32NBUF * B * 64 * 128 * kB32XC; }

// Every fragment-order operand stream of the fp32 recurrences in ONE launch, straight from the
// packed matrices (was nine launches per weight update): the forward's Wf (k_pack_wf32's order)
// and the BPTT's Wb (k_pack_wb32's) as fp32 copies and three-way bf16 splits (k_split_frag's
// layout), the dx rows' Wx split (DX: k_pack_wb32's order over W^T rows 0..63: chunk
// (((kh * kB32QP + q) * 2 + rb) * 64 + lane)) and the batched dx's WdT planes
// (split_planes over W^T rows 0..63).
struct FragPack {
  const float* WpXH;   // [512][1728]
  const float* WdT;    // [192][4608]
  float* Wf;           // fp32 fragment order (16 * kF32QP * 64 chunks)
  u32x2* Wf6;
  u32x4* Wf6p;         // the pre-split forward's paired stream (16 * kF32PP * 3 * 64 x 16 B)
  float* Wb;           // (8 * kB32QP * 4 * 64 chunks)
  u32x2* Wb6;
  u32x2* Wx6;          // (8 * kB32QP * 2 * 64 chunks)
  u32x4* Wb6p;         // DX's paired streams: [kh][pair][rb][part][lane] x 16 B
  u32x4* Wx6p;
  __bf16* WdT6;        // 3 planes of 64 * 4608
};
__device__ __forceinline__ void split_chunk(const f32x4& x, u32x2 (&part)[3]) {
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    uint32_t h2[2], m2[2], l2[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const float v = x[2 * e + k];
      const __bf16 hi = (__bf16)v;
      const float r = v - (float)hi;
      const __bf16 mid = (__bf16)r;
      const __bf16 lo = (__bf16)(r - (float)mid);
      h2[k] = __builtin_bit_cast(uint16_t, hi);
      m2[k] = __builtin_bit_cast(uint16_t, mid);
      l2[k] = __builtin_bit_cast(uint16_t, lo);
    }
    part[0][e] = h2[0] | (h2[1] << 16);
    part[1][e] = m2[0] | (m2[1] << 16);
    part[2][e] = l2[0] | (l2[1] << 16);
  }
}
constexpr int kFragNf = 16 * kF32QP * 64, kFragNb = 8 * kB32QP * 4 * 64, kFragNx = 8 * kB32QP * 2 * 64;
constexpr int kFragNd = 64 * 4608 / 4, kFragNp = 16 * kF32PP * 64;
constexpr int kFragNbp = 8 * kB32PP * 4 * 64, kFragNxp = 8 * kB32PP * 2 * 64;
static __global__ void __launch_bounds__(256) k_pack_frag_f32(FragPack a) {
  int c = blockIdx.x * 256 + (int)threadIdx.x;   // one 16-B chunk of one stream
  const int lane = c & 63;
  const float* src;
  float* f32dst = nullptr;
  u32x2* dst6;
  if (c < kFragNf) {
    const int rq = c >> 6, q = rq % kF32QP, rb = rq / kF32QP;
    src = a.WpXH + (size_t)(rb * 32 + (lane & 31)) * 1728 + f32_k(q % kF32Q) + (lane >> 5) * 4;
    f32dst = a.Wf;
    dst6 = a.Wf6;
  } else if ((c -= kFragNf) < kFragNb) {
    const int rb = (c >> 6) & 3, kq = c >> 8, q = kq % kB32QP, kh = kq / kB32QP, qq = q % kB32Q;
    src = a.WdT + (size_t)(64 + 32 * rb + (lane & 31)) * 4608 + (qq >> 3) * 512 + 64 * kh + 8 * (qq & 7) +
          4 * (lane >> 5);
    f32dst = a.Wb;
    dst6 = a.Wb6;
  } else if ((c -= kFragNb) < kFragNx) {
    const int rb = (c >> 6) & 1, kq = c >> 7, q = kq % kB32QP, kh = kq / kB32QP, qq = q % kB32Q;
    src = a.WdT + (size_t)(32 * rb + (lane & 31)) * 4608 + (qq >> 3) * 512 + 64 * kh + 8 * (qq & 7) + 4 * (lane >> 5);
    dst6 = a.Wx6;
  } else if ((c -= kFragNx) < kFragNp) {   // Wf6p: (row block, pair, lane) -> parts of quads 2 pj, 2 pj + 1
    const int rp = c >> 6, pj = rp % kF32PP, rb = rp / kF32PP;
    u32x2 part[2][3];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int q = (2 * pj + k) % kF32Q;
      const f32x4 x = *reinterpret_cast<const f32x4*>(a.WpXH + (size_t)(rb * 32 + (lane & 31)) * 1728 + f32_k(q) +
                                                      (lane >> 5) * 4);
      split_chunk(x, part[k]);
    }
#pragma unroll
    for (int p = 0; p < 3; ++p)
      a.Wf6p[(rp * 3 + p) * 64 + lane] = u32x4{part[0][p].x, part[0][p].y, part[1][p].x, part[1][p].y};
    return;
  } else if ((c -= kFragNp) < kFragNbp + kFragNxp) {   // DX's paired BPTT streams
    const bool x = c >= kFragNbp;
    if (x) c -= kFragNbp;
    const int nrb = x ? 2 : 4, rb = (c >> 6) % nrb, kp = (c >> 6) / nrb, pj = kp % kB32PP, kh = kp / kB32PP;
    u32x2 part[2][3];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int qq = (2 * pj + k) % kB32Q;
      const f32x4 v = *reinterpret_cast<const f32x4*>(
          a.WdT + (size_t)((x ? 0 : 64) + 32 * rb + (lane & 31)) * 4608 + (qq >> 3) * 512 + 64 * kh + 8 * (qq & 7) +
          4 * (lane >> 5));
      split_chunk(v, part[k]);
    }
    u32x4* d = x ? a.Wx6p : a.Wb6p;
#pragma unroll
    for (int p = 0; p < 3; ++p)
      d[((c >> 6) * 3 + p) * 64 + lane] = u32x4{part[0][p].x, part[0][p].y, part[1][p].x, part[1][p].y};
    return;
  } else if ((c -= kFragNbp + kFragNxp) < kFragNd) {   // planes: hi, mid, lo of W^T rows 0..63
    const f32x4 x = *reinterpret_cast<const f32x4*>(a.WdT + (size_t)c * 4);
    u32x2 part[3];
    split_chunk(x, part);
#pragma unroll
    for (int p = 0; p < 3; ++p) *reinterpret_cast<u32x2*>(a.WdT6 + (size_t)p * 64 * 4608 + (size_t)c * 4) = part[p];
    return;
  } else {
    return;
  }
  const f32x4 x = *reinterpret_cast<const f32x4*>(src);
  if (f32dst) *reinterpret_cast<f32x4*>(f32dst + (size_t)c * 4) = x;
  u32x2 part[3];
  split_chunk(x, part);
#pragma unroll
  for (int p = 0; p < 3; ++p) dst6[((c >> 6) * 3 + p) * 64 + lane] = part[p];
}

inline hipError_t pack_frag_f32(const FragPack& a, hipStream_t st) {
  constexpr int n = kFragNf + kFragNb + kFragNx + kFragNp + kFragNbp + kFragNxp + kFragNd;
  hipLaunchKernelGGL(k_pack_frag_f32, dim3((n + 255) / 256), dim3(256), 0, st, a);
  return hipGetLastError();
}

struct RecBwdF32Params {
  const float* Wb;     // fragment-order W_h^T (k_pack_wb32)
  const float* dO;     // (T, B, P, 128) attention-path grad of h_t
  const float* Gt;     // (T, B, P, 512) gate activations
  const float* Cst;    // (T+1, B, P, 128): slot s+1 = c_s
  float* dC;           // (B, P, 128) dc carry: in = the carry after step T-1's gate backward, out = dc_0
  float* dZ;           // (T, B, P, 512): slot T-1 read, slots T-2 .. 0 written
  float* part;         // (T, B, 512) <- gate-bias partials per (step, frame)
  float* dh0;          // (B, P, 128) <- grad of h_{-1}, or null
  float* xp;           // partial-dh exchange (b32_xpart_floats)
  int* flags;          // [B][8] count of published partial steps (zeroed by the caller)
  int* report;         // partner-timeout report word (pair_wait)
  int spin;           // partner-wait budget, 100-MHz ticks (pair_wait)
  int T, B, h, w, P;
  short colhb[128];    // column -> top-left image pixel of its 3x3 window (padding columns: pixel P-1's)
  const u32x2* Wb6 = nullptr;   // S6: the three-way split of Wb (recur_f32.h k_split_frag)
  const u32x2* Wx6 = nullptr;   // DX: the three-way split of the dx rows (k_pack_frag_f32)
  const u32x4* Wb6p = nullptr;  // DX: Wb6 with quads 2j, 2j+1 of a part side by side per lane (one 16-B load)
  const u32x4* Wx6p = nullptr;  // DX: the dx rows, paired the same way
  float* dx = nullptr;          // DX: (T, B, P, 64) <- conv2's output gradient (dY2)
  float* dxb = nullptr;         // DX: (B, 64) <- its pixel-and-step sums (conv2's bias gradient per frame)
};

#ifdef AAA_STAMPS
__device__ uint64_t aaa_b32_stamps[512 * 64 * 4];
#define AAA_B32_STAMP(s, k)                                                                               \
  do {                                                                                                    \
    if (tid == 0 && (s) < 64) aaa_b32_stamps[(blk * 64 + (s)) * 4 + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define AAA_B32_STAMP(s, k) do {} while (0)
#endif

// ABL (diagnostic builds only, tools/ubench/f32rec): bit 0 = no partner waits,
// bit 1 = no MFMAs, bit 3 = no exchange (partials neither stored nor loaded),
// bit 4 (S6) = no three-way split of the B fragments (hi only).
// Production launches use 0.
// S6: the MFMAs on the bf16 MFMA at fp32 accuracy, two quads per k-step with
// three-way split operands (as recur_f32.h S6, gemm.h SPLIT6).
// PDS: the S6 kernel's A quads in flight (4 or 8).
// PS (S6 only): the dZ image held pre-split (recur_f32.h k_convlstm_fwd_f32ps's layout:
// borderless, the zero pixel kPsZP (the image's last), pixel pitch 400 B, chunk (part * 4 + g) * 2 + hh for the
// 16-row group g) -- the gate backward splits each dZ value once as it writes the image,
// and the K loop reads bf16 parts only (no per-wave split of the B fragments).
template <int ABL = 0, bool S6 = false, int PDS = kB32PD, bool PS = false, bool DX = false>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
k_convlstm_bwd_f32(RecBwdF32Params p) {
  static_assert(!PS || S6, "PS: the split-product kernel");
  static_assert(!DX || PS, "DX: the pre-split kernel");
  constexpr int NR = DX ? 3 : 2;                 // 32-row blocks per wave: two of dh (+ one of dx)
  constexpr int G = 8, NG = 2;                   // NG: (pixel, 4-channel) groups per thread (484 <= 512)
  constexpr int IMB = PS ? kPsXB : kB32IB;
  __shared__ __attribute__((aligned(16))) unsigned char zim[IMB];   // own dZ rows of the current step
  __shared__ __attribute__((aligned(16))) f32x4 own[128][DX ? 6 : 4];  // own partial dh [px][quad] (+ dx: quads 4, 5)
  __shared__ __attribute__((aligned(16))) float bred[4][64];           // per-wave bias partials

  const int blk = (int)blockIdx.x, xcd = blk & 7, loc = blk >> 3;
  const int b = xcd + 8 * (loc / G), kh = loc % G;
  if (b >= p.B) return;
  const int tid = (int)threadIdx.x, lane = tid & 63;
  uint64_t wdl = 0;   // partner-wait deadline (common.h wait_expired), set by the first wait that polls
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r32 = lane & 31, hh = lane >> 5;
  const int rw = wave & 1, cw = wave >> 1;
  const int P = p.P, W2 = p.w + 2;
  const size_t M = (size_t)p.B * P;
  auto hidx = [&](int pp) { return (pp / p.w + 1) * W2 + pp % p.w + 1; };
  // 16-B chunk q of image pixel (y, x) at slot q ^ (key & 15), key = y * w + x (recur_f32.h)
  auto sw16 = [](int q, int key) { return (q ^ (key & 15)) << 4; };
  // exchange slot of (buffer, destination, source): [128 px][16 ch]
  auto xslot = [&](int buf, int dst, int src) {
    return p.xp + ((((size_t)buf * p.B + b) * 8 + dst) * 8 + src) * 128 * kB32XC;
  };

  {  // zero the image (borders / the zero pixel stay zero)
    u32x4* z = reinterpret_cast<u32x4*>(zim);
    for (int i = tid; i < IMB / 16; i += 256) z[i] = u32x4{0u, 0u, 0u, 0u};
  }
  __syncthreads();

  // per-thread gate-backward groups: g = tid + 256 n -> pixel g / 4, channels 16 kh + 4 (g % 4) .. + 3
  const int cq = tid & 3;
  float dcr[NG][4];
#pragma unroll
  for (int n = 0; n < NG; ++n) {
    const int px = (tid + 256 * n) >> 2;
#pragma unroll
    for (int e = 0; e < 4; ++e) dcr[n][e] = px < P ? p.dC[((size_t)b * P + px) * 128 + 16 * kh + 4 * cq + e] : 0.f;
  }
  // gate-bias partials of this workgroup's 64 rows of dZ_s over the frame's pixels -> part[s][b]
  auto bias_flush = [&](int s, f32x4 (&bs)[4]) {
    // lanes of one wave with equal cq (lane % 4) hold the same 16 rows: reduce over lane / 4
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        float v = bs[e][g];
        v += __shfl_xor(v, 4, 64);
        v += __shfl_xor(v, 8, 64);
        v += __shfl_xor(v, 16, 64);
        v += __shfl_xor(v, 32, 64);
        bs[e][g] = v;
      }
    if (lane < 4)
#pragma unroll
      for (int e = 0; e < 4; ++e) *reinterpret_cast<f32x4*>(&bred[wave][16 * cq + 4 * e]) = bs[e];
    __syncthreads();
    if (tid < 64)
      p.part[((size_t)s * p.B + b) * 512 + 64 * kh + tid] = bred[0][tid] + bred[1][tid] + bred[2][tid] + bred[3][tid];
  };
  {  // dZ_{T-1} (step T-1's gate backward ran before this kernel): own rows into the image, bias partials
    f32x4 bs[4] = {};
#pragma unroll
    for (int n = 0; n < NG; ++n) {
      const int px = (tid + 256 * n) >> 2;
      if (px < P) {
        const int ip = hidx(px);
        f32x4 zg[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const f32x4 z = *reinterpret_cast<const f32x4*>(p.dZ + ((size_t)(p.T - 1) * M + (size_t)b * P + px) * 512 +
                                                          64 * kh + 16 * cq + 4 * e);
          bs[e] += z;
          zg[e] = z;
          if constexpr (!PS) *reinterpret_cast<f32x4*>(zim + ip * 256 + sw16(4 * cq + e, px)) = z;
        }
        if constexpr (PS) ps_store_group(zim, px * kPsXP, 4, cq, zg);
      }
    }
    bias_flush(p.T - 1, bs);   // (its barrier also completes the image)
  }

  int hb[2], sb[2];   // sb: swizzle key of the window's top-left pixel
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int col = 32 * (2 * cw + c) + r32;
    hb[c] = p.colhb[col];
    sb[c] = (col < P ? col : P - 1) - p.w - 1;
  }
  // PS: per column block, the column and its valid-tap mask under the transposed gather
  // (tap (ky, kx) reads pixel (y + 1 - ky, x + 1 - kx); padding columns: none valid)
  int colc[2], vmk[2];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    colc[c] = 32 * (2 * cw + c) + r32;
    vmk[c] = 0;
    if (colc[c] < P) {
      const int y = colc[c] / p.w, x = colc[c] % p.w;
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int yy = y + 1 - tap / 3, xx = x + 1 - tap % 3;
        if ((unsigned)yy < (unsigned)p.h && (unsigned)xx < (unsigned)p.w) vmk[c] |= 1 << tap;
      }
    }
  }
  auto psbase = [&](int c, int tap) -> uint32_t {   // off-grid taps: the zero pixel kPsZP (recur_f32.h)
    const int nb = colc[c] + (1 - tap / 3) * p.w + (1 - tap % 3);
    return ps_tap_base((vmk[c] >> tap) & 1, nb, kPsXP, hh);
  };
  const __amdgpu_buffer_rsrc_t rsw = make_rsrc(p.Wb, (uint32_t)(8 * kB32QP * 4 * 1024));
  auto lda = [&](int q, int r) {
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                         rsw, lane * 16, ((kh * kB32QP + q) * 4 + 2 * rw + r) * 1024, 0));
  };
  constexpr int PD = S6 ? PDS : kB32PD;
  static_assert(kB32Q % PD == 0 && 8 % PD == 0 && PD >= 4 && PD <= kB32PD, "slot = q8 % PD");
  f32x4 af[PD][2];
  // S6: the pre-split stream (recur_f32.h k_split_frag), part p of chunk group g at (g * 3 + p) * 512 B
  const __amdgpu_buffer_rsrc_t rsw6 = make_rsrc(p.Wb6, S6 ? (uint32_t)(8 * kB32QP * 4 * 3 * 512) : 0u);
  auto lda6 = [&](int q, int r, int part) {
    return __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(
                                         rsw6, lane * 8, (((kh * kB32QP + q) * 4 + 2 * rw + r) * 3 + part) * 512, 0));
  };
  // DX: the dx rows' stream (k_pack_frag_f32): row block rw of the two
  const __amdgpu_buffer_rsrc_t rsx6 = make_rsrc(p.Wx6, DX ? (uint32_t)(8 * kB32QP * 2 * 3 * 512) : 0u);
  auto ldx6 = [&](int q, int part) {
    return __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(
                                         rsx6, lane * 8, (((kh * kB32QP + q) * 2 + rw) * 3 + part) * 512, 0));
  };
  auto lda6r = [&](int q, int r, int part) { return r < 2 ? lda6(q, r, part) : ldx6(q, part); };
  // DX: the paired streams -- one 16-B load per lane brings a part of both quads of a pair (half the
  // load instructions of two 8-B loads); PD / 2 pairs in flight
  const __amdgpu_buffer_rsrc_t rsbp = make_rsrc(p.Wb6p, DX ? (uint32_t)(8 * kB32PP * 4 * 3 * 1024) : 0u);
  const __amdgpu_buffer_rsrc_t rsxp = make_rsrc(p.Wx6p, DX ? (uint32_t)(8 * kB32PP * 2 * 3 * 1024) : 0u);
  auto ldp = [&](int pj, int r, int part) {
    return r < 2 ? __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                 rsbp, lane * 16, (((kh * kB32PP + pj) * 4 + 2 * rw + r) * 3 + part) * 1024, 0))
                 : __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                 rsxp, lane * 16, (((kh * kB32PP + pj) * 2 + rw) * 3 + part) * 1024, 0));
  };
  u32x2 a6[S6 && !DX ? PD : 1][NR][3];
  u32x4 a6p[DX ? PD / 2 : 1][NR][3];
  if constexpr (DX) {
#pragma unroll
    for (int s = 0; s < PD / 2; ++s)
#pragma unroll
      for (int r = 0; r < NR; ++r)
#pragma unroll
        for (int part = 0; part < 3; ++part) a6p[s][r][part] = ldp(s, r, part);
  } else {
#pragma unroll
    for (int s = 0; s < PD - 1; ++s)
#pragma unroll
      for (int r = 0; r < NR; ++r) {
        if constexpr (S6) {
#pragma unroll
          for (int part = 0; part < 3; ++part) a6[s][r][part] = lda6r(s, r, part);
        } else {
          af[s][r] = lda(s, r);
        }
      }
  }

  // the dgrad is the transposed conv: tap (ky, kx) of W^T (packed in the forward's
  // orientation) reads dZ at (y + 1 - ky, x + 1 - kx) (ConvGeo transposed gather)
  auto tapoff = [&](int tap) { return (2 - tap / 3) * W2 + 2 - tap % 3; };
  auto tapkey = [&](int tap) { return (2 - tap / 3) * p.w + 2 - tap % 3; };
  // dgrads: dZ_{T-1} .. dZ_1 (+ dZ_0 for dh0, or, with DX, for dx_0)
  const int nsteps = p.T - 1 + ((p.dh0 || DX) ? 1 : 0);
  f32x4 dxs = {0.f, 0.f, 0.f, 0.f};   // DX: this thread's dx quad summed over its pixel and the steps
  for (int it = 0; it < nsteps; ++it) {
    const int s = p.T - 1 - it;   // this dgrad reads dZ_s and yields dh_{s-1}
    const int buf = it % kB32NBUF;
    AAA_B32_STAMP(it, 0);
    f32x16 acc[NR][2];
#pragma unroll
    for (int r = 0; r < NR; ++r)
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[r][c][e] = 0.f;
    int hbs[2], sbs[2];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      hbs[c] = hb[c];
      sbs[c] = sb[c];
      asm volatile("" : "+v"(hbs[c]), "+v"(sbs[c]));
    }
    // gate-backward inputs of step s-1, loaded at the start (they land under the K loop)
    f32x4 gpre[NG][7];
    if (s >= 1) {
#pragma unroll
      for (int n = 0; n < NG; ++n) {
        const int px = min((tid + 256 * n) >> 2, P - 1), ch = 16 * kh + 4 * cq;
        const size_t r = (size_t)(s - 1) * M + (size_t)b * P + px;
        gpre[n][0] = *reinterpret_cast<const f32x4*>(p.dO + r * 128 + ch);
#pragma unroll
        for (int e = 0; e < 4; ++e) gpre[n][1 + e] = *reinterpret_cast<const f32x4*>(p.Gt + r * 512 + 4 * (ch + e));
        gpre[n][5] = *reinterpret_cast<const f32x4*>(p.Cst + r * 128 + ch);         // c_{s-2}
        gpre[n][6] = *reinterpret_cast<const f32x4*>(p.Cst + (r + M) * 128 + ch);   // c_{s-1}
      }
    }
    auto ldb = [&](int tap, int q8, f32x4 (&bf)[2]) {
      const int toff = tapoff(tap), tk = tapkey(tap);
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int ip = hbs[c] + toff;
        bf[c] = *reinterpret_cast<const f32x4*>(zim + ip * 256 + sw16(2 * q8 + hh, sbs[c] + tk));
      }
    };
    f32x4 bfr[2][2];
    if constexpr (S6 && PS) {
      bf16x8 bq[2][2][3];   // [pair parity][column block][part]
      auto ldq = [&](int tap, int g, bf16x8 (&o)[2][3]) {
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const uint32_t base = psbase(c, tap);
#pragma unroll
          for (int part = 0; part < 3; ++part)
            o[c][part] = *reinterpret_cast<const bf16x8*>(zim + base + (part * 4 + g) * 32);
        }
      };
      ldq(0, 0, bq[0]);
      for (int tap = 0; tap < 9; ++tap) {
        int qt = tap * 8;
        asm volatile("" : "+s"(qt));
#pragma unroll
        for (int q8 = 0; q8 < 8; q8 += 2) {
          const int pb = (q8 >> 1) & 1, nb = pb ^ 1;
          bf16x8 a3[NR][3];
          if constexpr (DX) {   // slot pair (q8 % PD) / 2, refilled with pair (qt + q8) / 2 + PD / 2 (wraps)
#pragma unroll
            for (int r = 0; r < NR; ++r)
#pragma unroll
              for (int part = 0; part < 3; ++part) {
                a3[r][part] = __builtin_bit_cast(bf16x8, a6p[(q8 % PD) / 2][r][part]);
                a6p[(q8 % PD) / 2][r][part] = ldp((qt + q8) / 2 + PD / 2, r, part);
              }
          } else {
#pragma unroll
            for (int r = 0; r < NR; ++r)
#pragma unroll
              for (int part = 0; part < 3; ++part)
                a3[r][part] = __builtin_bit_cast(bf16x8, u32x4{a6[q8 % PD][r][part].x, a6[q8 % PD][r][part].y,
                                                               a6[q8 % PD + 1][r][part].x, a6[q8 % PD + 1][r][part].y});
#pragma unroll
            for (int r = 0; r < NR; ++r)
#pragma unroll
              for (int part = 0; part < 3; ++part) {
                a6[(q8 + PD - 1) % PD][r][part] = lda6r(qt + q8 + PD - 1, r, part);
                a6[q8 % PD][r][part] = lda6r(qt + q8 + PD, r, part);
              }
          }
          if (q8 < 6) ldq(tap, (q8 >> 1) + 1, bq[nb]);
          else if (tap < 8) ldq(tap + 1, 0, bq[nb]);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int r = 0; r < NR; ++r) {
            const bf16x8 ah = a3[r][0], am = a3[r][1], al = a3[r][2];
#pragma unroll
            for (int c = 0; c < 2; ++c) {
              const bf16x8 bh = bq[pb][c][0], bm = bq[pb][c][1], bl = bq[pb][c][2];
              acc[r][c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc[r][c], 0, 0, 0);
              acc[r][c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc[r][c], 0, 0, 0);
              acc[r][c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bm, acc[r][c], 0, 0, 0);
              acc[r][c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bh, acc[r][c], 0, 0, 0);
              acc[r][c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bm, acc[r][c], 0, 0, 0);
              acc[r][c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc[r][c], 0, 0, 0);
            }
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    } else if constexpr (S6) {
      f32x4 bp[4][2];   // B fragments of two pairs of quads
      ldb(0, 0, bp[0]);
      ldb(0, 1, bp[1]);
      for (int tap = 0; tap < 9; ++tap) {
        int qt = tap * 8;
        asm volatile("" : "+s"(qt));
#pragma unroll
        for (int q8 = 0; q8 < 8; q8 += 2) {
          const int pb = (q8 >> 1) & 1, nb = pb ^ 1;
          bf16x8 a3[2][3];
#pragma unroll
          for (int r = 0; r < 2; ++r)
#pragma unroll
            for (int part = 0; part < 3; ++part)
              a3[r][part] = __builtin_bit_cast(bf16x8, u32x4{a6[q8 % PD][r][part].x, a6[q8 % PD][r][part].y,
                                                             a6[q8 % PD + 1][r][part].x, a6[q8 % PD + 1][r][part].y});
#pragma unroll
          for (int r = 0; r < 2; ++r)
#pragma unroll
            for (int part = 0; part < 3; ++part) {
              a6[(q8 + PD - 1) % PD][r][part] = lda6(qt + q8 + PD - 1, r, part);
              a6[q8 % PD][r][part] = lda6(qt + q8 + PD, r, part);
            }
          if (q8 < 6) {
            ldb(tap, q8 + 2, bp[2 * nb]);
            ldb(tap, q8 + 3, bp[2 * nb + 1]);
          } else if (tap < 8) {
            ldb(tap + 1, 0, bp[2 * nb]);
            ldb(tap + 1, 1, bp[2 * nb + 1]);
          }
          __builtin_amdgcn_sched_barrier(0);
          bf16x8 bh[2], bm[2], bl[2];
#pragma unroll
          for (int c = 0; c < 2; ++c) {
            const float b8[8] = {bp[2 * pb][c][0],     bp[2 * pb][c][1],     bp[2 * pb][c][2],     bp[2 * pb][c][3],
                                 bp[2 * pb + 1][c][0], bp[2 * pb + 1][c][1], bp[2 * pb + 1][c][2], bp[2 * pb + 1][c][3]};
            if constexpr ((ABL & 16) != 0) {   // ablation: hi part only (the split's VALU cost)
#pragma unroll
              for (int e = 0; e < 8; ++e) bh[c][e] = (__bf16)b8[e];
              bm[c] = bh[c];
              bl[c] = bh[c];
            } else {
              split3_bf16(b8, bh[c], bm[c], bl[c]);
            }
          }
#pragma unroll
          for (int r = 0; r < 2; ++r) {
            const bf16x8 ah = a3[r][0], am = a3[r][1], al = a3[r][2];
#pragma unroll
            for (int c = 0; c < 2; ++c) {
              acc[r][c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh[c], acc[r][c], 0, 0, 0);
              acc[r][c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl[c], acc[r][c], 0, 0, 0);
              acc[r][c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bm[c], acc[r][c], 0, 0, 0);
              acc[r][c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bh[c], acc[r][c], 0, 0, 0);
              acc[r][c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bm[c], acc[r][c], 0, 0, 0);
              acc[r][c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh[c], acc[r][c], 0, 0, 0);
            }
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    } else {
    ldb(0, 0, bfr[0]);
    for (int tap = 0; tap < 9; ++tap) {
      int qt = tap * 8;
      asm volatile("" : "+s"(qt));
#pragma unroll
      for (int q8 = 0; q8 < 8; ++q8) {
#pragma unroll
        for (int r = 0; r < 2; ++r) af[(q8 + PD - 1) % PD][r] = lda(qt + q8 + PD - 1, r);
        if (q8 < 7) ldb(tap, q8 + 1, bfr[(q8 + 1) & 1]);
        else if (tap < 8) ldb(tap + 1, 0, bfr[0]);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int r = 0; r < 2; ++r)
#pragma unroll
            for (int c = 0; c < 2; ++c) {
              if constexpr (ABL & 2)
                acc[r][c][j] += af[q8][r][j] * bfr[q8 & 1][c][j];
              else
                acc[r][c] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[q8][r][j], bfr[q8 & 1][c][j], acc[r][c], 0, 0, 0);
            }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    }
    AAA_B32_STAMP(it, 1);
    // partial dh: lane (r32, hh) of tile (r, c), element 4g + e = channel
    // 32 (2 rw + r) + 8 g + 4 hh + e at column 32 (2 cw + c) + r32, i.e. the
    // 16-B quad 8 (g & 1) + 4 hh of destination 2 (2 rw + r) + (g >> 1)
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int px = 32 * (2 * cw + c) + r32;
        if (px >= P) continue;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int dst = 2 * (2 * rw + r) + (g >> 1), cl = 8 * (g & 1) + 4 * hh;
          const f32x4 v{acc[r][c][4 * g], acc[r][c][4 * g + 1], acc[r][c][4 * g + 2], acc[r][c][4 * g + 3]};
          if (dst == kh) {
            own[px][cl >> 2] = v;
          } else if constexpr (!(ABL & 8)) {
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v),
                                                   make_rsrc(xslot(buf, dst, kh), 128 * kB32XC * 4),
                                                   (uint32_t)((px * kB32XC + cl) * 4), 0, kSC1);
          }
        }
      }
    if constexpr (DX) {   // dx tile (row block rw): element 4g + e = dx channel 32 rw + 8 g + 4 hh + e,
      // owned by workgroup 4 rw + g at its quad hh
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int px = 32 * (2 * cw + c) + r32;
        if (px >= P) continue;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int dst = 4 * rw + g;
          const f32x4 v{acc[2][c][4 * g], acc[2][c][4 * g + 1], acc[2][c][4 * g + 2], acc[2][c][4 * g + 3]};
          if (dst == kh)
            own[px][4 + hh] = v;
          else
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v),
                                                   make_rsrc(xslot(buf, dst, kh), 128 * kB32XC * 4),
                                                   (uint32_t)((px * kB32XC + 16 + 4 * hh) * 4), 0, kSC1);
        }
      }
    }
    // publish this step's partials: every wave's stores retired, a barrier, one flag store
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    barrier_lds();
    if (tid == 0) __hip_atomic_store(p.flags + b * G + kh, it + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // every wave waits for the seven partners, then sums their partials into its groups
    if constexpr (!(ABL & 1)) wave_wait_flags(p.flags + b * G, ((1ull << G) - 1) & ~(1ull << kh), it + 1, p.report, p.spin, wdl);
    AAA_B32_STAMP(it, 2);
    f32x4 dhv[NG];
#pragma unroll
    for (int n = 0; n < NG; ++n) {
      const int px = min((tid + 256 * n) >> 2, 127);
      dhv[n] = own[px][cq];
      if constexpr (!(ABL & 8)) {
        f32x4 pv[G - 1];
#pragma unroll
        for (int j = 0; j < G - 1; ++j) {
          const int src = j < kh ? j : j + 1;
          pv[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                make_rsrc(xslot(buf, kh, src), 128 * kB32XC * 4),
                                                (uint32_t)((px * kB32XC + 4 * cq) * 4), 0, kSC1));
        }
#pragma unroll
        for (int j = 0; j < G - 1; ++j) dhv[n] += pv[j];
      }
    }
    if constexpr (DX) {   // dx_s of the workgroup's 8 channels: thread -> (pixel tid / 2, quad tid % 2)
      const int px = tid >> 1, xq = tid & 1;
      f32x4 v = own[px][4 + xq];
      f32x4 pv[G - 1];
#pragma unroll
      for (int j = 0; j < G - 1; ++j) {
        const int src = j < kh ? j : j + 1;
        pv[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                              make_rsrc(xslot(buf, kh, src), 128 * kB32XC * 4),
                                              (uint32_t)((px * kB32XC + 16 + 4 * xq) * 4), 0, kSC1));
      }
#pragma unroll
      for (int j = 0; j < G - 1; ++j) v += pv[j];   // summed in source order: the same whoever is last
      if (px < P) {
        *reinterpret_cast<f32x4*>(p.dx + ((size_t)s * M + (size_t)b * P + px) * 64 + 8 * kh + 4 * xq) = v;
        dxs += v;
      }
    }
    if (s == 0) {   // dh0 = dh_{-1}: no gate backward
      if (p.dh0) {
#pragma unroll
        for (int n = 0; n < NG; ++n) {
          const int px = (tid + 256 * n) >> 2;
          if (px < P) *reinterpret_cast<f32x4*>(p.dh0 + ((size_t)b * P + px) * 128 + 16 * kh + 4 * cq) = dhv[n];
        }
      }
      break;
    }
    // (every wave is past the K loop -- the barrier behind the flag store -- so
    // the image and own[] are free to rewrite)
    // gate backward of step s-1 (EpiConvLstmBwd's math): dZ_{s-1} into the
    // image (the next dgrad's B operand) and to HBM (the weight gradient's)
    f32x4 bs[4] = {};
#pragma unroll
    for (int n = 0; n < NG; ++n) {
      const int px = (tid + 256 * n) >> 2;
      if (px >= P) continue;
      const int ip = hidx(px);
      float* zo = p.dZ + ((size_t)(s - 1) * M + (size_t)b * P + px) * 512 + 64 * kh;
      f32x4 zg[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float di, df, dcg, dout;
        gate_bwd(dhv[n][e] + gpre[n][0][e], gpre[n][1 + e], gpre[n][5][e], gpre[n][6][e], dcr[n][e], di, df, dcg,
                 dout);
        const f32x4 z{di, df, dcg, dout};
        bs[e] += z;
        zg[e] = z;
        const int q = 4 * cq + e;   // 16-B chunk (4 rows) of the workgroup's 64 rows
        if constexpr (!PS) *reinterpret_cast<f32x4*>(zim + ip * 256 + sw16(q, px)) = z;
        *reinterpret_cast<f32x4*>(zo + 4 * q) = z;
      }
      if constexpr (PS) ps_store_group(zim, px * kPsXP, 4, cq, zg);
    }
    bias_flush(s - 1, bs);   // (its barrier also completes the image before the next dgrad)
    AAA_B32_STAMP(it, 3);
  }
  // the final dc carry (dc_0) back to dC
#pragma unroll
  for (int n = 0; n < NG; ++n) {
    const int px = (tid + 256 * n) >> 2;
    if (px < P)
      *reinterpret_cast<f32x4*>(p.dC + ((size_t)b * P + px) * 128 + 16 * kh + 4 * cq) =
          f32x4{dcr[n][0], dcr[n][1], dcr[n][2], dcr[n][3]};
  }
  if constexpr (DX) {   // conv2's bias gradient of this frame's 8 channels: sum the pixels (lanes of equal parity)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float v = dxs[e];
      v += __shfl_xor(v, 2, 64);
      v += __shfl_xor(v, 4, 64);
      v += __shfl_xor(v, 8, 64);
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      dxs[e] = v;
    }
    __syncthreads();   // (bred's last readers: bias_flush)
    if (lane < 2)
#pragma unroll
      for (int e = 0; e < 4; ++e) bred[wave][4 * lane + e] = dxs[e];
    __syncthreads();
    if (tid < 8) p.dxb[(size_t)b * 64 + 8 * kh + tid] = bred[0][tid] + bred[1][tid] + bred[2][tid] + bred[3][tid];
  }
}

inline hipError_t convlstm_bwd_f32(RecBwdF32Params& p, hipStream_t st, bool s6 = false) {
  if (!f32_rec_fits(p.h, p.w) || p.P != p.h * p.w || p.B < 1 || p.T < 1 || !p.flags || !p.report || p.spin < 0 ||
      !p.part || !p.xp)
    return hipErrorInvalidValue;
  for (int c = 0; c < 128; ++c) {
    const int pp = c < p.P ? c : p.P - 1;
    p.colhb[c] = (short)((pp / p.w) * (p.w + 2) + pp % p.w);
  }
  // S6: 4 A quads in flight (tools/ubench/f32rec: 3% under 8, fewer registers parked in AGPRs)
  // S6: the dZ image pre-split (PS; the in-loop split of AAA_F32_PRESPLIT=0 in ablation builds only)
#ifdef AAA_ABLATION
  if (s6 && std::getenv("AAA_F32_PRESPLIT") != nullptr)
    return launch_resident(reinterpret_cast<const void*>(&k_convlstm_bwd_f32<0, true, 4>), f32_grid(p.B, 8), 256, p,
                           st);
#endif
  if (s6 && p.dx) {   // the production kernel: dx fused (DX)
    if (!p.Wb6p || !p.Wx6p || !p.dxb) return hipErrorInvalidValue;
    return launch_resident(reinterpret_cast<const void*>(&k_convlstm_bwd_f32<0, true, 4, true, true>),
                           f32_grid(p.B, 8), 256, p, st);
  }
  return launch_resident(s6 ? reinterpret_cast<const void*>(&k_convlstm_bwd_f32<0, true, 4, true>)
                            : reinterpret_cast<const void*>(&k_convlstm_bwd_f32<0>),
                         f32_grid(p.B, 8), 256, p, st);
}

}  // namespace aaa
