// Frame-resident ConvLSTM BPTT (bf16 operands, fp32 accumulate, fp16 gates).
//
// The backward of the recurrence (what autograd runs for attention.py:110-126
// over the unroll) couples a frame only to itself, like the forward (recur.h):
// one workgroup owns a frame for the whole chain t = T-1 .. 0.  Per step t it
// runs the transposed h-conv  dh_{t-1}[ch][q] = sum_{tap,r} W_h[r][ch][tap] *
// dZ_t[r][q - d(tap)]  as one 128 x P x 4608 GEMM whose B operand is gathered
// from zero-bordered LDS images of dZ_t, and the gate backward of step t-1 in
// its epilogue (dh + the attention-path grad dO -> dZ_{t-1}, the dc carry),
// which writes dZ_{t-1} straight into those images for the next step.
//
// dZ_t has 512 rows per pixel (173 KB per frame: more than the LDS), split in
// four chunks of 128 rows = the 32 channels of one wave: wave w's epilogue
// produces chunk w.  Chunks 0 and 1 stay in the two LDS images, written by the
// epilogue; chunks 2 and 3 go through HBM like every chunk (dZ is the
// weight-gradient operand) and are LDS-DMA'd into image 0 / 1 once chunk 0 / 1
// has been consumed.  The lane's dc carry lives in LDS (lane-native), and the
// epilogue's HBM inputs (dO, c_s, c_{s-1}, gates) are requested one column
// block ahead -- the first during the last chunk of the GEMM.
//
// Geometry: 4 waves, one per SIMD; wave w owns the GEMM rows (h channels)
// 32w..32w+31 for all P <= 128 pixel columns: acc 4 tiles of 32x32 (one per
// column block cb); lane (r32, hh) holds channels 32w + 8g + 4hh + e (e = 0..3)
// at pixel 32cb + r32, so its gate backward reads / writes 4 consecutive
// channels (16-B fp32, 32-B fp16 / bf16 pieces) and keeps its dc carry in
// registers across steps.  A operand: fragment-order W_h^T (k_pack_wbfrag), K
// ordered (chunk, tap, 16-row group) to follow the images.
#pragma once
#include "recur.h"

namespace aaa {

constexpr int kBwKS = 4608 / 16;   // k steps: 4 chunks x 9 taps x 8 groups of 16 rows
constexpr int kBwPD = 8;           // A register slots (PD-1 k steps in flight); divides 8
constexpr int kBwKSP = kBwKS + kBwPD - 1;
constexpr int kBwIP = 136;         // chunk image pixel pitch (bf16): 128 rows + 8 pad (272 B)
constexpr int kBwIB = 46080;       // chunk image bytes: 169 px x 272 B rounded up to whole 1-KB DMA pieces

// k step ks -> k of the dgrad GEMM (k = tap*512 + gate row)
__host__ __device__ constexpr int bw_k(int ks) { return ((ks % 72) >> 3) * 512 + (ks / 72) * 128 + (ks & 7) * 16; }

// Wb[((rb*kBwKSP + ks)*64 + lane)*8 + e] = W[rb*32 + lane%32][bw_k(ks % kBwKS) + (lane/32)*8 + e], W = the h
// rows of the packed dgrad weights ([128][4608], rows 64..191 of k_WdTl)
__global__ void __launch_bounds__(256) k_pack_wbfrag(const __bf16* __restrict__ W, __bf16* __restrict__ Wb) {
  const int c = blockIdx.x * 256 + (int)threadIdx.x;
  if (c >= 4 * kBwKSP * 64) return;
  const int lane = c & 63, rk = c >> 6, ks = rk % kBwKSP, rb = rk / kBwKSP;
  const int row = rb * 32 + (lane & 31), k = bw_k(ks % kBwKS) + (lane >> 5) * 8;
  *reinterpret_cast<bf16x8*>(Wb + (size_t)c * 8) = *reinterpret_cast<const bf16x8*>(W + (size_t)row * 4608 + k);
}

inline hipError_t pack_wbfrag(const __bf16* W, __bf16* Wb, hipStream_t st) {
  hipLaunchKernelGGL(k_pack_wbfrag, dim3((4 * kBwKSP * 64 + 255) / 256), dim3(256), 0, st, W, Wb);
  return hipGetLastError();
}

struct RecBwdParams {
  const __bf16* Wb;       // fragment-order W_h^T
  const float* dO;        // (T, B, P, 128) attention-path grad of h_t
  const _Float16* Gt;     // (T, B, P, 512) gate activations
  const float* Cst;       // (T+1, B, P, 128): slot s+1 = c_s
  const float* dhT;       // (B, P, 128) extra grad of h_{T-1}, or null
  float* dC;              // (B, P, 128) dc carry: in = dc_T, out = dc_0
  __bf16* dZ;             // (T, B, P, 512) <- gate pre-activation grads
  float* part;            // (T, B, 512) <- gate-bias partials per (step, frame)
  float* dh0;             // (B, P, 128) <- grad of h_{-1}, or null
  int T, B, h, w, P;
};

// ABL (diagnostic A/B only, AAA_RECB_ABL): bit 0 = no A loads in the K loop,
// bit 1 = no epilogue HBM loads / stores, bit 2 = no MFMAs, bit 3 = no chunk-3 DMA.
template <int ABL = 0>
__global__ void __launch_bounds__(256) k_convlstm_bwd_frames(RecBwdParams p) {
  __shared__ __attribute__((aligned(16))) unsigned char zim[2 * kBwIB];   // chunk images (0: chunks 0, 2; 1: 1, 3)
  __shared__ __attribute__((aligned(16))) f32x4 dcl[4 * 16 * 64];         // dc carry, lane-native [wave][g*4+cb][lane]
  const int b = blockIdx.x, tid = (int)threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r32 = lane & 31, hh = lane >> 5;
  const int P = p.P, W2 = p.w + 2, NPH = (p.h + 2) * W2;
  const size_t M = (size_t)p.B * P;
  auto hidx = [&](int pp) { return (pp / p.w + 1) * W2 + pp % p.w + 1; };

  {  // zero the images (borders and pads stay zero)
    u32x4* z = reinterpret_cast<u32x4*>(zim);
    for (int i = tid; i < 2 * kBwIB / 16; i += 256) z[i] = u32x4{0u, 0u, 0u, 0u};
  }
  // chunk c (rows 128c .. 128c+127) of dZ_t from HBM into image c & 1: 16-B
  // slot s of the image = pixel s / 17, row group s % 17 (16 = pad); borders,
  // pads and the tail read outside the descriptor and land as zeros
  auto dma_chunk = [&](int t, int c) {
    const __amdgpu_buffer_rsrc_t rs =
        make_rsrc(p.dZ + ((size_t)t * M + (size_t)b * P) * 512, (uint32_t)(P * 512 * 2));
    for (int i = wave; i < kBwIB / 1024; i += 4) {
      const int sl = i * 64 + lane, ip = sl / 17, q = sl - ip * 17;
      const int py = ip / W2 - 1, px = ip % W2 - 1;
      const bool v = q < 16 && ip < NPH && (unsigned)py < (unsigned)p.h && (unsigned)px < (unsigned)p.w;
      dma16(rs, zim + (c & 1) * kBwIB + i * 1024, v ? (uint32_t)(((py * p.w + px) * 512 + 128 * c + q * 8) * 2) : kOOB);
    }
  };

  int hb[4];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) {
    const int pp = min(cb * 32 + r32, P - 1);
    hb[cb] = (pp / p.w) * W2 + pp % p.w;
  }
  // dc carry of the lane's 64 (channel, pixel) pairs: channels 32w + 8g + 4hh + e at pixel 32cb + r32
  f32x4* dcw = dcl + wave * 16 * 64 + lane;   // + (g*4 + cb) * 64
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      const int pp = cb * 32 + r32;
      dcw[(g * 4 + cb) * 64] =
          pp < P ? *reinterpret_cast<const f32x4*>(p.dC + ((size_t)b * P + pp) * 128 + 32 * wave + 8 * g + 4 * hh)
                 : f32x4{0.f, 0.f, 0.f, 0.f};
    }

  const __amdgpu_buffer_rsrc_t rsw = make_rsrc(p.Wb, (uint32_t)(4 * kBwKSP * 1024));
  const int wofs = wave * kBwKSP * 1024;
  auto lda = [&](int ks) {
    return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rsw, lane * 16, wofs + ks * 1024, 0));
  };
  constexpr int PD = kBwPD;
  bf16x8 af[PD];
#pragma unroll
  for (int s = 0; s < PD - 1; ++s) af[s] = lda(s);

  // The epilogue's HBM inputs for one column block (4 channel groups g of the lane)
  struct EpIn { f32x4 dO[4], cc[4], cp[4]; u32x4 gt[4][2]; };
  auto load_in = [&](int s, int cb, int ln) {
    EpIn in;
    const int pp = cb * 32 + (ln & 31);
    if (pp < P && !(ABL & 2)) {
      const size_t row = (size_t)s * M + (size_t)b * P + pp;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int ch = 32 * wave + 4 * (ln >> 5) + 8 * g;
        in.dO[g] = *reinterpret_cast<const f32x4*>(p.dO + row * 128 + ch);
        in.cc[g] = *reinterpret_cast<const f32x4*>(p.Cst + (row + M) * 128 + ch);   // c_s
        in.cp[g] = *reinterpret_cast<const f32x4*>(p.Cst + row * 128 + ch);         // c_{s-1}
        const u32x4* gp = reinterpret_cast<const u32x4*>(p.Gt + row * 512 + 4 * ch);
        in.gt[g][0] = gp[0];
        in.gt[g][1] = gp[1];
      }
    } else {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        in.dO[g] = in.cc[g] = in.cp[g] = f32x4{0.f, 0.f, 0.f, 0.f};
        in.gt[g][0] = in.gt[g][1] = u32x4{0u, 0u, 0u, 0u};
      }
    }
    return in;
  };

  // Gate backward of step s on the GEMM result (acc = dh_s from step s+1, zero
  // for s = T-1): dZ_s to HBM (bf16) and, for chunks 0 and 1, into image w; the
  // lane's dc carry advances to step s-1; gate-bias partials of step s.
  // ``in0``: the inputs of column block 0, already requested.
  auto epilogue = [&](int s, const f32x16 (&acc)[4], bool gemm, EpIn in0) {
    int ln = lane;   // laundered: the epilogue's addresses are recomputed per step, not hoisted
    asm volatile("" : "+v"(ln));
    const int pl = ln & 31, hq = ln >> 5;
    const int c0 = 32 * wave + 4 * hq;   // + 8g + e
    const size_t rows = (size_t)s * M + (size_t)b * P;
    float bs[4][4][4];   // [g][e][gate] sums over the lane's pixels
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int q = 0; q < 4; ++q) bs[g][e][q] = 0.f;
    EpIn cur = in0;
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      EpIn nxt;
      if (cb < 3) nxt = load_in(s, cb + 1, ln);   // one column block ahead
      const int pp = cb * 32 + pl;
      if (pp < P) {
        const size_t row = rows + pp;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int ch = c0 + 8 * g;
          f32x4 dh = cur.dO[g];
          if (gemm) {
            dh[0] += acc[cb][4 * g]; dh[1] += acc[cb][4 * g + 1]; dh[2] += acc[cb][4 * g + 2]; dh[3] += acc[cb][4 * g + 3];
          } else if (p.dhT) {
            const f32x4 x = *reinterpret_cast<const f32x4*>(p.dhT + ((size_t)b * P + pp) * 128 + ch);
            dh[0] += x[0]; dh[1] += x[1]; dh[2] += x[2]; dh[3] += x[3];
          }
          f32x4* dcp = dcl + wave * 16 * 64 + ln + (g * 4 + cb) * 64;
          f32x4 dc = *dcp;
          float dz[16];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const uint32_t w01 = cur.gt[g][e >> 1][2 * (e & 1)], w23 = cur.gt[g][e >> 1][2 * (e & 1) + 1];
            typedef _Float16 h2 __attribute__((ext_vector_type(2)));
            const h2 a = __builtin_bit_cast(h2, w01), c2 = __builtin_bit_cast(h2, w23);
            const f32x4 gv{(float)a[0], (float)a[1], (float)c2[0], (float)c2[1]};
            float d = dc[e], di, df, dcg, dout;
            gate_bwd(dh[e], gv, cur.cp[g][e], cur.cc[g][e], d, di, df, dcg, dout);
            dc[e] = d;
            dz[4 * e] = di; dz[4 * e + 1] = df; dz[4 * e + 2] = dcg; dz[4 * e + 3] = dout;
            bs[g][e][0] += di; bs[g][e][1] += df; bs[g][e][2] += dcg; bs[g][e][3] += dout;
          }
          *dcp = dc;
          bf16x8 z0, z1;
#pragma unroll
          for (int i = 0; i < 8; ++i) { z0[i] = (__bf16)dz[i]; z1[i] = (__bf16)dz[8 + i]; }
          __bf16* zo = p.dZ + row * 512 + 4 * ch;
          if constexpr (!(ABL & 2)) {
            *reinterpret_cast<bf16x8*>(zo) = z0;
            *reinterpret_cast<bf16x8*>(zo + 8) = z1;
          }
          if (wave < 2) {   // chunk w of the next step's B operand, rows 4(ch - 32w) + gate
            unsigned char* zi = zim + wave * kBwIB + hidx(pp) * (kBwIP * 2) + (4 * (ch - 32 * wave)) * 2;
            *reinterpret_cast<bf16x8*>(zi) = z0;
            *reinterpret_cast<bf16x8*>(zi + 16) = z1;
          }
        }
      }
      if (cb < 3) cur = nxt;
      __builtin_amdgcn_sched_barrier(0);
    }
    // gate-bias partials: butterfly transpose-reduce of the 64 row sums over the
    // 32 pixel lanes of each half: after 5 exchange steps lane r32 holds the
    // totals of rows 2*r32 and 2*r32+1 of its half's 64 (g, e, gate) rows
    float v[64];
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int q = 0; q < 4; ++q) v[16 * g + 4 * e + q] = bs[g][e][q];
    int n = 64;
#pragma unroll
    for (int m = 16; m >= 1; m >>= 1) {
      const bool up = (pl & m) != 0;
      n >>= 1;
#pragma unroll
      for (int i = 0; i < 32; ++i) {
        if (i < n) {
          const float send = up ? v[i] : v[i + n];
          const float keep = up ? v[i + n] : v[i];
          v[i] = keep + __shfl_xor(send, m, 64);
        }
      }
    }
    // lane pl now owns rows ridx, ridx+1 of its half: the exchange at distance m
    // kept the upper half of the remaining rows where pl has bit m set
    const int ridx = ((pl & 16) ? 32 : 0) + ((pl & 8) ? 16 : 0) + ((pl & 4) ? 8 : 0) + ((pl & 2) ? 4 : 0) + ((pl & 1) ? 2 : 0);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int r = ridx + j, g = r >> 4, e = (r >> 2) & 3, q = r & 3;
      p.part[((size_t)s * p.B + b) * 512 + 4 * (c0 + 8 * g + e) + q] = v[j];
    }
  };

  {  // step T-1: no GEMM (dh = dO_{T-1} + dhT)
    f32x16 zero[4];
    epilogue(p.T - 1, zero, false, load_in(p.T - 1, 0, lane));
  }
  barrier_lds();   // chunk images 0, 1 of dZ_{T-1}

  for (int t = p.T - 1; t >= 0; --t) {
    if (t == 0 && !p.dh0) break;
    f32x16 acc[4];
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[cb][e] = 0.f;
    int hbs[4];
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      hbs[cb] = hb[cb];
      asm volatile("" : "+v"(hbs[cb]));
    }
    // transposed gather: output pixel q reads dZ at q - d(tap): image offset (2-ky)*W2 + (2-kx)
    auto tapoff = [&](int tap) { return (2 - tap / 3) * W2 + (2 - tap % 3); };
    auto ldb = [&](const unsigned char* img, int toff, int c16, bf16x8 (&bf)[4]) {
#pragma unroll
      for (int cb = 0; cb < 4; ++cb)
        bf[cb] = *reinterpret_cast<const bf16x8*>(img + (hbs[cb] + toff) * (kBwIP * 2) + c16 * 32 + hh * 16);
    };
    constexpr int BD = 4;   // B fragment ring: BD-1 k steps of lookahead (LDS latency vs 4 MFMAs per k step)
    bf16x8 bfr[BD][4];
    EpIn in0;
#pragma unroll 1
    for (int ck = 0; ck < 4; ++ck) {
      const unsigned char* img = zim + (ck & 1) * kBwIB;
      if (ck == 1 || ck == 2) {   // every wave is done with image ck-1 and every wave's dZ_t stores have
                                  // retired (its later A loads did): refill it with chunk ck+1 from HBM
        if constexpr (!(ABL & 8)) dma_chunk(t, ck + 1);
      }
      if (ck == 3 && t > 0) in0 = load_in(t - 1, 0, lane);   // the epilogue's first inputs, under chunk 3
#pragma unroll
      for (int j = 0; j < BD - 1; ++j) ldb(img, tapoff(0), j, bfr[j]);
      for (int tap = 0; tap < 9; ++tap) {
        const int toff = tapoff(tap), tn = tap < 8 ? tapoff(tap + 1) : 0;
        int kt = ck * 72 + tap * 8;
        asm volatile("" : "+s"(kt));
#pragma unroll
        for (int c16 = 0; c16 < 8; ++c16) {
          if constexpr (!(ABL & 1)) af[(c16 + PD - 1) % PD] = lda(kt + c16 + PD - 1);
          {  // B of k step + BD - 1 (same chunk)
            const int cn = c16 + BD - 1;
            if (cn < 8) ldb(img, toff, cn, bfr[cn % BD]);
            else if (tap < 8) ldb(img, tn, cn - 8, bfr[cn % BD]);
          }
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int cb = 0; cb < 4; ++cb) {
            if constexpr (ABL & 4) acc[cb][0] += (float)af[c16 % PD][0] * (float)bfr[c16 % BD][cb][0];
            else acc[cb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[c16 % PD], bfr[c16 % BD][cb], acc[cb], 0, 0, 0);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      barrier_lds();   // image ck & 1 free; (ck >= 1) the DMA'd chunk ck+1 has landed in every wave
    }
    if (t > 0) {
      epilogue(t - 1, acc, true, in0);
    } else {   // dh_{-1}: the gradient of the initial state h0
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
        const int pp = cb * 32 + r32;
        if (pp < P)
#pragma unroll
          for (int g = 0; g < 4; ++g)
            *reinterpret_cast<f32x4*>(p.dh0 + ((size_t)b * P + pp) * 128 + 32 * wave + 8 * g + 4 * hh) =
                f32x4{acc[cb][4 * g], acc[cb][4 * g + 1], acc[cb][4 * g + 2], acc[cb][4 * g + 3]};
      }
    }
    barrier_lds();   // chunk images 0, 1 of dZ_{t-1} complete
  }
  // dc carry out (dc_0)
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      const int pp = cb * 32 + r32;
      if (pp < P)
        *reinterpret_cast<f32x4*>(p.dC + ((size_t)b * P + pp) * 128 + 32 * wave + 8 * g + 4 * hh) = dcw[(g * 4 + cb) * 64];
    }
}

inline hipError_t convlstm_bwd_frames(const RecBwdParams& p, hipStream_t st) {
  if (!rec_fits(p.h, p.w) || p.P != p.h * p.w || p.B < 1 || p.T < 1) return hipErrorInvalidValue;
  const char* e = getenv("AAA_RECB_ABL");
  switch (e ? atoi(e) : 0) {
#define AAA_RECB_CASE(a) \
  case a: hipLaunchKernelGGL((k_convlstm_bwd_frames<a>), dim3(p.B), dim3(256), 0, st, p); break;
    AAA_RECB_CASE(1) AAA_RECB_CASE(2) AAA_RECB_CASE(3) AAA_RECB_CASE(4) AAA_RECB_CASE(8) AAA_RECB_CASE(6)
#undef AAA_RECB_CASE
    default: hipLaunchKernelGGL((k_convlstm_bwd_frames<0>), dim3(p.B), dim3(256), 0, st, p); break;
  }
  return hipGetLastError();
}

}  // namespace aaa
