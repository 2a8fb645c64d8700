// Frame-resident ConvLSTM BPTT with split roles (bf16 operands, fp32
// accumulate, fp16 gates): the same chain as k_convlstm_bwd_frames
// (recur_bwd.h; attention.py:110-126 through autograd over the unroll) on 8
// waves per workgroup, two per SIMD, in two roles:
//
//   MFMA waves 0-3   the dgrad GEMM of every step (wave w: h rows 32w.. over
//                    the 4 column blocks and the dx rows of x row block w % 2
//                    over 2 of them, as before), then the GEMM result dh into
//                    an LDS hand-off buffer and dx to HBM;
//   epilogue waves   the gate backward of step s-1 (wave 4+e: the units of h
//   4-7              rows 32e.., the same lane mapping as MFMA wave e), the dc
//                    carry in registers, the refills of the chunk images (LDS-DMA),
//                    the band halo exchange.
//
// Why: in the single-role kernel a step's epilogue (HBM inputs dO, c, gates and
// the dZ stores: ~400 KB per band workgroup at config 5) runs serially after
// its GEMM with only a 4-unit register ring in flight, and its stores sit in
// the same in-order vmcnt queue as the next GEMM's weight stream -- the first
// weight wait of every step waits for the whole store burst (MI355X_MICROARCH:
// loads, stores and LDS-DMA retire in issue order).  Here the epilogue waves
// request the next epilogue's first NA units during the GEMM (their registers
// are idle then), the MFMA waves' queue holds weight loads only, and the
// chunk refills leave it too.  Measured at config 5 before this: without the
// epilogue's HBM traffic the single-role band BPTT ran 2423 instead of 3712 us,
// without its MFMAs 3639 (profiles/r03/ab/bptt_ablation.txt).
//
// LDS: the two chunk images (as before) + the dh hand-off [4][16 units][64
// lanes] f32x4 = 64 KB, which replaces the LDS dc carry (now in registers).
#pragma once
#include "recur_bwd.h"

namespace aaa {

constexpr int kSpNA = 8;   // epilogue units per lane requested during the GEMM (of 16; the rest stream behind them)

template <bool BAND = false>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2))) k_convlstm_bwd_split(RecBwdParams p) {
  constexpr bool SWZ = BAND;             // swizzled 256-B pixel rows (band: LDS capacity) or 272-B rows
  constexpr int PIT = SWZ ? 256 : 272;   // image pixel pitch (bytes)
  constexpr int IB = SWZ ? kBwIBS : kBwIB;
  __shared__ __attribute__((aligned(16))) unsigned char zim[2 * IB];   // chunk images (0: chunks 0, 2; 1: 1, 3)
  __shared__ __attribute__((aligned(16))) f32x4 dhl[4 * 16 * 64];      // dh hand-off [wave][g*4+cb][lane]
  int b = (int)blockIdx.x, band = 0, r0 = 0, r1 = p.h;
  if constexpr (BAND) {
    const int blk = (int)blockIdx.x, loc = blk >> 3;
    b = (blk & 7) + 8 * (loc / kRecBands);
    band = loc % kRecBands;
    if (b >= p.B) return;
    r0 = band * p.h / kRecBands;
    r1 = (band + 1) * p.h / kRecBands;
  }
  const int tid = (int)threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool mw = wave < 4;            // MFMA wave (wave-uniform)
  const int w = wave & 3;              // row block / channel group of either role
  const int r32 = lane & 31, hh = lane >> 5;
  const int P = p.P, W2 = p.w + 2, NPH = (r1 - r0 + 2) * W2;
  const int Pb = (r1 - r0) * p.w, pix0 = r0 * p.w;
  const size_t M = (size_t)p.B * P;
  auto hidx = [&](int pp) { return (pp / p.w - r0 + 1) * W2 + pp % p.w + 1; };

  {  // zero the images (borders and pads stay zero)
    u32x4* z = reinterpret_cast<u32x4*>(zim);
    for (int i = tid; i < 2 * IB / 16; i += 512) z[i] = u32x4{0u, 0u, 0u, 0u};
  }
  // (epilogue waves) chunk c of dZ_t from HBM into image c & 1, whole 1-KB pieces
  auto dma_chunk = [&](int t, int c) {
    const __amdgpu_buffer_rsrc_t rs =
        make_rsrc(p.dZ + ((size_t)t * M + (size_t)b * P) * 512, (uint32_t)(P * 512 * 2));
    for (int i = w; i < (SWZ ? (NPH + 3) >> 2 : kBwIB / 1024); i += 4) {
      const int sl = i * 64 + lane, ip = SWZ ? sl >> 4 : sl / 17, iy = ip / W2, ix = ip - iy * W2;
      const int q = SWZ ? sl & 15 : sl - 17 * ip;
      const int py = r0 + iy - 1, px = ix - 1, lq = SWZ ? q ^ ((ip - 2 * iy) & 15) : q;
      const bool v = (SWZ || q < 16) && ip < NPH && (unsigned)py < (unsigned)p.h && (unsigned)px < (unsigned)p.w;
      const uint32_t vo = v ? (uint32_t)(((py * p.w + px) * 512 + 128 * c + lq * 8) * 2) : kOOB;
      if constexpr (BAND) dma16_sc1(rs, zim + (c & 1) * IB + i * 1024, vo);
      else dma16(rs, zim + (c & 1) * IB + i * 1024, vo);
    }
  };

  // Both roles run the same barrier sequence per step; each keeps its own state
  // in its own branch (one role's registers are not live in the other's code).
  if (mw) {
    int hb[4], fb[4];
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      const int col = min(cb * 32 + r32, Pb - 1), pp = pix0 + col;
      hb[cb] = (pp / p.w - r0) * W2 + pp % p.w;
      fb[cb] = col;
    }
    const __amdgpu_buffer_rsrc_t rsw = make_rsrc(p.Wb, (uint32_t)(6 * kBwKSP * 1024));
    const int wofs = w * kBwKSP * 1024, xofs = (4 + (w & 1)) * kBwKSP * 1024;
    auto lda = [&](int ks, int x) {
      return __builtin_bit_cast(bf16x8,
                                __builtin_amdgcn_raw_buffer_load_b128(rsw, lane * 16, (x ? xofs : wofs) + ks * 1024, 0));
    };
    constexpr int PD = kBwPD;
    bf16x8 af[PD][2];
#pragma unroll
    for (int s = 0; s < PD - 1; ++s) {
      af[s][0] = lda(s, 0);
      af[s][1] = lda(s, 1);
    }
    const int xcb = 2 * (w >> 1);
    float xbs[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) xbs[i] = 0.f;
    __syncthreads();   // images zeroed
    barrier_lds();     // the epilogue waves' dZ_{T-1} chunk images
    for (int t = p.T - 1; t >= 0; --t) {
      if constexpr (BAND) {   // the epilogue waves fetch the halo rows
        barrier_lds();
        barrier_lds();
      }
      f32x16 acc[4], accx[2];
#pragma unroll
      for (int cb = 0; cb < 4; ++cb)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[cb][e] = 0.f;
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) accx[j][e] = 0.f;
      int hbs[4], fbs[4];
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
        hbs[cb] = hb[cb];
        fbs[cb] = fb[cb];
        asm volatile("" : "+v"(hbs[cb]), "+v"(fbs[cb]));
      }
      auto bases = [&](int tap, int (&tb)[4]) {   // as k_convlstm_bwd_frames
        const int ky = tap / 3, kx = tap - 3 * ky;
        const int toff = (2 - ky) * W2 + (2 - kx), tf = (2 - ky) * p.w + (2 - kx);
#pragma unroll
        for (int cb = 0; cb < 4; ++cb)
          tb[cb] = SWZ ? ((hbs[cb] + toff) << 8) | (((((fbs[cb] + tf) & 15) ^ hh)) << 4) : toff * PIT;
      };
      auto ldb = [&](const unsigned char* img, const int (&tb)[4], int c16, bf16x8 (&bf)[4]) {
#pragma unroll
        for (int cb = 0; cb < 4; ++cb)
          bf[cb] = SWZ ? *reinterpret_cast<const bf16x8*>(img + (tb[cb] ^ (c16 << 5)))
                       : *reinterpret_cast<const bf16x8*>(img + tb[0] + hbs[cb] * PIT + hh * 16 + c16 * 32);
      };
      constexpr int BD = 4;
      bf16x8 bfr[BD][4];
      auto kloop = [&](auto xc) {
        constexpr int XC = decltype(xc)::value;
#pragma unroll 1
        for (int ck = 0; ck < 4; ++ck) {
          const unsigned char* img = zim + (ck & 1) * IB;
          int tcur[4], tnxt[4];
          bases(0, tcur);
#pragma unroll
          for (int j = 0; j < BD - 1; ++j) ldb(img, tcur, j, bfr[j]);
          for (int tap = 0; tap < 9; ++tap) {
            if (tap < 8) bases(tap + 1, tnxt);
            int kt = ck * 72 + tap * 8;
            asm volatile("" : "+s"(kt));
#pragma unroll
            for (int c16 = 0; c16 < 8; ++c16) {
              af[(c16 + PD - 1) % PD][0] = lda(kt + c16 + PD - 1, 0);
              af[(c16 + PD - 1) % PD][1] = lda(kt + c16 + PD - 1, 1);
              {
                const int cn = c16 + BD - 1;
                if (cn < 8) ldb(img, tcur, cn, bfr[cn % BD]);
                else if (tap < 8) ldb(img, tnxt, cn - 8, bfr[cn % BD]);
              }
              __builtin_amdgcn_sched_barrier(0);
#pragma unroll
              for (int cb = 0; cb < 4; ++cb)
                acc[cb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[c16 % PD][0], bfr[c16 % BD][cb], acc[cb], 0, 0, 0);
#pragma unroll
              for (int j = 0; j < 2; ++j)
                accx[j] =
                    __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[c16 % PD][1], bfr[c16 % BD][XC + j], accx[j], 0, 0, 0);
              __builtin_amdgcn_sched_barrier(0);
            }
#pragma unroll
            for (int cb = 0; cb < 4; ++cb) tcur[cb] = tnxt[cb];
          }
          barrier_lds();   // image ck & 1 free; (ck = 1, 2) the epilogue waves' refill of chunk ck+1 has landed
        }
      };
      if (w >> 1) kloop(std::integral_constant<int, 2>{});
      else kloop(std::integral_constant<int, 0>{});
      if (t > 0) {   // dh_{t-1} to the epilogue waves first: they wait for it
#pragma unroll
        for (int cb = 0; cb < 4; ++cb)
#pragma unroll
          for (int g = 0; g < 4; ++g)
            dhl[(w * 16 + g * 4 + cb) * 64 + lane] =
                f32x4{acc[cb][4 * g], acc[cb][4 * g + 1], acc[cb][4 * g + 2], acc[cb][4 * g + 3]};
      }
      barrier_lds();   // dh_{t-1} handed off
      {  // dx_t to HBM (bf16) and its fp32 sums, under the epilogue
        const size_t rows = (size_t)t * M + (size_t)b * P;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int col = (xcb + j) * 32 + r32;
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const float v[4] = {accx[j][4 * g], accx[j][4 * g + 1], accx[j][4 * g + 2], accx[j][4 * g + 3]};
            if (col < Pb) {
              *reinterpret_cast<bf16x4*>(p.dY2 + (rows + pix0 + col) * 64 + 32 * (w & 1) + 8 * g + 4 * hh) =
                  bf16x4{(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
#pragma unroll
              for (int e = 0; e < 4; ++e) xbs[4 * g + e] += v[e];
            }
          }
        }
      }
      if (t == 0 && p.dh0) {   // dh_{-1}: the gradient of the initial state h0
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) {
          const int col = cb * 32 + r32;
          if (col < Pb)
#pragma unroll
            for (int g = 0; g < 4; ++g)
              *reinterpret_cast<f32x4*>(p.dh0 + ((size_t)b * P + pix0 + col) * 128 + 32 * w + 8 * g + 4 * hh) =
                  f32x4{acc[cb][4 * g], acc[cb][4 * g + 1], acc[cb][4 * g + 2], acc[cb][4 * g + 3]};
        }
      }
      barrier_lds();   // the epilogue waves' dZ_{t-1} chunk images
    }
    {  // conv2 bias partials: reduce the 16 x-channel sums over the 32 pixel lanes of each half
      float v[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) v[i] = xbs[i];
      int n = 16;
#pragma unroll
      for (int m = 16; m >= 2; m >>= 1) {
        const bool up = (r32 & m) != 0;
        n >>= 1;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          if (i < n) {
            const float send = up ? v[i] : v[i + n];
            const float keep = up ? v[i + n] : v[i];
            v[i] = keep + __shfl_xor(send, m, 64);
          }
        }
      }
      v[0] += __shfl_xor(v[0], 1, 64);
      const int ridx = ((r32 & 16) ? 8 : 0) + ((r32 & 8) ? 4 : 0) + ((r32 & 4) ? 2 : 0) + ((r32 & 2) ? 1 : 0);
      if ((r32 & 1) == 0) {
        const int g = ridx >> 2, e = ridx & 3;
        atomicAdd(p.dxb + (size_t)b * 64 + 32 * (w & 1) + 8 * g + 4 * hh + e, v[0]);
      }
    }
  } else {
    // unit u = (g, cb) = (u >> 2, u & 3): channels 32w + 8g + 4hh + e (e = 0..3) at column 32cb + r32
    struct EpIn { f32x4 dO, cp; u32x4 gt[2]; };
    f32x4 dcr[16];   // the dc carry of the lane's 16 units
    EpIn pre[kSpNA];
    auto load_in = [&](int s, int u) {
      EpIn in;
      int ln = lane;
      asm volatile("" : "+v"(ln));
      const int g = u >> 2, cb = u & 3, col = cb * 32 + (ln & 31);
      if (col < Pb) {
        const size_t row = (size_t)s * M + (size_t)b * P + pix0 + col;
        const int ch = 32 * w + 4 * (ln >> 5) + 8 * g;
        in.dO = *reinterpret_cast<const f32x4*>(p.dO + row * 128 + ch);
        in.cp = *reinterpret_cast<const f32x4*>(p.Cst + row * 128 + ch);   // c_{s-1}
        const u32x4* gp = reinterpret_cast<const u32x4*>(p.Gt + row * 512 + 4 * ch);
        in.gt[0] = gp[0];
        in.gt[1] = gp[1];
      } else {
        in.dO = in.cp = f32x4{0.f, 0.f, 0.f, 0.f};
        in.gt[0] = in.gt[1] = u32x4{0u, 0u, 0u, 0u};
      }
      return in;
    };
    // gate backward of step s for the lane's 16 units: dh from the hand-off buffer
    // (gemm) or dO + dhT (s = T-1); units 0..kSpNA-1 already requested in pre[],
    // unit kSpNA + j requested into pre[j] once unit j is done
    auto epilogue = [&](int s, bool gemm) {
      int ln = lane;
      asm volatile("" : "+v"(ln));
      const int pl = ln & 31, hq = ln >> 5;
      const int c0 = 32 * w + 4 * hq;
      const size_t rows = (size_t)s * M + (size_t)b * P;
      const __amdgpu_buffer_rsrc_t rz = make_rsrc(p.dZ + rows * 512, (uint32_t)(P * 512 * 2));
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        float bs[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) bs[i] = 0.f;
        const int ch = c0 + 8 * g;
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) {
          const int u = g * 4 + cb;
          const EpIn in = pre[u % kSpNA];
          if (u + kSpNA < 16) pre[u % kSpNA] = load_in(s, u + kSpNA);
          const int col = cb * 32 + pl;
          if (col < Pb) {
            const int pp = pix0 + col;
            f32x4 dh = in.dO;
            if (gemm) {
              const f32x4 a = dhl[(w * 16 + u) * 64 + ln];
              dh[0] += a[0]; dh[1] += a[1]; dh[2] += a[2]; dh[3] += a[3];
            } else if (p.dhT) {
              const f32x4 x = *reinterpret_cast<const f32x4*>(p.dhT + ((size_t)b * P + pp) * 128 + ch);
              dh[0] += x[0]; dh[1] += x[1]; dh[2] += x[2]; dh[3] += x[3];
            }
            f32x4 dc = dcr[u];
            float dz[16];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const uint32_t w01 = in.gt[e >> 1][2 * (e & 1)], w23 = in.gt[e >> 1][2 * (e & 1) + 1];
              typedef _Float16 h2 __attribute__((ext_vector_type(2)));
              const h2 a = __builtin_bit_cast(h2, w01), c2 = __builtin_bit_cast(h2, w23);
              const f32x4 gv{(float)a[0], (float)a[1], (float)c2[0], (float)c2[1]};
              float d = dc[e], di, df, dcg, dout;
              gate_bwd_fast(dh[e], gv, in.cp[e], gv[1] * in.cp[e] + gv[0] * gv[2], d, di, df, dcg, dout);
              dc[e] = d;
              dz[4 * e] = di; dz[4 * e + 1] = df; dz[4 * e + 2] = dcg; dz[4 * e + 3] = dout;
              bs[4 * e] += di; bs[4 * e + 1] += df; bs[4 * e + 2] += dcg; bs[4 * e + 3] += dout;
            }
            dcr[u] = dc;
            bf16x8 z0, z1;
#pragma unroll
            for (int i = 0; i < 8; ++i) { z0[i] = (__bf16)dz[i]; z1[i] = (__bf16)dz[8 + i]; }
            const uint32_t zo = (uint32_t)((pp * 512 + 4 * ch) * 2);
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, z0), rz, zo, 0, BAND ? kSC1 : 0);
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, z1), rz, zo + 16, 0, BAND ? kSC1 : 0);
            if (w < 2) {   // chunk w of the next GEMM's B operand: rows 4(ch - 32w) + gate = slots 4g + 2hq, +1
              unsigned char* zi = zim + w * IB + hidx(pp) * PIT;
              const int fz = SWZ ? (col + p.w + 1) & 15 : 0, s0 = 4 * g + 2 * hq;
              *reinterpret_cast<bf16x8*>(zi + ((s0 ^ fz) << 4)) = z0;
              *reinterpret_cast<bf16x8*>(zi + (((s0 + 1) ^ fz) << 4)) = z1;
            }
          }
          __builtin_amdgcn_sched_barrier(0);
        }
        int n = 16;   // gate-bias partials of channel group g (recur_bwd.h's butterfly)
#pragma unroll
        for (int m = 16; m >= 2; m >>= 1) {
          const bool up = (pl & m) != 0;
          n >>= 1;
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            if (i < n) {
              const float send = up ? bs[i] : bs[i + n];
              const float keep = up ? bs[i + n] : bs[i];
              bs[i] = keep + __shfl_xor(send, m, 64);
            }
          }
        }
        bs[0] += __shfl_xor(bs[0], 1, 64);
        const int ridx = ((pl & 16) ? 8 : 0) + ((pl & 8) ? 4 : 0) + ((pl & 4) ? 2 : 0) + ((pl & 2) ? 1 : 0);
        if ((pl & 1) == 0)
          p.part[(((size_t)s * p.B + b) * (BAND ? kRecBands : 1) + band) * 512 + 4 * (ch + (ridx >> 2)) + (ridx & 3)] =
              bs[0];
      }
      if constexpr (BAND) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // dZ_s retired before the publish
    };
#pragma unroll
    for (int u = 0; u < 16; ++u) {   // dc_T
      const int col = (u & 3) * 32 + r32;
      dcr[u] = col < Pb ? *reinterpret_cast<const f32x4*>(p.dC + ((size_t)b * P + pix0 + col) * 128 + 32 * w +
                                                           8 * (u >> 2) + 4 * hh)
                        : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    if ((b >> 3) & 1) stagger_wait(p.stagger);
    __syncthreads();   // images zeroed
#pragma unroll
    for (int u = 0; u < kSpNA; ++u) pre[u] = load_in(p.T - 1, u);
    epilogue(p.T - 1, false);   // step T-1: no GEMM (dh = dO_{T-1} + dhT)
    barrier_lds();   // chunk images 0, 1 of dZ_{T-1}; (band) its stores retired
    if constexpr (BAND)
      if (tid == 256) __hip_atomic_store(p.flags + b * kRecBands + band, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int t = p.T - 1; t >= 0; --t) {
      if constexpr (BAND) {   // the neighbours' boundary rows of dZ_t, chunks 0 and 1, into the halo rows
        if (wave == 4)
          wave_wait_flags(p.flags + b * kRecBands,
                          (band > 0 ? 1ull << (band - 1) : 0ull) | (band < kRecBands - 1 ? 1ull << (band + 1) : 0ull),
                          p.T - t, p.report, p.spin);
        barrier_lds();
        const __amdgpu_buffer_rsrc_t rs =
            make_rsrc(p.dZ + ((size_t)t * M + (size_t)b * P) * 512, (uint32_t)(P * 512 * 2));
        const int nh = p.w * 16, et = tid - 256;
        constexpr int NHL = 6;
        for (int i0 = 0; i0 < 4 * nh; i0 += 256 * NHL) {
          u32x4 v[NHL];
#pragma unroll
          for (int r = 0; r < NHL; ++r) {
            const int i = i0 + et + 256 * r, k = i / nh, j = i - k * nh;
            const int gy = (k >> 1) ? r1 : r0 - 1;
            const bool ok = i < 4 * nh && (unsigned)gy < (unsigned)p.h;
            v[r] = __builtin_amdgcn_raw_buffer_load_b128(
                rs, ok ? (uint32_t)(((gy * p.w + (j >> 4)) * 512 + 128 * (k & 1) + (j & 15) * 8) * 2) : kOOB, 0, kSC1);
          }
#pragma unroll
          for (int r = 0; r < NHL; ++r) {
            const int i = i0 + et + 256 * r, k = i / nh, j = i - k * nh;
            const int gy = (k >> 1) ? r1 : r0 - 1, iy = (k >> 1) ? r1 - r0 + 1 : 0, gx = j >> 4;
            if (i < 4 * nh && (unsigned)gy < (unsigned)p.h) {
              const int ip = iy * W2 + gx + 1, fz = (iy * p.w + gx + 1) & 15;
              *reinterpret_cast<u32x4*>(zim + (k & 1) * IB + ip * 256 + (((j & 15) ^ fz) << 4)) = v[r];
            }
          }
        }
        barrier_lds();
      }
      if (t > 0) {   // the next epilogue's first units, under this GEMM
#pragma unroll
        for (int u = 0; u < kSpNA; ++u) pre[u] = load_in(t - 1, u);
      }
#pragma unroll 1
      for (int ck = 0; ck < 4; ++ck) {   // during the GEMM: refill image 0 with chunk 2 and image 1 with chunk 3
        if (ck == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every epilogue wave's dZ_t stores retired
        if (ck == 1 || ck == 2) {   // image ck-1 is free (the barrier behind chunk ck-1)
          dma_chunk(t, ck + 1);
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // landed before the MFMA waves pass the next barrier
        }
        barrier_lds();
      }
      barrier_lds();   // dh_{t-1} handed off (the chunk images are free)
      if (t > 0) epilogue(t - 1, true);
      barrier_lds();   // chunk images 0, 1 of dZ_{t-1}; (band) its stores retired
      if constexpr (BAND)
        if (tid == 256 && t > 0)
          __hip_atomic_store(p.flags + b * kRecBands + band, p.T - t + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) {   // dc carry out (dc_0)
      const int col = (u & 3) * 32 + r32;
      if (col < Pb)
        *reinterpret_cast<f32x4*>(p.dC + ((size_t)b * P + pix0 + col) * 128 + 32 * w + 8 * (u >> 2) + 4 * hh) = dcr[u];
    }
  }
}

inline hipError_t convlstm_bwd_split(const RecBwdParams& p, bool band, hipStream_t st) {
  if (p.P != p.h * p.w || p.B < 1 || p.T < 1) return hipErrorInvalidValue;
  RecBwdParams q = p;
  if (band) {
    if (!bw_band_fits(p.h, p.w) || !p.flags || !p.report || p.spin < 0) return hipErrorInvalidValue;
    return launch_resident(reinterpret_cast<const void*>(&k_convlstm_bwd_split<true>), 8 * kRecBands * ((p.B + 7) / 8),
                           512, q, st);
  }
  if (!rec_fits(p.h, p.w)) return hipErrorInvalidValue;
  hipLaunchKernelGGL((k_convlstm_bwd_split<false>), dim3(p.B), dim3(512), 0, st, q);
  return hipGetLastError();
}

}  // namespace aaa
