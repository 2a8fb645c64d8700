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
constexpr int kBwPD = 4;           // A register slots (PD-1 k steps in flight); divides 8
constexpr int kBwPD2 = 8;          // the paired kernel's (3 MFMAs per k step: twice the k steps in flight)
constexpr int kBwKSP = kBwKS + kBwPD2 - 1;   // packed k steps per row block: the first PD2-1 repeated at the end
constexpr int kBwIP = 136;         // chunk image pixel pitch (bf16) of the unswizzled images: 128 rows + 8 pad (272 B)
constexpr int kBwIB = 46080;       // unswizzled chunk image bytes: 169 px x 272 B rounded up to whole 1-KB DMA pieces

// k step ks -> k of the dgrad GEMM (k = tap*512 + gate row)
__host__ __device__ constexpr int bw_k(int ks) { return ((ks % 72) >> 3) * 512 + (ks / 72) * 128 + (ks & 7) * 16; }

// Wb[((rb*kBwKSP + ks)*64 + lane)*8 + e] = W[row(rb, lane%32)][bw_k(ks % kBwKS) + (lane/32)*8 + e], W = the
// packed dgrad weights [192][4608] (k_WdTl: rows 0..63 x channels, 64..191 h channels); row blocks 0..3 =
// the h rows (the BPTT GEMM proper), 4..5 = the x rows (dx: conv2's output gradient, fused in the same pass)
static __global__ void __launch_bounds__(256) k_pack_wbfrag(const __bf16* __restrict__ W, __bf16* __restrict__ Wb) {
  const int c = blockIdx.x * 256 + (int)threadIdx.x;
  if (c >= 6 * kBwKSP * 64) return;
  const int lane = c & 63, rk = c >> 6, ks = rk % kBwKSP, rb = rk / kBwKSP;
  const int row = (rb < 4 ? 64 + rb * 32 : (rb - 4) * 32) + (lane & 31), k = bw_k(ks % kBwKS) + (lane >> 5) * 8;
  *reinterpret_cast<bf16x8*>(Wb + (size_t)c * 8) = *reinterpret_cast<const bf16x8*>(W + (size_t)row * 4608 + k);
}

inline hipError_t pack_wbfrag(const __bf16* W, __bf16* Wb, hipStream_t st) {
  hipLaunchKernelGGL(k_pack_wbfrag, dim3((6 * kBwKSP * 64 + 255) / 256), dim3(256), 0, st, W, Wb);
  return hipGetLastError();
}

// gate_bwd (epilogues.h) with the branch-free tanh of the bf16 recurrence (recur.h)
__device__ __forceinline__ void gate_bwd_fast(float dh, const f32x4& g, float cprev, float ccur, float& dc, float& di,
                                              float& df, float& dcg, float& dout) {
  const float gi = g[0], gf = g[1], gc = g[2], go = g[3];
  const float tc = tanh_fast(ccur);
  const float dcc = dc + dh * go * (1.f - tc * tc);
  dout = dh * tc * (1.f - go) * go;
  di = dcc * gc * (1.f - gi) * gi;
  df = dcc * cprev * (1.f - gf) * gf;
  dcg = dcc * gi * (1.f - gc * gc);
  dc = dcc * gf;
}

struct RecBwdParams {   // dO, Gt, Cst: per-(frame, step) slices, channel-quad-major per cqm (recur.h cqm4)
  const __bf16* Wb;       // fragment-order W_h^T
  const float* dO;        // (T, B, P, 128) attention-path grad of h_t
  const _Float16* Gt;     // (T, B, P, 512) gate activations
  const float* Cst;       // (T+1, B, P, 128): slot s+1 = c_s
  const float* dhT;       // (B, P, 128) extra grad of h_{T-1}, or null
  float* dC;              // (B, P, 128) dc carry: in = dc_T, out = dc_0
  __bf16* dZ;             // (T, B, P, 512) <- gate pre-activation grads
  float* part;            // (T, B, 512) <- gate-bias partials per (step, frame); paired: (T, B, 2, 512)
  float* dh0;             // (B, P, 128) <- grad of h_{-1}, or null
  __bf16* dY2;            // (T, B, P, 64) <- dx_t, the conv2 output gradient (bf16: its readers' operand type)
  float* dxb;             // (B, 64) <- conv2 bias-gradient partials per frame (fp32 sums of dx)
  int* flags;             // paired kernel: per (frame, half) count of published dZ steps ([2B], zeroed)
  int T, B, h, w, P;
  int* report;            // paired kernel: partner-timeout report word (pinned host, device-mapped; pair_wait)
  int spin;               // paired / band kernels: partner-wait budget, 100-MHz ticks (pair_wait)
  int stagger;            // start offset (100-MHz ticks) of the frames with (b / 8) odd (stagger_wait)
  int cqm = kCqmC | kCqmG | kCqmDO;   // which slices are channel-quad-major (recur.h kCqm*)
  int rowpad = 0;         // single-workgroup kernel: 16-B slots after each image row (0 or 14: bw_rowpad)
  int sc1_all = 0;        // band kernel: every dZ store / chunk piece sc1 (A/B), not only the exchanged rows
  int ring = 0;           // single-workgroup kernel: the LDS-DMA epilogue ring (k_convlstm_bwd_frames RING)
};

// Chunk images of the band kernel: image pixel ip (a (rows+2) x (w+2)
// zero-bordered grid) holds its 16 row groups of 8 bf16 at 16-B slots
// s ^ bw_fz(ip) of a 256-B row, bw_fz = the pixel's index with the two border
// columns of every image row skipped (mod 16): 184 pixels of a band image fit
// two images and the dc carry in the LDS only at a 256-B pitch, and a
// B-fragment read of 16 consecutive GEMM columns then covers 16 consecutive
// bw_fz values across grid-row ends (each ds_read_b128 lane group hits 16
// distinct bank groups).  The single-workgroup kernel keeps the 272-B pitch
// (slot ip mod 16 + s; conflicting where a column group crosses a row end):
// the swizzle's XOR addressing (no immediate offsets) measured slower there
// (C3 BPTT 1340 -> 1358 us, C4 paired 756 -> 790; profiles/r03/ab/swizzle.txt).
__device__ __forceinline__ int bw_fz(int ip, int W2) { return (ip - 2 * (ip / W2)) & 15; }
constexpr int kBwIBS = 47104;   // swizzled chunk image bytes: 184 px x 256 B (46 whole 1-KB DMA pieces)
// The single-workgroup kernel's row-padded images: pixel ip at byte 272 ip + 16 rowpad (ip / W2).
// With rowpad = 14 the slot group of (pixel, slot j) is (ip - 2 (ip / W2) + j) mod 16 = bw_fz + j:
// a B-fragment read's consecutive columns stay on consecutive bank groups across grid-row ends
// (272-B rows alone skip two groups at every row end), and a tap and a k step still move the
// address by a wave-uniform amount and an immediate -- window columns never cross an image row.
constexpr int kBwIBP = 49152;   // row-padded chunk image bytes (48 whole 1-KB DMA pieces)
inline int bw_rowpad(int h, int w) { return (h + 2) * (17 * (w + 2) + 14) * 16 <= kBwIBP ? 14 : 0; }

#ifdef AAA_STAMPS
// Diagnostic builds only (tools/ubench/bwband): per (workgroup, step) phase stamps
// (s_memrealtime, 100 MHz): step start, halo in, chunks 0..3 done, dx stored, epilogue done.
__device__ uint64_t aaa_bw_stamps[1024 * 64 * 8];
#define AAA_BW_STAMP(t, k)                                                                                    \
  do {                                                                                                        \
    if (tid == 0 && (t) < 64) aaa_bw_stamps[((size_t)blockIdx.x * 64 + (t)) * 8 + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define AAA_BW_STAMP(t, k) do {} while (0)
#endif

// ABL (diagnostic A/B only: AAA_RECB_ABL, honoured only in a -DAAA_ABLATION build): bit 0 = no A loads in the K loop,
// bit 1 = no epilogue HBM loads / stores, bit 2 = no MFMAs, bit 3 = no chunk-3 DMA, bit 4 = no halo exchange (band),
// bit 5 = no dZ stores (epilogue loads kept), bit 6 = no epilogue loads (dZ stores kept), bit 7 = no c_{s-1}
// loads, bit 8 = no gate loads, bit 9 = no dO loads (single-workgroup kernel).
//
// BAND: 21x21 grids (168x168 frames) do not fit one workgroup's images, so
// kRecBands workgroups split a frame by whole grid rows (recur.h band mode:
// 5-6 rows = <= 126 GEMM columns each, all 128 h rows and the 64 dx rows).
// A band's images hold its rows plus one halo row above and below.  Each step
// the band stores dZ_s with sc1 stores and publishes a count; before the GEMM
// over dZ_t it waits for its neighbours' counts and reads their boundary rows
// of chunks 0 and 1 (its own are in the images, written by its epilogue) with
// sc1 loads into the halo rows; chunks 2 and 3 come whole, halo rows included,
// by LDS-DMA with the sc1 policy.  The bands of a frame get block indices of
// equal residue mod 8 (one XCD under round-robin placement).
//
// RING (single-workgroup kernel only): the epilogue's inputs -- c_{s-1}, the 16 fp16 gates and the dc
// carry of a unit -- arrive by LDS-DMA (inline asm, dma16a) into a wave-private ring of kBwEpD unit
// slots that replaces the LDS dc carry (the carry lives in p.dC in HBM: read with the unit's inputs,
// written back with its dZ), and the epilogue waits for a unit with its own counted vmcnt.  The
// register ring's loads are compiler-visible: with the unit's dZ stores pending (gfx9 counts stores in
// vmcnt) the compiler treats the counter as out of order and waits vmcnt(0) before every unit, so the
// register ring never had more than one unit in flight; the DMA'd ring keeps kBwEpD units in flight.
constexpr int kBwEpD = 4;   // RING: unit slots per wave (4 pieces of 1 KB each: c_{s-1}, gates 0-7, gates 8-15, dc)
template <int ABL = 0, bool BAND = false, bool DOACC = !BAND, bool RING = false>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) k_convlstm_bwd_frames(RecBwdParams p) {
  static_assert(!RING || (!BAND && DOACC), "the DMA'd epilogue ring is the single-workgroup DOACC kernel's");
  constexpr bool SWZ = BAND;             // swizzled 256-B pixel rows (band) or 272-B rows
  constexpr int PIT = SWZ ? 256 : 272;   // image pixel pitch (bytes)
  constexpr int IMG = SWZ ? kBwIBS : kBwIBP;   // bytes per chunk image
  __shared__ __attribute__((aligned(16))) unsigned char zim[2 * IMG];   // chunk images (0: chunks 0, 2; 1: 1, 3)
  __shared__ __attribute__((aligned(16))) f32x4 dcl[RING ? 1 : 4 * 16 * 64];   // dc carry, lane-native [wave][g*4+cb][lane]
  __shared__ __attribute__((aligned(16))) unsigned char ering[RING ? 4 * kBwEpD * 4096 : 16];   // [wave][slot][piece][lane]
  int b = (int)blockIdx.x, band = 0, r0 = 0, r1 = p.h;   // band mode: this workgroup's grid rows [r0, r1)
  if constexpr (BAND) {
    const int blk = (int)blockIdx.x, loc = blk >> 3;
    b = (blk & 7) + 8 * (loc / kRecBands);
    band = loc % kRecBands;
    if (b >= p.B) return;   // padding group of the last XCD column
    r0 = band * p.h / kRecBands;
    r1 = (band + 1) * p.h / kRecBands;
  }
  const int tid = (int)threadIdx.x, lane = tid & 63;
  uint64_t wdl = 0;   // partner-wait deadline (common.h wait_expired), set by the first wait that polls
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r32 = lane & 31, hh = lane >> 5;
  const int P = p.P, W2 = p.w + 2, NPH = (r1 - r0 + 2) * W2;
  const int Pb = (r1 - r0) * p.w, pix0 = r0 * p.w;   // the band's pixels (the whole frame without BAND)
  const size_t M = (size_t)p.B * P;
  auto hidx = [&](int pp) { return (pp / p.w - r0 + 1) * W2 + pp % p.w + 1; };   // interior pixel -> image index
  const int rp = SWZ ? 0 : p.rowpad;   // (the host checked that the padded image fits: bw_rowpad)
  auto pixb = [&](int ip) { return SWZ ? ip * PIT : 272 * ip + 16 * rp * (ip / W2); };   // image pixel -> byte
  const int RS = 17 * W2 + rp;         // unswizzled: 16-B slots per image row

  {  // zero the images (borders and pads stay zero)
    u32x4* z = reinterpret_cast<u32x4*>(zim);
    for (int i = tid; i < 2 * IMG / 16; i += 256) z[i] = u32x4{0u, 0u, 0u, 0u};
  }
  // chunk c (rows 128c .. 128c+127) of dZ_t from HBM into image c & 1, whole
  // 1-KB pieces of 4 image pixels; borders and the tail read outside the
  // descriptor and land as zeros
  auto dma_chunk = [&](int t, int c) {
    const __amdgpu_buffer_rsrc_t rs =
        make_rsrc(p.dZ + ((size_t)t * M + (size_t)b * P) * 512, (uint32_t)(P * 512 * 2));
    for (int i = wave; i < (SWZ ? (NPH + 3) >> 2 : ((r1 - r0 + 2) * RS + 63) >> 6); i += 4) {
      const int sl = i * 64 + lane;
      int iy, ix, q;   // image row, column, 16-B slot of the pixel row (unswizzled: 16 = the pixel pad, ix = W2 the row pad)
      if constexpr (SWZ) {
        iy = (sl >> 4) / W2;
        ix = (sl >> 4) - iy * W2;
        q = (sl & 15) ^ (((sl >> 4) - 2 * iy) & 15);
      } else {
        iy = sl / RS;
        const int rem = sl - iy * RS;
        ix = rem / 17;
        q = rem - 17 * ix;
      }
      const int py = r0 + iy - 1, px = ix - 1;
      const bool v = q < 16 && iy < r1 - r0 + 2 && (unsigned)py < (unsigned)p.h && (unsigned)px < (unsigned)p.w;
      const uint32_t vo = v ? (uint32_t)(((py * p.w + px) * 512 + 128 * c + q * 8) * 2) : kOOB;
      if constexpr (BAND) {
        // sc1 only for pieces that reach a halo row (the neighbours' sc1-stored boundary rows); the
        // band's own rows come from its own plain stores, still in the XCD's L2
        const int fp = 4 * i, lp = 4 * i + 3, nr = r1 - r0 + 1;
        if (p.sc1_all || fp < W2 || lp >= nr * W2) dma16_sc1(rs, zim + (c & 1) * IMG + i * 1024, vo);
        else dma16(rs, zim + (c & 1) * IMG + i * 1024, vo);
      } else {
        dma16(rs, zim + (c & 1) * IMG + i * 1024, vo);
      }
    }
  };

  int hb[4], fb[4];   // per column block: top-left image pixel of the lane's window, and its bw_fz (= the column)
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) {
    const int col = min(cb * 32 + r32, Pb - 1), pp = pix0 + col;   // columns >= Pb read column Pb-1: never stored
    hb[cb] = (pp / p.w - r0) * W2 + pp % p.w;
    fb[cb] = col;
  }
  // dc carry of the lane's 64 (channel, pixel) pairs: channels 32w + 8g + 4hh + e at pixel 32cb + r32
  f32x4* dcw = dcl + (RING ? 0 : wave * 16 * 64 + lane);   // + (g*4 + cb) * 64
  if constexpr (!RING) {
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
        const int col = cb * 32 + r32;
        dcw[(g * 4 + cb) * 64] =
            col < Pb ? *reinterpret_cast<const f32x4*>(p.dC + ((size_t)b * P + pix0 + col) * 128 + 32 * wave + 8 * g + 4 * hh)
                     : f32x4{0.f, 0.f, 0.f, 0.f};
      }
  }
  // RING: unit u = (g, cb) of step s into the wave's slot u % kBwEpD -- four 1-KB DMA pieces, lane-native
  // (lane i's 16 B at 16 i); columns past the band read out of range and land as zeros, whose gate
  // backward is exactly zero (every gate 0)
  unsigned char* const eslots = ering + wave * kBwEpD * 4096;
  auto ring_issue = [&](int s, int u) {
    int ln = lane;   // laundered: the unit's offsets are recomputed per step (hoisted, they spill)
    asm volatile("" : "+v"(ln));
    const int g = u >> 2, cb = u & 3, col = cb * 32 + (ln & 31);
    const bool v = col < Pb && !(ABL & 66);
    const int ch = 32 * wave + 4 * (ln >> 5) + 8 * g, pp = pix0 + col;
    const size_t fr = (size_t)s * M + (size_t)b * P;
    const __amdgpu_buffer_rsrc_t rc = make_rsrc(p.Cst + fr * 128, (uint32_t)(P * 128 * 4));
    const __amdgpu_buffer_rsrc_t rg = make_rsrc(p.Gt + fr * 512, (uint32_t)(P * 512 * 2));
    const __amdgpu_buffer_rsrc_t rd = make_rsrc(p.dC + (size_t)b * P * 128, (uint32_t)(P * 128 * 4));
    unsigned char* slot = eslots + (u % kBwEpD) * 4096;
    const uint32_t go = v ? (uint32_t)(slcg(pp, ch, P, p.cqm & kCqmG) * 2) : kOOB;
    dma16a(rc, slot, v ? (uint32_t)(slc4(pp, ch, P, p.cqm & kCqmC) * 4) : kOOB);
    dma16a(rg, slot + 1024, go);
    dma16a(rg, slot + 2048, go, 16);
    dma16a(rd, slot + 3072, v ? (uint32_t)((pp * 128 + ch) * 4) : kOOB);
  };
  // Wait until unit u's pieces have landed.  vmcnt(N) waits for all but the wave's N youngest
  // vector-memory operations, loads, stores and LDS-DMA alike, in issue order (MI355X_MICROARCH), so N
  // counts every operation issued after the unit's four pieces: per epilogue iteration v its two dZ
  // stores, its dc store, the pieces of unit v + kBwEpD (v + kBwEpD < 16) and its dO load -- all
  // unconditional (out-of-range columns use out-of-range offsets), so the count is exact; the
  // operations it leaves out (dx stores between the pre-issue and the epilogue, gate-bias partial
  // stores) only make the wait longer.
  auto ring_wait = [&](int u) {
    auto ops = [](int v) { return 3 + (v + kBwEpD < 16 ? 4 : 0) + 1; };
    int n = 0;
    if (u < kBwEpD) {   // pre-issued in unit order before iteration 0
      n = 4 * (kBwEpD - 1 - u);
      for (int v = 0; v < u; ++v) n += ops(v);
    } else {            // issued in iteration u - kBwEpD, before that iteration's dO load
      n = 1;
      for (int v = u - kBwEpD + 1; v < u; ++v) n += ops(v);
    }
    switch (n) {   // (u is a constant of the unrolled epilogue: the switch folds)
#define AAA_RW(k) case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
      AAA_RW(0) AAA_RW(1) AAA_RW(2) AAA_RW(3) AAA_RW(4) AAA_RW(5) AAA_RW(6) AAA_RW(7) AAA_RW(8) AAA_RW(9)
      AAA_RW(10) AAA_RW(11) AAA_RW(12) AAA_RW(13) AAA_RW(14) AAA_RW(15) AAA_RW(16) AAA_RW(17) AAA_RW(18)
      AAA_RW(19) AAA_RW(20) AAA_RW(21) AAA_RW(22) AAA_RW(23) AAA_RW(24) AAA_RW(25) AAA_RW(26) AAA_RW(27)
      AAA_RW(28) AAA_RW(29) AAA_RW(30) AAA_RW(31) AAA_RW(32)
#undef AAA_RW
      default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    }
  };

  // A stream: per k step the wave's h row block (wave) and its dx row block (4 + wave % 2)
  const __amdgpu_buffer_rsrc_t rsw = make_rsrc(p.Wb, (uint32_t)(6 * kBwKSP * 1024));
  const int wofs = wave * kBwKSP * 1024, xofs = (4 + (wave & 1)) * kBwKSP * 1024;
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
  const int xcb = 2 * (wave >> 1);   // the wave's dx tiles: x row block wave % 2, column blocks xcb, xcb + 1
  float xbs[16];                     // conv2 bias partials of the lane's 16 x channels, all steps
#pragma unroll
  for (int i = 0; i < 16; ++i) xbs[i] = 0.f;

  // The epilogue's HBM inputs of one unit u = (g, cb) (g-major): c_{s-1} (16 B)
  // and the 16 fp16 gates (32 B) of the lane's 4 channels at one pixel; c_s =
  // f c_{s-1} + i c~ is recomputed from them (not read).  A ring of kRing units is
  // in flight: the first kRing-1 are requested under the GEMM's last chunk, each
  // later one as the unit kRing-1 before it is processed.  DOACC: the
  // attention-path grad dO_s is not in the ring but the initial value of the
  // GEMM's accumulators (acc = dO_{t-1} + W^T dZ_t = dh_{t-1}), requested into
  // each accumulator slot as soon as the epilogue before has consumed it (the
  // band kernel keeps dO in the ring: its accumulators carried across steps
  // spill there).
  struct EpIn { f32x4 dO, cp; u32x4 gt[2]; };
  constexpr int kRing = 4;
  auto load_in = [&](int s, int u, int ln) {
    EpIn in;
    const int g = u >> 2, cb = u & 3, col = cb * 32 + (ln & 31);
    // buffer loads, out-of-range offsets past the band (the hardware returns zeros): no branch, and no
    // zero-fill of the destinations on the other path -- a write to a register with a load in flight
    // made the compiler wait vmcnt(0) right after issuing the ring's loads, so the ring held nothing
    const bool v = col < Pb && !(ABL & 66);
    const size_t fr = (size_t)s * M + (size_t)b * P;
    const int ch = 32 * wave + 4 * (ln >> 5) + 8 * g, pp = pix0 + col;
    const __amdgpu_buffer_rsrc_t rc = make_rsrc(p.Cst + fr * 128, (uint32_t)(P * 128 * 4));
    const __amdgpu_buffer_rsrc_t rg = make_rsrc(p.Gt + fr * 512, (uint32_t)(P * 512 * 2));
    if constexpr (!DOACC) {
      const __amdgpu_buffer_rsrc_t ro = make_rsrc(p.dO + fr * 128, (uint32_t)(P * 128 * 4));
      in.dO = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                            ro, v ? (uint32_t)(slc4(pp, ch, P, p.cqm & kCqmDO) * 4) : kOOB, 0, 0));
    }
    in.cp = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                          rc, v && !(ABL & 128) ? (uint32_t)(slc4(pp, ch, P, p.cqm & kCqmC) * 4) : kOOB,
                                          0, 0));
    const uint32_t go = v && !(ABL & 256) ? (uint32_t)(slcg(pp, ch, P, p.cqm & kCqmG) * 2) : kOOB;
    in.gt[0] = __builtin_amdgcn_raw_buffer_load_b128(rg, go, 0, 0);
    in.gt[1] = __builtin_amdgcn_raw_buffer_load_b128(rg, go, 16, 0);
    return in;
  };
  // dO_s of unit u into its accumulator slot (zero past the band's columns, or for s < 0: dh_{-1} has no dO)
  auto load_dO = [&](f32x16 (&acc)[4], int s, int u, int ln) {
    const int g = u >> 2, cb = u & 3, col = cb * 32 + (ln & 31);
    f32x4 v{0.f, 0.f, 0.f, 0.f};
    if constexpr (RING || !BAND) {   // always one load (RING: ring_wait counts it; no branch): out of range for s < 0 / past the band
      const bool ok = s >= 0 && col < Pb && !(ABL & (66 | 512));
      const __amdgpu_buffer_rsrc_t ro = make_rsrc(p.dO + ((size_t)max(s, 0) * M + (size_t)b * P) * 128,
                                                  (uint32_t)(P * 128 * 4));
      v = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                        ro, ok ? (uint32_t)(slc4(pix0 + col, 32 * wave + 4 * (ln >> 5) + 8 * g, P,
                                                                 p.cqm & kCqmDO) * 4)
                                           : kOOB, 0, 0));
    } else if (s >= 0 && col < Pb && !(ABL & (66 | 512))) {   // (ABL 512: without the dO loads)
      v = *reinterpret_cast<const f32x4*>(p.dO + ((size_t)s * M + (size_t)b * P) * 128 +
                                          slc4(pix0 + col, 32 * wave + 4 * (ln >> 5) + 8 * g, P, p.cqm & kCqmDO));
    }
    acc[cb][4 * g] = v[0]; acc[cb][4 * g + 1] = v[1]; acc[cb][4 * g + 2] = v[2]; acc[cb][4 * g + 3] = v[3];
  };

  // Gate backward of step s on dh_s = acc (dO_s + the GEMM of step s+1, dO_{T-1} +
  // dhT for s = T-1): dZ_s to HBM (bf16) and, for chunks 0 and 1, into image w;
  // the lane's dc carry advances to step s-1; gate-bias partials of step s; each
  // consumed accumulator slot is refilled with dO_{s-1} (the next GEMM's start).
  // ``ring``: units 0 .. kRing-2 already requested.  BAND: then publishes dZ_s.
  auto epilogue = [&](int s, f32x16 (&acc)[4], EpIn (&ring)[kRing], bool first) {
    int ln = lane;   // laundered: the epilogue's addresses are recomputed per step, not hoisted
    asm volatile("" : "+v"(ln));
    const int pl = ln & 31, hq = ln >> 5;
    const int c0 = 32 * wave + 4 * hq;   // + 8g + e
    const size_t rows = (size_t)s * M + (size_t)b * P;
    const __amdgpu_buffer_rsrc_t rz = make_rsrc(p.dZ + rows * 512, (uint32_t)(P * 512 * 2));
    const __amdgpu_buffer_rsrc_t rdc = make_rsrc(p.dC + (size_t)b * P * 128, (uint32_t)(P * 128 * 4));   // RING
    (void)rdc;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      float bs[16];   // [e][gate] sums over the lane's pixels (this channel group)
#pragma unroll
      for (int i = 0; i < 16; ++i) bs[i] = 0.f;
      const int ch = c0 + 8 * g;
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
        const int u = g * 4 + cb;
        if constexpr (RING) {   // branch-free: out-of-range columns read zeros and store out of range
          ring_wait(u);
          const unsigned char* sl = eslots + (u % kBwEpD) * 4096 + ln * 16;
          const f32x4 cp = *reinterpret_cast<const f32x4*>(sl);
          const u32x4 gt[2] = {*reinterpret_cast<const u32x4*>(sl + 1024), *reinterpret_cast<const u32x4*>(sl + 2048)};
          f32x4 dc = *reinterpret_cast<const f32x4*>(sl + 3072);
          const int col = cb * 32 + pl, pp = pix0 + col;
          const bool v = col < Pb;
          const f32x4 dh{acc[cb][4 * g], acc[cb][4 * g + 1], acc[cb][4 * g + 2], acc[cb][4 * g + 3]};
          float dz[16];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const uint32_t w01 = gt[e >> 1][2 * (e & 1)], w23 = gt[e >> 1][2 * (e & 1) + 1];
            typedef _Float16 h2 __attribute__((ext_vector_type(2)));
            const h2 a = __builtin_bit_cast(h2, w01), c2 = __builtin_bit_cast(h2, w23);
            const f32x4 gv{(float)a[0], (float)a[1], (float)c2[0], (float)c2[1]};
            float d = dc[e], di, df, dcg, dout;
            gate_bwd_fast(dh[e], gv, cp[e], gv[1] * cp[e] + gv[0] * gv[2], d, di, df, dcg, dout);
            dc[e] = d;
            dz[4 * e] = di; dz[4 * e + 1] = df; dz[4 * e + 2] = dcg; dz[4 * e + 3] = dout;
            bs[4 * e] += di; bs[4 * e + 1] += df; bs[4 * e + 2] += dcg; bs[4 * e + 3] += dout;
          }
          bf16x8 z0, z1;
#pragma unroll
          for (int i = 0; i < 8; ++i) { z0[i] = (__bf16)dz[i]; z1[i] = (__bf16)dz[8 + i]; }
          if constexpr (!(ABL & 34)) {
            const uint32_t zo = v ? (uint32_t)((pp * 512 + 4 * ch) * 2) : kOOB;
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, z0), rz, zo, 0, 0);
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, z1), rz, zo, 16, 0);
          }
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, dc), rdc,
                                                 v ? (uint32_t)((pp * 128 + ch) * 4) : kOOB, 0, 0);
          if (wave < 2 && v) {   // chunk w of the next step's B operand: rows 4(ch - 32w) + gate = slots 4g + 2hq, +1
            unsigned char* zi = zim + wave * IMG + pixb(hidx(pp));
            const int s0 = 4 * g + 2 * hq;
            *reinterpret_cast<bf16x8*>(zi + (s0 << 4)) = z0;
            *reinterpret_cast<bf16x8*>(zi + ((s0 + 1) << 4)) = z1;
          }
          if (u + kBwEpD < 16) ring_issue(s, u + kBwEpD);   // the slot just read: unit u + kBwEpD
          load_dO(acc, s - 1, u, ln);   // the slot's next value: dO_{s-1}
          __builtin_amdgcn_sched_barrier(0);
          continue;
        }
        if (u + kRing - 1 < 16) ring[(u + kRing - 1) % kRing] = load_in(s, u + kRing - 1, ln);
        const EpIn& in = ring[u % kRing];
        const int col = cb * 32 + pl;
        if (col < Pb) {
          const int pp = pix0 + col;
          f32x4 dh{acc[cb][4 * g], acc[cb][4 * g + 1], acc[cb][4 * g + 2], acc[cb][4 * g + 3]};
          if constexpr (!DOACC) {
            dh[0] += in.dO[0]; dh[1] += in.dO[1]; dh[2] += in.dO[2]; dh[3] += in.dO[3];
            if (first && p.dhT) {
              const f32x4 x = *reinterpret_cast<const f32x4*>(p.dhT + ((size_t)b * P + pp) * 128 + ch);
              dh[0] += x[0]; dh[1] += x[1]; dh[2] += x[2]; dh[3] += x[3];
            }
          }
          f32x4* dcp = dcl + wave * 16 * 64 + ln + (g * 4 + cb) * 64;
          f32x4 dc = *dcp;
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
          *dcp = dc;
          bf16x8 z0, z1;
#pragma unroll
          for (int i = 0; i < 8; ++i) { z0[i] = (__bf16)dz[i]; z1[i] = (__bf16)dz[8 + i]; }
          if constexpr (!(ABL & 34) && BAND) {
            // the band's first and last grid rows are the neighbours' halo rows: sc1 (write-through)
            // stores; the interior rows plain, so they stay in the XCD's L2 for this band's own
            // chunk 2 / 3 refills (an sc1 store drops the line: MI355X_MICROARCH hand-off table)
            const uint32_t zo = (uint32_t)((pp * 512 + 4 * ch) * 2);
            const int gy = pp / p.w;
            if (p.sc1_all || gy == r0 || gy == r1 - 1) {
              __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, z0), rz, zo, 0, kSC1);
              __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, z1), rz, zo + 16, 0, kSC1);
            } else {
              __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, z0), rz, zo, 0, 0);
              __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, z1), rz, zo + 16, 0, 0);
            }
          } else if constexpr (!(ABL & 34)) {
            __bf16* zo = p.dZ + (rows + pp) * 512 + 4 * ch;
            *reinterpret_cast<bf16x8*>(zo) = z0;
            *reinterpret_cast<bf16x8*>(zo + 8) = z1;
          }
          if (wave < 2) {   // chunk w of the next step's B operand: rows 4(ch - 32w) + gate = slots 4g + 2hq, +1
            unsigned char* zi = zim + wave * IMG + pixb(hidx(pp));
            const int fz = SWZ ? (col + p.w + 1) & 15 : 0, s0 = 4 * g + 2 * hq;
            *reinterpret_cast<bf16x8*>(zi + ((s0 ^ fz) << 4)) = z0;
            *reinterpret_cast<bf16x8*>(zi + (((s0 + 1) ^ fz) << 4)) = z1;
          }
        }
        if constexpr (DOACC) load_dO(acc, s - 1, u, ln);   // the slot's next value: dO_{s-1}
        __builtin_amdgcn_sched_barrier(0);
      }
      // gate-bias partials of channel group g: butterfly transpose-reduce of the 16
      // row sums over the 32 pixel lanes of each half; after 4 exchange steps and a
      // final pair add, lanes pl and pl^1 hold row ridx's total
      int n = 16;
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
      if ((pl & 1) == 0)   // row ridx = 4e + gate of channel ch + e; band mode: a row of partials per band
        p.part[(((size_t)s * p.B + b) * (BAND ? kRecBands : 1) + band) * 512 + 4 * (ch + (ridx >> 2)) + (ridx & 3)] =
            bs[0];
    }
    if constexpr (BAND) {   // publish dZ_s: every wave's sc1 stores retired, a barrier, one lane's flag store
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      barrier_lds();
      if (tid == 0) __hip_atomic_store(p.flags + b * kRecBands + band, p.T - s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  };

  if ((b >> 3) & 1) stagger_wait(p.stagger);
  f32x16 acc_carry[4];   // DOACC: the GEMM accumulators, carried across steps (dO_{t-1} at the start of step t's GEMM)
  {  // step T-1: no GEMM (dh = dO_{T-1} + dhT)
    f32x16 (&acc)[4] = acc_carry;
    EpIn ring[kRing];
    if constexpr (RING) {
#pragma unroll
      for (int u = 0; u < kBwEpD; ++u) ring_issue(p.T - 1, u);
    } else {
#pragma unroll
      for (int u = 0; u < kRing - 1; ++u) ring[u] = load_in(p.T - 1, u, lane);
    }
    if constexpr (DOACC) {
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        load_dO(acc, p.T - 1, u, lane);
        const int g = u >> 2, cb = u & 3, col = cb * 32 + r32;
        if (p.dhT && col < Pb) {
          const f32x4 x =
              *reinterpret_cast<const f32x4*>(p.dhT + ((size_t)b * P + pix0 + col) * 128 + 32 * wave + 8 * g + 4 * hh);
          acc[cb][4 * g] += x[0]; acc[cb][4 * g + 1] += x[1]; acc[cb][4 * g + 2] += x[2]; acc[cb][4 * g + 3] += x[3];
        }
      }
    } else {   // dO (ring) and dhT (epilogue) are added in the epilogue
#pragma unroll
      for (int cb = 0; cb < 4; ++cb)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[cb][e] = 0.f;
    }
    epilogue(p.T - 1, acc, ring, true);
  }
  barrier_lds();   // chunk images 0, 1 of dZ_{T-1}

  for (int t = p.T - 1; t >= 0; --t) {
    AAA_BW_STAMP(t, 0);
    if constexpr (BAND && !(ABL & 16)) {   // the neighbours' boundary rows of dZ_t, chunks 0 and 1, into the halo rows
      if (wave == 0)   // the neighbour bands' flags, both in one poll
        wave_wait_flags(p.flags + b * kRecBands,
                        ((band > 0 ? 1ull : 0ull) << (band - 1 + (band == 0))) | (band < kRecBands - 1 ? 2ull << band : 0ull),
                        p.T - t, p.report, p.spin, wdl);
      barrier_lds();
      const __amdgpu_buffer_rsrc_t rs =
          make_rsrc(p.dZ + ((size_t)t * M + (size_t)b * P) * 512, (uint32_t)(P * 512 * 2));
      const int nh = p.w * 16;   // 16-B pieces of one grid row of one chunk
      constexpr int NHL = 3;     // pieces per thread in flight
      for (int i0 = 0; i0 < 4 * nh; i0 += 256 * NHL) {
        u32x4 v[NHL];
#pragma unroll
        for (int r = 0; r < NHL; ++r) {   // piece i: (side, chunk) = i / nh, pixel (i % nh) / 16, slot i % 16
          const int i = i0 + tid + 256 * r, k = i / nh, j = i - k * nh;
          const int gy = (k >> 1) ? r1 : r0 - 1;
          const bool ok = i < 4 * nh && (unsigned)gy < (unsigned)p.h;
          v[r] = __builtin_amdgcn_raw_buffer_load_b128(
              rs, ok ? (uint32_t)(((gy * p.w + (j >> 4)) * 512 + 128 * (k & 1) + (j & 15) * 8) * 2) : kOOB, 0, kSC1);
        }
#pragma unroll
        for (int r = 0; r < NHL; ++r) {
          const int i = i0 + tid + 256 * r, k = i / nh, j = i - k * nh;
          const int gy = (k >> 1) ? r1 : r0 - 1, iy = (k >> 1) ? r1 - r0 + 1 : 0, gx = j >> 4;
          if (i < 4 * nh && (unsigned)gy < (unsigned)p.h) {
            const int ip = iy * W2 + gx + 1, fz = (iy * p.w + gx + 1) & 15;
            *reinterpret_cast<u32x4*>(zim + (k & 1) * IMG + ip * 256 + (((j & 15) ^ fz) << 4)) = v[r];
          }
        }
      }
      barrier_lds();
    }
    AAA_BW_STAMP(t, 1);
    f32x16 acc_local[4];
    f32x16 (&acc)[4] = *(DOACC ? &acc_carry : &acc_local);
    if constexpr (!DOACC) {
#pragma unroll
      for (int cb = 0; cb < 4; ++cb)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[cb][e] = 0.f;
    }
    f32x16 accx[2];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) accx[j][e] = 0.f;
    int hbs[4], fbs[4];
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      hbs[cb] = SWZ ? hb[cb] : pixb(hb[cb]);   // unswizzled: the window's top-left pixel as a byte offset
      fbs[cb] = fb[cb];
      asm volatile("" : "+v"(hbs[cb]), "+v"(fbs[cb]));
    }
    // transposed gather: output pixel q reads dZ at q - d(tap): image offset (2-ky)*W2 + (2-kx),
    // bw_fz offset (2-ky)*w + (2-kx).  Per tap and column block: the byte address of the
    // lane's pixel row or'ed with its swizzled slot for c16 = 0; row group c16 xors in c16 << 5.
    // (unswizzled: the lane's part hbs + hh * 16 is per step, the tap's offset wave-uniform, the row
    // group an immediate; tb then carries the tap offset only)
    auto bases = [&](int tap, int (&tb)[4]) {
      const int ky = tap / 3, kx = tap - 3 * ky;
      const int toff = (2 - ky) * W2 + (2 - kx), tf = (2 - ky) * p.w + (2 - kx);
#pragma unroll
      for (int cb = 0; cb < 4; ++cb)
        tb[cb] = SWZ ? ((hbs[cb] + toff) << 8) | (((((fbs[cb] + tf) & 15) ^ hh)) << 4) : toff * PIT + 16 * rp * (2 - ky);
    };
    auto ldb = [&](const unsigned char* img, const int (&tb)[4], int c16, bf16x8 (&bf)[4]) {
#pragma unroll
      for (int cb = 0; cb < 4; ++cb)
        bf[cb] = SWZ ? *reinterpret_cast<const bf16x8*>(img + (tb[cb] ^ (c16 << 5)))
                     : *reinterpret_cast<const bf16x8*>(img + tb[0] + hbs[cb] + hh * 16 + c16 * 32);
    };
    constexpr int BD = 4;   // B fragment ring: BD-1 k steps of lookahead (LDS latency vs 4 MFMAs per k step); divides 8
    bf16x8 bfr[BD][4];
    EpIn ring[kRing];
    // the K loop, with the wave's dx column blocks XC, XC+1 a compile-time constant
    // (a uniform select between fragment registers would be a per-k-step copy)
    auto kloop = [&](auto xc) {
      constexpr int XC = decltype(xc)::value;
  #pragma unroll 1
      for (int ck = 0; ck < 4; ++ck) {
        const unsigned char* img = zim + (ck & 1) * IMG;
        if (ck == 1 || ck == 2) {   // every wave is done with image ck-1 and every wave's dZ_t stores have
                                    // retired (its later A loads did): refill it with chunk ck+1 from HBM
          if constexpr (!(ABL & 8)) dma_chunk(t, ck + 1);
        }
        if (!RING && ck == 3 && t > 0) {   // the epilogue's first inputs, under chunk 3
          int ln = lane;
          asm volatile("" : "+v"(ln));
  #pragma unroll
          for (int u = 0; u < kRing - 1; ++u) ring[u] = load_in(t - 1, u, ln);
        }
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
            if constexpr (!(ABL & 1)) {
              af[(c16 + PD - 1) % PD][0] = lda(kt + c16 + PD - 1, 0);
              af[(c16 + PD - 1) % PD][1] = lda(kt + c16 + PD - 1, 1);
            }
            {  // B of k step + BD - 1 (same chunk)
              const int cn = c16 + BD - 1;
              if (cn < 8) ldb(img, tcur, cn, bfr[cn % BD]);
              else if (tap < 8) ldb(img, tnxt, cn - 8, bfr[cn % BD]);
            }
            __builtin_amdgcn_sched_barrier(0);
  #pragma unroll
            for (int cb = 0; cb < 4; ++cb) {
              if constexpr (ABL & 4) acc[cb][0] += (float)af[c16 % PD][0][0] * (float)bfr[c16 % BD][cb][0];
              else acc[cb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[c16 % PD][0], bfr[c16 % BD][cb], acc[cb], 0, 0, 0);
            }
  #pragma unroll
            for (int j = 0; j < 2; ++j) {   // dx rows: the B fragments of column blocks xcb, xcb + 1
              const bf16x8 bx = bfr[c16 % BD][XC + j];
              if constexpr (!(ABL & 4))
                accx[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[c16 % PD][1], bx, accx[j], 0, 0, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
          }
  #pragma unroll
          for (int cb = 0; cb < 4; ++cb) tcur[cb] = tnxt[cb];
        }
        barrier_lds();   // image ck & 1 free; (ck >= 1) the DMA'd chunk ck+1 has landed in every wave
        AAA_BW_STAMP(t, 2 + ck);
      }
    };
    if (wave >> 1) kloop(std::integral_constant<int, 2>{});
    else kloop(std::integral_constant<int, 0>{});
    if constexpr (RING) {
      if (t > 0) {   // the next epilogue's first kBwEpD units, under the dx stores; the dc carries
                     // they read were stored by the last epilogue (retired: vmcnt(0) first)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int u = 0; u < kBwEpD; ++u) ring_issue(t - 1, u);
      }
    }
    {  // dx_t (conv2 output grad) to HBM in bf16; its fp32 sums into the conv2 bias partials
      const size_t rows = (size_t)t * M + (size_t)b * P;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int col = (xcb + j) * 32 + r32;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const float v[4] = {accx[j][4 * g], accx[j][4 * g + 1], accx[j][4 * g + 2], accx[j][4 * g + 3]};
          if (col < Pb) {
            *reinterpret_cast<bf16x4*>(p.dY2 + (rows + pix0 + col) * 64 + 32 * (wave & 1) + 8 * g + 4 * hh) =
                bf16x4{(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
#pragma unroll
            for (int e = 0; e < 4; ++e) xbs[4 * g + e] += v[e];
          }
        }
      }
    }
    AAA_BW_STAMP(t, 6);
    if (t > 0) {
      epilogue(t - 1, acc, ring, false);
    } else if (p.dh0) {   // dh_{-1}: the gradient of the initial state h0
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
        const int col = cb * 32 + r32;
        if (col < Pb)
#pragma unroll
          for (int g = 0; g < 4; ++g)
            *reinterpret_cast<f32x4*>(p.dh0 + ((size_t)b * P + pix0 + col) * 128 + 32 * wave + 8 * g + 4 * hh) =
                f32x4{acc[cb][4 * g], acc[cb][4 * g + 1], acc[cb][4 * g + 2], acc[cb][4 * g + 3]};
      }
    }
    barrier_lds();   // chunk images 0, 1 of dZ_{t-1} complete
    AAA_BW_STAMP(t, 7);
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
    v[0] += __shfl_xor(v[0], 1, 64);   // lanes r32 and r32 ^ 1 now both hold row ridx's total
    const int ridx = ((r32 & 16) ? 8 : 0) + ((r32 & 8) ? 4 : 0) + ((r32 & 4) ? 2 : 0) + ((r32 & 2) ? 1 : 0);
    if ((r32 & 1) == 0) {   // row ridx = 4g + e: x channel 32(w%2) + 8g + 4hh + e; two waves (and the bands) share each
      const int g = ridx >> 2, e = ridx & 3;
      atomicAdd(p.dxb + (size_t)b * 64 + 32 * (wave & 1) + 8 * g + 4 * hh + e, v[0]);
    }
  }
  // dc carry out (dc_0; RING: already in p.dC, written by the last epilogue)
  if constexpr (!RING) {
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
        const int col = cb * 32 + r32;
        if (col < Pb)
          *reinterpret_cast<f32x4*>(p.dC + ((size_t)b * P + pix0 + col) * 128 + 32 * wave + 8 * g + 4 * hh) =
              dcw[(g * 4 + cb) * 64];
      }
  }
}

// Paired variant, for batches below the CU count: two workgroups per frame.
// Half kh owns the h channels [64kh, 64kh+64) -- dZ chunks 2kh and 2kh+1, the
// dh rows of those channels, their dc carry -- and the x channels [32kh,
// 32kh+32) of dx.  Per step it runs its own two chunks first (LDS images its
// epilogue wrote), then the partner's two, read from HBM once the partner has
// published dZ_t: the partner's dZ stores are sc1, its flag an sc1 store behind
// every wave's vmcnt(0) and a barrier, and the chunks come back with sc1 loads
// to registers (then ds_write), so neither side pays an agent fence
// (MI355X_MICROARCH: inter-workgroup visibility, hand-off table row 1).  Wave w:
// h row block 2kh + w%2 over column blocks 2(w/2), 2(w/2)+1 and the dx row block
// 4 + kh over column block w -- 3 MFMAs per k step, so the A stream runs
// kBwPD2-1 = 7 k steps ahead.  K order: own chunks, then the partner's (the
// packed stream read from k step 144kh on, wrapping through the repeated tail).
// Launched as one residency wave (launch_resident); the spins are bounded and reported.
template <int ABL = 0>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) k_convlstm_bwd_pairs(RecBwdParams p) {
  __shared__ __attribute__((aligned(16))) unsigned char zim[2 * kBwIBP];   // chunk images (c & 1)
  __shared__ __attribute__((aligned(16))) f32x4 dcl[4 * 8 * 64];          // dc carry, lane-native [wave][g*2+j][lane]
  const int b = (int)blockIdx.x % p.B, kh = (int)blockIdx.x / p.B;
  const int tid = (int)threadIdx.x, lane = tid & 63;
  uint64_t wdl = 0;   // partner-wait deadline (common.h wait_expired), set by the first wait that polls
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r32 = lane & 31, hh = lane >> 5;
  const int P = p.P, W2 = p.w + 2;
  const size_t M = (size_t)p.B * P;
  const int hrb = 2 * kh + (wave & 1);   // the wave's h row block (channels 32 hrb ..) = the dZ chunk it produces
  const int cbA = 2 * (wave >> 1);       // its column blocks cbA, cbA + 1
  auto hidx = [&](int pp) { return (pp / p.w + 1) * W2 + pp % p.w + 1; };
  // row-padded images as in k_convlstm_bwd_frames (kBwIBP; the host checked bw_rowpad)
  const int rp = p.rowpad;
  auto pixb = [&](int ip) { return 272 * ip + 16 * rp * (ip / W2); };   // image pixel -> byte

  {  // zero the images (borders and pads stay zero)
    u32x4* z = reinterpret_cast<u32x4*>(zim);
    for (int i = tid; i < 2 * kBwIBP / 16; i += 256) z[i] = u32x4{0u, 0u, 0u, 0u};
  }
  // the partner's chunk c of dZ_t: sc1 loads of the P x 256 B into registers
  // (issued at the start of a chunk), then into image c & 1 (three taps later)
  constexpr int NPR = 8;   // 16-B pieces per thread: P * 16 <= 2048
  auto pld = [&](int t, int c, u32x4 (&v)[NPR]) {
    const __amdgpu_buffer_rsrc_t rs =
        make_rsrc(p.dZ + ((size_t)t * M + (size_t)b * P) * 512, (uint32_t)(P * 512 * 2));
#pragma unroll
    for (int r = 0; r < NPR; ++r) {
      const int i = tid + 256 * r, px = i >> 4, q = i & 15;
      v[r] = __builtin_amdgcn_raw_buffer_load_b128(rs, px < P ? (uint32_t)((px * 512 + 128 * c + q * 8) * 2) : kOOB, 0,
                                                   kSC1);
    }
  };
  auto pst = [&](int c, const u32x4 (&v)[NPR]) {
#pragma unroll
    for (int r = 0; r < NPR; ++r) {
      const int i = tid + 256 * r, px = i >> 4, q = i & 15;
      if (px < P) *reinterpret_cast<u32x4*>(zim + (c & 1) * kBwIBP + pixb(hidx(px)) + q * 16) = v[r];
    }
  };

  int hb[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int pp = min((cbA + j) * 32 + r32, P - 1);
    hb[j] = (pp / p.w) * W2 + pp % p.w;
  }
  // dc carry of the lane's 32 (channel, pixel) pairs: channels 32hrb + 8g + 4hh + e at pixel 32(cbA+j) + r32
  f32x4* dcw = dcl + wave * 8 * 64 + lane;   // + (g*2 + j) * 64
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int pp = (cbA + j) * 32 + r32;
      dcw[(g * 2 + j) * 64] =
          pp < P ? *reinterpret_cast<const f32x4*>(p.dC + ((size_t)b * P + pp) * 128 + 32 * hrb + 8 * g + 4 * hh)
                 : f32x4{0.f, 0.f, 0.f, 0.f};
    }

  const __amdgpu_buffer_rsrc_t rsw = make_rsrc(p.Wb, (uint32_t)(6 * kBwKSP * 1024));
  const int wofs = hrb * kBwKSP * 1024, xofs = (4 + kh) * kBwKSP * 1024;
  auto lda = [&](int ks, int x) {
    return __builtin_bit_cast(bf16x8,
                              __builtin_amdgcn_raw_buffer_load_b128(rsw, lane * 16, (x ? xofs : wofs) + ks * 1024, 0));
  };
  constexpr int PD = kBwPD2;
  bf16x8 af[PD][2];
#pragma unroll
  for (int s = 0; s < PD - 1; ++s) {
    af[s][0] = lda(144 * kh + s, 0);
    af[s][1] = lda(144 * kh + s, 1);
  }
  float xbs[16];   // conv2 bias partials of the lane's 16 x channels, all steps
#pragma unroll
  for (int i = 0; i < 16; ++i) xbs[i] = 0.f;

  struct EpIn { f32x4 dO, cp; u32x4 gt[2]; };
  constexpr int kRing = 4, kU = 8;   // units u = (g, j), g-major
  auto load_in = [&](int s, int u, int ln) {   // channel-quad-major slices (recur.h cqm4 / cqmg)
    // buffer loads with out-of-range offsets past P (zeros), no branch: k_convlstm_bwd_frames' load_in
    EpIn in;
    const int g = u >> 1, j = u & 1, pp = (cbA + j) * 32 + (ln & 31);
    const bool v = pp < P;
    const size_t fr = (size_t)s * M + (size_t)b * P;
    const int ch = 32 * hrb + 4 * (ln >> 5) + 8 * g;
    const __amdgpu_buffer_rsrc_t ro = make_rsrc(p.dO + fr * 128, (uint32_t)(P * 128 * 4));
    const __amdgpu_buffer_rsrc_t rc = make_rsrc(p.Cst + fr * 128, (uint32_t)(P * 128 * 4));
    const __amdgpu_buffer_rsrc_t rg = make_rsrc(p.Gt + fr * 512, (uint32_t)(P * 512 * 2));
    in.dO = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                          ro, v ? (uint32_t)(slc4(pp, ch, P, p.cqm & kCqmDO) * 4) : kOOB, 0, 0));
    in.cp = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                          rc, v ? (uint32_t)(slc4(pp, ch, P, p.cqm & kCqmC) * 4) : kOOB, 0, 0));
    const uint32_t go = v ? (uint32_t)(slcg(pp, ch, P, p.cqm & kCqmG) * 2) : kOOB;
    in.gt[0] = __builtin_amdgcn_raw_buffer_load_b128(rg, go, 0, 0);
    in.gt[1] = __builtin_amdgcn_raw_buffer_load_b128(rg, go, 16, 0);
    return in;
  };

  // gate backward of step s (as the single-workgroup kernel's), then publish
  // dZ_s: every wave's sc1 stores retired, a barrier, one lane's sc1 flag store
  auto epilogue = [&](int s, const f32x16 (&acc)[2], bool gemm, EpIn (&ring)[kRing]) {
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const int pl = ln & 31, hq = ln >> 5;
    const int c0 = 32 * hrb + 4 * hq;   // + 8g + e
    const size_t rows = (size_t)s * M + (size_t)b * P;
    const __amdgpu_buffer_rsrc_t rz = make_rsrc(p.dZ + rows * 512, (uint32_t)(P * 512 * 2));
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      float bs[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) bs[i] = 0.f;
      const int ch = c0 + 8 * g;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int u = g * 2 + j;
        if (u + kRing - 1 < kU) ring[(u + kRing - 1) % kRing] = load_in(s, u + kRing - 1, ln);
        const EpIn& in = ring[u % kRing];
        const int pp = (cbA + j) * 32 + pl;
        if (pp < P) {
          f32x4 dh = in.dO;
          if (gemm) {
            dh[0] += acc[j][4 * g]; dh[1] += acc[j][4 * g + 1]; dh[2] += acc[j][4 * g + 2]; dh[3] += acc[j][4 * g + 3];
          } else if (p.dhT) {
            const f32x4 x = *reinterpret_cast<const f32x4*>(p.dhT + ((size_t)b * P + pp) * 128 + ch);
            dh[0] += x[0]; dh[1] += x[1]; dh[2] += x[2]; dh[3] += x[3];
          }
          f32x4* dcp = dcl + wave * 8 * 64 + ln + u * 64;
          f32x4 dc = *dcp;
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
          *dcp = dc;
          bf16x8 z0, z1;
#pragma unroll
          for (int i = 0; i < 8; ++i) { z0[i] = (__bf16)dz[i]; z1[i] = (__bf16)dz[8 + i]; }
          const uint32_t zo = (uint32_t)((pp * 512 + 4 * ch) * 2);
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, z0), rz, zo, 0, kSC1);
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, z1), rz, zo + 16, 0, kSC1);
          unsigned char* zi = zim + (wave & 1) * kBwIBP + pixb(hidx(pp)) + (4 * (ch - 32 * hrb)) * 2;
          *reinterpret_cast<bf16x8*>(zi) = z0;
          *reinterpret_cast<bf16x8*>(zi + 16) = z1;
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      int n = 16;
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
      if ((pl & 1) == 0)   // row 4(ch + e) + gate; the two pixel halves (w / 2) in rows of their own
        p.part[(((size_t)s * p.B + b) * 2 + (wave >> 1)) * 512 + 4 * (ch + (ridx >> 2)) + (ridx & 3)] = bs[0];
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    barrier_lds();   // own chunk images of dZ_s complete; every wave's dZ_s stores retired
    if (tid == 0) __hip_atomic_store(p.flags + 2 * b + kh, p.T - s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };

  if ((b >> 3) & 1) stagger_wait(p.stagger);
  {  // step T-1: no GEMM
    f32x16 zero[2];
    EpIn ring[kRing];
#pragma unroll
    for (int u = 0; u < kRing - 1; ++u) ring[u] = load_in(p.T - 1, u, lane);
    epilogue(p.T - 1, zero, false, ring);
  }

  for (int t = p.T - 1; t >= 0; --t) {
    f32x16 acc[2], accx;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[j][e] = 0.f;
#pragma unroll
    for (int e = 0; e < 16; ++e) accx[e] = 0.f;
    int hbs[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      hbs[j] = pixb(hb[j]);   // the window's top-left pixel as a byte offset
      asm volatile("" : "+v"(hbs[j]));
    }
    // a tap's byte offset (window columns never cross an image row: the row pad is per tap row)
    auto tapoff = [&](int tap) { return ((2 - tap / 3) * W2 + (2 - tap % 3)) * 272 + 16 * rp * (2 - tap / 3); };
    auto ldb = [&](const unsigned char* img, int toff, int c16, bf16x8 (&bf)[2]) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
        bf[j] = *reinterpret_cast<const bf16x8*>(img + hbs[j] + toff + c16 * 32 + hh * 16);
    };
    constexpr int BD = 4;
    bf16x8 bfr[BD][2];
    EpIn ring[kRing];
    auto kloop = [&](auto xj) {
      constexpr int XJ = decltype(xj)::value;   // the dx column block's fragment (w % 2)
#pragma unroll 1
      for (int ck = 0; ck < 4; ++ck) {
        const int c = (ck + 2 * kh) & 3;   // own chunks first, then the partner's
        const unsigned char* img = zim + (c & 1) * kBwIBP;
        u32x4 pv[NPR];
        const bool refill = ck == 1 || ck == 2;   // the partner's chunk c+1 into the image chunk ck-1 freed
        if (refill) pld(t, (c + 1) & 3, pv);
        if (ck == 3 && t > 0) {
          int ln = lane;
          asm volatile("" : "+v"(ln));
#pragma unroll
          for (int u = 0; u < kRing - 1; ++u) ring[u] = load_in(t - 1, u, ln);
        }
#pragma unroll
        for (int j = 0; j < BD - 1; ++j) ldb(img, tapoff(0), j, bfr[j]);
        for (int tap = 0; tap < 9; ++tap) {
          const int toff = tapoff(tap), tn = tap < 8 ? tapoff(tap + 1) : 0;
          int kt = c * 72 + tap * 8;
          asm volatile("" : "+s"(kt));
          if (refill && tap == 3) pst((c + 1) & 3, pv);
#pragma unroll
          for (int c16 = 0; c16 < 8; ++c16) {
            if constexpr (!(ABL & 1)) {
              af[(c16 + PD - 1) % PD][0] = lda(kt + c16 + PD - 1, 0);
              af[(c16 + PD - 1) % PD][1] = lda(kt + c16 + PD - 1, 1);
            }
            {
              const int cn = c16 + BD - 1;
              if (cn < 8) ldb(img, toff, cn, bfr[cn % BD]);
              else if (tap < 8) ldb(img, tn, cn - 8, bfr[cn % BD]);
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int j = 0; j < 2; ++j)
              acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[c16 % PD][0], bfr[c16 % BD][j], acc[j], 0, 0, 0);
            accx = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[c16 % PD][1], bfr[c16 % BD][XJ], accx, 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
          }
        }
        if (ck == 0 && tid == 0) {   // the partner's dZ_t published? (the other waves load after the barrier)
          pair_wait(p.flags + 2 * b + (1 - kh), p.T - t, p.report, p.spin, wdl);
        }
        barrier_lds();   // image c & 1 free for the partner's chunk; (ck = 1, 2) its refill complete
      }
    };
    if (wave & 1) kloop(std::integral_constant<int, 1>{});
    else kloop(std::integral_constant<int, 0>{});
    {  // dx_t: x channels 32kh + 8g + 4hh + e at pixel 32w + r32
      const size_t rows = (size_t)t * M + (size_t)b * P;
      const int pp = wave * 32 + r32;
      if (pp < P) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const float v[4] = {accx[4 * g], accx[4 * g + 1], accx[4 * g + 2], accx[4 * g + 3]};
          *reinterpret_cast<bf16x4*>(p.dY2 + (rows + pp) * 64 + 32 * kh + 8 * g + 4 * hh) =
              bf16x4{(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
#pragma unroll
          for (int e = 0; e < 4; ++e) xbs[4 * g + e] += v[e];
        }
      }
    }
    if (t > 0) {
      epilogue(t - 1, acc, true, ring);
    } else if (p.dh0) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int pp = (cbA + j) * 32 + r32;
        if (pp < P)
#pragma unroll
          for (int g = 0; g < 4; ++g)
            *reinterpret_cast<f32x4*>(p.dh0 + ((size_t)b * P + pp) * 128 + 32 * hrb + 8 * g + 4 * hh) =
                f32x4{acc[j][4 * g], acc[j][4 * g + 1], acc[j][4 * g + 2], acc[j][4 * g + 3]};
      }
    }
  }
  {  // conv2 bias partials (4 waves = 4 column blocks share each channel set)
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
      atomicAdd(p.dxb + (size_t)b * 64 + 32 * kh + 8 * g + 4 * hh + e, v[0]);
    }
  }
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int pp = (cbA + j) * 32 + r32;
      if (pp < P)
        *reinterpret_cast<f32x4*>(p.dC + ((size_t)b * P + pp) * 128 + 32 * hrb + 8 * g + 4 * hh) = dcw[(g * 2 + j) * 64];
    }
}

inline hipError_t convlstm_bwd_pairs(const RecBwdParams& p, hipStream_t st) {
  if (!rec_fits(p.h, p.w) || p.P != p.h * p.w || p.B < 1 || p.T < 1 || !p.flags || !p.report || p.spin < 0 ||
      (p.rowpad && p.rowpad != bw_rowpad(p.h, p.w)))
    return hipErrorInvalidValue;
  RecBwdParams q = p;
  return launch_resident(reinterpret_cast<const void*>(&k_convlstm_bwd_pairs<0>), 2 * p.B, 256, q, st);
}

inline hipError_t convlstm_bwd_frames(const RecBwdParams& p, hipStream_t st) {
  if (!rec_fits(p.h, p.w) || p.P != p.h * p.w || p.B < 1 || p.T < 1 || (p.rowpad && p.rowpad != bw_rowpad(p.h, p.w)))
    return hipErrorInvalidValue;
#ifdef AAA_ABLATION   // diagnostic builds only (tools/ubench): the product library never reads AAA_RECB_ABL
  const char* e = getenv("AAA_RECB_ABL");
  switch (e ? atoi(e) : 0) {
#define AAA_RECB_CASE(a) \
  case a: hipLaunchKernelGGL((k_convlstm_bwd_frames<a>), dim3(p.B), dim3(256), 0, st, p); return hipGetLastError();
    AAA_RECB_CASE(1) AAA_RECB_CASE(2) AAA_RECB_CASE(3) AAA_RECB_CASE(4) AAA_RECB_CASE(8) AAA_RECB_CASE(6)
    AAA_RECB_CASE(32) AAA_RECB_CASE(64) AAA_RECB_CASE(128) AAA_RECB_CASE(256) AAA_RECB_CASE(512)
#undef AAA_RECB_CASE
    default: break;
  }
#endif
#ifdef AAA_ABLATION   // the LDS-DMA epilogue ring (RING): measured slower, profiles/r06/ab/bw_ring/
  if (p.ring) {
    hipLaunchKernelGGL((k_convlstm_bwd_frames<0, false, true, true>), dim3(p.B), dim3(256), 0, st, p);
    return hipGetLastError();
  }
#endif
  hipLaunchKernelGGL((k_convlstm_bwd_frames<0>), dim3(p.B), dim3(256), 0, st, p);
  return hipGetLastError();
}

// Band mode (recur.h rec_band_fits; the image holds <= kRecNPHB = 184 pixels, kBwIBS
// bytes): kRecBands workgroups per frame in one residency wave (launch_resident;
// p.flags [B][kRecBands] zeroed by the caller, p.part rows per (step, frame, band)).
inline bool bw_band_fits(int h, int w) { return rec_band_fits(h, w) && kRecNPHB * 256 <= kBwIBS; }
inline hipError_t convlstm_bwd_band(const RecBwdParams& p, hipStream_t st) {
  if (!bw_band_fits(p.h, p.w) || p.P != p.h * p.w || p.B < 1 || p.T < 1 || !p.flags || !p.report || p.spin < 0)
    return hipErrorInvalidValue;
  RecBwdParams q = p;
  const void* k = reinterpret_cast<const void*>(&k_convlstm_bwd_frames<0, true>);
#ifdef AAA_ABLATION   // diagnostic builds only
  const char* e = getenv("AAA_RECB_ABL");
  switch (e ? atoi(e) : 0) {
#define AAA_RECB_BCASE(a) \
  case a: k = reinterpret_cast<const void*>(&k_convlstm_bwd_frames<a, true>); break;
    AAA_RECB_BCASE(1) AAA_RECB_BCASE(2) AAA_RECB_BCASE(4) AAA_RECB_BCASE(8) AAA_RECB_BCASE(16) AAA_RECB_BCASE(6)
    AAA_RECB_BCASE(18) AAA_RECB_BCASE(32) AAA_RECB_BCASE(64)
#undef AAA_RECB_BCASE
    default: break;
  }
#endif
  return launch_resident(k, 8 * kRecBands * ((p.B + 7) / 8), 256, q, st);
}

}  // namespace aaa
