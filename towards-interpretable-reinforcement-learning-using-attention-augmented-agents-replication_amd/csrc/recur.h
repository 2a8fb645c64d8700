// Frame-resident ConvLSTM recurrence (bf16 operands, fp32 accumulate).
//
// The recurrence of one frame depends only on that frame (attention.py:110-126:
// the gate convs are 3x3 over the frame's own grid, no batch coupling), so one
// workgroup owns a frame for ALL T steps of the unroll: the zero-bordered
// images of x_t and h_{t-1} live in LDS, the cell state c in LDS, and a step is
// one 512 x P x 1728 GEMM whose B operand (the im2col of [x_t | h_{t-1}]) is
// read straight out of the LDS images by all nine taps -- no per-step launch,
// no prologue, no re-gathering of the pixel operand from L2, and the epilogue's
// HBM stores of step t drain under the MFMAs of step t+1.
//
// Geometry: 4 waves, one per SIMD (512 registers each); wave w owns gate rows
// [128w, 128w+128) (row = 4*channel + gate: channels 32w..32w+31) for all
// P <= 128 pixel columns, acc 4x4 v_mfma_f32_32x32x16_bf16 tiles (row block
// rb, column block cb).  Lane (r32, hh) of tile (rb, cb) holds rows 8g + 4hh + e:
// the four gates of channel 32w + 8rb + 2g + hh at pixel 32cb + r32 -- the whole
// cell update is lane-local.
//
// A operand (weights): fragment-order copy of the packed [512][1728] matrix
// (k_pack_wfrag), one contiguous 1 KB wave load per (row block, k step) from a
// buffer descriptor, kRecPD-1 k steps in flight, streamed from L2 continuously
// across steps (the packed copy repeats its first k steps at the end).  K runs
// x-part first (9 taps x 64 channels), then the h-part (9 taps x 128 channels),
// so the single x image can be refilled (LDS-DMA) while the h-part runs.
#pragma once
#include <cstdlib>
#include "common.h"
#include "epilogues.h"
#include "glds.h"

namespace aaa {

constexpr int kRecKS = 1728 / 16;   // k steps of one [x|h] step GEMM: 36 x-part, then 72 h-part
constexpr int kRecKX = 36;
constexpr int kRecPD = 4;           // A k steps in flight + 1 (register slots); divides 4 and 8
constexpr int kRecKSP = kRecKS + kRecPD - 1;   // packed k steps per row block: the first PD-1 repeated at
                                               // the end, so the prefetch runs into the next step unwrapped
constexpr int kRecNPH = 169;        // whole-frame LDS images: (h+2)*(w+2) <= 169 (11x11 grids: 84x84 frames)
constexpr int kRecNPHB = 184;       // image buffer pixels: also one band of <= 6 rows of a 21-wide grid + its halo rows
constexpr int kRecXB = 23 * 1024;   // x image bytes: 184 pixels x 128 B (whole 1-KB DMA pieces)
constexpr int kRecBands = 4;        // grid bands per frame in band mode (168x168 frames: 21 rows -> 5,5,5,6)
constexpr int kRecHS = 136;         // h image pixel pitch (bf16): 128 + 8 pad (272 B = 17 x 16 B)
constexpr int kRecStg = 4608;       // per-wave epilogue staging bytes (16 px x 272 B gates; c + h 2 x 16 x 144 B)
constexpr int kSC1 = 16;            // buffer load / store cache policy: sc1 (cross-workgroup hand-off bytes)

// Channel-quad-major layout ("CQM") of the per-(frame, step) slices the
// frame-resident forward writes and the frame-resident BPTT reads (the cell
// state Cst, the gate activations Gt, the attention-path grad dO): inside a
// frame's P x 128 slice, channel quad q = ch / 4 of pixel pp sits at
// (q * P + pp) * 4 floats (Cst, dO) or (q * P + pp) * 16 fp16 (Gt: 4 channels
// x 4 gates).  The BPTT epilogue's lanes hold 4 consecutive channels at 32
// consecutive pixels, so each of its loads reads two contiguous 512-B runs
// (c, dO) or 1-KB runs (gates) instead of 16 B of every 512-B pixel row, which
// left the rest of each line to later loads (PMC: 2.4x the algorithmic bytes;
// tools/ubench/bwband "coalesced epilogue loads" -14 % per launch).  Slices
// keep their row-major positions and sizes; only their inside is permuted.
__host__ __device__ __forceinline__ int cqm4(int pp, int ch, int P) { return ((ch >> 2) * P + pp) * 4 + (ch & 3); }
__host__ __device__ __forceinline__ int cqmg(int pp, int ch, int P) { return ((ch >> 2) * P + pp) * 16 + (ch & 3) * 4; }
// Which slices are channel-quad-major (cqm_layout's mask; the others row-major):
constexpr int kCqmC = 1, kCqmG = 2, kCqmDO = 4;
// offset of channel ch of pixel pp in a 128-channel fp32 slice / in a gate slice (4 gates per channel)
__host__ __device__ __forceinline__ int slc4(int pp, int ch, int P, bool q) { return q ? cqm4(pp, ch, P) : pp * 128 + ch; }
__host__ __device__ __forceinline__ int slcg(int pp, int ch, int P, bool q) { return q ? cqmg(pp, ch, P) : pp * 512 + ch * 4; }

// k step ks of the x-first order -> element offset k of the [x|h] GEMM (k = tap*192 + c)
__host__ __device__ constexpr int rec_k(int ks) {
  return ks < kRecKX ? (ks >> 2) * 192 + (ks & 3) * 16 : ((ks - kRecKX) >> 3) * 192 + 64 + ((ks - kRecKX) & 7) * 16;
}

// Wf[((rb*kRecKSP + ks)*64 + lane)*8 + e] = W[rb*32 + lane%32][rec_k(ks % kRecKS) + (lane/32)*8 + e]
static __global__ void __launch_bounds__(256) k_pack_wfrag(const __bf16* __restrict__ W, __bf16* __restrict__ Wf) {
  const int c = blockIdx.x * 256 + (int)threadIdx.x;   // one 16-B chunk
  if (c >= 16 * kRecKSP * 64) return;
  const int lane = c & 63, rk = c >> 6, ks = rk % kRecKSP, rb = rk / kRecKSP;
  const int row = rb * 32 + (lane & 31), k = rec_k(ks % kRecKS) + (lane >> 5) * 8;
  *reinterpret_cast<bf16x8*>(Wf + (size_t)c * 8) = *reinterpret_cast<const bf16x8*>(W + (size_t)row * 1728 + k);
}

// Branch-free gate math for the bf16 path (operands already rounded to 8
// mantissa bits): sigma(x) = 1 / (1 + 2^(-x log2 e)) on v_exp_f32 / v_rcp_f32,
// tanh(x) = 2 sigma(2x) - 1 (absolute error ~1e-7).
__device__ __forceinline__ float sigm_fast(float x) {
  return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-1.4426950408889634f * x));
}
__device__ __forceinline__ float tanh_fast(float x) { return 2.0f * sigm_fast(2.0f * x) - 1.0f; }

inline hipError_t pack_wfrag(const __bf16* W, __bf16* Wf, hipStream_t st) {
  hipLaunchKernelGGL(k_pack_wfrag, dim3((16 * kRecKSP * 64 + 255) / 256), dim3(256), 0, st, W, Wf);
  return hipGetLastError();
}

// Whether a grid runs on the frame-resident kernels.
inline bool rec_fits(int h, int w) { return h * w <= 128 && (h + 2) * (w + 2) <= kRecNPH; }
// Row-padded h image of the single-workgroup and paired forward (round 6; the BPTT's
// bw_rowpad layout, recur_bwd.h): image pixel ip at byte 272 ip + 16 rowpad (ip / W2).  With
// rowpad = 14 the 16-B slot of (pixel, chunk j) is (ip - 2 (ip / W2) + j) mod 16, so a B-fragment
// read of 16 consecutive GEMM columns covers 16 consecutive slots across grid-row ends (272-B
// rows alone skip two slots at every row end: SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE 0.49 at
// C3); a tap still moves every lane's address by one wave-uniform amount.  0 if the padded image
// does not fit the h-image buffer.
inline int rec_rowpad(int h, int w) { return (h + 2) * (17 * (w + 2) + 14) * 16 <= kRecNPHB * kRecHS * 2 ? 14 : 0; }
// Band mode: the grid split into kRecBands bands of whole rows, each band's
// pixels (<= 128 columns) plus one halo row above and below in the LDS images.
inline int rec_band_rows(int h, int k) { return (k + 1) * h / kRecBands - k * h / kRecBands; }
inline bool rec_band_fits(int h, int w) {
  const int rmax = (h + kRecBands - 1) / kRecBands;
  return h >= kRecBands && rmax * w <= 128 && (rmax + 2) * (w + 2) <= kRecNPHB;
}

template <typename GT>
struct RecFwdParams {
  const __bf16* Wf;    // fragment-order [x|h] weights
  const float* bias;   // [512] gate-interleaved x-conv biases
  __bf16* XH;          // (T+1, B, P, 192): slot t = [x_t | h_{t-1}]; writes h_t into slot t+1
  float* Cst;          // (T+1, B, P, 128): slot 0 = c_0 (read), slot t+1 <- c_t
  float* Hs;           // (T, B, P, 128) <- h_t (fp32), or null (the readout reads h_t from XH)
  GT* Gt;              // (T, B, P, 512) <- gate activations (i, f, c~, o)
  int* flags;          // G = 2: per (frame, half) count of published h steps ([2B], zeroed); band mode: [B][bands]
  int T, B, h, w, P;
  int* report;         // G = 2: partner-timeout report word (pinned host, device-mapped; pair_wait)
  int spin;            // G = 2 / band: partner-wait budget, 100-MHz ticks (pair_wait)
  int stagger;         // start offset (100-MHz ticks) of the frames with (b / 8) odd (stagger_wait)
  int cqm;             // kCqmC / kCqmG: Cst / Gt slices channel-quad-major (cqm4 / cqmg) instead of row-major
  int rowpad;          // G = 1 / 2 (not band): 16-B slots after each h-image row (0 or 14: rec_rowpad)
  // GEMM column c -> pixel (colpp, -1 = padding column) and the top-left image
  // index of its 3x3 window (colhb); filled by convlstm_fwd_frames (rec_columns)
  short colpp[128], colhb[128];
};

// Column order of the frame-resident GEMMs.  A B-fragment ds_read_b128 serves
// 16 lanes (16 consecutive columns) per 256-B LDS row, and both images put
// image pixel ip at 16-B slot ip (mod 16) (+ a per-read constant), so a lane
// group is conflict-free iff its 16 pixels' image indices differ mod 16.  In
// raster order every 16-column group of an 11-wide grid crosses a row end,
// where the index jumps by 3 (the border): two slots collide, the read takes
// two passes (SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE = 0.50 at C3).  Here
// the columns are the pixels bucketed by image index mod 16 and dealt out one
// per residue to each 16-column group (padding columns read a spare interior
// index of the missing residue).  Measured (profiles/r02/ab/rec_perm.txt): the
// conflict cycles drop 61 % but the forward gets slower (C3 1136 -> 1177 us,
// C4 618 -> 652 us): the epilogue's pixel rows of a 16-column half are then
// scattered over the frame instead of one contiguous run, and the kernel is
// not bound by these reads.  So the raster order is the default and the
// dealt order an A/B option (AAA_REC_PERM=1; also kept when a residue holds
// more than 8 pixels).
inline void rec_columns(int h, int w, short* colpp, short* colhb) {
  const int W2 = w + 2, P = h * w, NPH = (h + 2) * W2;
  auto raster = [&] {
    for (int c = 0; c < 128; ++c) {
      const int pp = c < P ? c : P - 1;
      colpp[c] = (short)(c < P ? c : -1);
      colhb[c] = (short)((pp / w) * W2 + pp % w);
    }
  };
  raster();
#ifndef AAA_ABLATION
  (void)NPH;
  return;
#else
  const char* e = getenv("AAA_REC_PERM");
  if (!(e && atoi(e) == 1) || P > 128) return;
  int bucket[16][9], nb[16] = {0};
  for (int pp = 0; pp < P; ++pp) {
    const int r = ((pp / w + 1) * W2 + pp % w + 1) & 15;
    if (nb[r] == 8) return;   // a residue with more pixels than groups: keep the raster order
    bucket[r][nb[r]++] = pp;
  }
  int spare[16];
  for (int r = 0; r < 16; ++r) {   // a padding column's window must stay inside the image for all 9 taps
    spare[r] = -1;
    for (int ip = W2 + 1; ip <= NPH - W2 - 2 && spare[r] < 0; ++ip)
      if ((ip & 15) == r) spare[r] = ip;
    if (spare[r] < 0 && nb[r] < 8) return;
  }
  int used[16] = {0};
  for (int g = 0; g < 8; ++g)
    for (int r = 0; r < 16; ++r) {
      const int c = 16 * g + r;
      if (used[r] < nb[r]) {
        const int pp = bucket[r][used[r]++];
        colpp[c] = (short)pp;
        colhb[c] = (short)((pp / w) * W2 + pp % w);
      } else {
        colpp[c] = -1;
        colhb[c] = (short)(spare[r] - W2 - 1);
      }
    }
#endif
}

#ifdef AAA_STAMPS
// Diagnostic builds only (tools/ubench/bwband): per (workgroup, step) phase stamps
// (s_memrealtime, 100 MHz): step start, x-part done, neighbour h in, h-part done,
// epilogue done, h_t stored / published.
__device__ uint64_t aaa_fw_stamps[1024 * 64 * 8];
#define AAA_FW_STAMP(t, k)                                                                                    \
  do {                                                                                                        \
    if (tid == 0 && (t) < 64) aaa_fw_stamps[((size_t)blockIdx.x * 64 + (t)) * 8 + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define AAA_FW_STAMP(t, k) do {} while (0)
#endif

// ABL (diagnostic A/B only: AAA_REC_ABL, honoured only in a -DAAA_ABLATION build): bit 0 = no A loads in the K loop,
// bit 1 = no epilogue HBM stores, bit 2 = no MFMAs, bit 3 = no B fragment reads, bit 6 = the in-loop x-image
// LDS-DMA compiler-visible (the pre-round-6 form).
//
// G = 2 (batches too small to give every CU a frame): two workgroups per frame,
// half kh owning gate rows [256kh, 256kh+256) (its 64 channels); each step it
// publishes its half of h_t through XH slot t+1 (written anyway: the weight-
// gradient operand) with sc1 stores and an sc1 flag, and reads the partner's half
// (sc1 loads) into its h image after its own x-part -- the hand-off's latency
// hides under the x-part GEMM, and no agent release / acquire fence is paid
// (ABL bit 4 = the fenced hand-off, for A/B).  Launched as one residency wave
// (launch_resident, co-residency checked), spins bounded and reported.
//
// BAND (G = 1): 168x168 frames (21x21 grid) do not fit one workgroup's LDS,
// so kRecBands workgroups split a frame by whole grid rows (5-6 rows = <= 126
// pixel columns each) and all 512 gate rows.  A band's images hold its rows
// plus one halo row above and below; per step each band publishes its h_t rows
// (XH slot t+1, written anyway) with sc1 stores and a flag, and after its own
// x-part reads the neighbours' boundary rows into its halo rows (sc1 loads),
// like the G = 2 hand-off.  The bands of a frame get block indices of equal
// residue mod 8 (one XCD under round-robin placement).
template <typename GT, int G = 1, int ABL = 0, bool BAND = false>
__global__ void __launch_bounds__(256) k_convlstm_fwd_frames(RecFwdParams<GT> p) {
  static_assert(!BAND || G == 1, "band mode splits pixels, not channels");
  constexpr int NRB = 4 / G, GCH = 8 * NRB;     // row blocks and channels per wave
  constexpr int GTP = GCH * 8 + 16, CHP = GCH * 4 + 16;   // staging pixel pitches (gates fp16x4, c / h fp32)
  __shared__ __attribute__((aligned(16))) unsigned char xim[kRecXB];
  __shared__ __attribute__((aligned(16))) __bf16 him[kRecNPHB * kRecHS];
  __shared__ __attribute__((aligned(16))) float cstl[4 * NRB * 16 * 64];   // c, lane-native: [wave][rb][cb][g][lane]
  __shared__ __attribute__((aligned(16))) float sbias[512];
  __shared__ __attribute__((aligned(16))) unsigned char stg[4 * 16 * (GTP > 2 * CHP ? GTP : 2 * CHP)];
  __shared__ short scol[128];   // column -> pixel (LDS: the epilogue's lookups stay off the vmcnt queue of the A stream)
  constexpr int STG = 16 * (GTP > 2 * CHP ? GTP : 2 * CHP);
  int b = (int)blockIdx.x % p.B;
  const int kh = G == 1 ? 0 : (int)blockIdx.x / p.B;
  int band = 0, r0 = 0, r1 = p.h;   // band mode: this workgroup's grid rows [r0, r1)
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
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform (SGPR) for the buffer soffsets
  const int r32 = lane & 31, hh = lane >> 5;
  const int P = p.P, W2 = p.w + 2, NPH = (r1 - r0 + 2) * W2;
  const int Pb = (r1 - r0) * p.w, pix0 = r0 * p.w;   // the band's pixels (the whole frame without BAND)
  const size_t M = (size_t)p.B * P;
  auto hidx = [&](int pp) { return (pp / p.w - r0 + 1) * W2 + pp % p.w + 1; };   // interior pixel -> image index
  const int rp = BAND ? 0 : p.rowpad;
  auto pixb = [&](int ip) { return 272 * ip + 16 * rp * (ip / W2); };   // h image pixel -> byte (rec_rowpad)
  unsigned char* const himb = reinterpret_cast<unsigned char*>(him);
  const int rb0 = kh * (16 / G) + wave * NRB;   // the wave's first global row block (32 rows = 8 channels)
  const int cbase = 8 * rb0;                     // its first channel
  float* cw = cstl + wave * NRB * 16 * 64 + lane;   // + (rb*16 + cb*4 + g) * 64

  {  // zero the h image (its border stays zero), bias into LDS
    u32x4* z = reinterpret_cast<u32x4*>(him);
    for (int i = tid; i < kRecNPHB * kRecHS / 8; i += 256) z[i] = u32x4{0u, 0u, 0u, 0u};
    sbias[tid] = p.bias[tid];
    sbias[tid + 256] = p.bias[tid + 256];
    if (tid < 128) scol[tid] = BAND ? (short)(tid < Pb ? pix0 + tid : -1) : p.colpp[tid];
  }
  // x image of step t (XH slot t, channels 0..63) by LDS-DMA, border included:
  // image pixel ip holds its 8 16-B channel chunks at slots q ^ xswz(ip) (the
  // fragment reads of 16 consecutive pixels then hit 16 distinct bank groups);
  // border pixels read outside the descriptor and land as zeros.  Wave w issues
  // the 1-KB pieces w, w+4, ... of the 22 (8 pixels each).
  // In the step loop (asm = true) the pieces are issued from inline asm (dma16a): a compiler-visible
  // LDS-DMA in flight makes the compiler wait vmcnt(0) before every LDS read that might alias it -- the
  // epilogue's staging, c and bias reads, each then also waiting for the gate / c / h stores issued just
  // before it (~40 drains per step).  Nothing reads the x image before the h-part's A-stream waits, which
  // retire these older pieces (vmcnt retires in issue order) ahead of the barrier that ends the step.
  auto dma_x = [&](int t, bool asm_issue) {
    const __amdgpu_buffer_rsrc_t rs =
        make_rsrc_u(p.XH + ((size_t)t * M + (size_t)b * P) * 192, (uint32_t)(P * 192 * 2));
    int ln = lane;   // laundered: the pieces' offsets are recomputed per step (hoisted, they spill)
    asm volatile("" : "+v"(ln));
    for (int i = wave; i < kRecXB / 1024; i += 4) {
      const int sl = i * 64 + ln, ip = sl >> 3, q = (sl & 7) ^ ((ip >> 1) & 7);
      const int py = r0 + ip / W2 - 1, px = ip % W2 - 1;
      const bool v = ip < NPH && (unsigned)py < (unsigned)p.h && (unsigned)px < (unsigned)p.w;
      const uint32_t vo = v ? (uint32_t)(((py * p.w + px) * 192 + q * 8) * 2) : kOOB;
      if (asm_issue) dma16a(rs, xim + i * 1024, vo);
      else dma16(rs, xim + i * 1024, vo);
    }
  };
  dma_x(0, false);
  // cell state c_0 (Cst slot 0) into the lane-native LDS copy
#pragma unroll
  for (int rb = 0; rb < NRB; ++rb)
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int pp = BAND ? (cb * 32 + r32 < Pb ? pix0 + cb * 32 + r32 : -1) : p.colpp[cb * 32 + r32];
        const int ch = cbase + 8 * rb + 2 * g + hh;
        cw[(rb * 16 + cb * 4 + g) * 64] =
            pp >= 0 ? p.Cst[(size_t)b * P * 128 + slc4(pp, ch, P, p.cqm & kCqmC)] : 0.f;
      }
  __syncthreads();   // h image zeroed
  {  // h_0 (slot 0, channels 64..191) into the image (band mode: the band's rows and its halo rows)
    const __bf16* src = p.XH + (size_t)b * P * 192 + 64;
    const int hr0 = BAND ? max(r0 - 1, 0) : 0, hr1 = BAND ? min(r1 + 1, p.h) : p.h;
    for (int i = hr0 * p.w * 16 + tid; i < hr1 * p.w * 16; i += 256)
      *reinterpret_cast<u32x4*>(himb + pixb(hidx(i >> 4)) + (i & 15) * 16) =
          *reinterpret_cast<const u32x4*>(src + (size_t)(i >> 4) * 192 + (i & 15) * 8);
  }

  // per-lane B fragment bases: top-left image pixel of each column block's 3x3
  // window (columns >= P read pixel P-1: their outputs are never stored)
  int hb[4];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) {
    if constexpr (BAND) {
      const int pp = pix0 + min(cb * 32 + r32, Pb - 1);
      hb[cb] = (pp / p.w - r0) * W2 + pp % p.w;
    } else {
      hb[cb] = p.colhb[cb * 32 + r32];
    }
  }

  // A stream: one buffer descriptor over the fragment-order weights, the lane's
  // 16 B at voffset lane*16, the (row block, k step) in the wave-uniform soffset
  const __amdgpu_buffer_rsrc_t rsw = make_rsrc(p.Wf, (uint32_t)(16 * kRecKSP * 1024));
  const int wofs = rb0 * kRecKSP * 1024;
  auto lda = [&](int ks, int j) {
    return __builtin_bit_cast(bf16x8,
                              __builtin_amdgcn_raw_buffer_load_b128(rsw, lane * 16, wofs + (j * kRecKSP + ks) * 1024, 0));
  };
  constexpr int PD = kRecPD;
  bf16x8 af[PD][NRB];
#pragma unroll
  for (int s = 0; s < PD - 1; ++s)
#pragma unroll
    for (int j = 0; j < NRB; ++j) af[s][j] = lda(s, j);
  __syncthreads();   // images of step 0 complete (this wave's x DMA retired before: vmcnt in order)

  unsigned char* sw = stg + wave * STG;   // this wave's epilogue staging
  if ((b >> 3) & 1) stagger_wait(p.stagger);
  for (int t = 0; t < p.T; ++t) {
    AAA_FW_STAMP(t, 0);
    f32x16 acc[NRB][4];
#pragma unroll
    for (int j = 0; j < NRB; ++j)
#pragma unroll
      for (int cb = 0; cb < 4; ++cb)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[j][cb][e] = 0.f;
    int hbs[4], hbb[4];   // laundered per step: no per-tap address tables hoisted out of the step loop
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      hbs[cb] = hb[cb];
      asm volatile("" : "+v"(hbs[cb]));
    }
    // the h image's lane bases (the window's top-left pixel as a byte offset), made where the
    // h-part starts so they never live beside the x-part's bases
    auto h_bases = [&] {
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
        hbb[cb] = pixb(hb[cb]) + hh * 16;
        asm volatile("" : "+v"(hbb[cb]));
      }
    };
    // B fragments of a k step: x image (chunk c4 of 4 at tap offset toff) or h image (chunk c8 of 8)
    auto ldx = [&](int toff, int c4, bf16x8 (&bf)[4]) {
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
        const int ip = hbs[cb] + toff;
        bf[cb] = *reinterpret_cast<const bf16x8*>(xim + ip * 128 + (((2 * c4 + hh) ^ ((ip >> 1) & 7)) << 4));
      }
    };
    // (the window's columns never cross an image row, so a tap adds 272 toff + 16 rowpad ky: wave-uniform)
    auto ldh = [&](int toffb, int c8, bf16x8 (&bf)[4]) {
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) bf[cb] = *reinterpret_cast<const bf16x8*>(himb + hbb[cb] + toffb + c8 * 32);
    };
    auto tapoff = [&](int tap) { return (tap / 3) * W2 + tap % 3; };
    auto tapoffb = [&](int tap) { return 272 * tapoff(tap) + 16 * rp * (tap / 3); };
    // one k step: A prefetch PD-1 ahead, next B fragments, 16 MFMAs
    auto kstep = [&](int ks, int slot, bf16x8 (&bc)[4], auto&& load_next_b) {
      if constexpr (!(ABL & 1)) {
#pragma unroll
        for (int j = 0; j < NRB; ++j) af[(slot + PD - 1) % PD][j] = lda(ks + PD - 1, j);
      }
      if constexpr (!(ABL & 8)) load_next_b();
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < NRB; ++j)
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) {
          if constexpr (ABL & 4)
            acc[j][cb][0] += (float)af[slot][j][0] * (float)bc[cb][0];
          else
            acc[j][cb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[slot][j], bc[cb], acc[j][cb], 0, 0, 0);
        }
      __builtin_amdgcn_sched_barrier(0);
    };
    bf16x8 bfr[2][4];
    ldx(0, 0, bfr[0]);
    // x-part: 9 taps x 4 chunks (k steps 0..35)
    for (int tap = 0; tap < 9; ++tap) {
      const int toff = tapoff(tap), tn = tap < 8 ? tapoff(tap + 1) : 0;
      int kt = tap * 4;
      asm volatile("" : "+s"(kt));
#pragma unroll
      for (int c4 = 0; c4 < 4; ++c4)
        kstep(kt + c4, c4 % PD, bfr[c4 & 1], [&] {
          if (c4 < 3) ldx(toff, c4 + 1, bfr[(c4 + 1) & 1]);
          else if (tap < 8) ldx(tn, 0, bfr[0]);
          else if (G == 1 && !BAND) {
            h_bases();
            ldh(0, 0, bfr[0]);
          }
        });
    }
    barrier_lds();   // every wave is done with x_t: refill the image with x_{t+1} under the h-part
    AAA_FW_STAMP(t, 1);
    if (t + 1 < p.T) dma_x(t + 1, !(ABL & 64));   // (ABL 64, A/B: the compiler-visible form)
    if constexpr (BAND) {
      if (t > 0) {   // the neighbour bands' boundary rows of h_{t-1} (XH slot t) into the halo rows
        if (wave == 0)   // the neighbour bands' flags, both in one poll
          wave_wait_flags(p.flags + b * kRecBands,
                          (band > 0 ? 1ull << (band - 1) : 0ull) | (band < kRecBands - 1 ? 1ull << (band + 1) : 0ull), t,
                          p.report, p.spin, wdl);
        barrier_lds();
        const __amdgpu_buffer_rsrc_t rs = make_rsrc(p.XH + ((size_t)t * M + (size_t)b * P) * 192, (uint32_t)(P * 192 * 2));
        const int nh = p.w * 16;   // 16-B pieces of one grid row
        for (int i = tid; i < 2 * nh; i += 256) {
          const int gy = i < nh ? r0 - 1 : r1, j = i < nh ? i : i - nh;
          if ((unsigned)gy < (unsigned)p.h) {
            const int pp = gy * p.w + (j >> 4);
            *reinterpret_cast<u32x4*>(himb + pixb(hidx(pp)) + (j & 15) * 16) =
                __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)((pp * 192 + 64 + (j & 15) * 8) * 2), 0, kSC1);
          }
        }
        barrier_lds();
      }
      h_bases();
      ldh(0, 0, bfr[0]);
    }
    if constexpr (G == 2) {
      if (t > 0) {   // the partner's half of h_{t-1} (XH slot t) into the image, once it has published it
        if (tid == 0) {
          pair_wait(p.flags + 2 * b + (1 - kh), t, p.report, p.spin, wdl);   // bounded: a stranded partner reports
          if constexpr (ABL & 16) {   // fenced hand-off (A/B only)
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          }
        }
        barrier_lds();
        // the partner's bytes: sc1 loads (L2-served) of sc1-stored data behind an
        // sc1 flag poll -- no acquire needed (MI355X_MICROARCH: inter-workgroup
        // visibility, hand-off table row 1)
        const __amdgpu_buffer_rsrc_t rs = make_rsrc(p.XH + ((size_t)t * M + (size_t)b * P) * 192, (uint32_t)(P * 192 * 2));
        for (int i = tid; i < P * 8; i += 256)
          *reinterpret_cast<u32x4*>(himb + pixb(hidx(i >> 3)) + 128 * (1 - kh) + (i & 7) * 16) =
              __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)(((i >> 3) * 192 + 64 + 64 * (1 - kh) + (i & 7) * 8) * 2),
                                                    0, (ABL & 16) ? 0 : kSC1);
        barrier_lds();
      }
      h_bases();
      ldh(0, 0, bfr[0]);
    }
    AAA_FW_STAMP(t, 2);
    // h-part: 9 taps x 8 chunks (k steps 36..107)
    for (int tap = 0; tap < 9; ++tap) {
      const int toff = tapoffb(tap), tn = tap < 8 ? tapoffb(tap + 1) : 0;
      int kt = kRecKX + tap * 8;
      asm volatile("" : "+s"(kt));
#pragma unroll
      for (int c8 = 0; c8 < 8; ++c8)
        kstep(kt + c8, c8 % PD, bfr[c8 & 1], [&] {
          if (c8 < 7) ldh(toff, c8 + 1, bfr[(c8 + 1) & 1]);
          else if (tap < 8) ldh(tn, 0, bfr[0]);
        });
    }
    barrier_lds();   // every wave is done with h_{t-1}: the epilogue overwrites the image with h_t
    AAA_FW_STAMP(t, 3);

    // Epilogue, one column block (32 pixels) at a time: gate math + cell update
    // lane-local, h_t into the h image, c_t into its LDS copy, and the HBM
    // outputs staged through the wave's LDS scratch in two halves of 16 pixels
    // so every store instruction writes whole 128-B / 256-B pixel rows (gates, c,
    // h are [pixel][channel]: a lane's own values are one channel at 32 pixels).
    // the lane index laundered per step: every epilogue address is recomputed
    // here instead of hoisted out of the step loop into spilled registers
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const int pl = ln & 31, hl_ = ln >> 5;
    const size_t rowt = (size_t)t * M + (size_t)b * P;   // this frame's rows of step t (Hs, Gt)
    const int c0 = cbase + hl_;                          // + 8*rb + 2*g
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      const int pp = scol[cb * 32 + pl];   // -1: padding column
      __bf16* hl = reinterpret_cast<__bf16*>(himb + pixb(hidx(max(pp, 0)))) + c0;
      uint32_t gq[NRB][4][2];   // fp16 gate quads (i, f, c~, o), packed
      float hv[NRB][4], cv[NRB][4];
#pragma unroll
      for (int rb = 0; rb < NRB; ++rb)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int co = 8 * rb + 2 * g;
          const f32x4 bz = *reinterpret_cast<const f32x4*>(sbias + 4 * (c0 + co));
          const float gi = sigm_fast(acc[rb][cb][4 * g] + bz[0]);
          const float gf = sigm_fast(acc[rb][cb][4 * g + 1] + bz[1]);
          const float gc = tanh_fast(acc[rb][cb][4 * g + 2] + bz[2]);
          const float go = sigm_fast(acc[rb][cb][4 * g + 3] + bz[3]);
          float* cl = cstl + wave * NRB * 16 * 64 + ln + (rb * 16 + cb * 4 + g) * 64;
          const float c = gf * *cl + gi * gc;
          const float h = go * tanh_fast(c);
          *cl = c;
          cv[rb][g] = c;
          hv[rb][g] = h;
          typedef _Float16 h2 __attribute__((ext_vector_type(2)));
          gq[rb][g][0] = __builtin_bit_cast(uint32_t, h2{(_Float16)gi, (_Float16)gf});
          gq[rb][g][1] = __builtin_bit_cast(uint32_t, h2{(_Float16)gc, (_Float16)go});
          if (pp >= 0) hl[co] = (__bf16)h;
        }
      if constexpr (!(ABL & 2)) {
#pragma unroll
        for (int half = 0; half < 2; ++half) {
          const int pxl = pl & 15;
          const bool mine = (pl >> 4) == half;
          const int pbase = cb * 32 + half * 16;   // first column of this half
          // gates: staging [16 px][GCH ch][4] fp16 at pixel pitch GTP
          if (mine) {
#pragma unroll
            for (int rb = 0; rb < NRB; ++rb)
#pragma unroll
              for (int g = 0; g < 4; ++g)
                *reinterpret_cast<uint2*>(sw + pxl * GTP + (8 * rb + 2 * g + hl_) * 8) = uint2{gq[rb][g][0], gq[rb][g][1]};
          }
          constexpr int CG = GCH / 2, CC = GCH / 4;   // 16-B chunks per pixel row: gates, c / h
          if (p.cqm & kCqmG) {   // quad-major: lane pairs walk the 16 pixels of one quad (512-B runs)
#pragma unroll
            for (int k = 0; k < NRB; ++k) {
              const int q = k * 64 + ln, hf = q & 1, px = (q >> 1) & 15, qi = q >> 5, pix = scol[pbase + px];
              const u32x4 v = *reinterpret_cast<const u32x4*>(sw + px * GTP + (2 * qi + hf) * 16);
              if (pix >= 0)
                *reinterpret_cast<u32x4*>(p.Gt + rowt * 512 + ((size_t)(cbase / 4 + qi) * P + pix) * 16 + hf * 8) = v;
            }
          } else {
#pragma unroll
            for (int k = 0; k < NRB; ++k) {   // 1 KB each: 64 / CG pixel rows of 8 * GCH B
              const int q = k * 64 + ln, px = q / CG, pix = scol[pbase + px];
              const u32x4 v = *reinterpret_cast<const u32x4*>(sw + px * GTP + (q % CG) * 16);
              if (pix >= 0)
                *reinterpret_cast<u32x4*>(reinterpret_cast<unsigned char*>(p.Gt + (rowt + pix) * 512 + 4 * cbase) +
                                          (q % CG) * 16) = v;
            }
          }
          // c_t and h_t: staging [16 px][GCH ch] fp32 at pixel pitch CHP (c), then (h) 16 * CHP B on
          if (mine) {
#pragma unroll
            for (int rb = 0; rb < NRB; ++rb)
#pragma unroll
              for (int g = 0; g < 4; ++g) {
                *reinterpret_cast<float*>(sw + pxl * CHP + (8 * rb + 2 * g + hl_) * 4) = cv[rb][g];
                if (p.Hs) *reinterpret_cast<float*>(sw + 16 * CHP + pxl * CHP + (8 * rb + 2 * g + hl_) * 4) = hv[rb][g];
              }
          }
#pragma unroll
          for (int k = 0; k < NRB / 2; ++k) {   // 1 KB each of c and h: 64 / CC pixel rows of 4 * GCH B
            const int q = k * 64 + ln, px = q / CC, pix = scol[pbase + px];
            if (p.cqm & kCqmC) {   // c quad-major: 16 lanes walk the 16 pixels of one quad (256-B runs)
              const int pxq = q & 15, qi = q >> 4, pixq = scol[pbase + pxq];
              const u32x4 vc = *reinterpret_cast<const u32x4*>(sw + pxq * CHP + qi * 16);
              if (pixq >= 0) *reinterpret_cast<u32x4*>(p.Cst + (rowt + M) * 128 + ((size_t)(cbase / 4 + qi) * P + pixq) * 4) = vc;
            } else {
              const u32x4 vc = *reinterpret_cast<const u32x4*>(sw + px * CHP + (q % CC) * 16);
              if (pix >= 0) *reinterpret_cast<u32x4*>(p.Cst + (rowt + M + pix) * 128 + cbase + (q % CC) * 4) = vc;
            }
            if (p.Hs) {
              const u32x4 vh = *reinterpret_cast<const u32x4*>(sw + 16 * CHP + px * CHP + (q % CC) * 16);
              if (pix >= 0) *reinterpret_cast<u32x4*>(p.Hs + (rowt + pix) * 128 + cbase + (q % CC) * 4) = vh;
            }
          }
        }
      }
      __builtin_amdgcn_sched_barrier(0);   // one column block at a time (register pressure)
    }
    barrier_lds();   // h_t image and x_{t+1} image complete (this wave's DMA retired under its h-part A loads)
    AAA_FW_STAMP(t, 4);
    // h_t (bf16, this workgroup's channels) into XH slot t+1 (the weight-gradient operand), from the image
    const size_t rown = rowt + M;   // slot t+1
    constexpr int HC = 16 / G;      // 16-B chunks (8 channels) per pixel of this workgroup
    if constexpr (BAND) {   // the neighbours read these rows: sc1 stores, then publish
      const __amdgpu_buffer_rsrc_t rs = make_rsrc(p.XH + rown * 192, (uint32_t)(P * 192 * 2));
      for (int i = tid; i < Pb * HC; i += 256) {
        const int px = pix0 + i / HC, q = i % HC;
        __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const u32x4*>(himb + pixb(hidx(px)) + q * 16), rs,
                                               (uint32_t)((px * 192 + 64 + q * 8) * 2), 0, kSC1);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      barrier_lds();
      if (tid == 0)
        __hip_atomic_store(p.flags + b * kRecBands + band, t + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else if constexpr (G == 1) {
      for (int i = tid; i < ((ABL & 2) ? 0 : P * HC); i += 256) {
        const int px = i / HC, q = i % HC;
        *reinterpret_cast<u32x4*>(p.XH + (rown + px) * 192 + 64 + q * 8) =
            *reinterpret_cast<const u32x4*>(himb + pixb(hidx(px)) + q * 16);
      }
    } else {   // the partner reads these: sc1 stores (write through to the coherent level)
      const __amdgpu_buffer_rsrc_t rs = make_rsrc(p.XH + rown * 192, (uint32_t)(P * 192 * 2));
      for (int i = tid; i < P * HC; i += 256) {
        const int px = i / HC, q = i % HC + HC * kh;
        __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const u32x4*>(himb + pixb(hidx(px)) + q * 16), rs,
                                               (uint32_t)((px * 192 + 64 + q * 8) * 2), 0, (ABL & 16) ? 0 : kSC1);
      }
      // publish h_t's half: every wave's stores retired, a barrier, then one
      // lane's flag store (sc1; the fenced variant adds an agent release)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      barrier_lds();
      if (tid == 0) {
        if constexpr (ABL & 16) {
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __hip_atomic_store(p.flags + 2 * b + kh, t + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    AAA_FW_STAMP(t, 5);
  }
}

// G = 1: one workgroup per frame; G = 2: two per frame in one residency wave
// (launch_resident: p.flags zeroed by the caller; the launch fails rather than
// strand a half; a partner wait that still times out is reported via p.report).
template <typename GT>
inline hipError_t convlstm_fwd_frames_band(RecFwdParams<GT>& p, hipStream_t st) {
  if (!rec_band_fits(p.h, p.w) || p.P != p.h * p.w || p.B < 1 || p.T < 1 || !p.flags || !p.report || p.spin < 0)
    return hipErrorInvalidValue;
  return launch_resident(reinterpret_cast<const void*>(&k_convlstm_fwd_frames<GT, 1, 0, true>),
                         8 * kRecBands * ((p.B + 7) / 8), 256, p, st);
}

template <typename GT>
inline hipError_t convlstm_fwd_frames(const RecFwdParams<GT>& p, int G, hipStream_t st) {
  if (!rec_fits(p.h, p.w) || p.P != p.h * p.w || p.B < 1 || p.T < 1 || (G != 1 && G != 2)) return hipErrorInvalidValue;
  RecFwdParams<GT> q = p;
  rec_columns(p.h, p.w, q.colpp, q.colhb);
  if (G == 2) {
    if (!p.flags || !p.report || p.spin < 0) return hipErrorInvalidValue;
    const void* k = reinterpret_cast<const void*>(&k_convlstm_fwd_frames<GT, 2, 0>);
#ifdef AAA_ABLATION   // diagnostic builds only (tools/ubench): the product library never reads AAA_REC_ABL
    const char* e = getenv("AAA_REC_ABL");
    if (e && atoi(e) == 16) k = reinterpret_cast<const void*>(&k_convlstm_fwd_frames<GT, 2, 16>);
#endif
    return launch_resident(k, 2 * p.B, 256, q, st);
  }
#ifdef AAA_ABLATION
  const char* e = getenv("AAA_REC_ABL");
  switch (e ? atoi(e) : 0) {
#define AAA_REC_CASE(a) \
  case a: hipLaunchKernelGGL((k_convlstm_fwd_frames<GT, 1, a>), dim3(p.B), dim3(256), 0, st, q); return hipGetLastError();
    AAA_REC_CASE(1) AAA_REC_CASE(2) AAA_REC_CASE(3) AAA_REC_CASE(4) AAA_REC_CASE(8) AAA_REC_CASE(12) AAA_REC_CASE(64)
#undef AAA_REC_CASE
    default: break;
  }
#endif
  hipLaunchKernelGGL((k_convlstm_fwd_frames<GT, 1, 0>), dim3(p.B), dim3(256), 0, st, q);
  return hipGetLastError();
}

}  // namespace aaa
