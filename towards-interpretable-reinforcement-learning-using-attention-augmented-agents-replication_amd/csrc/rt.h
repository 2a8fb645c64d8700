// Internal header of the host runtime (csrc/runtime.hip and the rt_*.hip
// translation units): the buffer layout, error/timing/stream state (defined
// once in rt_core.hip), the tile configurations and the GEMM launch helpers
// shared by the forward (rt_forward.hip), the backward (rt_backward.hip) and
// the component entries (rt_components.hip).
#pragma once
#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <type_traits>
#include <utility>
#include <vector>

#include "aaa.h"
#include "epilogues.h"
#include "gemm.h"
#include "loaders_b.h"
#include "glds.h"
#include "gemm_deep.h"
#include "halo.h"
#include "recur.h"
#include "recur_bwd.h"
#include "recur_f32.h"
#include "recur_bwd_f32.h"
#include "vision.h"
#include "vision_bwd.h"
#include "misc.h"
#include "optim.h"
#include "actor.h"


namespace aaa {

extern thread_local std::string g_err;   // aaa_last_error()

int fail(int code, const char* fmt, ...);

#define HIPCHK(expr)                                                                      \
  do {                                                                                    \
    hipError_t e_ = (expr);                                                               \
    if (e_ != hipSuccess)                                                                 \
      return fail(AAA_E_LAUNCH, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_),   \
                  __FILE__, __LINE__);                                                    \
  } while (0)

inline size_t al256(size_t x) { return (x + 255) & ~size_t(255); }
inline int cdiv(int a, int b) { return (a + b - 1) / b; }
inline int conv_out(int n, int k, int s, int p) { return (n + 2 * p - k) / s + 1; }

enum PIdx {
  C0W = 0, C0B, C1W, C1B,
  XI_W, XI_B, HI_W, XF_W, XF_B, HF_W, XC_W, XC_B, HC_W, XO_W, XO_B, HO_W,
  Q0W, Q0B, Q2W, Q2B, Q4W, Q4B, A0W, A0B, A2W, A2B, WIH, WHH, BIH, BHH, PW, PB, VW, VB, NPARAM
};

struct Layout {
  int B, T, F, H, W, H1, W1, P1, h, w, P, nq, A, dt, esz;
  int sc;   // stateful policy core (AAA_FLAG_STATEFUL_CORE)
  int fu8;  // frames are uint8 (AAA_FLAG_FRAMES_U8)
  int fchunk;   // frames per launch of the whole-batch conv GEMMs (< 2 GiB per descriptor, check_ranges)
  int xpc;      // frames of the Xp chunk buffer (conv1's bordered RGBx operand, rebuilt per chunk)
  int qd, da, ans_in, ans_ld, ldy;
  size_t poff[NPARAM], psz[NPARAM], ptotal;
  size_t k_Wp1, k_Wp2, k_WdT2, k_WpX, k_WpH, k_WpXH, k_Wfr, k_Wbf, k_Wf32, k_Wb32, k_Wf6, k_Wf6p, k_Wb6, k_Wx6, k_Wb6p, k_Wx6p, k_WdTl, k_WdTc, k_WdT6, k_bl, k_Wihhp, k_q1, k_q2, k_Q, k_W1p, k_Wihp, k_blc, k_Whd, k_bhd, packed;
  size_t Xp, Y1, XH, Hs, Cst, Gt, SQ, Am, ans, hid1, AO, LG, LC, LH;
  size_t dY, dLG, dAO, dH1, dAns, dO, dQp, dQs, dC, dZ, dZp, dY2, dY1, dxb, rflags, xpart, dhs, dZ6;
  size_t gWp1, gWp2, gWpl, gbl, gW1p, gWihp, gblc, gWhd, gbhd, ws;
  // stateful core: state slots, per-step query activations, [answer | h] rows, their grads
  size_t CH, CC, AOX, Qf, q1s, q2s, dAOX, dQf, dq2s, dq1s, dhc, dcc, gWihhp;
};

// Algorithmic FLOP per frame of the other timer classes:
// conv1 (K = 8*8*3) and conv2 (K = 4*4*32) forward; the answer MLP + LSTMCell
// (zero state: W_ih only); their backward is twice that (dgrad + wgrad); the
// conv2 wgrad + dgrad and conv1 wgrad of the vision backward.
inline double vision_fwd_flop(const Layout& L) { return 2.0 * L.P1 * 32 * 192 + 2.0 * L.P * 64 * 512; }
inline double tail_fwd_flop(const Layout& L) {
  return 2.0 * ((double)L.ans_in * 512 + 512.0 * 256 + 256.0 * 1024);
}
inline double vision_bwd_flop(const Layout& L) { return 2.0 * (2.0 * L.P * 64 * 512) + 2.0 * L.P1 * 32 * 192; }

// min_frames: the frames one launch must be able to address (a step's B for
// the unroll; 1 for the frame-independent vision encoder entries).
int build_layout(const aaa_cfg* c, Layout& L, int min_frames = 0);
int check_device();

inline bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// ------------------------------------------------- paired-kernel reports --
// The paired frame-resident kernels (two cooperating workgroups per frame)
// bound their partner waits (common.h pair_wait).  A timed-out wait adds 1 to
// this device's report word: pinned host memory mapped into the device, so the
// host reads it without a copy or a sync.  Every aaa_forward / aaa_backward
// entry consumes pending reports and fails with AAA_E_STRANDED (the results of
// the call that stranded are invalid); aaa_pair_status syncs a stream first.
// Allocated once per process on first use, never freed (no HIP call at exit).
int pair_budget(int T);    // partner-wait budget of a T-step launch, 100-MHz ticks
int* pair_report(int dev);  // this device's report word, device-mapped (nullptr: cannot map)
int* pair_flag_base(int dev);  // aaa_pair_flag's own snapshot of it, device-mapped
int pair_take();            // pending reports of the current device (consumed)
int pair_peek();            // ... (left pending)
int pair_check();           // AAA_E_STRANDED if any are pending

// ------------------------------------------------------------ aux stream --
// Work that is off the sequential ConvLSTM chain (the batched x-part of the
// forward, every weight/bias gradient and dx/conv backward) is issued on a
// per-device low-priority stream, chunked every few steps and ordered against
// the caller's stream by events; the caller's stream waits for it before the
// call returns (fork/join inside each call).  Created lazily, once per device.
hipStream_t aux_stream();   // nullptr unless AAA_OVERLAP=1 (measured slower on C2, round 1)
hipStream_t side_stream();  // the backward HEAD phase's weight gradients (rt_core.hip); nullptr: AAA_SIDE=0
// Record a pooled event on ``s`` (everything enqueued on s so far).
hipError_t record_event(hipStream_t s, hipEvent_t* out);
// ``to`` waits for everything enqueued on ``from`` so far.
hipError_t stream_order(hipStream_t from, hipStream_t to);

// ------------------------------------------------- optional kernel timing --
// Per timer class: the HIP event pairs of each launch, the launches'
// algorithmic work (FLOP for the MFMA classes, bytes for the HBM ones) and
// the kernel variant dispatched -- so a benchmark reads the roofline inputs
// from the library instead of re-deriving its dispatch rules.
struct Timers {
  std::mutex mu;
  bool on = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> pending[AAA_TIMER_N];
  double work[AAA_TIMER_N] = {};
  std::string variant[AAA_TIMER_N];
  std::vector<hipEvent_t> pool;
  hipEvent_t get() {
    if (!pool.empty()) { hipEvent_t e = pool.back(); pool.pop_back(); return e; }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
  }
};
extern Timers g_timers;

struct TimerScope {
  int kind;
  hipStream_t st;
  hipEvent_t a = nullptr, b = nullptr;
  double work;
  std::string variant;
  TimerScope(int k, hipStream_t s, double w, std::string v) : kind(k), st(s), work(w), variant(std::move(v)) {
    std::lock_guard<std::mutex> lk(g_timers.mu);
    if (!g_timers.on) return;
    a = g_timers.get();
    b = g_timers.get();
    if (a && b) (void)hipEventRecord(a, st);
  }
  ~TimerScope() {
    if (!a || !b) return;
    (void)hipEventRecord(b, st);
    std::lock_guard<std::mutex> lk(g_timers.mu);
    g_timers.pending[kind].emplace_back(a, b);
    g_timers.work[kind] += work;
    g_timers.variant[kind] = variant;
  }
};

std::string strf(const char* fmt, ...);

// Algorithmic bytes per frame of the fused attention readout kernels (fp32):
// forward reads the frame's O rows (128 ch) and writes its map and answer row;
// backward reads O, the map and the answer grad, writes dO and dQ.
// per frame: O read (oesz bytes per element: 4 fp32 Hs, 2 the bf16 XH copy), A and the answer row written
inline double attn_fwd_bytes(int P, int nq, int ans_ld, int oesz = 4) {
  return oesz * 128.0 * P + 4.0 * (nq * P + ans_ld);
}
// per frame: O read, dO written (fp32), A / da / Q read, dQ written
inline double attn_bwd_bytes(int P, int nq, int oesz = 4) {
  return oesz * 128.0 * P + 4.0 * (128.0 * P + nq * P + 184.0 * nq + 72.0 * nq);
}

// --------------------------------------------------------- tile configs ---
// fp32 uses the exact v_mfma_f32_32x32x2_f32; bf16 v_mfma_f32_32x32x16_bf16 (fp32 accumulate).
using CF = GemmCfg<float, 64, 64, 32, 2, 2>;      // default 64x64 tile, 4 waves
using CF32 = GemmCfg<float, 32, 64, 32, 1, 2>;    // 32-row tile, 2 waves: small-Mi GEMMs / more WGs
using CFW = GemmCfg<float, 128, 128, 32, 2, 2>;   // long-K weight gradients: 64x64 per wave
using CFK = GemmCfg<float, 32, 64, 64, 1, 2, 2>;  // per-step ConvLSTM kernels: 2-way split-K in the WG
using CFK4 = GemmCfg<float, 32, 64, 64, 1, 2, 4>; // 4-way split-K (8 waves)
using CFK4B = GemmCfg<float, 32, 64, 128, 1, 2, 4>; // 4-way split-K, 2 k-steps per wave per barrier
using CF64 = GemmCfg<float, 64, 64, 64, 2, 2>;     // 64x64, BK 64
using CFJ = GemmCfg<float, 64, 128, 32, 2, 2>;     // 64-row GEMMs with long N (batched dx)
using CFS = GemmCfg<float, 128, 64, 32, 4, 2>;     // forward step: 8 waves, ~1 WG per CU at C2 (balanced)
using CB = GemmCfg<__bf16, 64, 64, 64, 2, 2>;
using CB32 = GemmCfg<__bf16, 32, 64, 64, 1, 2>;
using CBW = GemmCfg<__bf16, 128, 128, 64, 2, 2>;
using CBK = GemmCfg<__bf16, 32, 64, 64, 1, 2, 2>;
using CBK4 = GemmCfg<__bf16, 32, 64, 64, 1, 2, 4>;
using CBK4B = GemmCfg<__bf16, 32, 64, 128, 1, 2, 4>;
using CB64 = GemmCfg<__bf16, 64, 64, 128, 2, 2>;
using CBJ = GemmCfg<__bf16, 64, 128, 64, 2, 2>;
using CBS = GemmCfg<__bf16, 128, 64, 64, 4, 2>;
template <typename T> using CfgFor = std::conditional_t<std::is_same<T, float>::value, CF, CB>;
template <typename T> using Cfg32For = std::conditional_t<std::is_same<T, float>::value, CF32, CB32>;
template <typename T> using CfgWFor = std::conditional_t<std::is_same<T, float>::value, CFW, CBW>;
template <typename T> using CfgKFor = std::conditional_t<std::is_same<T, float>::value, CFK, CBK>;
template <typename T> using CfgK4For = std::conditional_t<std::is_same<T, float>::value, CFK4, CBK4>;
template <typename T> using CfgK4BFor = std::conditional_t<std::is_same<T, float>::value, CFK4B, CBK4B>;
template <typename T> using Cfg64For = std::conditional_t<std::is_same<T, float>::value, CF64, CB64>;
template <typename T> using CfgJFor = std::conditional_t<std::is_same<T, float>::value, CFJ, CBJ>;
template <typename T> using CfgSFor = std::conditional_t<std::is_same<T, float>::value, CFS, CBS>;

// Step-kernel tile choice (env AAA_STEP_TILE / AAA_BPTT_TILE override):
//   0 64x64 BK32 | 1 32x64 BK64 2-way in-WG split-K | 2 ... 4-way | 3 32x64 BK128 4-way
//   (forward: 3 = 64x64 BK64) | 4-6 the same shapes on the LDS-DMA ring of glds.h
//   (forward 4 = 128x64 8 waves, 5 = 32x64 split-K, 6 = 64x64 BK64; BPTT 4 = 32x64 BK128
//   4-way, 5 = BK64 4-way, 6 = 64x64, 9 = 64x32 BK128 4-way).  The default picks by how many 32x32
//   output tiles the step has, i.e. how many waves it can feed; measured on C2.
inline int env_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return e ? atoi(e) : dflt;
}
// A/B-only knobs (the same-box comparisons of tools/gpu_ab*.sh): read from the
// environment only in -DAAA_ABLATION builds (make ablation -> libaaa_ablation.so,
// loaded through AAA_LIB); the product library takes the default.  env_int stays
// for the path selectors the parity tests drive.
inline int ab_int(const char* name, int dflt) {
#ifdef AAA_ABLATION
  return env_int(name, dflt);
#else
  (void)name;
  return dflt;
#endif
}
// Steps per off-chain chunk: the whole unroll unless overlapping, and never
// more than the frames one launch may address (Layout::fchunk).
static int chunk_steps(const Layout& L) {
  const int c = ab_int("AAA_CHUNK", ab_int("AAA_OVERLAP", 0) ? 4 : L.T);
  return std::max(1, std::min({c, L.T, L.fchunk / L.B}));
}
bool f32_split6();   // fp32 path: large GEMMs as bf16x6 split products (rt_core.hip)
static int step_tile(long out_tiles32, const char* env, bool bptt, bool bf16 = false) {
  const int v = env_int(env, -1);
  if (v >= 0) {   // 7, 8: bf16 only; 9-11, 13, 15, 16: BPTT only; 14, 17, 18: forward only
    const bool bptt_only = v == 9 || v == 10 || v == 11 || v == 13 || v == 15 || v == 16 || (v >= 19 && v <= 24) ||
                           (v >= 27 && v <= 33);
    if (v >= 19 && v <= 24 && !bf16) return 4;   // 19-24: bf16 BPTT tiles (fp16 gate storage)
    if (v >= 27 && v <= 33 && bf16) return 4;    // 27-33: fp32 split-product BPTT tiles (30-33 split-K)
    const bool fwd_only = v == 14 || v == 17 || v == 18 || v == 25 || v == 26;
    return ((v == 7 || v == 8) && !bf16) || (bptt_only && !bptt) || (fwd_only && bptt) ? 4 : v;
  }
  // bf16 BPTT: 128x128 from ~3/4 of a workgroup per CU (C3: 242 WGs), else 128x64
  // (tools/ubench/bf16_tiles at B=128: 34.6 vs 39.6 us)
  // below that, 128x64 with a 4-way in-WG split-K (8 waves; C4: 50.0 vs 52.5 us for the 4-wave
  // 2-way tile 8, tools/ab_bptt_bf16.sh)
  if (bptt && bf16) return out_tiles32 >= 4L * 4 * 192 ? 7 : 22;
  // fp32 (C2: 484 BPTT / 1936 forward tiles): 32x32 BK64 4-way BPTT on a 3-stage ring, two WGs
  // per CU whose barriers are not in step (51.6 vs 54.4 us for 64x32 BK128, 54.6 vs 55.9 for
  // 32x64); 64x64 BK64 forward 47.4 us (32x64 / 32x32 / 64x32 split-K rings: 52-55 us)
  // (bench.py kernel table, tools/ab_bptt.sh)
  // fp32 with f32_split6(): below 1024 tiles (the B=1 episode / actor: 68) the split-K
  // split-product tile 31 (15.0 + 5.6 us per step vs 37 us for the fp32 tile 16 at the
  // episode's 27x20 grid; C2 itself runs the frame-group BPTT, recur_bwd_f32.h)
  if (bptt) return out_tiles32 < 1024 ? (f32_split6() ? 31 : 16) : (out_tiles32 < 1536 ? 1 : 0);
  return out_tiles32 < 1024 ? 5 : 6;
}

// Split-K BPTT (fp32 tiles 30/31): K slices of the per-step dh dgrad, summed by
// the gate backward (misc.hip k_gate_bwd_last).  Only where the step has few
// output tiles (the B=1 episode: 4 x 17), so the partials stay small.
constexpr int kBpttSplitMax = 8;
constexpr int kSplitBj = 8;   // pixels per gate-backward workgroup (and gate-bias partial row) of the split-K chain
static bool bptt_splitk_fits(int M) { return 4L * ((M + 31) / 32) < 1024; }
static int bptt_splitk() { return std::max(2, std::min(kBpttSplitMax, env_int("AAA_BPTT_SPLITK", 4))); }
// K slices launch_pipe actually runs for a requested nsplit (glds.h: whole BK tiles per slice)
inline int splitk_slices(int K, int BK, int nsplit) {
  const int kc = ((K + nsplit - 1) / nsplit + BK - 1) / BK * BK;
  return (K + kc - 1) / kc;
}

// fp16 gate-activation storage (halves the step epilogues' largest stream):
// bf16 operands, fused x-part (the gate buffer then holds activations only)
// and the bf16 BPTT tiles 7/8.  AAA_GATES_F16=0 keeps fp32.  Forward and
// backward evaluate this identically (same env, same shapes).
// The x-part rides in the step GEMM for bf16 and for small steps (M = B*P
// pixels; the actor's B = 1: one launch instead of two latency-bound ones);
// fp32 at C2 (M = 3872) keeps the batched x-part (measured 5.02 vs 5.09 ms).
// bf16 ConvLSTM forward on the frame-resident kernel (recur.h): one workgroup
// per frame for the whole unroll, on grids whose images fit its LDS (84x84
// frames), once the batch fills most of the chip's 256 CUs (C3, B=256: 55 vs
// 79 us per step; C4's B=128 leaves half the CUs idle: 49 vs 43 us,
// profiles/r02/frames).  AAA_FRAMES_FWD=1/0 forces it on/off.
int frames_fwd(const Layout& L);
static bool fused_x(int dt, int M) { return env_int("AAA_FUSED_X", dt == AAA_BF16 || M <= 1024 ? 1 : 0) != 0; }
static bool gates_f16(int dt, int M) {
  if (dt != AAA_BF16 || !fused_x(dt, M) || !ab_int("AAA_GATES_F16", 1)) return false;
  const int bt = step_tile((long)(128 / 32) * ((M + 31) / 32), "AAA_BPTT_TILE", true, true);
  return bt == 7 || bt == 8 || bt >= 19;
}

// Whether the LDS-DMA ring can run tile config CK (every wave issues the same DMA count).
template <class CK>
constexpr bool pipe_even() {
  constexpr int VG = 16 / (int)sizeof(typename CK::type);
  return (CK::BI * CK::BK / VG) % CK::NT == 0 && (CK::BJ * CK::BK / VG) % CK::NT == 0;
}

// One per-step ConvLSTM GEMM: D[Mi][M] = W[Mi][K] x im2col(src)[K][M] with
// epilogue ep.  PIPE = LDS-DMA ring (glds.h; needs src already in T),
// otherwise the register-staged kernel (which can convert fp32 -> bf16).
template <class CK, bool PIPE, typename T, typename G, class EP, int NBUF = 2, bool ILV = false>
static hipError_t step_gemm(const T* W, int ldw, int wrows, const G* src, const ConvGeo& g, int M, uint32_t src_bytes,
                            const EP& ep, int Mi, int K, hipStream_t st, int nsplit = 1) {
  if constexpr (PIPE && pipe_even<CK>() && std::is_same<G, T>::value) {
    using LA = GRowsB<T, CK::BI, CK::BK, CK::NT>;
    using LB = GIm2colB<T, CK::BJ, CK::BK, CK::NT>;
    return launch_pipe<CK, LA, LB, EP, NBUF, ILV>(typename LA::Params{W, ldw, wrows},
                                                  typename LB::Params{src, g, M, src_bytes}, ep, Mi, M, K, nsplit, st);
  } else {
    if (nsplit != 1) return hipErrorInvalidValue;   // split-K: ring tiles only
    using LA = LdRowsB<T, T, CK::BI, CK::BK, CK::NT>;
    using LB = LdIm2colB<G, T, CK::BJ, CK::BK, CK::NT>;
    return launch_gemm<CK, LA, LB>(typename LA::Params{W, ldw, wrows}, typename LB::Params{src, g, M, src_bytes}, ep,
                                   Mi, M, K, 1, st);
  }
}

// Small GEMMs of the head (F = T*B rows; answer MLP, LSTMCell, policy/value
// heads): 64x64 tiles leave most CUs idle, so below ~192 tiles use the 32x64
// tile with a 4-way in-WG split-K (8 waves per WG: the serial K loop of these
// long-K, few-tile GEMMs is what they wait on; C2 4.487 -> 4.414 ms per
// iteration vs the plain 32x64 tile, tools/ab_head.sh).  AAA_HEAD_TILE=1 forces
// 64x64, =2 the plain 32x64, =3/4/5 the 2-way / 4-way / 4-way BK128 split-K tiles.  (128x128 and 64x128
// tiles, fewer split fragments per MFMA, measured slower: C2 tail 190 -> 370 / 290 us, C3 367 -> 536 / 433.)
// g_tail3 (set per forward / backward call of the bf16 path, TailPrecision):
// the same tiles with fp32 operands split into bf16 pairs on the bf16 MFMA
// (gemm.h GemmCfgS3), ~1e-5 relative per product.
// g_tail6 (set per call of the fp32 path when f32_split6()): the three-way
// split at fp32 accuracy (gemm.h GemmCfgS6).
extern thread_local bool g_tail3, g_tail6;
struct TailPrecision {
  bool prev3, prev6;
  explicit TailPrecision(bool split3, bool split6 = false) : prev3(g_tail3), prev6(g_tail6) {
    g_tail3 = split3;
    g_tail6 = split6;
  }
  ~TailPrecision() {
    g_tail3 = prev3;
    g_tail6 = prev6;
  }
};
template <class C> struct S3Of { using type = GemmCfgS3<C::BI, C::BJ, C::BK, C::WI, C::WJ, C::WK>; };
template <class C> struct S6Of { using type = GemmCfgS6<C::BI, C::BJ, C::BK, C::WI, C::WJ, C::WK>; };

// The deep-pipeline (gemm_deep.h) form of a tail loader: LdRows -> LdRowsN, LdRowsT -> LdRowsTN.
template <template <typename, typename, int, int, int> class L> struct DeepLd;
template <> struct DeepLd<LdRows> {
  template <typename G, typename T, int R, int BK, int NT> using type = LdRowsN<G, T, R, BK, NT>;
  static bool fits(const void*, int ld, int nrows) { return ld % 4 == 0 && (size_t)nrows * ld * 4 < (1u << 31); }
};
template <> struct DeepLd<LdRowsT> {
  template <typename G, typename T, int R, int BK, int NT> using type = LdRowsTN<G, T, R, BK, NT>;
  static bool fits(const void*, int ld, int nrows) { return ld % 4 == 0 && nrows % 4 == 0; }
};
constexpr int kTailStages = 8;
#ifdef AAA_ABLATION
constexpr bool kAblationBuild = true;
#else
constexpr bool kAblationBuild = false;
#endif   // K tiles of global loads in flight per workgroup (gemm_kernel_deep)

template <template <typename, typename, int, int, int> class LA_,
          template <typename, typename, int, int, int> class LB_, class PA, class PB, class EP>
static hipError_t head_gemm(const PA& pa, const PB& pb, const EP& ep, int Mi, int Nj, int K, int nsplit,
                            hipStream_t st) {
  const int mode = ab_int("AAA_HEAD_TILE", 0);
  const long tiles = (long)cdiv(Mi, 64) * cdiv(Nj, 64) * std::max(nsplit, 1);
  // ablation builds, AAA_TAIL_DEEP=1: kTailStages register stages of K tiles in flight (gemm_kernel_deep)
#ifdef AAA_ABLATION   // measured no faster (profiles/r06/ab/tail_deep/): ablation builds only
  const bool deep = ab_int("AAA_TAIL_DEEP", 0) && DeepLd<LA_>::fits(pa.src, pa.ld, pa.nrows) &&
                    DeepLd<LB_>::fits(pb.src, pb.ld, pb.nrows) && (size_t)K * pa.ld * 4 < (1u << 31) &&
                    (size_t)K * pb.ld * 4 < (1u << 31);
#else
  constexpr bool deep = false;
#endif
  auto run = [&](auto cfg) {
    using C = decltype(cfg);
    if constexpr (!kAblationBuild) {
      (void)deep;
    } else if (deep) {
      using A = typename DeepLd<LA_>::template type<float, float, C::BI, C::BK, C::NT>;
      using B = typename DeepLd<LB_>::template type<float, float, C::BJ, C::BK, C::NT>;
      return launch_gemm_deep<C, A, B, EP, kTailStages>(typename A::Params{pa.src, pa.ld, pa.nrows},
                                                        typename B::Params{pb.src, pb.ld, pb.nrows}, ep, Mi, Nj, K,
                                                        nsplit, st);
    }
    using A = LA_<float, float, C::BI, C::BK, C::NT>;
    using B = LB_<float, float, C::BJ, C::BK, C::NT>;
    return launch_gemm<C, A, B>(typename A::Params{pa.src, pa.ld, pa.nrows}, typename B::Params{pb.src, pb.ld, pb.nrows},
                                ep, Mi, Nj, K, nsplit, st);
  };
  auto splitk = [&](auto cfg0) {   // 32x64 tile, in-WG split-K over 2-4 waves (long K, few tiles)
    if (g_tail6) return run(typename S6Of<decltype(cfg0)>::type{});
    if (g_tail3) return run(typename S3Of<decltype(cfg0)>::type{});
    return run(cfg0);
  };
  if (mode == 0 && tiles < 192) return splitk(CFK4{});
  // bf16 path, 64x64 tiles: the operands split once at their LDS commit (hi, lo part tiles, gemm_kernel_s6l),
  // not per wave per fragment read -- the same products in the same order (AAA_TAIL_S3L=1, ablation builds: A/B)
  if (mode == 0 && g_tail3 && ab_int("AAA_TAIL_S3L", 0) && DeepLd<LA_>::fits(pa.src, pa.ld, pa.nrows) &&
      DeepLd<LB_>::fits(pb.src, pb.ld, pb.nrows) && (size_t)K * pa.ld * 4 < (1u << 31) &&
      (size_t)K * pb.ld * 4 < (1u << 31)) {
    using C = GemmCfgS3L<64, 64, 32, 2, 2, 2>;
    using A = typename DeepLd<LA_>::template type<float, float, C::BI, C::BK, C::NT>;
    using B = typename DeepLd<LB_>::template type<float, float, C::BJ, C::BK, C::NT>;
    return launch_gemm<C, A, B>(typename A::Params{pa.src, pa.ld, pa.nrows}, typename B::Params{pb.src, pb.ld, pb.nrows},
                                ep, Mi, Nj, K, nsplit, st);
  }
  if (mode == 1 || (mode == 0 && tiles >= 192)) return splitk(CF{});
#ifdef AAA_ABLATION   // the measured-slower tail tiles (AAA_HEAD_TILE 2-5)
  if (mode == 3) return splitk(CFK{});
  if (mode == 4) return splitk(CFK4{});
  if (mode == 5) return splitk(CFK4B{});
  if (g_tail3 || g_tail6) return splitk(CF32{});
  using C = CF32;
  using A = LA_<float, float, C::BI, C::BK, C::NT>;
  using B = LB_<float, float, C::BJ, C::BK, C::NT>;
  return launch_gemm<C, A, B>(typename A::Params{pa.src, pa.ld, pa.nrows}, typename B::Params{pb.src, pb.ld, pb.nrows}, ep,
                              Mi, Nj, K, nsplit, st);
#else
  return hipErrorInvalidValue;   // unreachable: mode is 0 outside ablation builds
#endif
}

// Tail GEMMs with very few columns (the actor's B=1, T=1 step: F = 1):
// D[i][j] = sum_k W[i][k] X[j][k], one wavefront per 4-row group, lanes split
// K in 16-B pieces (coalesced weight rows), butterfly reduction, then the same
// epilogue functor.  A 64x64 tile spends ~20 us on its serial K loop there;
// this reads the weight matrix once at full width.
constexpr int kSkinnyMaxCols = 8;
template <class EP, int NJ>
__global__ void __launch_bounds__(256)
k_skinny_gemm(const float* __restrict__ W, int ldw, int Mi, const float* __restrict__ X, int ldx, int Nj, int K,
              EP ep) {
  const int lane = threadIdx.x & 63;
  const int i = (blockIdx.x * 4 + (int)(threadIdx.x >> 6)) * 4;
  if (i >= Mi) return;
  float acc[4][NJ];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[r][j] = 0.f;
  for (int k = lane * 4; k < K; k += 256) {
    f32x4 w[4];
#pragma unroll
    for (int r = 0; r < 4; ++r)
      w[r] = i + r < Mi ? *reinterpret_cast<const f32x4*>(W + (size_t)(i + r) * ldw + k) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      if (j < Nj) {
        const f32x4 x = *reinterpret_cast<const f32x4*>(X + (size_t)j * ldx + k);
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[r][j] += w[r][0] * x[0] + w[r][1] * x[1] + w[r][2] * x[2] + w[r][3] * x[3];
      }
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) acc[r][j] += __shfl_xor(acc[r][j], o, 64);
  if (lane == 0)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
      if (j < Nj) ep(i, j, acc[0][j], acc[1][j], acc[2][j], acc[3][j]);
}

// Forward tail GEMM (row-major weights [Mi][K] x activations [Nj][K]): the
// skinny kernel for <= kSkinnyMaxCols columns (AAA_SKINNY=0 disables), else head_gemm.
template <class PA, class PB, class EP>
static hipError_t tail_gemm(const PA& pa, const PB& pb, const EP& ep, int Mi, int Nj, int K, hipStream_t st) {
  if (Nj <= kSkinnyMaxCols && K % 4 == 0 && pa.ld % 4 == 0 && pb.ld % 4 == 0 && ab_int("AAA_SKINNY", 1)) {
    const int blocks = cdiv(cdiv(Mi, 4), 4);
    if (Nj == 1)
      hipLaunchKernelGGL((k_skinny_gemm<EP, 1>), dim3(blocks), dim3(256), 0, st, pa.src, pa.ld, Mi, pb.src, pb.ld, Nj,
                         K, ep);
    else
      hipLaunchKernelGGL((k_skinny_gemm<EP, kSkinnyMaxCols>), dim3(blocks), dim3(256), 0, st, pa.src, pa.ld, Mi,
                         pb.src, pb.ld, Nj, K, ep);
    return hipGetLastError();
  }
  return head_gemm<LdRows, LdRows>(pa, pb, ep, Mi, Nj, K, 1, st);
}

// Batched (off-chain) conv GEMMs on the LDS-DMA ring (env AAA_PIPE_BATCHED=0: register-staged).
static bool pipe_batched() { return env_int("AAA_PIPE_BATCHED", 1) != 0; }

static int wgrad_splits(int tiles, int K, int BK) {
  int s = std::max(1, 1024 / std::max(tiles, 1));
  int maxs = std::max(1, K / (8 * BK));
  return std::min(s, maxs);
}

// One fused ConvLSTM forward step (attention.py:110-126): D[512][M] = WpXH x
// im2col([x_t | h_{t-1}]) (K = 9*192), gate math and cell update in the
// epilogue ``ep``.  Tile: AAA_FUSED_TILE, default bf16 128x128 of 4 waves
// (64x64 per wave; tools/ab_fused.sh), fp32 (small M only, e.g. the B=1 actor
// and the standalone cell) 128x64 of 8 waves.
// zpart (fp32, B*P < 8192: Layout::dhs) enables the split-K tiles 17/18: K-slice
// partials of the gate pre-activations, then the cell in gate_fwd_zx.
static int fused_splitk() { return std::max(2, std::min(4, env_int("AAA_FUSED_SPLITK", 3))); }
// Ring depth of the split-K launches (2-4 stages: tiles in flight per workgroup; their few
// k-steps per slice are latency-bound, not MFMA-bound).  AAA_SPLITK_NBUF.
static int splitk_nbuf() { return std::max(2, std::min(4, ab_int("AAA_SPLITK_NBUF", 2))); }
template <class CK, class EP, typename T>
static hipError_t step_gemm_splitk(const T* W, int ldw, int wrows, const T* src, const ConvGeo& g, int M,
                                   uint32_t src_bytes, const EP& ep, int Mi, int K, hipStream_t st, int nsplit,
                                   bool ilv = false) {
  switch (splitk_nbuf() * 2 + (ilv ? 1 : 0)) {
    case 4: return step_gemm<CK, true, T, T, EP, 2, false>(W, ldw, wrows, src, g, M, src_bytes, ep, Mi, K, st, nsplit);
    case 5: return step_gemm<CK, true, T, T, EP, 2, true>(W, ldw, wrows, src, g, M, src_bytes, ep, Mi, K, st, nsplit);
    case 6: return step_gemm<CK, true, T, T, EP, 3, false>(W, ldw, wrows, src, g, M, src_bytes, ep, Mi, K, st, nsplit);
    case 7: return step_gemm<CK, true, T, T, EP, 3, true>(W, ldw, wrows, src, g, M, src_bytes, ep, Mi, K, st, nsplit);
    case 8: return step_gemm<CK, true, T, T, EP, 4, false>(W, ldw, wrows, src, g, M, src_bytes, ep, Mi, K, st, nsplit);
    default: return step_gemm<CK, true, T, T, EP, 4, true>(W, ldw, wrows, src, g, M, src_bytes, ep, Mi, K, st, nsplit);
  }
}
template <typename T, typename GT>
static int fused_step(const T* WpXH, const T* xht, int h, int w, int M, const EpiConvLstmFwd<T, GT>& ep,
                      hipStream_t st, float* zpart = nullptr) {
  using EF = EpiConvLstmFwd<T, GT>;
  const ConvGeo g = ConvGeo{192, 192, 0, h, w, h, w, 3, 1, 1, 0}.prep();
  const uint32_t xh_bytes = (uint32_t)((size_t)M * 192 * sizeof(T));
  constexpr bool f32 = std::is_same<T, float>::value;
  // fp32 with f32_split6(): the split-product tiles 13-18 (bf16x6 on the bf16
  // MFMA): default 18 = 64x64 BK64 2-way in-WG split-K x 3 K slices + gate_fwd_zx
  // (B=1 episode step, 27x20 grid: 16.2 + 5.0 us vs 68 us for the fp32 128x64
  // tile, 23 us for 13 = 32x64 4-way in-WG; tools/gpu_episode_ab.sh), 13 where
  // there is no split-K scratch
  const int ftile = env_int("AAA_FUSED_TILE", f32 ? (f32_split6() ? (zpart ? 18 : 13) : 4) : 9);
  TimerScope tim(AAA_TIMER_FWD_STEP, st, 2.0 * M * 512 * 1728,
                 strf("%s fused [x|h] step, K=1728, AAA_FUSED_TILE %d%s [kernel: EpiConvLstmFwd]", f32 ? "fp32" : "bf16",
                      ftile, f32 && ftile >= 13 && ftile <= 16 ? " (bf16x6 split products)" : ""));
  if (ftile == 17 || ftile == 18) {   // split-K (bf16x6 split products)
    if constexpr (!f32 || !std::is_same<GT, float>::value) {
      return fail(AAA_E_ARG, "AAA_FUSED_TILE %d: fp32 split-product tiles only", ftile);
    } else {
      if (!zpart || !ep.bias) return fail(AAA_E_ARG, "AAA_FUSED_TILE %d: split-K needs B*P < 8192 (got %d)", ftile, M);
      const int ns = splitk_slices(1728, 64, fused_splitk());
      const EpiSliceT es{zpart, 512, 512, M, (size_t)M * 512};
      if (ftile == 17)
        HIPCHK((step_gemm_splitk<GemmCfgS6<32, 64, 64, 1, 2, 4>>(WpXH, 1728, 512, xht, g, M, xh_bytes, es, 512, 1728,
                                                                 st, ns)));
      else
        HIPCHK((step_gemm_splitk<GemmCfgS6<64, 64, 64, 2, 2, 2>>(WpXH, 1728, 512, xht, g, M, xh_bytes, es, 512, 1728,
                                                                 st, ns)));
      HIPCHK(gate_fwd_zx<T>(M, ep.cprev, ep.gates, ep.cnext, ep.hout, ep.xhnext, st, zpart, ns, (size_t)M * 512,
                            ep.bias));
      return AAA_OK;
    }
  }
  if (ftile >= 13 && ftile <= 16) {
    if constexpr (!f32) return fail(AAA_E_ARG, "AAA_FUSED_TILE %d: fp32 split-product tiles only", ftile);
    else if (ftile == 13)
      HIPCHK((step_gemm<GemmCfgS6<32, 64, 64, 1, 2, 4>, true>(WpXH, 1728, 512, xht, g, M, xh_bytes, ep, 512, 1728, st)));
    else if (ftile == 14)
      HIPCHK((step_gemm<GemmCfgS6<64, 64, 64, 2, 2, 2>, true>(WpXH, 1728, 512, xht, g, M, xh_bytes, ep, 512, 1728, st)));
    else if (ftile == 15)
      HIPCHK((step_gemm<GemmCfgS6<128, 64, 32, 4, 2>, true>(WpXH, 1728, 512, xht, g, M, xh_bytes, ep, 512, 1728, st)));
    else
      HIPCHK((step_gemm<GemmCfgS6<32, 32, 64, 1, 1, 4>, true, T, T, EF, 3>(WpXH, 1728, 512, xht, g, M, xh_bytes, ep,
                                                                             512, 1728, st)));
    return AAA_OK;
  }
  if (ftile == 7)
    HIPCHK((step_gemm<CfgFor<T>, true>(WpXH, 1728, 512, xht, g, M, xh_bytes, ep, 512, 1728, st)));
  else if (ftile == 8)   // 128x64, 8 waves, 3-stage ring
    HIPCHK((step_gemm<CfgSFor<T>, true, T, T, EF, 3, true>(WpXH, 1728, 512, xht, g, M, xh_bytes, ep, 512, 1728, st)));
  else if (ftile == 9)   // 128x128, 4 waves of 64x64
    HIPCHK((step_gemm<GemmCfg<T, 128, 128, 64, 2, 2>, true>(WpXH, 1728, 512, xht, g, M, xh_bytes, ep, 512, 1728, st)));
  else if (ftile == 10)   // 64x64, 4 waves, 3-stage ring
    HIPCHK((step_gemm<CfgFor<T>, true, T, T, EF, 3, true>(WpXH, 1728, 512, xht, g, M, xh_bytes, ep, 512, 1728, st)));
  else if (ftile == 11)   // 64x64, 2-way in-WG split-K (8 waves), BK64 (K = 1728 = 27 x 64)
    HIPCHK((step_gemm<GemmCfg<T, 64, 64, 64, 2, 2, 2>, true>(WpXH, 1728, 512, xht, g, M, xh_bytes, ep, 512, 1728, st)));
  else if (ftile == 12)   // 128x64, 2x2 waves of 64x32
    HIPCHK((step_gemm<GemmCfg<T, 128, 64, 64, 2, 2>, true>(WpXH, 1728, 512, xht, g, M, xh_bytes, ep, 512, 1728, st)));
  else
    HIPCHK((step_gemm<CfgSFor<T>, true>(WpXH, 1728, 512, xht, g, M, xh_bytes, ep, 512, 1728, st)));
  return AAA_OK;
}

// ---------------------------------------------- frame-resident dispatch ----
int device_cus();   // CUs of the current device
// Workgroups per frame of the bf16 frame-resident kernels (0: per-step launches).
int frames_g(const Layout& L, const char* env);
int frames_band(const Layout& L);   // band mode (recur.h BAND): kRecBands, else 0
int f32_frames(const Layout& L);    // fp32 frame-group G (recur_f32.h), else 0
int frames_bwd(const Layout& L, bool g16);
// Cst / Gt / dO slices channel-quad-major (recur.h cqm4): the frame-resident forward + BPTT pair
int cqm_layout(const Layout& L);   // recur.h kCqm* mask of the channel-quad-major slices (0: all row-major)
// h_t of all T*B frames as the attention readout reads it: the fp32 Hs slices
// (fp32 path), or the h half of XH slots 1..T (bf16 path: no fp32 copy of h_t
// is kept -- the readout reads the bf16 h the next step's conv and the weight
// gradient read, oracle/ref_cpu.py h_store).  Frame f = t*B + b sits at
// .frame(f, P) either way.
inline OSrc readout_h(const Layout& L, char* ws) {
  if (L.esz == 2) return o_bf16((const __bf16*)(ws + L.XH) + (size_t)L.B * L.P * 192 + 64, 192);
  return o_f32((const float*)(ws + L.Hs));
}
int rec_stagger(const char* env);   // start offset of half the frames, 100-MHz ticks
// fp32 path: its large GEMMs on the bf16 MFMA with three-way split operands (gemm.h SPLIT6)
bool f32_split6();

// ------------------------------------------------------- cross-unit paths --
template <typename T> int pack_impl(const Layout& L, const float* prm, char* pk, hipStream_t st);
template <typename T, typename OT>
int vision_fwd(const Layout& L, int F, const char* pk, const float* prm, const void* frames, T* Xp, T* Y1, OT* out,
               int out_ld, hipStream_t st, bool xp_full = true);
template <typename T> int forward_impl(const Layout& L, const aaa_io* io, hipStream_t st, int phases);
template <typename T>
int lstm_wgrad(const T* dz, const T* xh, int rows, int h, int w, float* gW, hipStream_t s, bool aux);
template <typename T>
int vision_bwd(const Layout& L, const char* pk, const T* dy2, const T* y1, T* xp, T* dy1, int F, float* gW2,
               float* gW1, float* gb1, hipStream_t s, const void* frames = nullptr);
template <typename T> int backward_impl(const Layout& L, const aaa_io* io, int phases, hipStream_t st);

}  // namespace aaa
