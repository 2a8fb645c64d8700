// Host runtime + C ABI (include/aaa.h): buffer layout, weight packing and the
// launch sequence of the batched unroll forward / hand-written BPTT backward.
//
// Forward (reference attention.py:298-368 over T steps from reset()):
//   conv1, conv2 over all T*B frames at once (no recurrence there), then one
//   fused ConvLSTM kernel per step (x- and h-convs as ONE implicit GEMM over
//   [x_t | h_{t-1}], gate math in the epilogue), then -- because the policy
//   core never carries state (Q1) -- the whole attention / answer / LSTMCell /
//   heads tail batched over all T*B frames.
// Backward (what autograd does for main_mp.py:77): the tail batched over T*B,
// then the only sequential part, the ConvLSTM BPTT (one dgrad GEMM per step
// with the previous step's gate backward fused in its epilogue), then all
// weight gradients as long-K GEMMs over every frame.
#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <cstdlib>
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
#include "halo.h"
#include "recur.h"
#include "recur_bwd.h"
#include "recur_f32.h"
#include "recur_bwd_f32.h"
#include "vision.h"
#include "misc.h"
#include "optim.h"
#include "actor.h"

namespace aaa {

static thread_local std::string g_err;

static int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIPCHK(expr)                                                                      \
  do {                                                                                    \
    hipError_t e_ = (expr);                                                               \
    if (e_ != hipSuccess)                                                                 \
      return fail(AAA_E_LAUNCH, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_),   \
                  __FILE__, __LINE__);                                                    \
  } while (0)

static inline size_t al256(size_t x) { return (x + 255) & ~size_t(255); }
static inline int cdiv(int a, int b) { return (a + b - 1) / b; }
static inline int conv_out(int n, int k, int s, int p) { return (n + 2 * p - k) / s + 1; }

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
  int qd, da, ans_in, ans_ld, ldy;
  size_t poff[NPARAM], psz[NPARAM], ptotal;
  size_t k_Wp1, k_Wp2, k_WdT2, k_WpX, k_WpH, k_WpXH, k_Wfr, k_Wbf, k_Wf32, k_Wb32, k_WdTl, k_bl, k_Wihhp, k_q1, k_q2, k_Q, k_W1p, k_Wihp, k_blc, k_Whd, k_bhd, packed;
  size_t Xp, Y1, XH, Hs, Cst, Gt, SQ, Am, ans, hid1, AO, LG, LC, LH;
  size_t dY, dLG, dAO, dH1, dAns, dO, dQp, dQs, dC, dZ, dZp, dY2, dY1, dxb, rflags, xpart;
  size_t gWp1, gWp2, gWpl, gbl, gW1p, gWihp, gblc, gWhd, gbhd, ws;
  // stateful core: state slots, per-step query activations, [answer | h] rows, their grads
  size_t CH, CC, AOX, Qf, q1s, q2s, dAOX, dQf, dq2s, dq1s, dhc, dcc, gWihhp;
};

static int check_ranges(Layout& L, int min_frames);

// min_frames: the frames one launch must be able to address (a step's B for
// the unroll; 1 for the frame-independent vision encoder entries).
static int build_layout(const aaa_cfg* c, Layout& L, int min_frames = 0) {
  if (!c) return fail(AAA_E_ARG, "cfg is NULL");
  if (c->B < 1 || c->T < 1) return fail(AAA_E_ARG, "B and T must be >= 1 (B=%d T=%d)", c->B, c->T);
  if (c->nq != 4 && c->nq != 8) return fail(AAA_E_ARG, "nq must be 4 or 8 (got %d)", c->nq);
  if (c->A < 1 || c->A > 256) return fail(AAA_E_ARG, "A out of range (%d)", c->A);
  if (c->dtype != AAA_F32 && c->dtype != AAA_BF16) return fail(AAA_E_ARG, "bad dtype %d", c->dtype);
  if (c->flags & ~(AAA_FLAG_STATEFUL_CORE | AAA_FLAG_FRAMES_U8)) return fail(AAA_E_ARG, "unknown flags 0x%x", c->flags);
  L.sc = (c->flags & AAA_FLAG_STATEFUL_CORE) != 0;
  L.fu8 = (c->flags & AAA_FLAG_FRAMES_U8) != 0;
  L.B = c->B; L.T = c->T; L.F = c->B * c->T; L.H = c->H; L.W = c->W;
  L.H1 = conv_out(c->H, 8, 4, 1); L.W1 = conv_out(c->W, 8, 4, 1);
  L.h = conv_out(L.H1, 4, 2, 2); L.w = conv_out(L.W1, 4, 2, 2);
  if (L.H1 < 1 || L.W1 < 1 || L.h < 1 || L.w < 1) return fail(AAA_E_ARG, "frame %dx%d too small", c->H, c->W);
  L.P1 = L.H1 * L.W1; L.P = L.h * L.w;
  L.nq = c->nq; L.A = c->A; L.dt = c->dtype; L.esz = c->dtype == AAA_BF16 ? 2 : 4;
  // dAns columns: the readout part, plus the query copy when Q depends on the state
  L.qd = 72 * L.nq; L.da = (L.sc ? 256 : 184) * L.nq; L.ans_in = 256 * L.nq + 2;
  L.ans_ld = (L.ans_in + 7) / 8 * 8;
  L.ldy = (2 * L.A + 3) / 4 * 4;
  const size_t shp[NPARAM] = {
      32 * 3 * 64, 32, 64 * 32 * 16, 64,
      128 * 64 * 9, 128, 128 * 128 * 9, 128 * 64 * 9, 128, 128 * 128 * 9,
      128 * 64 * 9, 128, 128 * 128 * 9, 128 * 64 * 9, 128, 128 * 128 * 9,
      128 * 256, 128, (size_t)L.qd * 128, (size_t)L.qd, (size_t)L.qd * L.qd, (size_t)L.qd,
      512 * (size_t)L.ans_in, 512, 256 * 512, 256,
      1024 * 256, 1024 * 256, 1024, 1024,
      (size_t)L.A * 256, (size_t)L.A, (size_t)L.A * 256, (size_t)L.A};
  size_t o = 0;
  for (int i = 0; i < NPARAM; ++i) { L.poff[i] = o; L.psz[i] = shp[i]; o += shp[i]; }
  L.ptotal = o;
  // packed weights
  size_t p = 0;
  auto take = [&](size_t bytes) { size_t r = p; p = al256(p + bytes); return r; };
  const size_t e = L.esz;
  L.k_Wp1 = take(32 * 256 * e);        // RGBx: 4th input channel zero
  L.k_Wp2 = take(64 * 512 * e);
  L.k_WdT2 = take(4 * 32 * 256 * e);   // conv2 dgrad, 4 parity classes
  L.k_WpX = take(512 * 576 * e);
  L.k_WpH = take(512 * 1152 * e);
  L.k_WpXH = take(512 * 1728 * e);     // [x | h] step operand (fused x-part, bf16 default)
  L.k_Wfr = take(e == 2 ? (size_t)16 * kRecKSP * 64 * 16 : 0);   // its fragment-order copy (frame-resident recurrence, recur.h)
  L.k_WdTl = take(192 * 4608 * e);
  L.k_Wbf = take(e == 2 ? (size_t)6 * kBwKSP * 64 * 16 : 0);   // fragment-order [W_h^T | W_x^T] (frame-resident BPTT)
  L.k_Wf32 = take(e == 4 ? (size_t)16 * kF32QP * 64 * 16 : 0);   // fp32 fragment-order [x|h] (frame-group recurrence, recur_f32.h)
  L.k_Wb32 = take(e == 4 ? (size_t)8 * kB32QP * 4 * 64 * 16 : 0);   // fp32 fragment-order W_h^T (frame-group BPTT, recur_bwd_f32.h)
  L.k_bl = take(512 * 4);
  L.k_W1p = take(512 * (size_t)L.ans_ld * 4);
  L.k_Wihp = take(1024 * 256 * 4);
  L.k_blc = take(1024 * 4);
  L.k_Whd = take((size_t)L.ldy * 256 * 4);
  L.k_bhd = take((size_t)L.ldy * 4);
  L.k_Wihhp = take(L.sc ? 1024 * 512 * 4 : 0);   // [W_ih | W_hh], rows 4u+g
  L.k_q1 = take(128 * 4);                          // the constant query (Q1) and its activations
  L.k_q2 = take((size_t)L.qd * 4);
  L.k_Q = take((size_t)L.qd * 4);
  L.packed = p;
  // workspace
  p = 0;
  const size_t F = L.F, P = L.P, M = (size_t)L.B * L.P;
  L.Xp = take(F * (L.H + 2) * (L.W + 2) * 4 * e);  // frames as zero-bordered RGBx (conv1 operand type)
  L.Y1 = take(F * L.P1 * 32 * e);
  L.XH = take((size_t)(L.T + 1) * M * 192 * e);
  L.Hs = take(F * P * 128 * 4);
  L.Cst = take((size_t)(L.T + 1) * M * 128 * 4);
  L.Gt = take(F * P * 512 * 4);
  L.SQ = take(P * L.nq * 4);
  L.Am = take(F * P * L.nq * 4);
  L.ans = take(F * L.ans_ld * 4);
  L.hid1 = take(F * 512 * 4);
  L.AO = take(F * 256 * 4);
  L.LG = take(F * 1024 * 4);
  L.LC = take(F * 256 * 4);
  L.LH = take(F * 256 * 4);
  L.dY = take(F * L.ldy * 4);
  L.dLG = take(F * 1024 * 4);
  L.dAO = take(F * 256 * 4);
  L.dH1 = take(F * 512 * 4);
  L.dAns = take(F * L.da * 4);
  L.dO = take(F * P * 128 * 4);
  L.dQp = take(F * L.qd * 4);
  L.dC = take(M * 128 * 4);
  L.dZ = take(F * P * 512 * e);                          // gate pre-activation grads, GEMM operand type
  L.dZp = take((size_t)L.T * std::max((M + 31) / 32, 2 * (size_t)L.B) * 512 * 4);  // gate-bias partials per (step, column tile | frame half)
  L.dY2 = take(F * P * 64 * e);       // conv-input grads in the operand type of the GEMMs reading them
  L.dY1 = take(F * L.P1 * 32 * e);
  L.dxb = take((size_t)L.B * 64 * 4);   // conv2 bias-gradient partials per frame (frame-resident BPTT)
  L.rflags = take((size_t)8 * L.B * 4);   // hand-off flags of the multi-workgroup frame kernels ([B][G], G <= 8)
  L.xpart = take(L.esz == 4 && rec_fits(L.h, L.w) ? b32_xpart_floats(L.B) * 4 : 0);   // fp32 frame-group BPTT exchange
  {
    const size_t sc = L.sc ? 1 : 0, B = L.B;
    L.CH = take(sc * (L.T + 1) * B * 256 * 4);
    L.CC = take(sc * (L.T + 1) * B * 256 * 4);
    L.AOX = take(sc * F * 512 * 4);
    L.Qf = take(sc * F * L.qd * 4);
    L.q1s = take(sc * F * 128 * 4);
    L.q2s = take(sc * F * L.qd * 4);
    L.dAOX = take(sc * F * 512 * 4);
    L.dQf = take(sc * F * L.qd * 4);
    L.dq2s = take(sc * F * L.qd * 4);
    L.dq1s = take(sc * F * 128 * 4);
    L.dhc = take(sc * B * 256 * 4);
    L.dcc = take(sc * B * 256 * 4);
  }
  // zero-initialised (atomic) accumulation region: one memset covers it
  L.dQs = take((size_t)L.qd * 4);
  L.gWp1 = take(32 * 256 * 4);
  L.gWp2 = take(64 * 512 * 4);
  L.gWpl = take(512 * 1728 * 4);
  L.gbl = take(512 * 4);
  L.gW1p = take(512 * (size_t)L.ans_ld * 4);
  L.gWihp = take(1024 * 256 * 4);
  L.gblc = take(1024 * 4);
  L.gWhd = take((size_t)L.ldy * 256 * 4);
  L.gbhd = take((size_t)L.ldy * 4);
  L.gWihhp = take(L.sc ? 1024 * 512 * 4 : 0);
  L.ws = p;
  return check_ranges(L, min_frames > 0 ? min_frames : L.B);
}

// The GEMM loaders address their operands through buffer descriptors with
// 32-bit byte offsets whose out-of-range sentinel is kOOB = 2^31, and index
// rows with int.  The whole-batch conv GEMMs (conv1/conv2 over all frames, the
// weight gradients, dx) therefore run in chunks of at most ``fchunk`` frames
// whose operands stay below 2 GiB (one HBM-sized batch is several launches,
// not a wrapped offset); the per-step GEMMs address one step.  A shape whose
// single step does not fit, or whose activations exceed the int element range,
// is refused (AAA_E_ARG) -- split the batch over ranks or calls.
static int check_ranges(Layout& L, int min_frames) {
  const size_t lim = size_t(1) << 31, F = (size_t)L.F, e = (size_t)L.esz;
  const size_t per_frame = std::max({(size_t)(L.H + 2) * (L.W + 2) * 4 * e,   // bordered frames (conv1 operand)
                                     (size_t)L.P1 * 32 * e,                 // Y1 / dY1
                                     (size_t)L.P * 512 * e,                 // dZ
                                     (size_t)L.P * 192 * e,                 // XH
                                     (size_t)L.P * 64 * e,                  // dY2
                                     (size_t)L.H * L.W * 3 * 4});           // input frames
  const size_t fc = (lim - 1) / per_frame;
  if (fc < (size_t)min_frames)
    return fail(AAA_E_ARG, "B=%d %dx%d: one step's operands (%zu bytes) exceed the 2 GiB a buffer descriptor "
                "addresses; split the batch (data-parallel ranks or several calls)", L.B, L.H, L.W,
                per_frame * min_frames);
  L.fchunk = (int)std::min(fc, F);
  const size_t elems[] = {F * L.P * 512, F * L.P * 128, F * (size_t)L.ans_ld, F * 1024, F * (size_t)L.P1 * 32,
                          F * (size_t)L.H * L.W * 3};
  for (size_t n : elems)
    if (n >= lim)
      return fail(AAA_E_ARG, "B=%d T=%d %dx%d: a %zu-element activation exceeds the int index range; split the batch",
                  L.B, L.T, L.H, L.W, n);
  return AAA_OK;
}

static int check_device() {
  static std::mutex mu;
  static int checked[64] = {0};  // 0 unknown, 1 ok, -1 bad
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return fail(AAA_E_DEVICE, "no HIP device");
  if (dev < 0 || dev >= 64) return AAA_OK;
  std::lock_guard<std::mutex> lk(mu);
  if (checked[dev] == 0) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return fail(AAA_E_DEVICE, "hipGetDeviceProperties failed");
    checked[dev] = strncmp(prop.gcnArchName, "gfx950", 6) == 0 ? 1 : -1;
    if (checked[dev] < 0) g_err = std::string("device is ") + prop.gcnArchName + ", need gfx950";
  }
  return checked[dev] > 0 ? AAA_OK : fail(AAA_E_DEVICE, "%s", g_err.c_str());
}

static bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// ------------------------------------------------- paired-kernel reports --
// The paired frame-resident kernels (two cooperating workgroups per frame)
// bound their partner waits (common.h pair_wait).  A timed-out wait adds 1 to
// this device's report word: pinned host memory mapped into the device, so the
// host reads it without a copy or a sync.  Every aaa_forward / aaa_backward
// entry consumes pending reports and fails with AAA_E_STRANDED (the results of
// the call that stranded are invalid); aaa_pair_status syncs a stream first.
// Allocated once per process on first use, never freed (no HIP call at exit).
static std::mutex g_pair_mu;
static int* g_pair_host = nullptr;    // [64] words, one per device ordinal
static int* g_pair_dev = nullptr;     // the same words, device-mapped
static long g_pair_spin = 1L << 24;   // partner-wait bound in polls (aaa_debug_pair_spin)

static int* pair_report(int dev) {
  std::lock_guard<std::mutex> lk(g_pair_mu);
  if (!g_pair_host) {
    void* h = nullptr;
    if (hipHostMalloc(&h, 64 * sizeof(int), hipHostMallocMapped | hipHostMallocPortable | hipHostMallocCoherent) !=
        hipSuccess)
      return nullptr;
    memset(h, 0, 64 * sizeof(int));
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) return nullptr;
    g_pair_host = (int*)h;
    g_pair_dev = (int*)d;
  }
  return g_pair_dev + dev;
}

// Pending reports of the current device (consumed).
static int pair_take() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
  std::lock_guard<std::mutex> lk(g_pair_mu);
  if (!g_pair_host) return 0;
  return __atomic_exchange_n(g_pair_host + dev, 0, __ATOMIC_ACQ_REL);
}

static int pair_check() {
  const int n = pair_take();
  return n ? fail(AAA_E_STRANDED,
                  "%d partner wait(s) of a paired frame-resident ConvLSTM kernel timed out in an earlier call on this "
                  "device: that call's outputs/gradients are invalid (the pair was not co-resident)", n)
           : AAA_OK;
}

// ------------------------------------------------------------ aux stream --
// Work that is off the sequential ConvLSTM chain (the batched x-part of the
// forward, every weight/bias gradient and dx/conv backward) is issued on a
// per-device low-priority stream, chunked every few steps and ordered against
// the caller's stream by events; the caller's stream waits for it before the
// call returns (fork/join inside each call).  Created lazily, once per device.
struct AuxStream {
  hipStream_t s = nullptr;
  hipEvent_t ev[64] = {};
  unsigned next = 0;
};
static AuxStream g_aux[64];
static std::mutex g_aux_mu;

static int env_int(const char* name, int dflt);

// Measured on C2 (round 1): running the off-chain chunks concurrently slows the
// chain's step kernels ~2x (stream priority does not keep CUs free for them),
// 6.31-6.55 ms vs 6.15 ms serial; so overlap is opt-in (AAA_OVERLAP=1).
static hipStream_t aux_stream() {
  if (env_int("AAA_OVERLAP", 0) == 0) return nullptr;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  std::lock_guard<std::mutex> lk(g_aux_mu);
  AuxStream& a = g_aux[dev];
  if (!a.s) {
    int lo = 0, hi = 0;
    (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
    if (hipStreamCreateWithPriority(&a.s, hipStreamNonBlocking, lo) != hipSuccess) { a.s = nullptr; return nullptr; }
    for (auto& e : a.ev)
      if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) { (void)hipStreamDestroy(a.s); a.s = nullptr; return nullptr; }
  }
  return a.s;
}

// Record a pooled event on ``s`` (everything enqueued on s so far).
static hipError_t record_event(hipStream_t s, hipEvent_t* out) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  {
    std::lock_guard<std::mutex> lk(g_aux_mu);
    AuxStream& a = g_aux[dev];
    *out = a.ev[a.next++ & 63];
  }
  return hipEventRecord(*out, s);
}

// ``to`` waits for everything enqueued on ``from`` so far.
static hipError_t stream_order(hipStream_t from, hipStream_t to) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  hipEvent_t ev;
  {
    std::lock_guard<std::mutex> lk(g_aux_mu);
    AuxStream& a = g_aux[dev];
    ev = a.ev[a.next++ & 63];
  }
  if ((e = hipEventRecord(ev, from)) != hipSuccess) return e;
  return hipStreamWaitEvent(to, ev, 0);
}

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
static Timers g_timers;

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

static std::string strf(const char* fmt, ...) {
  char buf[160];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  return buf;
}

// Algorithmic bytes per frame of the fused attention readout kernels (fp32):
// forward reads the frame's O rows (128 ch) and writes its map and answer row;
// backward reads O, the map and the answer grad, writes dO and dQ.
static double attn_fwd_bytes(int P, int nq, int ans_ld) { return 4.0 * (128.0 * P + nq * P + ans_ld); }
static double attn_bwd_bytes(int P, int nq) { return 4.0 * (2.0 * 128 * P + nq * P + 184.0 * nq + 72.0 * nq); }

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
static int env_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return e ? atoi(e) : dflt;
}
// Steps per off-chain chunk: the whole unroll unless overlapping, and never
// more than the frames one launch may address (Layout::fchunk).
static int chunk_steps(const Layout& L) {
  const int c = env_int("AAA_CHUNK", env_int("AAA_OVERLAP", 0) ? 4 : L.T);
  return std::max(1, std::min({c, L.T, L.fchunk / L.B}));
}
static int step_tile(long out_tiles32, const char* env, bool bptt, bool bf16 = false) {
  const int v = env_int(env, -1);
  if (v >= 0) {   // 7, 8: bf16 only; 9-11, 13, 15, 16: BPTT only; 14, 17, 18: forward only
    const bool bptt_only = v == 9 || v == 10 || v == 11 || v == 13 || v == 15 || v == 16 || (v >= 19 && v <= 24);
    if (v >= 19 && v <= 24 && !bf16) return 4;   // 19-24: bf16 BPTT tiles (fp16 gate storage)
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
  if (bptt) return out_tiles32 < 1024 ? 16 : (out_tiles32 < 1536 ? 1 : 0);
  return out_tiles32 < 1024 ? 5 : 6;
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
static int frames_fwd(const struct Layout& L);
static bool fused_x(int dt, int M) { return env_int("AAA_FUSED_X", dt == AAA_BF16 || M <= 1024 ? 1 : 0) != 0; }
static bool gates_f16(int dt, int M) {
  if (dt != AAA_BF16 || !fused_x(dt, M) || !env_int("AAA_GATES_F16", 1)) return false;
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
                            const EP& ep, int Mi, int K, hipStream_t st) {
  if constexpr (PIPE && pipe_even<CK>() && std::is_same<G, T>::value) {
    using LA = GRowsB<T, CK::BI, CK::BK, CK::NT>;
    using LB = GIm2colB<T, CK::BJ, CK::BK, CK::NT>;
    return launch_pipe<CK, LA, LB, EP, NBUF, ILV>(typename LA::Params{W, ldw, wrows},
                                                  typename LB::Params{src, g, M, src_bytes}, ep, Mi, M, K, 1, st);
  } else {
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
// 64x64, =2 the plain 32x64, =3/4/5 the 2-way / 4-way / 4-way BK128 split-K tiles.
template <template <typename, typename, int, int, int> class LA_,
          template <typename, typename, int, int, int> class LB_, class PA, class PB, class EP>
static hipError_t head_gemm(const PA& pa, const PB& pb, const EP& ep, int Mi, int Nj, int K, int nsplit,
                            hipStream_t st) {
  const int mode = env_int("AAA_HEAD_TILE", 0);
  const long tiles = (long)cdiv(Mi, 64) * cdiv(Nj, 64) * std::max(nsplit, 1);
  auto splitk = [&](auto cfg) {   // 32x64 tile, in-WG split-K over 2-4 waves (long K, few tiles)
    using C = decltype(cfg);
    using A = LA_<float, float, C::BI, C::BK, C::NT>;
    using B = LB_<float, float, C::BJ, C::BK, C::NT>;
    return launch_gemm<C, A, B>(typename A::Params{pa.src, pa.ld, pa.nrows}, typename B::Params{pb.src, pb.ld, pb.nrows},
                                ep, Mi, Nj, K, nsplit, st);
  };
  if (mode == 3) return splitk(CFK{});
  if (mode == 4) return splitk(CFK4{});
  if (mode == 5) return splitk(CFK4B{});
  if (mode == 0 && tiles < 192) return splitk(CFK4{});
  if (mode == 1 || (mode == 0 && tiles >= 192)) {
    using C = CF;
    using A = LA_<float, float, C::BI, C::BK, C::NT>;
    using B = LB_<float, float, C::BJ, C::BK, C::NT>;
    return launch_gemm<C, A, B>(typename A::Params{pa.src, pa.ld, pa.nrows}, typename B::Params{pb.src, pb.ld, pb.nrows},
                                ep, Mi, Nj, K, nsplit, st);
  }
  using C = CF32;
  using A = LA_<float, float, C::BI, C::BK, C::NT>;
  using B = LB_<float, float, C::BJ, C::BK, C::NT>;
  return launch_gemm<C, A, B>(typename A::Params{pa.src, pa.ld, pa.nrows}, typename B::Params{pb.src, pb.ld, pb.nrows}, ep,
                              Mi, Nj, K, nsplit, st);
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
  if (Nj <= kSkinnyMaxCols && K % 4 == 0 && pa.ld % 4 == 0 && pb.ld % 4 == 0 && env_int("AAA_SKINNY", 1)) {
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
template <typename T, typename GT>
static int fused_step(const T* WpXH, const T* xht, int h, int w, int M, const EpiConvLstmFwd<T, GT>& ep,
                      hipStream_t st) {
  using EF = EpiConvLstmFwd<T, GT>;
  const ConvGeo g = ConvGeo{192, 192, 0, h, w, h, w, 3, 1, 1, 0}.prep();
  const uint32_t xh_bytes = (uint32_t)((size_t)M * 192 * sizeof(T));
  const int ftile = env_int("AAA_FUSED_TILE", std::is_same<T, float>::value ? 4 : 9);
  TimerScope tim(AAA_TIMER_FWD_STEP, st, 2.0 * M * 512 * 1728,
                 strf("%s fused [x|h] step, K=1728, AAA_FUSED_TILE %d", std::is_same<T, float>::value ? "fp32" : "bf16",
                      ftile));
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

// ------------------------------------------------------------- packing ----
template <typename T>
static int pack_impl(const Layout& L, const float* prm, char* pk, hipStream_t st) {
  PackAll<T> a;
  a.c1w = prm + L.poff[C0W];
  a.c2w = prm + L.poff[C1W];
  a.Wp1 = (T*)(pk + L.k_Wp1); a.Wp2 = (T*)(pk + L.k_Wp2); a.WdT2 = (T*)(pk + L.k_WdT2);
  for (int g = 0; g < 4; ++g) {
    a.lstm.wx[g] = prm + L.poff[XI_W + 3 * g];
    a.lstm.bx[g] = prm + L.poff[XI_B + 3 * g];
    a.lstm.wh[g] = prm + L.poff[HI_W + 3 * g];
  }
  a.WpX = (T*)(pk + L.k_WpX); a.WpH = (T*)(pk + L.k_WpH); a.WdT = (T*)(pk + L.k_WdTl);
  a.WpXH = (T*)(pk + L.k_WpXH); a.bl = (float*)(pk + L.k_bl);
  F32Pack& fp = a.f32;
  fp.a0w = prm + L.poff[A0W]; fp.wih = prm + L.poff[WIH]; fp.bih = prm + L.poff[BIH]; fp.bhh = prm + L.poff[BHH];
  fp.pw = prm + L.poff[PW]; fp.vw = prm + L.poff[VW]; fp.pb = prm + L.poff[PB]; fp.vb = prm + L.poff[VB];
  fp.W1p = (float*)(pk + L.k_W1p); fp.Wihp = (float*)(pk + L.k_Wihp); fp.blc = (float*)(pk + L.k_blc);
  fp.Whd = (float*)(pk + L.k_Whd); fp.bhd = (float*)(pk + L.k_bhd);
  fp.ans_in = L.ans_in; fp.ans_ld = L.ans_ld; fp.A = L.A; fp.ldy = L.ldy;
  if (L.sc) {
    fp.whh = prm + L.poff[WHH];
    fp.Wihhp = (float*)(pk + L.k_Wihhp);
  }
  HIPCHK(pack_all<T>(a, st));   // conv1, conv2, conv2 dgrad classes, ConvLSTM layouts, fp32 tail: one launch
  if constexpr (!std::is_same<T, float>::value) {   // fragment orders of the frame-resident kernels (read WpXH / WdT)
    HIPCHK(pack_wfrag((const __bf16*)(pk + L.k_WpXH), (__bf16*)(pk + L.k_Wfr), st));
    HIPCHK(pack_wbfrag((const __bf16*)(pk + L.k_WdTl), (__bf16*)(pk + L.k_Wbf), st));
  } else {   // the fp32 frame-group recurrence's fragment order (recur_f32.h)
    HIPCHK(pack_wf32((const float*)(pk + L.k_WpXH), (float*)(pk + L.k_Wf32), st));
    HIPCHK(pack_wb32((const float*)(pk + L.k_WdTl), (float*)(pk + L.k_Wb32), st));
  }
  HIPCHK(query_pack(prm + L.poff[Q0B], prm + L.poff[Q2W], prm + L.poff[Q2B], prm + L.poff[Q4W], prm + L.poff[Q4B], L.nq,
                    (float*)(pk + L.k_q1), (float*)(pk + L.k_q2), (float*)(pk + L.k_Q), st));
  return AAA_OK;
}

// Vision encoder over F frames (VisionNetwork.vision_cnn, attention.py:155-170,
// on X.transpose(1,3), :179 -- Q3): frames (F,H,W,3) -> zero-bordered RGBx
// image Xp -> conv 8/4/1 -> Y1 (F,H1,W1,32) -> conv 4/2/2 -> out (F,h,w,64) at
// row pitch out_ld (the ConvLSTM operand slots, or a plain output), no
// activation in between.  Packed conv weights at L.k_Wp1 / L.k_Wp2, biases
// from the flat params (state_dict order: the vision tensors come first).
template <typename T, typename OT>
static int vision_fwd_chunk(const Layout& L, int F, const char* pk, const float* prm, const void* frames, T* Xp, T* Y1,
                      OT* out, int out_ld, hipStream_t st) {
  using C = CfgFor<T>;
  constexpr int NT = C::NT;
  const int P = L.P;
  bool banded = false;   // bf16 frames too large for the frame-resident encoder: the banded conv1 (vision.h)
  if constexpr (std::is_same<T, __bf16>::value) {
    if (band_fits(L.H, L.W, L.H1, L.W1) && env_int("AAA_VIS_BAND", 1)) {
      const VisBandParams bp{frames, (const __bf16*)(pk + L.k_Wp1), prm + L.poff[C0B], Xp, Y1, F, L.H, L.W, L.H1, L.W1};
      HIPCHK(L.fu8 ? vision_conv1_band<uint8_t>(bp, st) : vision_conv1_band<float>(bp, st));
      banded = true;
    }
  }
  if (!banded) {  // conv1 (attention.py:156-162): frames -> zero-bordered RGBx (Cin 4, pad 1 stored) -> Y1
    if (L.fu8) HIPCHK((frames_rgbx<T, uint8_t>(F, L.H, L.W, (const uint8_t*)frames, Xp, st)));
    else HIPCHK((frames_rgbx<T, float>(F, L.H, L.W, (const float*)frames, Xp, st)));
    // LDS-DMA ring, 32x128 tile over 4 waves (tools/ubench/conv_cfg: 62 vs 90 us register-staged)
    constexpr int BKc = std::is_same<T, float>::value ? 32 : 64;
    EpiStoreT<T> ep{Y1, 32, 32, F * L.P1, prm + L.poff[C0B], 0};
    auto conv1 = [&](auto cfg) -> int {
      using CP = decltype(cfg);
      using PA = GRowsB<T, CP::BI, CP::BK, CP::NT>;
      using PB = GIm2colB<T, CP::BJ, CP::BK, CP::NT>;
      HIPCHK((launch_pipe<CP, PA, PB, EpiStoreT<T>, 2>(
          typename PA::Params{(const T*)(pk + L.k_Wp1), 256, 32},
          typename PB::Params{Xp, ConvGeo{4, 4, 0, L.H + 2, L.W + 2, L.H1, L.W1, 8, 4, 0, 0}.prep(), F * L.P1,
                              (uint32_t)((size_t)F * (L.H + 2) * (L.W + 2) * 4 * L.esz)},
          ep, 32, F * L.P1, 256, 1, st)));
      return AAA_OK;
    };
    // K = 256 is four BK steps: a wider column tile does more MFMA work per DMA round trip (A/B: AAA_CONV1_TILE)
    const int c1t = env_int("AAA_CONV1_TILE", 0);
    const int rc = c1t == 1 ? conv1(GemmCfg<T, 32, 256, BKc, 1, 4>{}) : conv1(GemmCfg<T, 32, 128, BKc, 1, 4>{});
    if (rc) return rc;
  }
  if constexpr (std::is_same<T, __bf16>::value && std::is_same<OT, __bf16>::value) {
    // after the banded conv1: the banded conv2 (vision.h), Y1 rows staged in LDS per band
    if (banded && band2_fits(L.H1, L.W1, L.h, L.w) && env_int("AAA_VIS_BAND2", 1)) {
      const VisBand2Params bp{Y1, (const __bf16*)(pk + L.k_Wp2), prm + L.poff[C1B], out, out_ld, F, L.H1, L.W1, L.h, L.w};
      HIPCHK(vision_conv2_band(bp, st));
      return AAA_OK;
    }
  }
  {  // conv2 (attention.py:163-169): Y1 -> out
    using LA = LdRowsB<T, T, C::BI, C::BK, NT>;
    typename LA::Params pa{(const T*)(pk + L.k_Wp2), 512, 64};
    const ConvGeo g = ConvGeo{32, 32, 0, L.H1, L.W1, L.h, L.w, 4, 2, 2, 0}.prep();
    EpiStoreT<OT> ep{out, out_ld, 64, F * P, prm + L.poff[C1B], 0};
    const uint32_t y1b = (uint32_t)((size_t)F * L.P1 * 32 * L.esz);
    if constexpr (32 % C::BK == 0) {   // LDS-DMA ring (tools/ubench/conv_cfg: 62 vs 67 us)
      HIPCHK((step_gemm<C, true>((const T*)(pk + L.k_Wp2), 512, 64, (const T*)Y1, g, F * P, y1b, ep, 64, 512, st)));
    } else if (pipe_batched()) {   // bf16: a BK=32 ring, one 4x4 tap row's 32 channels per K tile
      HIPCHK((step_gemm<GemmCfg<T, 64, 128, 32, 2, 2>, true>((const T*)(pk + L.k_Wp2), 512, 64, (const T*)Y1, g,
                                                           F * P, y1b, ep, 64, 512, st)));
    } else {
      using LB = LdIm2col<T, T, C::BJ, C::BK, NT, true>;
      HIPCHK((launch_gemm<C, LA, LB>(pa, typename LB::Params{Y1, g, F * P}, ep, 64, F * P, 512, 1, st)));
    }
  }
  return AAA_OK;
}

static int device_cus();

template <typename T, typename OT>
static int vision_fwd(const Layout& L, int F, const char* pk, const float* prm, const void* frames, T* Xp, T* Y1,
                      OT* out, int out_ld, hipStream_t st) {
  if constexpr (std::is_same<T, __bf16>::value && std::is_same<OT, __bf16>::value) {
    // bf16: the frame-resident encoder (vision.h), one launch; AAA_VIS_FRAMES=0 -> the layered kernels
    if (vis_fits(L.H, L.W, L.H1, L.W1, L.h, L.w) && env_int("AAA_VIS_FRAMES", 1)) {
      VisFwdParams vp{frames, (const __bf16*)(pk + L.k_Wp1), prm + L.poff[C0B], (const __bf16*)(pk + L.k_Wp2),
                      prm + L.poff[C1B], Xp, Y1, out, out_ld, F, L.H, L.W, L.H1, L.W1, L.h, L.w};
      HIPCHK(L.fu8 ? vision_fwd_frames<uint8_t>(vp, device_cus(), st) : vision_fwd_frames<float>(vp, device_cus(), st));
      return AAA_OK;
    }
  }
  for (int f0 = 0; f0 < F; f0 += L.fchunk) {   // descriptor-sized frame chunks (check_ranges)
    const int n = std::min(L.fchunk, F - f0);
    const int rc = vision_fwd_chunk<T, OT>(L, n, pk, prm,
                                           (const char*)frames + (size_t)f0 * L.H * L.W * 3 * (L.fu8 ? 1 : 4),
                                           Xp + (size_t)f0 * (L.H + 2) * (L.W + 2) * 4, Y1 + (size_t)f0 * L.P1 * 32,
                                           out + (size_t)f0 * L.P * out_ld, out_ld, st);
    if (rc) return rc;
  }
  return AAA_OK;
}

// ------------------------------------------------------------- forward ----
static int device_cus() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    hipDeviceProp_t prop;
    cus = (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess) ? prop.multiProcessorCount
                                                                                                 : 256;
  }
  return cus;
}
// Workgroups per frame of the frame-resident kernels (0: per-step launches):
// 1 once the batch fills most of the CUs, 2 (paired workgroups) while two per
// frame still fit the chip, else the per-step kernels.  AAA_FRAMES_FWD /
// AAA_FRAMES_BWD = 0 / 1 / 2 force it.
static int frames_g(const Layout& L, const char* env) {
  if (L.dt != AAA_BF16 || !rec_fits(L.h, L.w)) return 0;
  const int cus = device_cus();
  const int v = env_int(env, L.B >= (cus * 5) / 8 ? 1 : (L.B >= 32 && 2 * L.B <= cus ? 2 : 0));
  return v == 1 ? 1 : (v == 2 && 2 * L.B <= cus ? 2 : 0);
}
static int frames_fwd(const Layout& L) { return frames_g(L, "AAA_FRAMES_FWD"); }
// bf16 forward on the band-mode frame-resident kernel (recur.h BAND): grids too
// large for one workgroup's images (168x168 frames: 21x21) split into kRecBands
// row bands, one workgroup each, when B * kRecBands workgroups fit one
// residency wave (config 5: B = 64 per GPU -> 256).  AAA_FRAMES_BAND = 0 keeps
// the per-step launches.
static int frames_band(const Layout& L) {
  if (L.dt != AAA_BF16 || rec_fits(L.h, L.w) || !rec_band_fits(L.h, L.w) || !env_int("AAA_FRAMES_BAND", 1)) return 0;
  return 8 * kRecBands * ((L.B + 7) / 8) <= device_cus() ? kRecBands : 0;
}
// fp32 ConvLSTM forward on the frame-group kernel (recur_f32.h): G workgroups
// per frame for all T steps, once B * G fills at least half the CUs in one
// residency wave (C2: B = 32, G = 8 on 256 CUs).  AAA_F32_FRAMES = 0 keeps the
// per-step launches (A/B and parity of both paths); 8 / 4 force that G.
static int f32_frames(const Layout& L) {
  if (L.dt != AAA_F32 || !f32_rec_fits(L.h, L.w)) return 0;
  const int v = env_int("AAA_F32_FRAMES", 1), cus = device_cus();
  if (v == 8 || v == 4) return f32_grid(L.B, v) <= cus ? v : 0;   // forced G (tests, A/B)
  if (v != 1) return 0;
  const int G = f32_rec_g(L.B, cus);
  return G && 2 * G * L.B >= cus ? G : 0;
}
// The BPTT chain on the frame-resident kernels (recur_bwd.h; fp16 gate storage):
// workgroups per frame as the forward's (AAA_FRAMES_BWD = 0 / 1 / 2 forces it).
static int frames_bwd(const Layout& L, bool g16) { return g16 ? frames_g(L, "AAA_FRAMES_BWD") : 0; }

template <typename T>
static int forward_tail(const Layout& L, const aaa_io* io, hipStream_t st);

template <typename T>
static int forward_impl(const Layout& L, const aaa_io* io, hipStream_t st) {
  using C = CfgFor<T>;
  char* ws = (char*)io->workspace;
  const char* pk = (const char*)io->packed;
  const float* prm = io->params;
  auto Wf = [&](size_t off) { return (float*)(ws + off); };
  auto Wt = [&](size_t off) { return (T*)(ws + off); };
  const int F = L.F, M = L.B * L.P;

  {  // conv1 + conv2 over all T*B frames -> XH[:, :, 0:64] of every slot
    const int rc = vision_fwd<T, T>(L, F, pk, prm, io->frames, Wt(L.Xp), Wt(L.Y1), Wt(L.XH), 192, st);
    if (rc) return rc;
  }
  // initial state (reset(): zeros, attention.py:142-149) or carried state
  HIPCHK(state_to_xh<T>(M, io->h0, Wt(L.XH), st));
  if (io->c0) HIPCHK(hipMemcpyAsync(Wf(L.Cst), io->c0, (size_t)M * 128 * 4, hipMemcpyDeviceToDevice, st));
  else HIPCHK(hipMemsetAsync(Wf(L.Cst), 0, (size_t)M * 128 * 4, st));
  if constexpr (std::is_same<T, float>::value) {
    if (const int G = f32_frames(L)) {   // one frame-group launch for all T steps, x-part included (recur_f32.h)
      HIPCHK(hipMemsetAsync(ws + L.rflags, 0, (size_t)G * L.B * 4, st));
      int dev = 0;
      HIPCHK(hipGetDevice(&dev));
      int* rep = pair_report(dev);
      if (!rep) return fail(AAA_E_LAUNCH, "cannot map the frame-group report word");
      RecF32Params rp{(const float*)(pk + L.k_Wf32), (const float*)(pk + L.k_bl), Wf(L.XH), Wf(L.Cst), Wf(L.Hs),
                      Wf(L.Gt), (int*)(ws + L.rflags), rep, (int)g_pair_spin, L.T, L.B, L.h, L.w, L.P,
                      io->h0 ? 0 : 1, {}};
      {
        TimerScope tim(AAA_TIMER_FWD_STEP, st, 2.0 * M * 512 * (576.0 * L.T + 1152.0 * (L.T - (io->h0 ? 0 : 1))),
                       strf("fp32 frame-group [x|h] recurrence, %d steps per launch, %d WG per frame", L.T, G));
        HIPCHK(convlstm_fwd_f32(rp, G, st));
      }
      return forward_tail<T>(L, io, st);
    }
  }
  // bf16: the x-part rides in each step's GEMM (K over the whole XH slot,
  // [x_t | h_{t-1}], bias in the epilogue): no batched x-part GEMM and no
  // fp32 x-part round trip through HBM (tools/ubench/bf16_tiles: the step's
  // epilogue traffic, not its MFMAs, is half its time).  AAA_FUSED_X=0/1 overrides.
  if (fused_x(L.dt, M)) {
    const T* WpXH = (const T*)(pk + L.k_WpXH);
    // bf16: 128x128 tiles of 4 waves (64x64 per wave: twice the MFMA work per
    // fragment read of the 128x64 8-wave tile) -- C3 94.7 -> 81-83 us, C4 51.5 ->
    // 44.6 us, C5 90.7 -> 78.6-79.5 us per step (tools/ab_fused.sh); fp32 (only
    // small M, e.g. the B=1 actor, fuses the x-part): 128x64 8 waves.
    auto steps = [&](auto gtag) -> int {
      using GT = decltype(gtag);
      if constexpr (!std::is_same<T, float>::value) {
        if (const int NBd = frames_band(L)) {   // one band-mode launch for all T steps (recur.h BAND)
          HIPCHK(hipMemsetAsync(ws + L.rflags, 0, (size_t)NBd * L.B * 4, st));
          int dev = 0;
          HIPCHK(hipGetDevice(&dev));
          int* rep = pair_report(dev);
          if (!rep) return fail(AAA_E_LAUNCH, "cannot map the band-mode report word");
          RecFwdParams<GT> rp{(const __bf16*)(pk + L.k_Wfr), (const float*)(pk + L.k_bl), Wt(L.XH), Wf(L.Cst),
                              Wf(L.Hs), (GT*)(ws + L.Gt), (int*)(ws + L.rflags), L.T, L.B, L.h, L.w, L.P,
                              rep, (int)g_pair_spin};
          TimerScope tim(AAA_TIMER_FWD_STEP, st, 2.0 * M * 512 * 1728 * L.T,
                         strf("bf16 band-mode frame-resident [x|h] recurrence, %d steps per launch, %d bands per frame",
                              L.T, NBd));
          HIPCHK(convlstm_fwd_frames_band<GT>(rp, st));
          return AAA_OK;
        }
        if (const int G = frames_fwd(L)) {   // one frame-resident launch for all T steps (recur.h)
          int* rep = nullptr;
          if (G == 2) {
            HIPCHK(hipMemsetAsync(ws + L.rflags, 0, (size_t)2 * L.B * 4, st));
            int dev = 0;
            HIPCHK(hipGetDevice(&dev));
            if (!(rep = pair_report(dev))) return fail(AAA_E_LAUNCH, "cannot map the paired-kernel report word");
          }
          RecFwdParams<GT> rp{(const __bf16*)(pk + L.k_Wfr), (const float*)(pk + L.k_bl), Wt(L.XH), Wf(L.Cst),
                              Wf(L.Hs), (GT*)(ws + L.Gt), (int*)(ws + L.rflags), L.T, L.B, L.h, L.w, L.P,
                              rep, (int)g_pair_spin};
          TimerScope tim(AAA_TIMER_FWD_STEP, st, 2.0 * M * 512 * 1728 * L.T,
                         strf("bf16 frame-resident [x|h] recurrence, %d steps per launch, %d WG per frame", L.T, G));
          HIPCHK(convlstm_fwd_frames<GT>(rp, G, st));
          return AAA_OK;
        }
      }
      for (int t = 0; t < L.T; ++t) {   // ConvLSTM (attention.py:110-126), x- and h-part together
        EpiConvLstmFwd<T, GT> ep{Wf(L.Cst) + (size_t)t * M * 128, Wf(L.Cst) + (size_t)(t + 1) * M * 128,
                                 Wf(L.Hs) + (size_t)t * M * 128, Wt(L.XH) + (size_t)(t + 1) * M * 192,
                                 (GT*)(ws + L.Gt) + (size_t)t * M * 512, M, (const float*)(pk + L.k_bl)};
        const int rc = fused_step<T, GT>(WpXH, Wt(L.XH) + (size_t)t * M * 192, L.h, L.w, M, ep, st);
        if (rc) return rc;
      }
      return AAA_OK;
    };
    const int rc = gates_f16(L.dt, M) ? steps(_Float16{}) : steps(float{});
    if (rc) return rc;
    return forward_tail<T>(L, io, st);
  }
  // x-part of the ConvLSTM steps (not recurrent): Gt <- Wx * x_t + b, in
  // chunks of ``cs`` steps on the aux stream; step t waits only for its chunk.
  hipStream_t ax = aux_stream();
  const int cs = chunk_steps(L);
  hipStream_t xs = ax ? ax : st;
  if (ax) HIPCHK(stream_order(st, ax));
  auto xpart = [&](int lo, int hi) -> int {
    // 64x64 tiles (128x128 measured slower: K is only 576)
    const ConvGeo g = ConvGeo{64, 192, 0, L.h, L.w, L.h, L.w, 3, 1, 1, 0}.prep();
    const int rows = (hi - lo) * M;
    EpiStoreT<float> ep{Wf(L.Gt) + (size_t)lo * M * 512, 512, 512, rows, (const float*)(pk + L.k_bl), 0};
    const T* WpX = (const T*)(pk + L.k_WpX);
    const T* xs0 = Wt(L.XH) + (size_t)lo * M * 192;
    const uint32_t xb = (uint32_t)((size_t)(hi - lo) * M * 192 * L.esz);
    using EX = EpiStoreT<float>;
    switch (pipe_batched() ? env_int("AAA_XPART_TILE", 0) : -1) {   // A/B: tools/ab_batched.sh
      case -1: HIPCHK((step_gemm<CfgFor<T>, false>(WpX, 576, 512, xs0, g, rows, xb, ep, 512, 576, xs))); break;
      case 1: HIPCHK((step_gemm<Cfg64For<T>, true>(WpX, 576, 512, xs0, g, rows, xb, ep, 512, 576, xs))); break;
      case 2: HIPCHK((step_gemm<CfgFor<T>, true, T, T, EX, 3, true>(WpX, 576, 512, xs0, g, rows, xb, ep, 512, 576, xs))); break;
      case 3: HIPCHK((step_gemm<CfgJFor<T>, true>(WpX, 576, 512, xs0, g, rows, xb, ep, 512, 576, xs))); break;
      case 4: HIPCHK((step_gemm<CfgSFor<T>, true>(WpX, 576, 512, xs0, g, rows, xb, ep, 512, 576, xs))); break;
      case 5:
        HIPCHK((step_gemm<GemmCfg<T, 128, 128, 32, 2, 2>, true>(WpX, 576, 512, xs0, g, rows, xb, ep, 512, 576, xs)));
        break;
      default: HIPCHK((step_gemm<CfgFor<T>, true>(WpX, 576, 512, xs0, g, rows, xb, ep, 512, 576, xs))); break;
    }
    return AAA_OK;
  };
  hipEvent_t xev[64];
  const int nchunks = (L.T + cs - 1) / cs;
  if (ax && nchunks > 48) return fail(AAA_E_ARG, "too many overlap chunks (T=%d, AAA_CHUNK=%d)", L.T, cs);
  for (int k = 0; k < nchunks; ++k) {
    int rc = xpart(k * cs, std::min(L.T, (k + 1) * cs));
    if (rc) return rc;
    if (ax) HIPCHK(record_event(ax, &xev[k]));
  }
  const int fwd_tile = step_tile((long)(512 / 32) * cdiv(M, 32), "AAA_STEP_TILE", false);
  const uint32_t xh_bytes = (uint32_t)((size_t)M * 192 * L.esz);  // one step slice of XH
  for (int t = 0; t < L.T; ++t) {  // ConvLSTM recurrence (attention.py:110-126): h-part only
    if (ax && t % cs == 0) HIPCHK(hipStreamWaitEvent(st, xev[t / cs], 0));   // x-part of steps [t, t+cs) done
    if (t == 0 && !io->h0) {       // zero state: gates come from the x-part alone
      HIPCHK(gate_fwd_zx<T>(M, Wf(L.Cst), Wf(L.Gt), Wf(L.Cst) + (size_t)M * 128, Wf(L.Hs), Wt(L.XH) + (size_t)M * 192,
                            st));
      continue;
    }
    EpiConvLstmFwd<T> ep{Wf(L.Cst) + (size_t)t * M * 128, Wf(L.Cst) + (size_t)(t + 1) * M * 128,
                         Wf(L.Hs) + (size_t)t * M * 128, Wt(L.XH) + (size_t)(t + 1) * M * 192,
                         Wf(L.Gt) + (size_t)t * M * 512, M};
    const ConvGeo g = ConvGeo{128, 192, 64, L.h, L.w, L.h, L.w, 3, 1, 1, 0}.prep();
    TimerScope tim(AAA_TIMER_FWD_STEP, st, 2.0 * M * 512 * 1152, strf("%s h-part step (x-part batched), K=1152, tile %d", std::is_same<T, float>::value ? "fp32" : "bf16", fwd_tile));
    const T* WpH = (const T*)(pk + L.k_WpH);
    const T* xh = Wt(L.XH) + (size_t)t * M * 192;
    hipError_t e;
    switch (fwd_tile) {
      case 1: case 2: e = step_gemm<CfgKFor<T>, false>(WpH, 1152, 512, xh, g, M, xh_bytes, ep, 512, 1152, st); break;
      case 3: e = step_gemm<Cfg64For<T>, false>(WpH, 1152, 512, xh, g, M, xh_bytes, ep, 512, 1152, st); break;
      case 4:   // 128x64, 8 waves
        e = step_gemm<CfgSFor<T>, true>(WpH, 1152, 512, xh, g, M, xh_bytes, ep, 512, 1152, st);
        break;
      case 7: e = step_gemm<C, true>(WpH, 1152, 512, xh, g, M, xh_bytes, ep, 512, 1152, st); break;
      case 5: e = step_gemm<CfgKFor<T>, true>(WpH, 1152, 512, xh, g, M, xh_bytes, ep, 512, 1152, st); break;
      case 6: e = step_gemm<Cfg64For<T>, true>(WpH, 1152, 512, xh, g, M, xh_bytes, ep, 512, 1152, st); break;
      case 12:   // 32x64 BK64, 2-way in-WG split-K, 3-stage ring
        e = step_gemm<CfgKFor<T>, true, T, T, EpiConvLstmFwd<T>, 3, true>(WpH, 1152, 512, xh, g, M, xh_bytes, ep, 512,
                                                                          1152, st);
        break;
      case 14:   // 32x32 BK64, 4-way in-WG split-K, 3-stage ring
        e = step_gemm<GemmCfg<T, 32, 32, 64, 1, 1, 4>, true, T, T, EpiConvLstmFwd<T>, 3, true>(WpH, 1152, 512, xh, g, M,
                                                                                              xh_bytes, ep, 512, 1152, st);
        break;
      case 17:   // 64x32 BK64, 2-way in-WG split-K, 3-stage ring
        e = step_gemm<GemmCfg<T, 64, 32, 64, 2, 1, 2>, true, T, T, EpiConvLstmFwd<T>, 3, true>(WpH, 1152, 512, xh, g, M,
                                                                                              xh_bytes, ep, 512, 1152, st);
        break;
      case 25:   // 64x64 BK64, 2-way in-WG split-K (8 waves), 2-stage ring
        e = step_gemm<GemmCfg<T, 64, 64, 64, 2, 2, 2>, true>(WpH, 1152, 512, xh, g, M, xh_bytes, ep, 512, 1152, st);
        break;
      case 26:   // 64x64 BK128, 2-way in-WG split-K (8 waves), 2-stage ring
        e = step_gemm<GemmCfg<T, 64, 64, 128, 2, 2, 2>, true>(WpH, 1152, 512, xh, g, M, xh_bytes, ep, 512, 1152, st);
        break;
      case 18:   // 64x64 BK64, 2x2 waves, 3-stage ring
        e = step_gemm<Cfg64For<T>, true, T, T, EpiConvLstmFwd<T>, 3, true>(WpH, 1152, 512, xh, g, M, xh_bytes, ep, 512,
                                                                           1152, st);
        break;
      default: e = step_gemm<C, false>(WpH, 1152, 512, xh, g, M, xh_bytes, ep, 512, 1152, st); break;
    }
    HIPCHK(e);
  }
  return forward_tail<T>(L, io, st);
}

// Stateful policy core (AAA_FLAG_STATEFUL_CORE; the reference's else branch,
// attention.py:324-331, 356-358): per step t, over the B frames of that step,
//   Q_t = QueryNetwork(h_{t-1}) -> attention readout with the per-frame Q_t ->
//   answer MLP -> LSTMCell([answer | h_{t-1}], c_{t-1}) -> (h_t, c_t).
// State slots CH/CC[t] hold (h, c) entering step t (slot 0 = io->core_*0 or
// zeros); the LSTMCell epilogue also writes h_t into step t+1's [answer | h]
// GEMM row, so each step is five small GEMMs and one attention launch.  The
// heads then run batched over all frames on CH[1..T].
static int forward_tail_stateful(const Layout& L, const aaa_io* io, hipStream_t st) {
  constexpr int NTF = CF::NT;
  char* ws = (char*)io->workspace;
  const char* pk = (const char*)io->packed;
  const float* prm = io->params;
  auto Wf = [&](size_t off) { return (float*)(ws + off); };
  const int B = L.B, P = L.P, qd = L.qd;
  const size_t sB = (size_t)B * 256 * 4;
  float *CH = Wf(L.CH), *CC = Wf(L.CC), *AOX = Wf(L.AOX);
  if (io->core_h0) HIPCHK(hipMemcpyAsync(CH, io->core_h0, sB, hipMemcpyDeviceToDevice, st));
  else HIPCHK(hipMemsetAsync(CH, 0, sB, st));
  if (io->core_c0) HIPCHK(hipMemcpyAsync(CC, io->core_c0, sB, hipMemcpyDeviceToDevice, st));
  else HIPCHK(hipMemsetAsync(CC, 0, sB, st));
  HIPCHK(hipMemcpy2DAsync(AOX + 256, 512 * 4, CH, 256 * 4, 256 * 4, B, hipMemcpyDeviceToDevice, st));
  using LRf = LdRows<float, float, CF::BI, CF::BK, NTF>;
  using LRfj = LdRows<float, float, CF::BJ, CF::BK, NTF>;
  for (int t = 0; t < L.T; ++t) {
    const size_t f0 = (size_t)t * B;
    float* q1 = Wf(L.q1s) + f0 * 128;
    float* q2 = Wf(L.q2s) + f0 * qd;
    float* Qt = Wf(L.Qf) + f0 * qd;
    {  // QueryNetwork(prev_output = h_{t-1}) (attention.py:184-198, 331)
      LRf::Params pa{prm + L.poff[Q0W], 256, 128};
      LRfj::Params pb{CH + f0 * 256, 256, B};
      EpiStoreT<float> ep{q1, 128, 128, B, prm + L.poff[Q0B], 1};
      HIPCHK((tail_gemm(pa, pb, ep, 128, B, 256, st)));
    }
    {
      LRf::Params pa{prm + L.poff[Q2W], 128, qd};
      LRfj::Params pb{q1, 128, B};
      EpiStoreT<float> ep{q2, qd, qd, B, prm + L.poff[Q2B], 1};
      HIPCHK((tail_gemm(pa, pb, ep, qd, B, 128, st)));
    }
    {
      LRf::Params pa{prm + L.poff[Q4W], qd, qd};
      LRfj::Params pb{q2, qd, B};
      EpiStoreT<float> ep{Qt, qd, qd, B, prm + L.poff[Q4B], 0};
      HIPCHK((tail_gemm(pa, pb, ep, qd, B, qd, st)));
    }
    // attention readout with this step's per-frame queries (basis logits in-kernel)
    {
      TimerScope tim(AAA_TIMER_ATTN_FWD, st, (double)B * attn_fwd_bytes(P, L.nq, L.ans_ld), "k_attn_fwd, per-frame query (stateful core)");
      HIPCHK(attn_fwd(Wf(L.Hs) + f0 * P * 128, io->basis, Qt, nullptr, io->prev_reward ? io->prev_reward + f0 : nullptr,
                      io->prev_action ? io->prev_action + f0 : nullptr, B, P, L.nq, Wf(L.Am) + f0 * P * L.nq,
                      Wf(L.ans) + f0 * L.ans_ld, L.ans_ld, st, qd));
    }
    {  // answer_processor.0 + ReLU
      LRf::Params pa{(const float*)(pk + L.k_W1p), L.ans_ld, 512};
      LRfj::Params pb{Wf(L.ans) + f0 * L.ans_ld, L.ans_ld, B};
      EpiStoreT<float> ep{Wf(L.hid1) + f0 * 512, 512, 512, B, prm + L.poff[A0B], 1};
      HIPCHK((tail_gemm(pa, pb, ep, 512, B, L.ans_ld, st)));
    }
    {  // answer_processor.2 -> the answer half of this step's [answer | h_{t-1}] rows
      LRf::Params pa{prm + L.poff[A2W], 512, 256};
      LRfj::Params pb{Wf(L.hid1) + f0 * 512, 512, B};
      EpiStoreT<float> ep{AOX + f0 * 512, 512, 256, B, prm + L.poff[A2B], 0};
      HIPCHK((tail_gemm(pa, pb, ep, 256, B, 512, st)));
    }
    {  // policy_core LSTMCell from (h_{t-1}, c_{t-1}) (attention.py:356-358)
      LRf::Params pa{(const float*)(pk + L.k_Wihhp), 512, 1024};
      LRfj::Params pb{AOX + f0 * 512, 512, B};
      EpiLstmCellFwdS ep{(const float*)(pk + L.k_blc), Wf(L.LG) + f0 * 1024, CC + f0 * 256, CC + (f0 + B) * 256,
                         CH + (f0 + B) * 256, t + 1 < L.T ? AOX + (f0 + B) * 512 + 256 : nullptr, B};
      HIPCHK((tail_gemm(pa, pb, ep, 1024, B, 512, st)));
    }
  }
  if (io->attn)
    HIPCHK(hipMemcpyAsync(io->attn, Wf(L.Am), (size_t)L.F * P * L.nq * 4, hipMemcpyDeviceToDevice, st));
  return AAA_OK;
}

// Everything after the ConvLSTM: query, attention readout, answer MLP,
// LSTMCell, heads (all batched over the T*B frames, Q1) and state outputs.
template <typename T>
static int forward_tail(const Layout& L, const aaa_io* io, hipStream_t st) {
  constexpr int NTF = CF::NT;
  char* ws = (char*)io->workspace;
  const char* pk = (const char*)io->packed;
  const float* prm = io->params;
  auto Wf = [&](size_t off) { return (float*)(ws + off); };
  const int F = L.F, P = L.P, M = L.B * L.P;
  if (L.sc) {   // stateful core: the tail runs step by step
    const int rc = forward_tail_stateful(L, io, st);
    if (rc) return rc;
  } else {
  // constant query (Q1) + fused attention readout over all T*B frames
  const float* Qc = (const float*)(pk + L.k_Q);
  HIPCHK(query_sq(io->basis, Qc, P, L.nq, Wf(L.SQ), st));
  {
    TimerScope tim(AAA_TIMER_ATTN_FWD, st, (double)F * attn_fwd_bytes(P, L.nq, L.ans_ld), "k_attn_fwd, 1 WG per frame");
    HIPCHK(attn_fwd(Wf(L.Hs), io->basis, Qc, Wf(L.SQ), io->prev_reward, io->prev_action, F, P, L.nq, Wf(L.Am),
                    Wf(L.ans), L.ans_ld, st));
  }
  if (io->attn) HIPCHK(hipMemcpyAsync(io->attn, Wf(L.Am), (size_t)F * P * L.nq * 4, hipMemcpyDeviceToDevice, st));
  using LRf = LdRows<float, float, CF::BI, CF::BK, NTF>;
  using LRfj = LdRows<float, float, CF::BJ, CF::BK, NTF>;
  {  // answer_processor.0 + ReLU (attention.py:277-282, 350)
    LRf::Params pa{(const float*)(pk + L.k_W1p), L.ans_ld, 512};
    LRfj::Params pb{Wf(L.ans), L.ans_ld, F};
    EpiStoreT<float> ep{Wf(L.hid1), 512, 512, F, prm + L.poff[A0B], 1};
    HIPCHK((tail_gemm(pa, pb, ep, 512, F, L.ans_ld, st)));
  }
  {  // answer_processor.2
    LRf::Params pa{prm + L.poff[A2W], 512, 256};
    LRfj::Params pb{Wf(L.hid1), 512, F};
    EpiStoreT<float> ep{Wf(L.AO), 256, 256, F, prm + L.poff[A2B], 0};
    HIPCHK((tail_gemm(pa, pb, ep, 256, F, 512, st)));
  }
  {  // policy_core LSTMCell from zero state (attention.py:354-355)
    LRf::Params pa{(const float*)(pk + L.k_Wihp), 256, 1024};
    LRfj::Params pb{Wf(L.AO), 256, F};
    EpiLstmCellFwd ep{(const float*)(pk + L.k_blc), Wf(L.LG), Wf(L.LC), Wf(L.LH), F};
    HIPCHK((tail_gemm(pa, pb, ep, 1024, F, 256, st)));
  }
  }
  {  // policy / values heads (attention.py:365-367), batched over all frames
    using LRf = LdRows<float, float, CF::BI, CF::BK, NTF>;
    using LRfj = LdRows<float, float, CF::BJ, CF::BK, NTF>;
    LRf::Params pa{(const float*)(pk + L.k_Whd), 256, 2 * L.A};
    LRfj::Params pb{L.sc ? Wf(L.CH) + (size_t)L.B * 256 : Wf(L.LH), 256, F};
    EpiHeads ep{io->logits, io->values, (const float*)(pk + L.k_bhd), L.A, F};
    HIPCHK((tail_gemm(pa, pb, ep, 2 * L.A, F, 256, st)));
  }
  if (io->hT)
    HIPCHK(hipMemcpyAsync(io->hT, Wf(L.Hs) + (size_t)(L.T - 1) * M * 128, (size_t)M * 128 * 4,
                          hipMemcpyDeviceToDevice, st));
  if (io->cT)
    HIPCHK(hipMemcpyAsync(io->cT, Wf(L.Cst) + (size_t)L.T * M * 128, (size_t)M * 128 * 4, hipMemcpyDeviceToDevice, st));
  if (L.sc && io->core_hT)
    HIPCHK(hipMemcpyAsync(io->core_hT, Wf(L.CH) + (size_t)L.T * L.B * 256, (size_t)L.B * 256 * 4,
                          hipMemcpyDeviceToDevice, st));
  if (L.sc && io->core_cT)
    HIPCHK(hipMemcpyAsync(io->core_cT, Wf(L.CC) + (size_t)L.T * L.B * 256, (size_t)L.B * 256 * 4,
                          hipMemcpyDeviceToDevice, st));
  return AAA_OK;
}

// conv2 dgrad (stride 2, k4, pad 2) as four parity-class 2x2 convs over dY2:
// output pixel (2a+py, 2b+px) only receives taps ky = py + 2(1-ty), kx = px + 2(1-tx).
template <typename T>
static int conv2_dgrad(const Layout& L, const char* pk, const T* dy2, T* dy1, int frames, float* gbias,
                       hipStream_t s) {
  {
    // small grids: the four classes share one gather (output (a, b) reads dY2
    // (a + ty, b + tx)), so one 128-row tile (class-major rows, [cls][32][256]
    // = k_WdT2) per frame reads the frame's dY2 once as a zero-bordered LDS
    // image (halo.h, KS = 2) -- one launch instead of four 32-row GEMMs whose
    // K = 256 loops were pure latency (4 x 65 us at C3, 0.06 of bf16 peak)
    constexpr int CKd = std::is_same<T, float>::value ? 32 : 64;
    const int Ha = (L.H1 + 1) / 2, Wa = (L.W1 + 1) / 2;
    auto halo4 = [&](auto cfg) -> int {
      using HC = decltype(cfg);
      EpiStoreParity4<T> ep(dy1, frames * Ha * Wa, Ha, Wa, L.H1, L.W1, gbias);
      const HaloParams hp{pk + L.k_WdT2, 256, 128, dy2, 64, 0, 64, (uint32_t)((size_t)frames * L.P * 64 * L.esz),
                          L.h, L.w, frames, 0, Ha, Wa};
      HIPCHK((launch_halo<HC, EpiStoreParity4<T>, 2>(hp, ep, s)));
      return AAA_OK;
    };
    auto fits = [&](int fr, int bj, int hmax) {
      return fr * Ha * Wa <= bj && fr * (L.h + 2) * (L.w + 2) + 1 <= hmax && Ha <= L.h && Wa <= L.w;
    };
    // bf16: FR = 2 frames per tile -- the 64 KB weight tile streamed once per two frames and twice the
    // MFMA work per DMA round trip (C3 4.97 -> 4.94 ms); fp32 keeps FR = 1 (C2 4.306 vs 4.341 ms)
    // (profiles/r02/ab/dgrad_fr.txt; AAA_DGRAD2_FR overrides)
    const int fr = env_int("AAA_DGRAD2_FR", std::is_same<T, float>::value ? 1 : 2);
    if (env_int("AAA_DGRAD2_HALO", 1)) {
      if (fr == 2 && fits(2, 256, 352)) return halo4(HaloCfg<T, 128, 256, CKd, 2, 2, 2, 352>{});
      if (fits(1, 128, 192)) return halo4(HaloCfg<T, 128, 128, CKd, 2, 2, 1, 192>{});
      // bf16, grids up to 21x21 (168x168 frames, C5): one frame per 512-column tile of 8 waves,
      // 32-channel chunks (two LDS images of 23x23 pixels), the epilogue in two column chunks
      if constexpr (!std::is_same<T, float>::value)
        if (fits(1, 512, 640) && env_int("AAA_DGRAD2_WIDE", 1)) return halo4(HaloCfg<T, 128, 512, 32, 2, 4, 1, 640>{});
    }
  }
  if (env_int("AAA_CONV2_DGRAD_RING", 1)) {
    // the LDS-DMA ring (dY2 is already in T), dY1 stored in T, conv1's bias
    // gradient summed from the fp32 values in the epilogue (no column-sum pass)
    constexpr int BKd = std::is_same<T, float>::value ? 32 : 64;
    auto classes = [&](auto cfg) -> int {
      using CP = decltype(cfg);
      using PA = GRowsB<T, CP::BI, CP::BK, CP::NT>;
      using PB = GIm2colB<T, CP::BJ, CP::BK, CP::NT>;
      for (int cls = 0; cls < 4; ++cls) {
        const int py = cls >> 1, px = cls & 1;
        const int Ha = (L.H1 - py + 1) / 2, Wa = (L.W1 - px + 1) / 2;
        if (Ha <= 0 || Wa <= 0) continue;
        const int rows = frames * Ha * Wa;
        EpiStoreParityBias<T> ep{dy1, 32, rows, Ha, Wa, L.H1, L.W1, py, px, gbias};
        HIPCHK((launch_pipe<CP, PA, PB, EpiStoreParityBias<T>, 2>(
            typename PA::Params{(const T*)(pk + L.k_WdT2) + (size_t)cls * 32 * 256, 256, 32},
            typename PB::Params{dy2, ConvGeo{64, 64, 0, L.h, L.w, Ha, Wa, 2, 1, 0, 0}.prep(), rows,
                                (uint32_t)((size_t)frames * L.P * 64 * L.esz)},
            ep, 32, rows, 256, 1, s)));
      }
      return AAA_OK;
    };
    // K = 256: four BK steps per tile, so 256 columns per workgroup (twice the MFMA work per DMA round
    // trip of 32x128): C5 14.945 -> 14.74 ms per iteration (profiles/r02/ab/vision_tiles.txt); AAA_DGRAD2_TILE=0 the old tile
    return env_int("AAA_DGRAD2_TILE", 1) == 1 ? classes(GemmCfg<T, 32, 256, BKd, 1, 4>{})
                                             : classes(GemmCfg<T, 32, 128, BKd, 1, 4>{});
  }
  // register-staged fallback (fp32 only: dY2's loader converts from fp32)
  if constexpr (!std::is_same<T, float>::value) return fail(AAA_E_ARG, "AAA_CONV2_DGRAD_RING=0 needs fp32");
  using C3 = Cfg32For<T>;
  using LA = LdRowsB<T, T, C3::BI, C3::BK, C3::NT>;
  using LB = LdIm2colB<float, T, C3::BJ, C3::BK, C3::NT>;
  for (int cls = 0; cls < 4; ++cls) {
    const int py = cls >> 1, px = cls & 1;
    const int Ha = (L.H1 - py + 1) / 2, Wa = (L.W1 - px + 1) / 2;
    if (Ha <= 0 || Wa <= 0) continue;
    const int rows = frames * Ha * Wa;
    typename LA::Params pa{(const T*)(pk + L.k_WdT2) + (size_t)cls * 32 * 256, 256, 32};
    typename LB::Params pb{(const float*)dy2, ConvGeo{64, 64, 0, L.h, L.w, Ha, Wa, 2, 1, 0, 0}.prep(), rows,
                           (uint32_t)((size_t)frames * L.P * 64 * 4)};
    EpiStoreParity ep{(float*)dy1, 32, rows, Ha, Wa, L.H1, L.W1, py, px, FastDiv((uint32_t)(Ha * Wa)),
                      FastDiv((uint32_t)Wa)};
    HIPCHK((launch_gemm<C3, LA, LB>(pa, pb, ep, 32, rows, 256, 1, s)));
  }
  return AAA_OK;
}

// conv2 weight gradient over ``frames`` frames: gW[64][(ky*4+kx)*32 + ci] +=
// dY2^T x im2col(Y1) (k = output pixel), split-K atomics into a zeroed gW.
template <typename T>
static int conv2_wgrad(const Layout& L, const T* dy2, const T* y1, int frames, float* gW, hipStream_t s) {
  using C = CfgFor<T>;
  using LA = LdRowsTB<T, T, C::BI, C::BK, C::NT>;
  using LB = LdIm2colTB<T, T, C::BJ, C::BK, C::NT>;
  const int rows = frames * L.P;
  if constexpr (!std::is_same<T, float>::value) {
    // bf16 (AAA_CONV2_WGRAD_PIPE, A/B): the LDS-DMA ring of the ConvLSTM weight gradient, 64x256
    // tiles of 4 waves, split-K over about one wave of workgroups, atomics from the accumulators
    if (rows % 32 == 0 && env_int("AAA_CONV2_WGRAD_PIPE", 0)) {
      using CW = GemmCfg<T, 64, 256, 32, 1, 4>;
      using PA = GRowsT<T, CW::BI, CW::BK, CW::NT>;
      using PB = GIm2colT<T, CW::BJ, CW::BK, CW::NT>;
      typename PA::Params pa{dy2, 64, 64, rows};
      typename PB::Params pb{y1, ConvGeo{32, 32, 0, L.H1, L.W1, L.h, L.w, 4, 2, 2, 0}.prep(), 512,
                             (uint32_t)((size_t)frames * L.P1 * 32 * L.esz)};
      EpiAtomicD ep{{gW, 512, 64, 512}};
      const int ns = std::max(1, std::min(env_int("AAA_CONV2_WGRAD_WGS", 256) / 2, rows / (8 * CW::BK)));
      HIPCHK((launch_pipe<CW, PA, PB, EpiAtomicD, 4, 2>(pa, pb, ep, 64, 512, rows, ns, s)));
      return AAA_OK;
    }
  }
  typename LA::Params pa{dy2, 64, 64, rows};
  typename LB::Params pb{y1, ConvGeo{32, 32, 0, L.H1, L.W1, L.h, L.w, 4, 2, 2, 0}.prep(), 512,
                         (uint32_t)((size_t)frames * L.P1 * 32 * L.esz)};
  EpiStore<true> ep{gW, 512, 64, 512};
  const int tiles = cdiv(64, C::BI) * cdiv(512, C::BJ);
  HIPCHK((launch_gemm<C, LA, LB>(pa, pb, ep, 64, 512, rows, wgrad_splits(tiles, rows, C::BK), s)));
  return AAA_OK;
}

// conv1 weight gradient over RGBx frames (Cin 4; the 4th channel's grad is dropped on unpack)
template <typename T>
static int conv1_wgrad(const Layout& L, const T* dy1, const T* xp, int frames, float* gW, hipStream_t s) {
  const int rows1 = frames * L.P1;
  auto run = [&](auto cfg) -> int {
    using C3 = decltype(cfg);
    using LA = LdRowsTB<T, T, C3::BI, C3::BK, C3::NT>;
    using LB = LdIm2colTB<T, T, C3::BJ, C3::BK, C3::NT>;   // bf16 chunks = 2 taps x 4 ch, in-bounds (bordered image)
    typename LA::Params pa{dy1, 32, 32, rows1};
    typename LB::Params pb{xp, ConvGeo{4, 4, 0, L.H + 2, L.W + 2, L.H1, L.W1, 8, 4, 0, 0}.prep(), 256,
                           (uint32_t)((size_t)frames * (L.H + 2) * (L.W + 2) * 4 * L.esz)};
    EpiStore<true> ep{gW, 256, 32, 256};
    const int tiles = cdiv(32, C3::BI) * cdiv(256, C3::BJ);
    HIPCHK((launch_gemm<C3, LA, LB>(pa, pb, ep, 32, 256, rows1, wgrad_splits(tiles, rows1, C3::BK), s)));
    return AAA_OK;
  };
  // AAA_CONV1_WGRAD_TILE=1 (A/B): one 32x256 tile covering every (tap, channel) column, so each
  // pixel's 8x8 window is gathered once instead of by four 64-column tiles
  if (env_int("AAA_CONV1_WGRAD_TILE", 0) == 1) return run(GemmCfg<T, 32, 256, Cfg32For<T>::BK, 1, 4>{});
  return run(Cfg32For<T>{});
}

// All 8 ConvLSTM weight gradients of ``rows`` pixels at once (attention.py:39-102
// as used at :119-122): gW[512 = 4ch+gate][1728 = tap*192 + c'] += dZ^T x
// im2col(XH) with k = pixel, accumulated (split-K atomics) into a zeroed gW.
// ``aux``: issued on the low-priority overlap stream.
template <typename T>
static int lstm_wgrad(const T* dz, const T* xh, int rows, int h, int w, float* gW, hipStream_t s, bool aux) {
  const uint32_t xh_bytes = (uint32_t)((size_t)rows * 192 * sizeof(T));
  auto wgrad_lstm = [&](auto cfg) -> int {   // all 8 ConvLSTM weight grads: D[512][1728] += dZ^T * im2col(XH)
    using CW = decltype(cfg);
    using LA = LdRowsTB<T, T, CW::BI, CW::BK, CW::NT>;
    using LB = LdIm2colTB<T, T, CW::BJ, CW::BK, CW::NT>;
    typename LA::Params pa{dz, 512, 512, rows};
    typename LB::Params pb{xh, ConvGeo{192, 192, 0, h, w, h, w, 3, 1, 1, 0}.prep(),
                           1728, xh_bytes};
    EpiStore<true> ep{gW, 1728, 512, 1728};
    const int tiles = cdiv(512, CW::BI) * cdiv(1728, CW::BJ);
    // about two workgroups per CU of splits (both fit a CU; the 1024-WG rule of
    // the other weight gradients doubled the output atomics for the same time:
    // profiles/r02/ab/wgrad_split.txt)
    const int ns = std::max(1, std::min(env_int("AAA_WGRAD_SPLIT", std::max(1, 512 / tiles)), rows / CW::BK));
    TimerScope tim(AAA_TIMER_CORE_WGRAD, s, 2.0 * 512 * 1728 * rows, strf("register-staged %dx%d BK%d, %d-way split-K atomics", CW::BI, CW::BJ, CW::BK, ns));
    HIPCHK((launch_gemm<CW, LA, LB>(pa, pb, ep, 512, 1728, rows, ns, s)));
    return AAA_OK;
  };
  // LDS-DMA ring with transposed fragment reads for both operands (k = pixel)
  // and the split-K atomics straight from the accumulators
  auto wgrad_lstm_pipe = [&](auto cfg, auto nbuf, auto ilv) -> int {
    using CW = decltype(cfg);
    constexpr int NB = decltype(nbuf)::value, IL = decltype(ilv)::value;
    using LA = GRowsT<T, CW::BI, CW::BK, CW::NT>;
    using LB = GIm2colT<T, CW::BJ, CW::BK, CW::NT>;
    typename LA::Params pa{dz, 512, 512, rows};
    typename LB::Params pb{xh, ConvGeo{192, 192, 0, h, w, h, w, 3, 1, 1, 0}.prep(),
                           1728, xh_bytes};
    EpiAtomicD ep{{gW, 1728, 512, 1728}};
    const int tiles = cdiv(512, CW::BI) * cdiv(1728, CW::BJ);
    TimerScope tim(AAA_TIMER_CORE_WGRAD, s, 2.0 * 512 * 1728 * rows, strf("LDS-DMA ring %dx%d BK%d, %d-deep", CW::BI, CW::BJ, CW::BK, NB));
    // split-K over pixels: about one resident wave of workgroups (fewer
    // passes of the output's atomics than the register path's ~1024)
    const int wgs = env_int("AAA_WGRAD_WGS", 256);
    const int ns = std::max(1, std::min(wgs / tiles, rows / (8 * CW::BK)));
    HIPCHK((launch_pipe<CW, LA, LB, EpiAtomicD, NB, IL>(pa, pb, ep, 512, 1728, rows, ns, s)));
    return AAA_OK;
  };
  // bf16 default: 256x256 (8 waves of 128x64), BK=32 in a 4-deep ring with the
  // DMA pieces spread over the k steps (tools/ubench/wgrad_ablate at C3: 1163 us
  // vs 1296 for BK=64 in a 2-deep ring and 1400 for the register-staged GEMM)
  constexpr int WBK = std::is_same<T, float>::value ? 32 : 64;
  // (not on the aux stream: its 128 KB of LDS would keep the chain's step kernels off the CU)
  const int wpipe = rows % WBK == 0 ? env_int("AAA_WGRAD_PIPE", std::is_same<T, float>::value || aux ? 0 : 6) : 0;
  if (wpipe) {
    using I0 = std::integral_constant<int, 0>;
    using I2 = std::integral_constant<int, 2>;
    using I3 = std::integral_constant<int, 3>;
    int rc;
    switch (wpipe) {
      case 2: rc = wgrad_lstm_pipe(GemmCfg<T, 256, 128, WBK, 2, 2>{}, I2{}, I0{}); break;
      case 3:   // 8 waves of 128x64 (fp32: spills, so 256x128)
        if constexpr (std::is_same<T, float>::value) rc = wgrad_lstm_pipe(GemmCfg<T, 256, 128, WBK, 2, 2>{}, I2{}, I0{});
        else rc = wgrad_lstm_pipe(GemmCfg<T, 256, 256, WBK, 2, 4>{}, I2{}, I0{});
        break;
      case 4: rc = wgrad_lstm_pipe(GemmCfg<T, 128, 256, WBK, 2, 2>{}, I2{}, I0{}); break;
      case 5: rc = wgrad_lstm_pipe(GemmCfg<T, 256, 128, WBK, 2, 2>{}, I3{}, I0{}); break;
      case 6:   // bf16: 8 waves, BK=32, 4-deep ring, spread DMA issue
      case 7:   // bf16: the same in a 3-deep ring
        if constexpr (std::is_same<T, float>::value)
          rc = wgrad_lstm_pipe(GemmCfg<T, 128, 128, WBK, 2, 2>{}, I3{}, I2{});
        else if (wpipe == 6)
          rc = wgrad_lstm_pipe(GemmCfg<T, 256, 256, 32, 2, 4>{}, std::integral_constant<int, 4>{}, I2{});
        else
          rc = wgrad_lstm_pipe(GemmCfg<T, 256, 256, 32, 2, 4>{}, I3{}, I2{});
        break;
      case 8:   // bf16: 4 waves of 128x128 (half the LDS fragment reads per MFMA of the 8-wave tile), 4-deep ring:
                // measured slower (C3 1367 vs 1079 us, C4 691 vs 561 us: one wave per SIMD hides less)
        if constexpr (std::is_same<T, float>::value)
          rc = wgrad_lstm_pipe(GemmCfg<T, 128, 128, WBK, 2, 2>{}, I3{}, I2{});
        else
          rc = wgrad_lstm_pipe(GemmCfg<T, 256, 256, 32, 2, 2>{}, std::integral_constant<int, 4>{}, I2{});
        break;
      default: rc = wgrad_lstm_pipe(GemmCfg<T, 128, 128, WBK, 2, 2>{}, I2{}, I0{}); break;
    }
    if (rc) return rc;
  } else {
    // on the aux stream a small-footprint tile lets the chain's step kernels co-reside on a CU
    const int wide = env_int("AAA_AUX_WIDE", aux ? 0 : 1);
    // AAA_WGRAD_TILE=1 (A/B): 128x192 tiles, 1728 = 9 x 192 columns without the half-empty last tile of 128
    const int rc = !wide ? wgrad_lstm(CfgFor<T>{})
                   : env_int("AAA_WGRAD_TILE", 0) == 1 ? wgrad_lstm(GemmCfg<T, 128, 192, 32, 2, 2>{})
                                                       : wgrad_lstm(CfgWFor<T>{});
    if (rc) return rc;
  }
  return AAA_OK;
}

// Vision encoder backward over F frames in descriptor-sized chunks: conv2
// weight grad (gW2 +=), conv2 dgrad -> dY1 with conv1's bias grad (gb1 +=),
// conv1 weight grad (gW1 +=); accumulators zeroed by the caller.
template <typename T>
static int vision_bwd(const Layout& L, const char* pk, const T* dy2, const T* y1, const T* xp, T* dy1, int F,
                      float* gW2, float* gW1, float* gb1, hipStream_t s) {
  for (int f0 = 0; f0 < F; f0 += L.fchunk) {
    const int n = std::min(L.fchunk, F - f0);
    const T* d2 = dy2 + (size_t)f0 * L.P * 64;
    T* d1 = dy1 + (size_t)f0 * L.P1 * 32;
    int rc = conv2_wgrad<T>(L, d2, y1 + (size_t)f0 * L.P1 * 32, n, gW2, s);
    if (!rc) rc = conv2_dgrad<T>(L, pk, d2, d1, n, gb1, s);
    if (!rc) rc = conv1_wgrad<T>(L, d1, xp + (size_t)f0 * (L.H + 2) * (L.W + 2) * 4, n, gW1, s);
    if (rc) return rc;
  }
  return AAA_OK;
}

// ------------------------------------------------------------ backward ----
// Stateful policy core, backward of the tail (phase HEAD): the dgrad chain runs
// step by step from t = T-1 (the carries dh, dc of the core state flow through
// the LSTMCell's W_hh and the query MLP into step t-1); every weight gradient
// is then one batched GEMM over all frames from the saved per-step operands.
static int head_backward_stateful(const Layout& L, const aaa_io* io, hipStream_t st) {
  constexpr int NTF = CF::NT;
  char* ws = (char*)io->workspace;
  const char* pk = (const char*)io->packed;
  const float* prm = io->params;
  float* grads = io->grads;
  auto Wf = [&](size_t off) { return (float*)(ws + off); };
  const int F = L.F, P = L.P, B = L.B, qd = L.qd, da = L.da;
  using LRfj = LdRows<float, float, CF::BJ, CF::BK, NTF>;
  using LTf = LdRowsT<float, float, CF::BI, CF::BK, NTF>;
  using LTfj = LdRowsT<float, float, CF::BJ, CF::BK, NTF>;
  float *CH = Wf(L.CH), *CC = Wf(L.CC), *AOX = Wf(L.AOX), *dAOX = Wf(L.dAOX), *dhc = Wf(L.dhc), *dcc = Wf(L.dcc);
  const size_t sB = (size_t)B * 256 * 4;
  if (io->dcore_hT) HIPCHK(hipMemcpyAsync(dhc, io->dcore_hT, sB, hipMemcpyDeviceToDevice, st));
  else HIPCHK(hipMemsetAsync(dhc, 0, sB, st));
  if (io->dcore_cT) HIPCHK(hipMemcpyAsync(dcc, io->dcore_cT, sB, hipMemcpyDeviceToDevice, st));
  else HIPCHK(hipMemsetAsync(dcc, 0, sB, st));
  for (int t = L.T - 1; t >= 0; --t) {
    const size_t f0 = (size_t)t * B;
    {  // heads dgrad + dh carry -> LSTMCell backward from (c_{t-1}, c_t), dc carry
      LTf::Params pa{(const float*)(pk + L.k_Whd), 256, 256};
      LRfj::Params pb{Wf(L.dY) + f0 * L.ldy, L.ldy, B};
      EpiLstmCellBwdS ep{Wf(L.LG) + f0 * 1024, CC + f0 * 256, CC + (f0 + B) * 256, dhc, dcc, Wf(L.dLG) + f0 * 1024, B};
      HIPCHK((head_gemm<LdRowsT, LdRows>(pa, pb, ep, 256, B, L.ldy, 1, st)));
    }
    {  // [d answer | d h_{t-1} (recurrent part)] = [W_ih | W_hh]^T dgates
      LTf::Params pa{(const float*)(pk + L.k_Wihhp), 512, 512};
      LRfj::Params pb{Wf(L.dLG) + f0 * 1024, 1024, B};
      EpiStoreT<float> ep{dAOX + f0 * 512, 512, 512, B, nullptr, 0};
      HIPCHK((head_gemm<LdRowsT, LdRows>(pa, pb, ep, 512, B, 1024, 1, st)));
    }
    {  // answer_processor.2 dgrad fused with the ReLU backward
      LTf::Params pa{prm + L.poff[A2W], 512, 512};
      LRfj::Params pb{dAOX + f0 * 512, 512, B};
      EpiReluBwdT ep{Wf(L.dH1) + f0 * 512, Wf(L.hid1) + f0 * 512, 512, 512, 512, B};
      HIPCHK((head_gemm<LdRowsT, LdRows>(pa, pb, ep, 512, B, 256, 1, st)));
    }
    {  // answer_processor.0 dgrad: readout and query columns of the answer row
      LTf::Params pa{(const float*)(pk + L.k_W1p), L.ans_ld, da};
      LRfj::Params pb{Wf(L.dH1) + f0 * 512, 512, B};
      EpiStoreT<float> ep{Wf(L.dAns) + f0 * da, da, da, B, nullptr, 0};
      HIPCHK((head_gemm<LdRowsT, LdRows>(pa, pb, ep, da, B, 512, 1, st)));
    }
    // readout / softmax / logits backward with this step's queries; dQ gets
    // the logits path plus the answer row's copy of Q
    {
      TimerScope tim(AAA_TIMER_ATTN_BWD, st, (double)B * attn_bwd_bytes(P, L.nq), "k_attn_bwd, per-frame query (stateful core)");
      HIPCHK(attn_bwd(Wf(L.Hs) + f0 * P * 128, io->basis, Wf(L.Qf) + f0 * qd, Wf(L.Am) + f0 * P * L.nq,
                      Wf(L.dAns) + f0 * da, da, B, P, L.nq, Wf(L.dO) + f0 * P * 128, Wf(L.dQf) + f0 * qd, st, qd, 1));
    }
    {  // query MLP backward to its input h_{t-1}
      LTf::Params pa{prm + L.poff[Q4W], qd, qd};
      LRfj::Params pb{Wf(L.dQf) + f0 * qd, qd, B};
      EpiReluBwdT ep{Wf(L.dq2s) + f0 * qd, Wf(L.q2s) + f0 * qd, qd, qd, qd, B};
      HIPCHK((head_gemm<LdRowsT, LdRows>(pa, pb, ep, qd, B, qd, 1, st)));
    }
    {
      LTf::Params pa{prm + L.poff[Q2W], 128, 128};
      LRfj::Params pb{Wf(L.dq2s) + f0 * qd, qd, B};
      EpiReluBwdT ep{Wf(L.dq1s) + f0 * 128, Wf(L.q1s) + f0 * 128, 128, 128, 128, B};
      HIPCHK((head_gemm<LdRowsT, LdRows>(pa, pb, ep, 128, B, qd, 1, st)));
    }
    {  // dh_{t-1} = W0^T dq1 (query path) + W_hh^T dgates (recurrent path)
      LTf::Params pa{prm + L.poff[Q0W], 256, 256};
      LRfj::Params pb{Wf(L.dq1s) + f0 * 128, 128, B};
      EpiStoreAddT ep{dhc, dAOX + f0 * 512 + 256, 256, 512, 256, B};
      HIPCHK((head_gemm<LdRowsT, LdRows>(pa, pb, ep, 256, B, 128, 1, st)));
    }
  }
  if (io->dcore_h0) HIPCHK(hipMemcpyAsync(io->dcore_h0, dhc, sB, hipMemcpyDeviceToDevice, st));
  if (io->dcore_c0) HIPCHK(hipMemcpyAsync(io->dcore_c0, dcc, sB, hipMemcpyDeviceToDevice, st));
  // weight gradients, batched over all T*B frames
  auto wgrad = [&](const float* dA, int lda, int Mi, const float* X, int ldx, int Nj, float* out, int ldo) -> int {
    LTf::Params pa{dA, lda, Mi};
    LTfj::Params pb{X, ldx, Nj};
    EpiStore<true> ep{out, ldo, Mi, Nj};
    HIPCHK((head_gemm<LdRowsT, LdRowsT>(pa, pb, ep, Mi, Nj, F, wgrad_splits(cdiv(Mi, 64) * cdiv(Nj, 64), F, CF::BK),
                                        st)));
    return AAA_OK;
  };
  int rc;
  if ((rc = wgrad(Wf(L.dY), L.ldy, L.ldy, CH + (size_t)B * 256, 256, 256, Wf(L.gWhd), 256))) return rc;
  HIPCHK(colsum(Wf(L.dY), L.ldy, F, L.ldy, Wf(L.gbhd), st));
  if ((rc = wgrad(Wf(L.dLG), 1024, 1024, AOX, 512, 512, Wf(L.gWihhp), 512))) return rc;
  HIPCHK(colsum(Wf(L.dLG), 1024, F, 1024, Wf(L.gblc), st));
  if ((rc = wgrad(dAOX, 512, 256, Wf(L.hid1), 512, 512, grads + L.poff[A2W], 512))) return rc;
  HIPCHK(colsum(dAOX, 512, F, 256, grads + L.poff[A2B], st));
  if ((rc = wgrad(Wf(L.dH1), 512, 512, Wf(L.ans), L.ans_ld, L.ans_ld, Wf(L.gW1p), L.ans_ld))) return rc;
  HIPCHK(colsum(Wf(L.dH1), 512, F, 512, grads + L.poff[A0B], st));
  if ((rc = wgrad(Wf(L.dQf), qd, qd, Wf(L.q2s), qd, qd, grads + L.poff[Q4W], qd))) return rc;
  HIPCHK(colsum(Wf(L.dQf), qd, F, qd, grads + L.poff[Q4B], st));
  if ((rc = wgrad(Wf(L.dq2s), qd, qd, Wf(L.q1s), 128, 128, grads + L.poff[Q2W], 128))) return rc;
  HIPCHK(colsum(Wf(L.dq2s), qd, F, qd, grads + L.poff[Q2B], st));
  if ((rc = wgrad(Wf(L.dq1s), 128, 128, CH, 256, 256, grads + L.poff[Q0W], 256))) return rc;
  HIPCHK(colsum(Wf(L.dq1s), 128, F, 128, grads + L.poff[Q0B], st));
  F32Unpack up;
  up.gW1p = Wf(L.gW1p); up.gWihp = Wf(L.gWihp); up.gblc = Wf(L.gblc); up.gWhd = Wf(L.gWhd); up.gbhd = Wf(L.gbhd);
  up.a0w = grads + L.poff[A0W]; up.wih = grads + L.poff[WIH]; up.bih = grads + L.poff[BIH];
  up.bhh = grads + L.poff[BHH]; up.pw = grads + L.poff[PW]; up.vw = grads + L.poff[VW];
  up.pb = grads + L.poff[PB]; up.vb = grads + L.poff[VB];
  up.ans_in = L.ans_in; up.ans_ld = L.ans_ld; up.A = L.A;
  up.gWihhp = Wf(L.gWihhp); up.whh = grads + L.poff[WHH];
  HIPCHK(unpack_f32(up, st));
  return AAA_OK;
}

template <typename T>
static int backward_impl(const Layout& L, const aaa_io* io, int phases, hipStream_t st) {
  using C = CfgFor<T>;
  constexpr int NTF = CF::NT;
  char* ws = (char*)io->workspace;
  const char* pk = (const char*)io->packed;
  const float* prm = io->params;
  float* grads = io->grads;
  auto Wf = [&](size_t off) { return (float*)(ws + off); };
  auto Wt = [&](size_t off) { return (T*)(ws + off); };
  const int F = L.F, P = L.P, M = L.B * L.P;
  using LRfj = LdRows<float, float, CF::BJ, CF::BK, NTF>;
  using LTf = LdRowsT<float, float, CF::BI, CF::BK, NTF>;
  using LTfj = LdRowsT<float, float, CF::BJ, CF::BK, NTF>;
  LstmGrads core_unpack{};   // the ConvLSTM grads' reference tensors, unpacked with the vision grads when both run here

  if (phases & AAA_BWD_HEAD) {
    HIPCHK(hipMemsetAsync(grads, 0, L.ptotal * 4, st));
    HIPCHK(hipMemsetAsync(ws + L.dQs, 0, L.ws - L.dQs, st));
    HIPCHK(concat_dy(F, L.A, L.ldy, io->dlogits, io->dvalues, Wf(L.dY), st));
    if (L.sc) {
      const int rc = head_backward_stateful(L, io, st);
      if (rc) return rc;
    } else {
    {  // heads dgrad fused with the zero-state LSTMCell backward
      LTf::Params pa{(const float*)(pk + L.k_Whd), 256, 256};
      LRfj::Params pb{Wf(L.dY), L.ldy, F};
      EpiLstmCellBwd ep{Wf(L.LG), Wf(L.LC), Wf(L.dLG), F};
      HIPCHK((head_gemm<LdRowsT, LdRows>(pa, pb, ep, 256, F, L.ldy, 1, st)));
    }
    {  // heads wgrad
      LTf::Params pa{Wf(L.dY), L.ldy, L.ldy};
      LTfj::Params pb{Wf(L.LH), 256, 256};
      EpiStore<true> ep{Wf(L.gWhd), 256, L.ldy, 256};
      HIPCHK((head_gemm<LdRowsT, LdRowsT>(pa, pb, ep, L.ldy, 256, F, wgrad_splits(cdiv(L.ldy, 64) * 4, F, CF::BK), st)));
    }
    {  // LSTMCell input dgrad
      LTf::Params pa{(const float*)(pk + L.k_Wihp), 256, 256};
      LRfj::Params pb{Wf(L.dLG), 1024, F};
      EpiStoreT<float> ep{Wf(L.dAO), 256, 256, F, nullptr, 0};
      HIPCHK((head_gemm<LdRowsT, LdRows>(pa, pb, ep, 256, F, 1024, 1, st)));
    }
    {  // LSTMCell weight_ih grad (weight_hh grad is exactly zero: h0 = 0, Q1)
      LTf::Params pa{Wf(L.dLG), 1024, 1024};
      LTfj::Params pb{Wf(L.AO), 256, 256};
      EpiStore<true> ep{Wf(L.gWihp), 256, 1024, 256};
      HIPCHK((head_gemm<LdRowsT, LdRowsT>(pa, pb, ep, 1024, 256, F, wgrad_splits(16 * 4, F, CF::BK), st)));
    }
    {  // answer_processor.2 dgrad fused with ReLU backward
      LTf::Params pa{prm + L.poff[A2W], 512, 512};
      LRfj::Params pb{Wf(L.dAO), 256, F};
      EpiReluBwdT ep{Wf(L.dH1), Wf(L.hid1), 512, 512, 512, F};
      HIPCHK((head_gemm<LdRowsT, LdRows>(pa, pb, ep, 512, F, 256, 1, st)));
    }
    {  // answer_processor.2 wgrad / bias
      LTf::Params pa{Wf(L.dAO), 256, 256};
      LTfj::Params pb{Wf(L.hid1), 512, 512};
      EpiStore<true> ep{grads + L.poff[A2W], 512, 256, 512};
      HIPCHK((head_gemm<LdRowsT, LdRowsT>(pa, pb, ep, 256, 512, F, wgrad_splits(4 * 8, F, CF::BK), st)));
    }
    {  // answer_processor.0 dgrad (readout columns only)
      LTf::Params pa{(const float*)(pk + L.k_W1p), L.ans_ld, L.da};
      LRfj::Params pb{Wf(L.dH1), 512, F};
      EpiStoreT<float> ep{Wf(L.dAns), L.da, L.da, F, nullptr, 0};
      HIPCHK((head_gemm<LdRowsT, LdRows>(pa, pb, ep, L.da, F, 512, 1, st)));
    }
    {  // answer_processor.0 wgrad / bias
      LTf::Params pa{Wf(L.dH1), 512, 512};
      LTfj::Params pb{Wf(L.ans), L.ans_ld, L.ans_ld};
      EpiStore<true> ep{Wf(L.gW1p), L.ans_ld, 512, L.ans_ld};
      HIPCHK((head_gemm<LdRowsT, LdRowsT>(pa, pb, ep, 512, L.ans_ld, F,
                                        wgrad_splits(8 * cdiv(L.ans_ld, 64), F, CF::BK), st)));
    }
    // attention readout / softmax / logits backward, then the query MLP
    {
      TimerScope tim(AAA_TIMER_ATTN_BWD, st, (double)F * attn_bwd_bytes(P, L.nq), "k_attn_bwd, 1 WG per frame");
      HIPCHK(attn_bwd(Wf(L.Hs), io->basis, (const float*)(pk + L.k_Q), Wf(L.Am), Wf(L.dAns), L.da, F, P, L.nq,
                      Wf(L.dO), Wf(L.dQp), st));
    }
    {  // the bias grads of the heads, the LSTMCell and both answer layers, and dQ summed over frames: one launch
      ColSums cs;
      cs.add(Wf(L.dY), L.ldy, L.ldy, Wf(L.gbhd));
      cs.add(Wf(L.dLG), 1024, 1024, Wf(L.gblc));
      cs.add(Wf(L.dAO), 256, 256, grads + L.poff[A2B]);
      cs.add(Wf(L.dH1), 512, 512, grads + L.poff[A0B]);
      cs.add(Wf(L.dQp), L.qd, L.qd, Wf(L.dQs));
      HIPCHK(colsum_multi(cs, F, st));
    }
    HIPCHK(query_bwd(Wf(L.dQs), grads + L.poff[A0B], prm + L.poff[A0W], L.ans_in, L.nq, prm + L.poff[Q2W],
                     prm + L.poff[Q4W], (const float*)(pk + L.k_q1), (const float*)(pk + L.k_q2), grads + L.poff[Q4W],
                     grads + L.poff[Q4B],
                     grads + L.poff[Q2W], grads + L.poff[Q2B], grads + L.poff[Q0B], st));
    F32Unpack up;
    up.gW1p = Wf(L.gW1p); up.gWihp = Wf(L.gWihp); up.gblc = Wf(L.gblc); up.gWhd = Wf(L.gWhd); up.gbhd = Wf(L.gbhd);
    up.a0w = grads + L.poff[A0W]; up.wih = grads + L.poff[WIH]; up.bih = grads + L.poff[BIH];
    up.bhh = grads + L.poff[BHH]; up.pw = grads + L.poff[PW]; up.vw = grads + L.poff[VW];
    up.pb = grads + L.poff[PB]; up.vb = grads + L.poff[VB];
    up.ans_in = L.ans_in; up.ans_ld = L.ans_ld; up.A = L.A;
    HIPCHK(unpack_f32(up, st));
    }
  }

  // Off-chain backward work for the steps [lo, hi): weight/bias grads of the
  // ConvLSTM, dx (conv2 output grad) and -- when VISION runs in the same call
  // -- the conv2/conv1 backward of those frames.  Every gradient accumulates
  // atomically into zeroed buffers, so chunks may run in any order.
  const bool vision_here = (phases & AAA_BWD_VISION) && (phases & AAA_BWD_CORE);
  bool dx_fused = false;   // the frame-resident BPTT computed dx (dY2) and conv2's bias gradient itself
  auto core_chunk = [&](int lo, int hi, hipStream_t s) -> int {
    const int rows = (hi - lo) * M;                       // pixels of these frames
    const int F1 = (hi - lo) * L.B;                       // frames
    const T* dz = Wt(L.dZ) + (size_t)lo * M * 512;
    {
      const int rc = lstm_wgrad<T>(dz, Wt(L.XH) + (size_t)lo * M * 192, rows, L.h, L.w, Wf(L.gWpl), s, s != st);
      if (rc) return rc;
    }
    if (!dx_fused) {  // dx_t for these steps: D[64][rows] = WdT[0:64] * gather(dZ)
      const ConvGeo g = ConvGeo{512, 512, 0, L.h, L.w, L.h, L.w, 3, 1, 1, 1}.prep();
      const T* WdT = (const T*)(pk + L.k_WdTl);
      const uint32_t zb = (uint32_t)((size_t)rows * 512 * L.esz);
      if constexpr (std::is_same<T, float>::value) {
        // 64x64 tiles (64x128 measured slower: occupancy); conv2's bias
        // gradient summed from the tile in the epilogue (no column-sum pass)
        EpiStoreBiasT<float> ep{Wf(L.dY2) + (size_t)lo * M * 64, 64, 64, rows, grads + L.poff[C1B]};
        using ED = EpiStoreBiasT<float>;
        switch (pipe_batched() ? env_int("AAA_DX_TILE", 0) : -1) {   // A/B: tools/ab_batched.sh
          case -1: HIPCHK((step_gemm<CfgFor<T>, false, T, T, ED>(WdT, 4608, 64, dz, g, rows, zb, ep, 64, 4608, s))); break;
          case 1: HIPCHK((step_gemm<Cfg64For<T>, true, T, T, ED>(WdT, 4608, 64, dz, g, rows, zb, ep, 64, 4608, s))); break;
          case 2: HIPCHK((step_gemm<CfgFor<T>, true, T, T, ED, 3, true>(WdT, 4608, 64, dz, g, rows, zb, ep, 64, 4608, s))); break;
          case 3: HIPCHK((step_gemm<CfgJFor<T>, true, T, T, ED>(WdT, 4608, 64, dz, g, rows, zb, ep, 64, 4608, s))); break;
          case 4:   // 64x64, 2-way in-WG split-K (8 waves), BK64
            HIPCHK((step_gemm<GemmCfg<T, 64, 64, 64, 2, 2, 2>, true, T, T, ED>(WdT, 4608, 64, dz, g, rows, zb, ep, 64, 4608,
                                                                                s)));
            break;
          default: HIPCHK((step_gemm<CfgFor<T>, true, T, T, ED>(WdT, 4608, 64, dz, g, rows, zb, ep, 64, 4608, s))); break;
        }
      } else {
        // bf16: dY2 stored bf16 (its readers round it to bf16 anyway), conv2's
        // bias gradient summed from the fp32 values in the epilogue
        EpiStoreBiasT<T> ep{Wt(L.dY2) + (size_t)lo * M * 64, 64, 64, rows, grads + L.poff[C1B]};
        // small grids: halo-staged conv, one frame per 64x128 tile
        // (tools/ubench/halo_tiles: 658 vs 771 us for the ring at C3)
        using HD = HaloCfg<__bf16, 64, 128, 64, 1, 2, 1, 176>;
        // 21x21 grids (168x168 frames): one frame per 512-column tile of 4 waves, 32-channel chunks
        using HW = HaloCfg<__bf16, 64, 512, 32, 1, 4, 1, 576>;
        if (halo_fits<HD>(L.h, L.w, 512) && env_int("AAA_HALO_DX", 1)) {
          const HaloParams hp{WdT, 4608, 64, dz, 512, 0, 512, zb, L.h, L.w, (hi - lo) * L.B, 1};
          HIPCHK((launch_halo<HD>(hp, ep, s)));
        } else if (halo_fits<HW>(L.h, L.w, 512) && env_int("AAA_HALO_DX", 1)) {
          const HaloParams hp{WdT, 4608, 64, dz, 512, 0, 512, zb, L.h, L.w, (hi - lo) * L.B, 1};
          HIPCHK((launch_halo<HW>(hp, ep, s)));
        } else {
          // larger grids (21x21 at 168x168): 64x128 on a 3-stage ring (bf16_tiles at C3: 643 vs 716 us for 64x64)
          HIPCHK((step_gemm<GemmCfg<T, 64, 128, 64, 2, 2>, true, T, T, EpiStoreBiasT<T>, 3>(WdT, 4608, 64, dz, g, rows,
                                                                                            zb, ep, 64, 4608, s)));
        }
      }
    }
    if (!vision_here) return AAA_OK;
    const T* dy2 = Wt(L.dY2) + (size_t)lo * M * 64;
    T* dy1 = Wt(L.dY1) + (size_t)lo * L.B * L.P1 * 32;
    const int rows1 = F1 * L.P1;
    constexpr bool f32 = std::is_same<T, float>::value;   // fp32 with AAA_CONV2_DGRAD_RING=0: conv1 bias by a column sum
    {  // conv2 wgrad
      const int rc = conv2_wgrad<T>(L, dy2, Wt(L.Y1) + (size_t)lo * L.B * L.P1 * 32, F1, Wf(L.gWp2), s);
      if (rc) return rc;
    }
    {  // conv2 dgrad (4 parity classes) -> dY1, then conv1 wgrad / bias
      int rc = conv2_dgrad<T>(L, pk, dy2, dy1, F1, grads + L.poff[C0B], s);
      if (!rc) rc = conv1_wgrad<T>(L, dy1, Wt(L.Xp) + (size_t)lo * L.B * (L.H + 2) * (L.W + 2) * 4, F1, Wf(L.gWp1), s);
      if (rc) return rc;
      if (f32 && !env_int("AAA_CONV2_DGRAD_RING", 1)) HIPCHK(colsum(dy1, 32, rows1, 32, grads + L.poff[C0B], s));
    }
    return AAA_OK;
  };

  if (phases & AAA_BWD_CORE) {
    hipStream_t ax = aux_stream();
    hipStream_t os = ax ? ax : st;     // stream for the off-chain chunks
    const int cs = chunk_steps(L);
    // ConvLSTM BPTT, t = T-1 .. 0
    if (io->dcT) HIPCHK(hipMemcpyAsync(Wf(L.dC), io->dcT, (size_t)M * 128 * 4, hipMemcpyDeviceToDevice, st));
    else HIPCHK(hipMemsetAsync(Wf(L.dC), 0, (size_t)M * 128 * 4, st));
    const int t1 = L.T - 1;
    // Sequential part: only the h rows (dh_{t-1}, fused with the gate backward
    // of step t-1); everything else runs in chunks off the chain.
    const int bwd_tile = step_tile((long)(128 / 32) * cdiv(M, 32), "AAA_BPTT_TILE", true, L.dt == AAA_BF16);
    // pipe (glds.h) tiles reduce the gate-bias partials in their epilogue;
    // the register-staged ones leave the bias to a column sum over dZ
    const int bj = bwd_tile == 7 || bwd_tile == 19 || bwd_tile == 20 ? 128 : (bwd_tile == 21 || bwd_tile == 22 || bwd_tile == 23 ? 64 : (bwd_tile >= 9 && bwd_tile != 14 ? 32 : 64));
    const bool pipe = (bwd_tile == 4 && pipe_even<CfgK4BFor<T>>()) || (bwd_tile == 5 && pipe_even<CfgK4For<T>>()) ||
                      (bwd_tile == 6 && pipe_even<C>()) || bwd_tile == 7 || bwd_tile == 8 || bwd_tile >= 19 ||
                      (bwd_tile == 9 && pipe_even<GemmCfg<T, 64, 32, 128, 2, 1, 4>>()) ||
                      (bwd_tile == 10 && pipe_even<GemmCfg<T, 32, 32, 128, 1, 1, 4>>()) ||
                      ((bwd_tile == 11 || bwd_tile == 12 || bwd_tile == 16) && pipe_even<GemmCfg<T, 32, 32, 64, 1, 1, 4>>()) ||
                      (bwd_tile == 13 && pipe_even<GemmCfg<T, 32, 32, 128, 1, 1, 8>>()) ||
                      (bwd_tile == 15 && pipe_even<GemmCfg<T, 64, 32, 64, 2, 1, 4>>());
    const int ntj = cdiv(M, bj);
    float* part = pipe ? Wf(L.dZp) : nullptr;
    const bool g16 = gates_f16(L.dt, M);
    const int fb = frames_bwd(L, g16);   // the whole chain in one frame-resident launch (workgroups per frame)
    // fp32: the frame-group BPTT (recur_bwd_f32.h, G = 8) behind the forward's frame-group kernel
    const bool fb32 = std::is_same<T, float>::value && f32_frames(L) == 8 && env_int("AAA_F32_FRAMES_BWD", 1);
    if (fb32) part = nullptr;   // the kernel writes per-(step, frame) bias partials, step T-1's included
    if (fb) {
    } else if (g16)
      HIPCHK((gate_bwd_last<T, _Float16>(M, bj, Wf(L.dO) + (size_t)t1 * M * 128, io->dhT,
                                         (const _Float16*)(ws + L.Gt) + (size_t)t1 * M * 512,
                                         Wf(L.Cst) + (size_t)t1 * M * 128, Wf(L.Cst) + (size_t)(t1 + 1) * M * 128,
                                         Wf(L.dC), Wt(L.dZ) + (size_t)t1 * M * 512,
                                         part ? part + (size_t)t1 * ntj * 512 : nullptr, st)));
    else
      HIPCHK((gate_bwd_last<T, float>(M, bj, Wf(L.dO) + (size_t)t1 * M * 128, io->dhT, Wf(L.Gt) + (size_t)t1 * M * 512,
                                      Wf(L.Cst) + (size_t)t1 * M * 128, Wf(L.Cst) + (size_t)(t1 + 1) * M * 128,
                                      Wf(L.dC), Wt(L.dZ) + (size_t)t1 * M * 512,
                                      part ? part + (size_t)t1 * ntj * 512 : nullptr, st)));
    const uint32_t dz_bytes = (uint32_t)((size_t)M * 512 * L.esz);  // one step slice of dZ
    const T* WdTh = (const T*)(pk + L.k_WdTl) + (size_t)64 * 4608;
    int done_hi = L.T;   // chunks [lo, done_hi) not yet issued
    auto flush = [&](int ready_lo) -> int {   // dz of steps >= ready_lo are final
      while (done_hi - ready_lo >= cs || (ready_lo == 0 && done_hi > 0)) {
        const int lo = std::max(ready_lo, done_hi - cs);
        if (ax) HIPCHK(stream_order(st, ax));
        int rc = core_chunk(lo, done_hi, os);
        if (rc) return rc;
        done_hi = lo;
      }
      return AAA_OK;
    };
    if (fb) {
      if constexpr (!std::is_same<T, float>::value) {
        RecBwdParams rp{(const __bf16*)(pk + L.k_Wbf), Wf(L.dO), (const _Float16*)(ws + L.Gt), Wf(L.Cst), io->dhT,
                        Wf(L.dC), Wt(L.dZ), Wf(L.dZp), io->dh0, Wt(L.dY2), Wf(L.dxb), (int*)(ws + L.rflags),
                        L.T, L.B, L.h, L.w, L.P, nullptr, (int)g_pair_spin};
        HIPCHK(hipMemsetAsync(Wf(L.dxb), 0, (size_t)L.B * 64 * 4, st));
        if (fb == 2) {
          HIPCHK(hipMemsetAsync(ws + L.rflags, 0, (size_t)2 * L.B * 4, st));
          int dev = 0;
          HIPCHK(hipGetDevice(&dev));
          if (!(rp.report = pair_report(dev))) return fail(AAA_E_LAUNCH, "cannot map the paired-kernel report word");
        }
        {
          // work: the h rows over T-1 steps (+ dh0) and the dx rows over all T (the batched dx it replaces)
          TimerScope tim(AAA_TIMER_BPTT_STEP, st, 2.0 * M * 4608 * (128.0 * (L.T - 1 + (io->dh0 ? 1 : 0)) + 64.0 * L.T),
                         strf("bf16 frame-resident BPTT + dx, %d steps per launch, %d WG per frame, fp16 gates", L.T, fb));
          HIPCHK(fb == 2 ? convlstm_bwd_pairs(rp, st) : convlstm_bwd_frames(rp, st));
        }
        HIPCHK(colsum<float>(Wf(L.dxb), 64, L.B, 64, grads + L.poff[C1B], st));
        dx_fused = true;
      }
    }
    if (fb32) {
      if constexpr (std::is_same<T, float>::value) {
        HIPCHK(hipMemsetAsync(ws + L.rflags, 0, (size_t)8 * L.B * 4, st));
        int dev = 0;
        HIPCHK(hipGetDevice(&dev));
        int* rep = pair_report(dev);
        if (!rep) return fail(AAA_E_LAUNCH, "cannot map the frame-group report word");
        RecBwdF32Params rp{(const float*)(pk + L.k_Wb32), Wf(L.dO), Wf(L.Gt), Wf(L.Cst), Wf(L.dC), Wf(L.dZ),
                           Wf(L.dZp), io->dh0, Wf(L.xpart), (int*)(ws + L.rflags), rep, (int)g_pair_spin,
                           L.T, L.B, L.h, L.w, L.P, {}};
        TimerScope tim(AAA_TIMER_BPTT_STEP, st, 2.0 * M * 128 * 4608 * (L.T - 1 + (io->dh0 ? 1 : 0)),
                       strf("fp32 frame-group BPTT (dh rows), %d steps per launch, 8 WG per frame", L.T));
        HIPCHK(convlstm_bwd_f32(rp, st));
      }
    }
    for (int t = (fb || fb32) ? -1 : t1; t >= 0; --t) {
      const int rc0 = flush(t);   // dz_t .. dz_{T-1} are final here
      if (rc0) return rc0;
      const bool prev = t > 0;
      if (!prev && !io->dh0) break;
      const ConvGeo g = ConvGeo{512, 512, 0, L.h, L.w, L.h, L.w, 3, 1, 1, 1}.prep();
      const T* dzt = Wt(L.dZ) + (size_t)t * M * 512;
      TimerScope tim(AAA_TIMER_BPTT_STEP, st, 2.0 * M * 128 * 4608, strf("%s dh dgrad + fused gate bwd, K=4608, AAA_BPTT_TILE %d%s", std::is_same<T, float>::value ? "fp32" : "bf16", bwd_tile, g16 ? ", fp16 gates" : ""));
      auto step = [&](auto gtag) -> hipError_t {
        using GT = decltype(gtag);
        using EB = EpiConvLstmBwd<T, GT>;
        EB ep{nullptr,
              prev ? (const GT*)(ws + L.Gt) + (size_t)(t - 1) * M * 512 : nullptr,
              prev ? Wf(L.Cst) + (size_t)(t - 1) * M * 128 : nullptr,
              Wf(L.Cst) + (size_t)t * M * 128,
              prev ? Wf(L.dO) + (size_t)(t - 1) * M * 128 : nullptr,
              Wf(L.dC),
              prev ? Wt(L.dZ) + (size_t)(t - 1) * M * 512 : nullptr,
              prev ? nullptr : io->dh0, prev ? 1 : 0, M, 64,
              part && prev ? part + (size_t)(t - 1) * ntj * 512 : nullptr};
        if constexpr (!std::is_same<GT, float>::value) {   // fp16 gates: the bf16 tiles only (gates_f16)
          if constexpr (std::is_same<T, float>::value) return hipErrorInvalidValue;
          else if (bwd_tile == 7)
            return step_gemm<GemmCfg<T, 128, 128, 128, 2, 2, 2>, true>(WdTh, 4608, 128, dzt, g, M, dz_bytes, ep, 128,
                                                                        4608, st);
          else if (bwd_tile == 19)   // 128x128, 4 waves of 64x64, BK64
            return step_gemm<GemmCfg<T, 128, 128, 64, 2, 2>, true>(WdTh, 4608, 128, dzt, g, M, dz_bytes, ep, 128, 4608,
                                                                    st);
          else if (bwd_tile == 20)   // the same on a 3-stage ring
            return step_gemm<GemmCfg<T, 128, 128, 64, 2, 2>, true, T, T, EB, 3, true>(WdTh, 4608, 128, dzt, g, M,
                                                                                      dz_bytes, ep, 128, 4608, st);
          else if (bwd_tile == 22)   // 128x64, BK128, 4-way in-WG split-K (8 waves)
            return step_gemm<GemmCfg<T, 128, 64, 128, 2, 1, 4>, true>(WdTh, 4608, 128, dzt, g, M, dz_bytes, ep, 128,
                                                                       4608, st);
          else if (bwd_tile == 23)   // 64x64, BK128, 2-way in-WG split-K (8 waves)
            return step_gemm<GemmCfg<T, 64, 64, 128, 2, 2, 2>, true>(WdTh, 4608, 128, dzt, g, M, dz_bytes, ep, 128,
                                                                      4608, st);
          else if (bwd_tile == 24)   // 64x32, BK128, 4-way in-WG split-K (8 waves)
            return step_gemm<GemmCfg<T, 64, 32, 128, 2, 1, 4>, true>(WdTh, 4608, 128, dzt, g, M, dz_bytes, ep, 128,
                                                                      4608, st);
          else if (bwd_tile == 21)   // 128x64, 4 waves of 64x32, BK64
            return step_gemm<GemmCfg<T, 128, 64, 64, 2, 2>, true>(WdTh, 4608, 128, dzt, g, M, dz_bytes, ep, 128, 4608,
                                                                   st);
          else
            return step_gemm<GemmCfg<T, 128, 64, 128, 2, 1, 2>, true>(WdTh, 4608, 128, dzt, g, M, dz_bytes, ep, 128,
                                                                       4608, st);
        } else {
          // tiles 19-24 other than 22 exist for fp16 gate storage only: fail loudly, never fall back
          if (bwd_tile >= 19 && bwd_tile != 22) return hipErrorInvalidValue;
          switch (bwd_tile) {
            case 1: return step_gemm<CfgKFor<T>, false>(WdTh, 4608, 128, dzt, g, M, dz_bytes, ep, 128, 4608, st);
            case 2: return step_gemm<CfgK4For<T>, false>(WdTh, 4608, 128, dzt, g, M, dz_bytes, ep, 128, 4608, st);
            case 3: return step_gemm<CfgK4BFor<T>, false>(WdTh, 4608, 128, dzt, g, M, dz_bytes, ep, 128, 4608, st);
            case 4:   // 3-stage ring, DMA interleaved with the MFMAs (tools/ubench/step_ablate: 57.9 vs 59.4 us)
              return step_gemm<CfgK4BFor<T>, true, T, T, EB, 3, true>(WdTh, 4608, 128, dzt, g, M, dz_bytes, ep, 128,
                                                                       4608, st);
            case 5: return step_gemm<CfgK4For<T>, true>(WdTh, 4608, 128, dzt, g, M, dz_bytes, ep, 128, 4608, st);
            case 6: return step_gemm<C, true>(WdTh, 4608, 128, dzt, g, M, dz_bytes, ep, 128, 4608, st);
            case 7:   // bf16: 128x128, BK128, 2-way in-WG split-K (tools/ubench/bf16_tiles: 48 vs 53-60 us at C3)
              if constexpr (std::is_same<T, float>::value) return hipErrorInvalidValue;
              else return step_gemm<GemmCfg<T, 128, 128, 128, 2, 2, 2>, true>(WdTh, 4608, 128, dzt, g, M, dz_bytes, ep,
                                                                              128, 4608, st);
            case 8:   // bf16: 128x64, BK128, 2-way in-WG split-K, 4 waves (small batches)
              if constexpr (std::is_same<T, float>::value) return hipErrorInvalidValue;
              else return step_gemm<GemmCfg<T, 128, 64, 128, 2, 1, 2>, true>(WdTh, 4608, 128, dzt, g, M, dz_bytes, ep,
                                                                             128, 4608, st);
            case 22:   // bf16 with fp32 gate storage (AAA_FUSED_X=0 / AAA_GATES_F16=0): the default small-batch tile
              if constexpr (std::is_same<T, float>::value) return hipErrorInvalidValue;
              else return step_gemm<GemmCfg<T, 128, 64, 128, 2, 1, 4>, true>(WdTh, 4608, 128, dzt, g, M, dz_bytes, ep,
                                                                             128, 4608, st);
            case 9:   // 64x32, BK128, 4-way in-WG split-K, 3-stage ring, interleaved DMA
              return step_gemm<GemmCfg<T, 64, 32, 128, 2, 1, 4>, true, T, T, EB, 3, true>(WdTh, 4608, 128, dzt, g, M,
                                                                                          dz_bytes, ep, 128, 4608, st);
            case 10:   // 32x32, BK128, 4-way in-WG split-K, 2-stage ring (2 WGs per CU, desynchronised barriers)
              return step_gemm<GemmCfg<T, 32, 32, 128, 1, 1, 4>, true, T, T, EB, 2, true>(WdTh, 4608, 128, dzt, g, M,
                                                                                         dz_bytes, ep, 128, 4608, st);
            case 11:   // 32x32, BK64, 4-way in-WG split-K, 3-stage ring
              return step_gemm<GemmCfg<T, 32, 32, 64, 1, 1, 4>, true, T, T, EB, 3, true>(WdTh, 4608, 128, dzt, g, M,
                                                                                        dz_bytes, ep, 128, 4608, st);
            case 12:   // 32x32, BK64, 4-way in-WG split-K, 4-stage ring
              return step_gemm<GemmCfg<T, 32, 32, 64, 1, 1, 4>, true, T, T, EB, 4, true>(WdTh, 4608, 128, dzt, g, M,
                                                                                        dz_bytes, ep, 128, 4608, st);
            case 13:   // 32x32, BK128, 8-way in-WG split-K (8 waves), 2-stage ring
              return step_gemm<GemmCfg<T, 32, 32, 128, 1, 1, 8>, true, T, T, EB, 2, true>(WdTh, 4608, 128, dzt, g, M,
                                                                                         dz_bytes, ep, 128, 4608, st);
            case 15:   // 64x32, BK64, 4-way in-WG split-K, 3-stage ring
              return step_gemm<GemmCfg<T, 64, 32, 64, 2, 1, 4>, true, T, T, EB, 3, true>(WdTh, 4608, 128, dzt, g, M,
                                                                                        dz_bytes, ep, 128, 4608, st);
            case 16:   // 32x32, BK64, 4-way in-WG split-K, 3-stage ring, DMA issued before the MFMAs
              return step_gemm<GemmCfg<T, 32, 32, 64, 1, 1, 4>, true, T, T, EB, 3, false>(WdTh, 4608, 128, dzt, g, M,
                                                                                         dz_bytes, ep, 128, 4608, st);
            default: return step_gemm<C, false>(WdTh, 4608, 128, dzt, g, M, dz_bytes, ep, 128, 4608, st);
          }
        }
      };
      const hipError_t e = g16 ? step(_Float16{}) : step(float{});
      HIPCHK(e);
    }
    { const int rc0 = flush(0); if (rc0) return rc0; }
    // gate-bias gradient: column sum of the per-(step, tile) partials, or of dZ itself
    if (fb)   // per (step, frame[, pixel half]) partials
      HIPCHK(colsum<float>(Wf(L.dZp), 512, L.T * L.B * fb, 512, Wf(L.gbl), st));
    else if (fb32)   // per (step, frame) partials
      HIPCHK(colsum<float>(Wf(L.dZp), 512, L.T * L.B, 512, Wf(L.gbl), st));
    else if (part) HIPCHK(colsum<float>(part, 512, L.T * ntj, 512, Wf(L.gbl), st));
    else HIPCHK(colsum<T>(Wt(L.dZ), 512, F * P, 512, Wf(L.gbl), st));
    if (io->dc0) HIPCHK(hipMemcpyAsync(io->dc0, Wf(L.dC), (size_t)M * 128 * 4, hipMemcpyDeviceToDevice, st));
    if (ax) HIPCHK(stream_order(ax, st));   // join
    LstmGrads lg;
    for (int g = 0; g < 4; ++g) {
      lg.wx[g] = grads + L.poff[XI_W + 3 * g];
      lg.bx[g] = grads + L.poff[XI_B + 3 * g];
      lg.wh[g] = grads + L.poff[HI_W + 3 * g];
    }
    // with VISION in this call the ConvLSTM grads unpack in the vision phase's launch
    if (!(phases & AAA_BWD_VISION)) HIPCHK(unpack_lstm(Wf(L.gWpl), Wf(L.gbl), lg, st));
    else core_unpack = lg;
  }

  if (phases & AAA_BWD_VISION) {
    if (!vision_here) {   // VISION alone: its chunk work over all frames, here
      const int rows1 = F * L.P1;
      constexpr bool f32 = std::is_same<T, float>::value;
      {
        const int rc = vision_bwd<T>(L, pk, Wt(L.dY2), Wt(L.Y1), Wt(L.Xp), Wt(L.dY1), F, Wf(L.gWp2), Wf(L.gWp1),
                                     grads + L.poff[C0B], st);
        if (rc) return rc;
        if (f32 && !env_int("AAA_CONV2_DGRAD_RING", 1)) HIPCHK(colsum(Wt(L.dY1), 32, rows1, 32, grads + L.poff[C0B], st));
      }
    }
    HIPCHK(unpack_cv((phases & AAA_BWD_CORE) ? Wf(L.gWpl) : nullptr, Wf(L.gbl), core_unpack, Wf(L.gWp2),
                     grads + L.poff[C1W], Wf(L.gWp1), grads + L.poff[C0W], st));
  }
  return AAA_OK;
}

// ------------------------------------------------------ component entries --
// One reference module per entry, on caller-owned buffers,
// through the same kernels aaa_forward / aaa_backward run for that module.

// ConvLSTMCell(64, 128, 3) at one step (attention.py:110-126): packed weights
// (the four ConvLSTM layouts of pack_lstm_all) and the workspace that carries
// the forward's saved activations to the backward.
struct CellLayout {
  int B, h, w, M, dt, esz;
  size_t k_WpX, k_WpH, k_WdTl, k_bl, k_WpXH, packed;
  size_t XH, Cst, Hs, Gt, dZ, dC, dO, dX, gW, gb, ws;
};

static int cell_layout(const aaa_cell_desc* d, CellLayout& C) {
  if (!d) return fail(AAA_E_ARG, "cell desc is NULL");
  if (d->B < 1 || d->h < 1 || d->w < 1) return fail(AAA_E_ARG, "cell: need B, h, w >= 1");
  if (d->dtype != AAA_F32 && d->dtype != AAA_BF16) return fail(AAA_E_ARG, "cell: bad dtype %d", d->dtype);
  const size_t M = (size_t)d->B * d->h * d->w, e = d->dtype == AAA_BF16 ? 2 : 4;
  if (M * 512 * 4 >= (size_t(1) << 31))   // dZ / gates: buffer descriptors and int indices
    return fail(AAA_E_ARG, "cell: B*h*w = %zu pixels is above the 2 GiB descriptor range; split the batch", M);
  C.B = d->B; C.h = d->h; C.w = d->w; C.M = (int)M; C.dt = d->dtype; C.esz = (int)e;
  size_t p = 0;
  auto take = [&](size_t bytes) { size_t r = p; p = al256(p + bytes); return r; };
  C.k_WpX = take(512 * 576 * e);
  C.k_WpH = take(512 * 1152 * e);
  C.k_WdTl = take(192 * 4608 * e);
  C.k_bl = take(512 * 4);
  C.k_WpXH = take(512 * 1728 * e);
  C.packed = p;
  p = 0;
  C.XH = take(2 * M * 192 * e);
  C.Cst = take(2 * M * 128 * 4);
  C.Hs = take(M * 128 * 4);
  C.Gt = take(M * 512 * 4);
  C.dZ = take(M * 512 * e);
  C.dC = take(M * 128 * 4);
  C.dO = take(M * 128 * 4);
  C.dX = take(M * 64 * 4);
  C.gW = take(512 * 1728 * 4);
  C.gb = take(512 * 4);
  C.ws = p;
  return AAA_OK;
}

// the cell's 12 state_dict tensors, concatenated in state_dict order
// (Wx{g}.weight (128,64,3,3), Wx{g}.bias (128), Wh{g}.weight (128,128,3,3) for g = i, f, c, o)
constexpr size_t kCellGate = 128 * 64 * 9 + 128 + 128 * 128 * 9;
template <typename P, typename Ptrs>
static void cell_ptrs(P* base, Ptrs& lp) {
  for (int g = 0; g < 4; ++g) {
    lp.wx[g] = base + g * kCellGate;
    lp.bx[g] = base + g * kCellGate + 128 * 64 * 9;
    lp.wh[g] = base + g * kCellGate + 128 * 64 * 9 + 128;
  }
}

template <typename T>
static int cell_fwd_impl(const CellLayout& C, const char* pk, const float* x, const float* h0, const float* c0,
                         float* h1, float* c1, char* ws, hipStream_t st) {
  const int M = C.M;
  T* xh = (T*)(ws + C.XH);
  float* cst = (float*)(ws + C.Cst);
  HIPCHK(cell_xh<T>(M, x, h0, xh, st));
  if (c0) HIPCHK(hipMemcpyAsync(cst, c0, (size_t)M * 128 * 4, hipMemcpyDeviceToDevice, st));
  else HIPCHK(hipMemsetAsync(cst, 0, (size_t)M * 128 * 4, st));
  auto run = [&](auto gtag) -> int {
    using GT = decltype(gtag);
    EpiConvLstmFwd<T, GT> ep{cst, cst + (size_t)M * 128, (float*)(ws + C.Hs), xh + (size_t)M * 192,
                             (GT*)(ws + C.Gt), M, (const float*)(pk + C.k_bl)};
    return fused_step<T, GT>((const T*)(pk + C.k_WpXH), xh, C.h, C.w, M, ep, st);
  };
  const int rc = gates_f16(C.dt, M) ? run(_Float16{}) : run(float{});
  if (rc) return rc;
  if (h1) HIPCHK(hipMemcpyAsync(h1, ws + C.Hs, (size_t)M * 128 * 4, hipMemcpyDeviceToDevice, st));
  if (c1) HIPCHK(hipMemcpyAsync(c1, cst + (size_t)M * 128, (size_t)M * 128 * 4, hipMemcpyDeviceToDevice, st));
  return AAA_OK;
}

template <typename T>
static int cell_bwd_impl(const CellLayout& C, const char* pk, const float* dh1, const float* dc1, float* dx,
                         float* dh0, float* dc0, float* grads, char* ws, hipStream_t st) {
  const int M = C.M;
  const T* xh = (const T*)(ws + C.XH);
  const float* cst = (const float*)(ws + C.Cst);
  float* dC = (float*)(ws + C.dC);
  T* dZ = (T*)(ws + C.dZ);
  if (dc1) HIPCHK(hipMemcpyAsync(dC, dc1, (size_t)M * 128 * 4, hipMemcpyDeviceToDevice, st));
  else HIPCHK(hipMemsetAsync(dC, 0, (size_t)M * 128 * 4, st));
  const float* dh = dh1;
  if (!dh) {
    HIPCHK(hipMemsetAsync(ws + C.dO, 0, (size_t)M * 128 * 4, st));
    dh = (const float*)(ws + C.dO);
  }
  auto run = [&](auto gtag) -> int {
    using GT = decltype(gtag);
    // gate backward (dz of the four gates, dc carry -> dc0)
    HIPCHK((gate_bwd_last<T, GT>(M, 64, dh, nullptr, (const GT*)(ws + C.Gt), cst, cst + (size_t)M * 128, dC, dZ,
                                 nullptr, st)));
    // [dx | dh0] = W^T dz: the dgrad of all eight gate convs into [x | h] in one GEMM
    EpiConvLstmBwd<T, GT> ep{dx ? dx : (float*)(ws + C.dX), nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                             dh0, 0, M, 0, nullptr};
    const ConvGeo g = ConvGeo{512, 512, 0, C.h, C.w, C.h, C.w, 3, 1, 1, 1}.prep();
    HIPCHK((step_gemm<CfgFor<T>, false>((const T*)(pk + C.k_WdTl), 4608, 192, (const T*)dZ, g, M,
                                         (uint32_t)((size_t)M * 512 * C.esz), ep, 192, 4608, st)));
    return AAA_OK;
  };
  int rc = gates_f16(C.dt, M) ? run(_Float16{}) : run(float{});
  if (rc) return rc;
  if (dc0) HIPCHK(hipMemcpyAsync(dc0, dC, (size_t)M * 128 * 4, hipMemcpyDeviceToDevice, st));
  if (grads) {   // weight grads (all 8 convs, one GEMM over the pixels) and the gate biases
    float* gW = (float*)(ws + C.gW);
    float* gb = (float*)(ws + C.gb);
    HIPCHK(hipMemsetAsync(gW, 0, (size_t)512 * 1728 * 4, st));
    HIPCHK(hipMemsetAsync(gb, 0, 512 * 4, st));
    if ((rc = lstm_wgrad<T>(dZ, xh, M, C.h, C.w, gW, st, false))) return rc;
    HIPCHK(colsum<T>(dZ, 512, M, 512, gb, st));
    LstmGrads lg;
    cell_ptrs(grads, lg);
    HIPCHK(unpack_lstm(gW, gb, lg, st));
  }
  return AAA_OK;
}

// VisionNetwork.vision_cnn over N frames: a Layout with B = N, T = 1 gives the
// geometry and the packed-weight offsets (the conv weights are the first three
// packed layouts, the vision params the first four state_dict tensors).
struct CnnLayout {
  Layout L;
  size_t Xp, Y1, dY2, dY1, gW1, gW2, ws;
};

static int cnn_layout(const aaa_cnn_desc* d, CnnLayout& C) {
  if (!d) return fail(AAA_E_ARG, "cnn desc is NULL");
  if (d->N < 1) return fail(AAA_E_ARG, "cnn: need N >= 1");
  const aaa_cfg cfg{d->N, 1, d->H, d->W, 4, 18, d->dtype, 0};
  int r = build_layout(&cfg, C.L, 1);
  if (r) return r;
  const Layout& L = C.L;
  const size_t F = L.F, e = L.esz;
  size_t p = 0;
  auto take = [&](size_t bytes) { size_t q = p; p = al256(p + bytes); return q; };
  C.Xp = take(F * (L.H + 2) * (L.W + 2) * 4 * e);
  C.Y1 = take(F * L.P1 * 32 * e);
  C.dY2 = take(F * L.P * 64 * e);
  C.dY1 = take(F * L.P1 * 32 * e);
  C.gW1 = take(32 * 256 * 4);
  C.gW2 = take(64 * 512 * 4);
  C.ws = p;
  return AAA_OK;
}

template <typename T>
static int cnn_pack_impl(const Layout& L, const float* prm, char* pk, hipStream_t st) {
  HIPCHK(pack_conv1_rgbx<T>(prm + L.poff[C0W], (T*)(pk + L.k_Wp1), st));
  HIPCHK(pack_conv<T>(prm + L.poff[C1W], 64, 32, 4, (T*)(pk + L.k_Wp2), st));
  HIPCHK(pack_conv2_classes<T>(prm + L.poff[C1W], (T*)(pk + L.k_WdT2), st));
  return AAA_OK;
}

template <typename T>
static int cnn_bwd_impl(const CnnLayout& CL, const char* pk, const float* dy2, float* dy1, float* grads, char* ws,
                        hipStream_t st) {
  const Layout& L = CL.L;
  const int N = L.F;
  const T* dy2t;
  if constexpr (std::is_same<T, float>::value) {
    dy2t = dy2;
  } else {
    HIPCHK((cast<float, T>((long)N * L.P * 64, dy2, (T*)(ws + CL.dY2), st)));
    dy2t = (const T*)(ws + CL.dY2);
  }
  float* gW1 = (float*)(ws + CL.gW1);
  float* gW2 = (float*)(ws + CL.gW2);
  T* dY1 = (T*)(ws + CL.dY1);
  HIPCHK(hipMemsetAsync(grads, 0, L.poff[XI_W] * 4, st));
  HIPCHK(hipMemsetAsync(gW1, 0, 32 * 256 * 4, st));
  HIPCHK(hipMemsetAsync(gW2, 0, 64 * 512 * 4, st));
  HIPCHK(colsum<float>(dy2, 64, N * L.P, 64, grads + L.poff[C1B], st));   // conv2 bias (fp32 grads)
  const int rc = vision_bwd<T>(L, pk, dy2t, (const T*)(ws + CL.Y1), (const T*)(ws + CL.Xp), dY1, N, gW2, gW1,
                               grads + L.poff[C0B], st);
  if (rc) return rc;
  if (std::is_same<T, float>::value && !env_int("AAA_CONV2_DGRAD_RING", 1))
    HIPCHK(colsum(dY1, 32, N * L.P1, 32, grads + L.poff[C0B], st));
  HIPCHK(unpack_conv(gW2, 64, 32, 4, grads + L.poff[C1W], st));
  HIPCHK(unpack_conv1_rgbx(gW1, grads + L.poff[C0W], st));
  if (dy1) HIPCHK((cast<T, float>((long)N * L.P1 * 32, dY1, dy1, st)));
  return AAA_OK;
}

// ----------------------------------------------------- unit-test entries --
template <typename T>
static int conv_nhwc_impl(const aaa_conv_desc* d, const float* x, const float* w, const float* bias, float* y,
                          hipStream_t st) {
  using C = CfgFor<T>;
  constexpr int NT = C::NT;
  const int K = d->KH * d->KW * d->Cin, M = d->N * d->Hout * d->Wout;
  using LA = LdRows<float, T, C::BI, C::BK, NT>;
  typename LA::Params pa{w, K, d->Cout};
  const ConvGeo g = ConvGeo{d->Cin, d->Cin, 0, d->Hin, d->Win, d->Hout, d->Wout, d->KW, d->stride, d->pad, 0}.prep();
  EpiStoreT<float> ep{y, d->Cout, d->Cout, M, bias, 0};
  const int tpt = C::BK / std::max(1, d->Cin);
  if (d->Cin % C::BK == 0 || (C::BK % d->Cin == 0 && (tpt % d->KW == 0 || d->KW % tpt == 0))) {   // hot-path loaders
    using LAB = LdRowsB<float, T, C::BI, C::BK, NT>;
    using LB = LdIm2colB<float, T, C::BJ, C::BK, NT>;
    const uint32_t xb = (uint32_t)((size_t)d->N * d->Hin * d->Win * d->Cin * 4);
    HIPCHK((launch_gemm<C, LAB, LB>(typename LAB::Params{w, K, d->Cout}, typename LB::Params{x, g, M, xb}, ep, d->Cout,
                                    M, K, 1, st)));
  } else if (d->Cin % 4 == 0) {
    using LB = LdIm2col<float, T, C::BJ, C::BK, NT, true>;
    HIPCHK((launch_gemm<C, LA, LB>(pa, typename LB::Params{x, g, M}, ep, d->Cout, M, K, 1, st)));
  } else {
    using LB = LdIm2col<float, T, C::BJ, C::BK, NT, false>;
    HIPCHK((launch_gemm<C, LA, LB>(pa, typename LB::Params{x, g, M}, ep, d->Cout, M, K, 1, st)));
  }
  return AAA_OK;
}

template <typename T>
static int dgrad_nhwc_impl(const aaa_conv_desc* d, const float* dy, const float* wT, float* dx, hipStream_t st) {
  using C = CfgFor<T>;
  constexpr int NT = C::NT;
  const int K = d->KH * d->KW * d->Cout, M = d->N * d->Hin * d->Win;
  using LA = LdRows<float, T, C::BI, C::BK, NT>;
  using LB = LdIm2col<float, T, C::BJ, C::BK, NT, true>;
  typename LA::Params pa{wT, K, d->Cin};
  const ConvGeo g = ConvGeo{d->Cout, d->Cout, 0, d->Hout, d->Wout, d->Hin, d->Win, d->KW, d->stride, d->pad, 1}.prep();
  EpiStoreT<float> ep{dx, d->Cin, d->Cin, M, nullptr, 0};
  if (d->stride == 1 && d->Cout % C::BK == 0) {
    using LAB = LdRowsB<float, T, C::BI, C::BK, NT>;
    using LBB = LdIm2colB<float, T, C::BJ, C::BK, NT>;
    const uint32_t yb = (uint32_t)((size_t)d->N * d->Hout * d->Wout * d->Cout * 4);
    HIPCHK((launch_gemm<C, LAB, LBB>(typename LAB::Params{wT, K, d->Cin}, typename LBB::Params{dy, g, M, yb}, ep,
                                     d->Cin, M, K, 1, st)));
    return AAA_OK;
  }
  HIPCHK((launch_gemm<C, LA, LB>(pa, typename LB::Params{dy, g, M}, ep, d->Cin, M, K, 1, st)));
  return AAA_OK;
}

template <typename T>
static int wgrad_nhwc_impl(const aaa_conv_desc* d, const float* x, const float* dy, float* dw, hipStream_t st) {
  using C = CfgFor<T>;
  constexpr int NT = C::NT;
  const int Kp = d->KH * d->KW * d->Cin, M = d->N * d->Hout * d->Wout;
  HIPCHK(hipMemsetAsync(dw, 0, (size_t)d->Cout * Kp * 4, st));
  using LA = LdRowsT<float, T, C::BI, C::BK, NT>;
  typename LA::Params pa{dy, d->Cout, d->Cout};
  const ConvGeo g = ConvGeo{d->Cin, d->Cin, 0, d->Hin, d->Win, d->Hout, d->Wout, d->KW, d->stride, d->pad, 0}.prep();
  EpiStore<true> ep{dw, Kp, d->Cout, Kp};
  const int tiles = cdiv(d->Cout, C::BI) * cdiv(Kp, C::BJ);
  const int ns = wgrad_splits(tiles, M, C::BK);
  if (d->Cin % 4 == 0 && d->Cout % 4 == 0) {   // hot-path loaders
    using LAB = LdRowsTB<float, T, C::BI, C::BK, NT>;
    using LB = LdIm2colTB<float, T, C::BJ, C::BK, NT>;
    const uint32_t xb = (uint32_t)((size_t)d->N * d->Hin * d->Win * d->Cin * 4);
    HIPCHK((launch_gemm<C, LAB, LB>(typename LAB::Params{dy, d->Cout, d->Cout, M}, typename LB::Params{x, g, Kp, xb},
                                    ep, d->Cout, Kp, M, ns, st)));
  } else if (d->Cin % 4 == 0) {
    using LB = LdIm2colT<float, T, C::BJ, C::BK, NT, true>;
    HIPCHK((launch_gemm<C, LA, LB>(pa, typename LB::Params{x, g, Kp}, ep, d->Cout, Kp, M, ns, st)));
  } else {
    using LB = LdIm2colT<float, T, C::BJ, C::BK, NT, false>;
    HIPCHK((launch_gemm<C, LA, LB>(pa, typename LB::Params{x, g, Kp}, ep, d->Cout, Kp, M, ns, st)));
  }
  return AAA_OK;
}

}  // namespace aaa

using namespace aaa;

extern "C" {

int aaa_abi_version(void) { return AAA_ABI_VERSION; }

int aaa_fastdiv_check(unsigned d, unsigned lo, unsigned hi, unsigned long long* mismatches) {
  if (!mismatches || d == 0 || d >= (1u << 31) || hi > (1u << 31) || lo > hi)
    return fail(AAA_E_ARG, "fastdiv_check: need 1 <= d < 2^31 and lo <= hi <= 2^31");
  const FastDiv fd(d);
  // exhaustive over [lo, hi): split over host threads; the exact quotient is
  // carried incrementally (no hardware division in the loop)
  const unsigned nthr = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  std::vector<unsigned long long> bad(nthr, 0);
  std::vector<std::thread> th;
  const unsigned long long span = hi - lo, per = (span + nthr - 1) / nthr;
  for (unsigned t = 0; t < nthr; ++t) {
    th.emplace_back([&, t]() {
      const unsigned long long a = lo + std::min(span, t * per), b = lo + std::min(span, (t + 1) * per);
      if (a >= b) return;
      uint32_t q = (uint32_t)(a / d), r = (uint32_t)(a % d);
      unsigned long long nb = 0;
      for (unsigned long long n = a; n < b; ++n) {
        nb += fd.div((uint32_t)n) != q;
        if (++r == d) { r = 0; ++q; }
      }
      bad[t] = nb;
    });
  }
  for (auto& x : th) x.join();
  unsigned long long tot = 0;
  for (auto v : bad) tot += v;
  *mismatches = tot;
  return AAA_OK;
}

int aaa_divisor_log(int enable, unsigned* out, int cap) {
  DivisorLog& g = divisor_log();
  std::lock_guard<std::mutex> lk(g.mu);
  const int n = (int)g.seen.size();
  if (out)
    for (int i = 0; i < std::min(n, cap); ++i) out[i] = g.seen[i];
  if (enable >= 0) {   // -1: read only
    g.on = enable != 0;
    if (!g.on) g.seen.clear();
  }
  return n;
}

const char* aaa_last_error(void) { return g_err.c_str(); }

int aaa_timing_enable(int on) {
  std::lock_guard<std::mutex> lk(g_timers.mu);
  g_timers.on = on != 0;
  for (double& w : g_timers.work) w = 0.0;
  for (auto& v : g_timers.pending) {
    for (auto& pr : v) { g_timers.pool.push_back(pr.first); g_timers.pool.push_back(pr.second); }
    v.clear();
  }
  return AAA_OK;
}

int aaa_timing_read(int kind, double* total_ms, long* launches) {
  if (!total_ms || !launches) return fail(AAA_E_ARG, "bad timer query");
  aaa_timer_stats s;
  const int rc = aaa_timing_stats(kind, &s);
  *total_ms = s.total_ms;
  *launches = s.launches;
  return rc;
}

int aaa_timing_stats(int kind, aaa_timer_stats* out) {
  if (kind < 0 || kind >= AAA_TIMER_N || !out) return fail(AAA_E_ARG, "bad timer query");
  std::vector<std::pair<hipEvent_t, hipEvent_t>> v;
  memset(out, 0, sizeof *out);
  {
    std::lock_guard<std::mutex> lk(g_timers.mu);
    v.swap(g_timers.pending[kind]);
    out->work = g_timers.work[kind];
    snprintf(out->variant, sizeof out->variant, "%s", g_timers.variant[kind].c_str());
    g_timers.work[kind] = 0.0;
  }
  double tot = 0.0;
  int rc = AAA_OK;
  for (auto& pr : v) {
    float ms = 0.f;
    if (hipEventSynchronize(pr.second) != hipSuccess || hipEventElapsedTime(&ms, pr.first, pr.second) != hipSuccess)
      rc = fail(AAA_E_LAUNCH, "event timing failed");
    tot += ms;
  }
  {
    std::lock_guard<std::mutex> lk(g_timers.mu);
    for (auto& pr : v) { g_timers.pool.push_back(pr.first); g_timers.pool.push_back(pr.second); }
  }
  out->total_ms = tot;
  out->launches = (long)v.size();
  return rc;
}

int aaa_grid(int H, int W, int* h, int* w) {
  if (!h || !w) return fail(AAA_E_ARG, "NULL output");
  *h = conv_out(conv_out(H, 8, 4, 1), 4, 2, 2);
  *w = conv_out(conv_out(W, 8, 4, 1), 4, 2, 2);
  return (*h >= 1 && *w >= 1) ? AAA_OK : fail(AAA_E_ARG, "frame too small");
}

int aaa_param_layout(const aaa_cfg* cfg, size_t* total, size_t* offsets, size_t* sizes) {
  Layout L;
  int r = build_layout(cfg, L);
  if (r) return r;
  if (total) *total = L.ptotal;
  for (int i = 0; i < NPARAM; ++i) {
    if (offsets) offsets[i] = L.poff[i];
    if (sizes) sizes[i] = L.psz[i];
  }
  return AAA_OK;
}

size_t aaa_packed_bytes(const aaa_cfg* cfg) {
  Layout L;
  return build_layout(cfg, L) ? 0 : L.packed;
}

size_t aaa_workspace_bytes(const aaa_cfg* cfg) {
  Layout L;
  return build_layout(cfg, L) ? 0 : L.ws;
}

int aaa_pack_weights(const aaa_cfg* cfg, const float* params, void* packed, hipStream_t stream) {
  Layout L;
  int r = build_layout(cfg, L);
  if (r) return r;
  if ((r = check_device())) return r;
  if (!params || !packed) return fail(AAA_E_ARG, "NULL params/packed");
  if (!aligned16(params) || !aligned16(packed)) return fail(AAA_E_ALIGN, "params/packed must be 16-byte aligned");
  return L.dt == AAA_BF16 ? pack_impl<__bf16>(L, params, (char*)packed, stream)
                          : pack_impl<float>(L, params, (char*)packed, stream);
}

static int check_io(const Layout& L, const aaa_io* io, bool bwd) {
  if (!io) return fail(AAA_E_ARG, "io is NULL");
  if (!io->params || !io->packed || !io->basis || !io->frames || !io->workspace)
    return fail(AAA_E_ARG, "params/packed/basis/frames/workspace must be set");
  if (!bwd && (!io->logits || !io->values)) return fail(AAA_E_ARG, "logits/values outputs must be set");
  if (bwd && (!io->dlogits || !io->grads)) return fail(AAA_E_ARG, "dlogits/grads must be set");
  const void* ptrs[] = {io->params, io->packed, io->basis, io->frames, io->workspace, io->h0, io->c0, io->hT,
                        io->cT, io->dhT, io->dcT, io->dh0, io->dc0, io->grads};
  for (const void* p : ptrs)
    if (p && !aligned16(p)) return fail(AAA_E_ALIGN, "buffers must be 16-byte aligned");
  (void)L;
  return AAA_OK;
}

int aaa_forward(const aaa_cfg* cfg, const aaa_io* io, hipStream_t stream) {
  Layout L;
  int r = build_layout(cfg, L);
  if (r) return r;
  if ((r = check_device())) return r;
  if ((r = check_io(L, io, false))) return r;
  if ((r = pair_check())) return r;
  return L.dt == AAA_BF16 ? forward_impl<__bf16>(L, io, stream) : forward_impl<float>(L, io, stream);
}

int aaa_backward(const aaa_cfg* cfg, const aaa_io* io, int phases, hipStream_t stream) {
  Layout L;
  int r = build_layout(cfg, L);
  if (r) return r;
  if ((r = check_device())) return r;
  if ((r = check_io(L, io, true))) return r;
  if (phases & ~AAA_BWD_ALL || !phases) return fail(AAA_E_ARG, "bad phase mask %d", phases);
  if ((r = pair_check())) return r;
  return L.dt == AAA_BF16 ? backward_impl<__bf16>(L, io, phases, stream)
                          : backward_impl<float>(L, io, phases, stream);
}

int aaa_pair_status(hipStream_t stream, int clear) {
  if (stream && hipStreamSynchronize(stream) != hipSuccess) return fail(AAA_E_LAUNCH, "stream synchronize failed");
  if (!stream && hipDeviceSynchronize() != hipSuccess) return fail(AAA_E_LAUNCH, "device synchronize failed");
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return fail(AAA_E_DEVICE, "no HIP device");
  std::lock_guard<std::mutex> lk(g_pair_mu);
  if (!g_pair_host) return 0;
  return clear ? __atomic_exchange_n(g_pair_host + dev, 0, __ATOMIC_ACQ_REL)
               : __atomic_load_n(g_pair_host + dev, __ATOMIC_ACQUIRE);
}

int aaa_debug_pair_spin(long polls) {
  if (polls < 0 || polls > (1L << 30)) return fail(AAA_E_ARG, "pair spin bound must be in [0, 2^30] (0 = default)");
  g_pair_spin = polls ? polls : (1L << 24);
  return AAA_OK;
}

static int check_conv(const aaa_conv_desc* d) {
  if (!d) return fail(AAA_E_ARG, "NULL desc");
  if (d->N < 1 || d->Cin < 1 || d->Cout < 1 || d->KH != d->KW || d->stride < 1 || d->pad < 0)
    return fail(AAA_E_ARG, "bad conv desc");
  if (d->Hout != conv_out(d->Hin, d->KH, d->stride, d->pad) || d->Wout != conv_out(d->Win, d->KW, d->stride, d->pad))
    return fail(AAA_E_ARG, "Hout/Wout inconsistent with Hin/Win/K/stride/pad");
  if ((d->KH * d->KW * d->Cin) % 4 || d->Cout % 4) return fail(AAA_E_ARG, "KH*KW*Cin and Cout must be multiples of 4");
  // buffer descriptors span the whole input / output gradient (32-bit byte offsets, kOOB = 2^31)
  const size_t lim = size_t(1) << 31;
  if ((size_t)d->N * d->Hin * d->Win * d->Cin * 4 >= lim || (size_t)d->N * d->Hout * d->Wout * d->Cout * 4 >= lim)
    return fail(AAA_E_ARG, "conv tensors must stay below 2 GiB (split N)");
  return check_device();
}

int aaa_conv2d_nhwc(const aaa_conv_desc* d, const float* x, const float* w, const float* bias, float* y,
                    hipStream_t stream) {
  int r = check_conv(d);
  if (r) return r;
  return d->dtype == AAA_BF16 ? conv_nhwc_impl<__bf16>(d, x, w, bias, y, stream)
                              : conv_nhwc_impl<float>(d, x, w, bias, y, stream);
}

int aaa_conv2d_nhwc_dgrad(const aaa_conv_desc* d, const float* dy, const float* wT, float* dx, hipStream_t stream) {
  int r = check_conv(d);
  if (r) return r;
  if (d->Cout % 4) return fail(AAA_E_ARG, "Cout must be a multiple of 4");
  return d->dtype == AAA_BF16 ? dgrad_nhwc_impl<__bf16>(d, dy, wT, dx, stream)
                              : dgrad_nhwc_impl<float>(d, dy, wT, dx, stream);
}

int aaa_conv2d_nhwc_wgrad(const aaa_conv_desc* d, const float* x, const float* dy, float* dw, hipStream_t stream) {
  int r = check_conv(d);
  if (r) return r;
  return d->dtype == AAA_BF16 ? wgrad_nhwc_impl<__bf16>(d, x, dy, dw, stream)
                              : wgrad_nhwc_impl<float>(d, x, dy, dw, stream);
}

int aaa_adam_step(const aaa_adam_hparams* hp, long step, int ntensors, float* const* params,
                  const float* const* grads, float* const* exp_avg, float* const* exp_avg_sq,
                  float* const* max_exp_avg_sq, const size_t* numel, hipStream_t stream) {
  if (!hp || ntensors < 0 || (ntensors > 0 && (!params || !grads || !exp_avg || !exp_avg_sq || !numel)))
    return fail(AAA_E_ARG, "adam: NULL argument");
  if (step < 1) return fail(AAA_E_ARG, "adam: step must be >= 1 (got %ld)", step);
  if (hp->amsgrad && !max_exp_avg_sq) return fail(AAA_E_ARG, "adam: amsgrad needs max_exp_avg_sq");
  if (!(hp->lr >= 0.0) || !(hp->eps >= 0.0) || !(hp->beta1 >= 0.0 && hp->beta1 < 1.0) ||
      !(hp->beta2 >= 0.0 && hp->beta2 < 1.0) || !(hp->weight_decay >= 0.0))
    return fail(AAA_E_ARG, "adam: invalid hyper-parameters");
  int r = check_device();
  if (r) return r;
  AdamHost h{hp->lr, hp->beta1, hp->beta2, hp->eps, hp->weight_decay, step, hp->amsgrad ? 1 : 0, hp->maximize ? 1 : 0};
  for (int t0 = 0; t0 < ntensors; t0 += kAdamMaxTensors) {
    AdamTable tab;
    memset(&tab, 0, sizeof tab);
    int nch = 0;
    for (int t = t0; t < std::min(ntensors, t0 + kAdamMaxTensors); ++t) {
      if (numel[t] == 0) continue;
      const int i = tab.n++;
      if (!params[t] || !grads[t] || !exp_avg[t] || !exp_avg_sq[t] || (h.amsgrad && !max_exp_avg_sq[t]))
        return fail(AAA_E_ARG, "adam: NULL pointer for tensor %d", t);
      tab.p[i] = params[t]; tab.g[i] = grads[t]; tab.m[i] = exp_avg[t]; tab.v[i] = exp_avg_sq[t];
      tab.vmax[i] = h.amsgrad ? max_exp_avg_sq[t] : nullptr;
      tab.numel[i] = numel[t];
      tab.chunk0[i] = nch;
      tab.vec[i] = aligned16(params[t]) && aligned16(grads[t]) && aligned16(exp_avg[t]) && aligned16(exp_avg_sq[t]) &&
                   (!tab.vmax[i] || aligned16(tab.vmax[i]));
      const long c = adam_chunks(numel[t]);
      if (nch + c > (1L << 30)) return fail(AAA_E_ARG, "adam: tensor %d too large", t);
      nch += (int)c;
    }
    HIPCHK(adam_launch(tab, nch, h, stream));
  }
  return AAA_OK;
}

int aaa_reinforce(int T, int B, int A, const float* logits, const int* actions, const float* rewards, double gamma,
                  float* loss, float* returns_norm, float* dlogits, hipStream_t stream) {
  if (T < 1 || B < 1 || A < 1) return fail(AAA_E_ARG, "reinforce: need T, B, A >= 1 (T=%d B=%d A=%d)", T, B, A);
  if (!logits || !actions || !rewards || !loss || !returns_norm || !dlogits)
    return fail(AAA_E_ARG, "reinforce: NULL argument");
  if (!(gamma >= 0.0 && gamma <= 1.0)) return fail(AAA_E_ARG, "reinforce: gamma must be in [0, 1]");
  int r = check_device();
  if (r) return r;
  HIPCHK(reinforce_launch(T, B, A, logits, actions, rewards, gamma, loss, returns_norm, dlogits, stream));
  return AAA_OK;
}

int aaa_sample_actions(int B, int A, const float* logits, unsigned long long seed, unsigned long long* counter,
                       int* actions, float* logp, float* dlogp_dlogits, hipStream_t stream) {
  if (B < 1 || A < 1) return fail(AAA_E_ARG, "sample_actions: need B, A >= 1 (B=%d A=%d)", B, A);
  if (!logits || !actions || !logp) return fail(AAA_E_ARG, "sample_actions: NULL argument");
  int r = check_device();
  if (r) return r;
  HIPCHK(sample_launch(B, A, logits, seed, counter, actions, logp, dlogp_dlogits, stream));
  return AAA_OK;
}

// ---- actor step (include/aaa.h; csrc/actor.hip) ----
// Workspace: conv2 output X (B,P,64), h_t Hs (B,P,128), hid1 (B,512), AO (B,256), LH (B,256).
static int actor_layout(const aaa_cfg* cfg, Layout& L, size_t off[5], size_t* total) {
  int r = build_layout(cfg, L);
  if (r) return r;
  if (cfg->T != 1) return fail(AAA_E_ARG, "actor_step: T must be 1 (got %d)", cfg->T);
  if (cfg->dtype != AAA_F32) return fail(AAA_E_ARG, "actor_step: fp32 weights only (bf16 agents use aaa_forward)");
  if (L.sc) return fail(AAA_E_ARG, "actor_step: the stateful policy core uses aaa_forward");
  if (cfg->B > 16) return fail(AAA_E_ARG, "actor_step: B <= 16 (got %d); larger batches use aaa_forward", cfg->B);
  const size_t B = cfg->B, P = L.P;
  const size_t sz[5] = {B * P * 64 * 4, B * P * 128 * 4, B * 512 * 4, B * 256 * 4, B * 256 * 4};
  size_t o = 0;
  for (int i = 0; i < 5; ++i) { off[i] = o; o = al256(o + sz[i]); }
  *total = o;
  return AAA_OK;
}

size_t aaa_actor_workspace_bytes(const aaa_cfg* cfg) {
  Layout L;
  size_t off[5], tot = 0;
  return actor_layout(cfg, L, off, &tot) ? 0 : tot;
}

int aaa_actor_step(const aaa_cfg* cfg, const aaa_actor_io* io, hipStream_t stream) {
  Layout L;
  size_t off[5], tot = 0;
  int r = actor_layout(cfg, L, off, &tot);
  if (r) return r;
  if (!io || !io->params || !io->packed || !io->basis || !io->frames || !io->h || !io->c || !io->logits ||
      !io->values || !io->workspace)
    return fail(AAA_E_ARG, "actor_step: NULL argument");
  if (!aligned16(io->packed) || !aligned16(io->basis) || !aligned16(io->h) || !aligned16(io->c) ||
      !aligned16(io->workspace) || !aligned16(io->params))
    return fail(AAA_E_ALIGN, "actor_step: params, packed, basis, h, c and workspace must be 16-byte aligned");
  if ((r = check_device())) return r;
  const char* pk = (const char*)io->packed;
  const float* prm = io->params;
  char* ws = (char*)io->workspace;
  ActorParams p;
  p.B = L.B; p.H = L.H; p.W = L.W; p.H1 = L.H1; p.W1 = L.W1; p.h = L.h; p.w = L.w; p.P = L.P;
  p.nq = L.nq; p.A = L.A; p.ldy = L.ldy; p.ans_in = L.ans_in; p.ans_ld = L.ans_ld; p.u8 = L.fu8;
  p.frames = io->frames; p.basis = io->basis; p.prev_reward = io->prev_reward; p.prev_action = io->prev_action;
  p.Wp1 = (const float*)(pk + L.k_Wp1); p.b1 = prm + L.poff[C0B];
  p.Wp2 = (const float*)(pk + L.k_Wp2); p.b2 = prm + L.poff[C1B];
  p.WpXH = (const float*)(pk + L.k_WpXH); p.bl = (const float*)(pk + L.k_bl);
  p.Q = (const float*)(pk + L.k_Q);
  p.W1p = (const float*)(pk + L.k_W1p); p.a0b = prm + L.poff[A0B];
  p.A2W = prm + L.poff[A2W]; p.a2b = prm + L.poff[A2B];
  p.Wihp = (const float*)(pk + L.k_Wihp); p.blc = (const float*)(pk + L.k_blc);
  p.Whd = (const float*)(pk + L.k_Whd); p.bhd = (const float*)(pk + L.k_bhd);
  p.hst = io->h; p.cst = io->c; p.logits = io->logits; p.values = io->values; p.attn = io->attn;
  p.X = (float*)(ws + off[0]); p.Hs = (float*)(ws + off[1]); p.hid1 = (float*)(ws + off[2]);
  p.AO = (float*)(ws + off[3]); p.LH = (float*)(ws + off[4]);
  p.seed = io->seed; p.counter = io->counter; p.actions = io->actions; p.logp = io->logp; p.jac = io->dlogp_dlogits;
  HIPCHK(actor_launch(p, stream));
  return AAA_OK;
}

// ---- component entries (include/aaa.h) ----
size_t aaa_convlstm_packed_bytes(const aaa_cell_desc* d) {
  CellLayout C;
  return cell_layout(d, C) ? 0 : C.packed;
}

size_t aaa_convlstm_workspace_bytes(const aaa_cell_desc* d) {
  CellLayout C;
  return cell_layout(d, C) ? 0 : C.ws;
}

int aaa_convlstm_pack(const aaa_cell_desc* d, const float* cell_params, void* packed, hipStream_t stream) {
  CellLayout C;
  int r = cell_layout(d, C);
  if (r) return r;
  if ((r = check_device())) return r;
  if (!cell_params || !packed) return fail(AAA_E_ARG, "convlstm_pack: NULL argument");
  if (!aligned16(packed)) return fail(AAA_E_ALIGN, "packed must be 16-byte aligned");
  LstmPtrs lp;
  cell_ptrs(cell_params, lp);
  char* pk = (char*)packed;
  if (C.dt == AAA_BF16)
    HIPCHK(pack_lstm_all<__bf16>(lp, (__bf16*)(pk + C.k_WpX), (__bf16*)(pk + C.k_WpH), (__bf16*)(pk + C.k_WdTl),
                                 (float*)(pk + C.k_bl), (__bf16*)(pk + C.k_WpXH), stream));
  else
    HIPCHK(pack_lstm_all<float>(lp, (float*)(pk + C.k_WpX), (float*)(pk + C.k_WpH), (float*)(pk + C.k_WdTl),
                                (float*)(pk + C.k_bl), (float*)(pk + C.k_WpXH), stream));
  return AAA_OK;
}

int aaa_convlstm_cell_fwd(const aaa_cell_desc* d, const void* packed, const float* x, const float* h0,
                          const float* c0, float* h1, float* c1, void* workspace, hipStream_t stream) {
  CellLayout C;
  int r = cell_layout(d, C);
  if (r) return r;
  if ((r = check_device())) return r;
  if (!packed || !x || !workspace) return fail(AAA_E_ARG, "convlstm_cell_fwd: packed/x/workspace must be set");
  const void* ptrs[] = {packed, x, h0, c0, h1, c1, workspace};
  for (const void* p : ptrs)
    if (p && !aligned16(p)) return fail(AAA_E_ALIGN, "buffers must be 16-byte aligned");
  return C.dt == AAA_BF16 ? cell_fwd_impl<__bf16>(C, (const char*)packed, x, h0, c0, h1, c1, (char*)workspace, stream)
                          : cell_fwd_impl<float>(C, (const char*)packed, x, h0, c0, h1, c1, (char*)workspace, stream);
}

int aaa_convlstm_cell_bwd(const aaa_cell_desc* d, const void* packed, const float* dh1, const float* dc1, float* dx,
                          float* dh0, float* dc0, float* cell_grads, void* workspace, hipStream_t stream) {
  CellLayout C;
  int r = cell_layout(d, C);
  if (r) return r;
  if ((r = check_device())) return r;
  if (!packed || !workspace) return fail(AAA_E_ARG, "convlstm_cell_bwd: packed/workspace must be set");
  const void* ptrs[] = {packed, dh1, dc1, dx, dh0, dc0, cell_grads, workspace};
  for (const void* p : ptrs)
    if (p && !aligned16(p)) return fail(AAA_E_ALIGN, "buffers must be 16-byte aligned");
  return C.dt == AAA_BF16
             ? cell_bwd_impl<__bf16>(C, (const char*)packed, dh1, dc1, dx, dh0, dc0, cell_grads, (char*)workspace, stream)
             : cell_bwd_impl<float>(C, (const char*)packed, dh1, dc1, dx, dh0, dc0, cell_grads, (char*)workspace, stream);
}

size_t aaa_vision_cnn_packed_bytes(const aaa_cnn_desc* d) {
  CnnLayout C;
  return cnn_layout(d, C) ? 0 : C.L.k_WpX;   // the first three packed layouts
}

size_t aaa_vision_cnn_workspace_bytes(const aaa_cnn_desc* d) {
  CnnLayout C;
  return cnn_layout(d, C) ? 0 : C.ws;
}

int aaa_vision_cnn_pack(const aaa_cnn_desc* d, const float* cnn_params, void* packed, hipStream_t stream) {
  CnnLayout C;
  int r = cnn_layout(d, C);
  if (r) return r;
  if ((r = check_device())) return r;
  if (!cnn_params || !packed) return fail(AAA_E_ARG, "vision_cnn_pack: NULL argument");
  if (!aligned16(packed)) return fail(AAA_E_ALIGN, "packed must be 16-byte aligned");
  return C.L.dt == AAA_BF16 ? cnn_pack_impl<__bf16>(C.L, cnn_params, (char*)packed, stream)
                            : cnn_pack_impl<float>(C.L, cnn_params, (char*)packed, stream);
}

int aaa_vision_cnn_fwd(const aaa_cnn_desc* d, const float* cnn_params, const void* packed, const float* frames,
                       float* y1, float* y2, void* workspace, hipStream_t stream) {
  CnnLayout C;
  int r = cnn_layout(d, C);
  if (r) return r;
  if ((r = check_device())) return r;
  if (!cnn_params || !packed || !frames || !y2 || !workspace)
    return fail(AAA_E_ARG, "vision_cnn_fwd: cnn_params/packed/frames/y2/workspace must be set");
  const void* ptrs[] = {packed, frames, y1, y2, workspace};
  for (const void* p : ptrs)
    if (p && !aligned16(p)) return fail(AAA_E_ALIGN, "buffers must be 16-byte aligned");
  const Layout& L = C.L;
  char* ws = (char*)workspace;
  auto run = [&](auto tag) -> int {
    using T = decltype(tag);
    int rc = vision_fwd<T, float>(L, L.F, (const char*)packed, cnn_params, frames, (T*)(ws + C.Xp), (T*)(ws + C.Y1),
                                  y2, 64, stream);
    if (rc) return rc;
    if (y1) HIPCHK((cast<T, float>((long)L.F * L.P1 * 32, (const T*)(ws + C.Y1), y1, stream)));
    return AAA_OK;
  };
  return L.dt == AAA_BF16 ? run(__bf16{}) : run(float{});
}

int aaa_vision_cnn_bwd(const aaa_cnn_desc* d, const void* packed, const float* dy2, float* dy1, float* cnn_grads,
                       void* workspace, hipStream_t stream) {
  CnnLayout C;
  int r = cnn_layout(d, C);
  if (r) return r;
  if ((r = check_device())) return r;
  if (!packed || !dy2 || !cnn_grads || !workspace)
    return fail(AAA_E_ARG, "vision_cnn_bwd: packed/dy2/cnn_grads/workspace must be set");
  const void* ptrs[] = {packed, dy2, dy1, cnn_grads, workspace};
  for (const void* p : ptrs)
    if (p && !aligned16(p)) return fail(AAA_E_ALIGN, "buffers must be 16-byte aligned");
  return C.L.dt == AAA_BF16
             ? cnn_bwd_impl<__bf16>(C, (const char*)packed, dy2, dy1, cnn_grads, (char*)workspace, stream)
             : cnn_bwd_impl<float>(C, (const char*)packed, dy2, dy1, cnn_grads, (char*)workspace, stream);
}

static int check_attn(int F, int h, int w, int nq, int q_stride) {
  if (F < 1 || h < 1 || w < 1) return fail(AAA_E_ARG, "attn: need F, h, w >= 1");
  if (nq != 4 && nq != 8) return fail(AAA_E_ARG, "attn: nq must be 4 or 8 (got %d)", nq);
  if (q_stride != 0 && q_stride != nq * 72) return fail(AAA_E_ARG, "attn: q_stride must be 0 or nq*72");
  if ((size_t)F * h * w * 128 >= (size_t(1) << 31)) return fail(AAA_E_ARG, "attn: F*h*w too large; split F");
  return check_device();
}

int aaa_attn_fwd(int F, int h, int w, int nq, const float* O, const float* S, const float* Q, int q_stride,
                 const float* prev_reward, const float* prev_action, float* attn, float* answer, hipStream_t stream) {
  int r = check_attn(F, h, w, nq, q_stride);
  if (r) return r;
  if (!O || !S || !Q || !attn || !answer) return fail(AAA_E_ARG, "attn_fwd: O/S/Q/attn/answer must be set");
  if (!aligned16(O) || !aligned16(S)) return fail(AAA_E_ALIGN, "O and S must be 16-byte aligned");
  TimerScope tim(AAA_TIMER_ATTN_FWD, stream, (double)F * attn_fwd_bytes(h * w, nq, 256 * nq + 2), "k_attn_fwd (aaa_attn_fwd)");
  HIPCHK(attn_fwd(O, S, Q, nullptr, prev_reward, prev_action, F, h * w, nq, attn, answer, 256 * nq + 2, stream,
                  q_stride));
  return AAA_OK;
}

int aaa_attn_bwd(int F, int h, int w, int nq, const float* O, const float* S, const float* Q, int q_stride,
                 const float* attn, const float* danswer, float* dO, float* dQ, hipStream_t stream) {
  int r = check_attn(F, h, w, nq, q_stride);
  if (r) return r;
  if (!O || !S || !Q || !attn || !danswer || !dO || !dQ)
    return fail(AAA_E_ARG, "attn_bwd: O/S/Q/attn/danswer/dO/dQ must be set");
  if (!aligned16(O) || !aligned16(S) || !aligned16(dO)) return fail(AAA_E_ALIGN, "O, S, dO must be 16-byte aligned");
  TimerScope tim(AAA_TIMER_ATTN_BWD, stream, (double)F * attn_bwd_bytes(h * w, nq), "k_attn_bwd (aaa_attn_bwd)");
  HIPCHK(attn_bwd(O, S, Q, attn, danswer, 256 * nq + 2, F, h * w, nq, dO, dQ, stream, q_stride, 1));
  return AAA_OK;
}

int aaa_linear(int M, int N, int K, const float* x, const float* w, const float* bias, float* y,
               hipStream_t stream) {
  if (M < 1 || N < 1 || K < 1 || K % 4) return fail(AAA_E_ARG, "linear: need M,N,K >= 1 and K %% 4 == 0");
  int r = check_device();
  if (r) return r;
  using LA = LdRows<float, float, CF::BI, CF::BK, CF::NT>;
  using LB = LdRows<float, float, CF::BJ, CF::BK, CF::NT>;
  EpiStoreT<float> ep{y, N, N, M, bias, 0};
  HIPCHK((launch_gemm<CF, LA, LB>(LA::Params{w, K, N}, LB::Params{x, K, M}, ep, N, M, K, 1, stream)));
  return AAA_OK;
}

}  // extern "C"
