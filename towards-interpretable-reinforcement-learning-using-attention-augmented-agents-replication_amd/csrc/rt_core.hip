// Host runtime state and layout (include/aaa.h): the error string, the buffer
// layout, the device check, the paired-kernel reports, the aux stream, the
// kernel timers and the frame-resident dispatch rules (rt.h).
#include "rt.h"

namespace aaa {

thread_local std::string g_err;
thread_local bool g_tail3 = false, g_tail6 = false;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

static int check_ranges(Layout& L, int min_frames);

int build_layout(const aaa_cfg* c, Layout& L, int min_frames) {
  if (!c) return fail(AAA_E_ARG, "cfg is NULL");
  if (c->B < 1 || c->T < 1) return fail(AAA_E_ARG, "B and T must be >= 1 (B=%d T=%d)", c->B, c->T);
  if (c->nq != 4 && c->nq != 8) return fail(AAA_E_ARG, "nq must be 4 or 8 (got %d)", c->nq);
  if (c->A < 1 || c->A > 256) return fail(AAA_E_ARG, "A out of range (%d)", c->A);
  if (c->dtype != AAA_F32 && c->dtype != AAA_BF16) return fail(AAA_E_ARG, "bad dtype %d", c->dtype);
  if (c->flags & ~(AAA_FLAG_STATEFUL_CORE | AAA_FLAG_FRAMES_U8 | AAA_FLAG_DEFER_STRANDED)) return fail(AAA_E_ARG, "unknown flags 0x%x", c->flags);
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
  L.k_WdTc = take(e == 4 ? 64 * 4608 * 4 : 0);   // its dx rows channel-chunk-major (BK 32: the fp32 dx ring, cmaj)
  L.k_WdT6 = take(e == 4 ? 3 * 64 * 4608 * 2 : 0);   // its dx rows as three bf16 planes (the split6 dx ring's A)
  L.k_Wbf = take(e == 2 ? (size_t)6 * kBwKSP * 64 * 16 : 0);   // fragment-order [W_h^T | W_x^T] (frame-resident BPTT)
  L.k_Wf32 = take(e == 4 ? (size_t)16 * kF32QP * 64 * 16 : 0);   // fp32 fragment-order [x|h] (frame-group recurrence, recur_f32.h)
  L.k_Wb32 = take(e == 4 ? (size_t)8 * kB32QP * 4 * 64 * 16 : 0);   // fp32 fragment-order W_h^T (frame-group BPTT, recur_bwd_f32.h)
  L.k_Wf6 = take(e == 4 ? (size_t)16 * kF32QP * 64 * 24 : 0);    // their three-way bf16 splits (S6, k_split_frag)
  L.k_Wf6p = take(e == 4 ? (size_t)16 * kF32PP * 3 * 64 * 16 : 0);   // ... paired for the pre-split forward
  L.k_Wb6 = take(e == 4 ? (size_t)8 * kB32QP * 4 * 64 * 24 : 0);
  L.k_Wx6 = take(e == 4 ? (size_t)8 * kB32QP * 2 * 64 * 24 : 0);   // the dx rows of W^T, split (DX)
  L.k_Wb6p = take(e == 4 ? (size_t)8 * kB32PP * 4 * 3 * 64 * 16 : 0);   // DX's paired streams
  L.k_Wx6p = take(e == 4 ? (size_t)8 * kB32PP * 2 * 3 * 64 * 16 : 0);
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
  // frames as zero-bordered RGBx (conv1's operand type): all F frames, written by the forward's encoder
  // and read by conv1's weight gradient; AAA_XP_CHUNK=n (A/B) keeps a chunk of n frames instead, rebuilt
  // from the observation right before conv1 (layered forward) or its weight gradient reads it (measured
  // slower: C3 vision backward 0.368 -> 0.666 ms for -0.03 ms in the forward)
  const int xc = ab_int("AAA_XP_CHUNK", 0);
  L.xpc = xc > 0 ? (int)std::min<size_t>(F, (size_t)std::max(64, xc)) : (int)F;
  L.Xp = take((size_t)L.xpc * (L.H + 2) * (L.W + 2) * 4 * e);
  L.Y1 = take(F * L.P1 * 32 * e);
  L.XH = take((size_t)(L.T + 1) * M * 192 * e);
  L.Hs = take(e == 4 ? F * P * 128 * 4 : 0);   // fp32 h_t for the readout (bf16: it reads XH, readout_h)
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
  // (A/B, AAA_DX_S6_TILE=5) fp32 dZ as three bf16 planes for the batched dx (0 = none)
  L.dZ6 = take(e == 4 && ab_int("AAA_DX_S6_TILE", 4) == 5 ? F * P * 512 * 6 : 0);
  // gate-bias partials per (step, column tile | frame half); the fp32 split-K chain's tiles are kSplitBj pixels
  const size_t zp_rows = std::max({(M + 31) / 32, 2 * (size_t)L.B,
                                   L.esz == 4 && bptt_splitk_fits(M) ? (M + kSplitBj - 1) / kSplitBj : 0});
  L.dZp = take((size_t)L.T * zp_rows * 512 * 4);
  L.dY2 = take(F * P * 64 * e);       // conv-input grads in the operand type of the GEMMs reading them
  L.dY1 = take(F * L.P1 * 32 * e);
  L.dxb = take((size_t)L.B * 64 * 4);   // conv2 bias-gradient partials per frame (frame-resident BPTT)
  L.rflags = take((size_t)8 * L.B * 4);   // hand-off flags of the multi-workgroup frame kernels ([B][G], G <= 8)
  L.xpart = take(L.esz == 4 && rec_fits(L.h, L.w) ? b32_xpart_floats(L.B) * 4 : 0);   // fp32 frame-group BPTT exchange
  // split-K partials: BPTT dh (<= kBpttSplitMax x 128 per pixel) or the fused forward step's gates (<= 4 x 512)
  // (0 = none: the split-K tiles then fail loudly)
  // (+ 4 KB: the split-K tiles' fixup counters, EpiSliceFix, after the partials)
  L.dhs = L.esz == 4 && bptt_splitk_fits(M) ? take((size_t)std::max(kBpttSplitMax * 128, 4 * 512) * M * 4 + 4096) : 0;
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

int check_device() {
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

// ------------------------------------------------- paired-kernel reports --
// The multi-workgroup frame-resident kernels bound their partner waits
// (common.h pair_wait).  A timed-out wait adds 1 to this device's report word:
// pinned host memory mapped into the device, so the host reads it without a
// copy or a sync.  The word is MONOTONIC -- nothing resets it -- and it has two
// independent readers, each holding its own snapshot:
//   * the host (pair_take / pair_peek): reports past g_pair_seen[dev]; every
//     aaa_forward / aaa_backward entry consumes them and fails with
//     AAA_E_STRANDED unless the call defers them (AAA_FLAG_DEFER_STRANDED);
//   * the device (aaa_pair_flag): k_pair_flag writes, in stream order, the
//     reports past its own base word (words [64, 128) of the same page) and
//     advances that base -- so a host-side consumption between the stranded
//     launch and the guard can never hide the timeout from the guarded Adam
//     (ADVICE r04).
// Allocated once per process on first use, never freed (no HIP call at exit).
static std::mutex g_pair_mu;
static int* g_pair_host = nullptr;    // [128] words: [0,64) reports, [64,128) device-side bases
static int* g_pair_dev = nullptr;     // the same words, device-mapped
static unsigned g_pair_seen[64] = {};  // host-side snapshot per device ordinal

// Partner-wait budget of one multi-workgroup launch of T steps: 1 s plus 20 ms
// per step (the slowest legitimate launch, C5's band BPTT, takes ~80 us per
// step), so only a partner that is not running at all exhausts it.
int pair_budget(int T) {
  return (int)std::min<long>(100000000L + 2000000L * (long)T, 0x7fffffffL);
}

int* pair_report(int dev) {
  std::lock_guard<std::mutex> lk(g_pair_mu);
  if (!g_pair_host) {
    void* h = nullptr;
    if (hipHostMalloc(&h, 128 * sizeof(int), hipHostMallocMapped | hipHostMallocPortable | hipHostMallocCoherent) !=
        hipSuccess)
      return nullptr;
    memset(h, 0, 128 * sizeof(int));
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) return nullptr;
    g_pair_host = (int*)h;
    g_pair_dev = (int*)d;
  }
  return g_pair_dev + dev;
}

int* pair_flag_base(int dev) {
  return pair_report(dev) ? g_pair_dev + 64 + dev : nullptr;
}

static int pair_pending(bool consume) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
  std::lock_guard<std::mutex> lk(g_pair_mu);
  if (!g_pair_host) return 0;
  const unsigned cur = (unsigned)__atomic_load_n(g_pair_host + dev, __ATOMIC_ACQUIRE);
  const unsigned n = cur - g_pair_seen[dev];
  if (consume) g_pair_seen[dev] = cur;
  return (int)std::min<unsigned>(n, 0x7fffffffu);
}

// Pending reports of the current device since the host last consumed them.
int pair_take() { return pair_pending(true); }
int pair_peek() { return pair_pending(false); }

int pair_check() {
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


// Measured on C2 (round 1): running the off-chain chunks concurrently slows the
// chain's step kernels ~2x (stream priority does not keep CUs free for them),
// 6.31-6.55 ms vs 6.15 ms serial; so overlap is opt-in (AAA_OVERLAP=1).
hipStream_t aux_stream() {
  if (ab_int("AAA_OVERLAP", 0) == 0) return nullptr;
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

// Side stream: the backward HEAD phase's weight gradients run on it beside the phase's dgrad chain
// (each waits only for the chain product it reads; the chain waits for all of them before the grads
// are unpacked), low priority so the chain's small GEMMs take CUs first.  AAA_SIDE=0: one stream.
static hipStream_t g_side[64];
hipStream_t side_stream() {
  if (!env_int("AAA_SIDE", 1)) return nullptr;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  std::lock_guard<std::mutex> lk(g_aux_mu);
  if (!g_side[dev]) {
    AuxStream& a = g_aux[dev];
    if (!a.ev[0])   // the event pool stream_order draws from (created with the aux stream otherwise)
      for (auto& e : a.ev)
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return nullptr;
    int lo = 0, hi = 0;
    (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
    if (hipStreamCreateWithPriority(&g_side[dev], hipStreamNonBlocking, lo) != hipSuccess) {
      g_side[dev] = nullptr;
      return nullptr;
    }
  }
  return g_side[dev];
}

// Record a pooled event on ``s`` (everything enqueued on s so far).
hipError_t record_event(hipStream_t s, hipEvent_t* out) {
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
hipError_t stream_order(hipStream_t from, hipStream_t to) {
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

Timers g_timers;

std::string strf(const char* fmt, ...) {
  char buf[256];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  return buf;
}

// ------------------------------------------------------------- forward ----
int device_cus() {   // per device ordinal, queried once
  static int cus[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cus[dev]) {
    hipDeviceProp_t prop;
    cus[dev] = hipGetDeviceProperties(&prop, dev) == hipSuccess ? prop.multiProcessorCount : 256;
  }
  return cus[dev];
}
// Workgroups per frame of the frame-resident kernels (0: per-step launches).
// Every frame-resident workgroup holds more than half a CU's LDS, so the chip
// has exactly one slot per CU (launch_resident re-checks the occupancy of the
// paired kernels).  G = 1 once the frames fill at least 5/8 of the slots (the
// measured crossover against the per-step launches: C3's B = 256 on 256 CUs
// 55 vs 79 us per step, B = 128 49 vs 43, profiles/r02/frames); G = 2 (paired)
// while both workgroups of every frame fit one residency wave and they still
// occupy at least a quarter of the slots; else the per-step kernels.
// AAA_FRAMES_FWD / AAA_FRAMES_BWD = 0 / 1 / 2 force it.
static_assert(2 * kBwIBS + 4 * 16 * 64 * 16 > 160 * 1024 / 2, "one frame-resident workgroup per CU");
int frames_g(const Layout& L, const char* env) {
  if (L.dt != AAA_BF16 || !rec_fits(L.h, L.w)) return 0;
  const int slots = device_cus();
  const int v = env_int(env, 8 * L.B >= 5 * slots ? 1 : (8 * L.B >= slots && 2 * L.B <= slots ? 2 : 0));
  return v == 1 ? 1 : (v == 2 && 2 * L.B <= slots ? 2 : 0);
}
int frames_fwd(const Layout& L) { return frames_g(L, "AAA_FRAMES_FWD"); }
// bf16 forward on the band-mode frame-resident kernel (recur.h BAND): grids too
// large for one workgroup's images (168x168 frames: 21x21) split into kRecBands
// row bands, one workgroup each, when B * kRecBands workgroups fit one
// residency wave (config 5: B = 64 per GPU -> 256).  AAA_FRAMES_BAND = 0 keeps
// the per-step launches.
int frames_band(const Layout& L) {
  if (L.dt != AAA_BF16 || rec_fits(L.h, L.w) || !rec_band_fits(L.h, L.w) || !env_int("AAA_FRAMES_BAND", 1)) return 0;
  return 8 * kRecBands * ((L.B + 7) / 8) <= device_cus() ? kRecBands : 0;
}
// fp32 ConvLSTM forward on the frame-group kernel (recur_f32.h): G workgroups
// per frame for all T steps, once B * G fills at least half the CUs in one
// residency wave (C2: B = 32, G = 8 on 256 CUs).  AAA_F32_FRAMES = 0 keeps the
// per-step launches (A/B and parity of both paths); 8 / 4 force that G.
int f32_frames(const Layout& L) {
  if (L.dt != AAA_F32 || !f32_rec_fits(L.h, L.w)) return 0;
  const int v = env_int("AAA_F32_FRAMES", 1), cus = device_cus();
  if (v == 8 || v == 4) return f32_grid(L.B, v) <= cus ? v : 0;   // forced G (tests, A/B)
  if (v != 1) return 0;
  const int G = f32_rec_g(L.B, cus);
  return G && 2 * G * L.B >= cus ? G : 0;
}
// The BPTT chain on the frame-resident kernels (recur_bwd.h; fp16 gate storage):
// workgroups per frame as the forward's (AAA_FRAMES_BWD = 0 / 1 / 2 forces it).
// Start offset of half the frames of the bf16 frame-resident kernels (common.h
// stagger_wait), in microseconds -> 100-MHz ticks.
int rec_stagger(const char* env) { return 100 * ab_int(env, 0); }
// default on: C2 150.6k -> 175.6k frames/s (profiles/r04/ab_split6); AAA_F32_SPLIT6=0 restores the fp32 MFMA
bool f32_split6() { return env_int("AAA_F32_SPLIT6", 1) != 0; }
// Band mode (recur_bwd.h BAND) wherever the forward runs in band mode: kRecBands.
// Only behind a frame-resident forward: the two share the channel-quad-major
// slices of Cst / Gt / dO (cqm_layout), which the per-step kernels do not read.
int frames_bwd(const Layout& L, bool g16) {
  if (!g16) return 0;
  if (const int nb = frames_band(L)) return bw_band_fits(L.h, L.w) ? nb : 0;
  return frames_fwd(L) ? frames_g(L, "AAA_FRAMES_BWD") : 0;
}
int cqm_layout(const Layout& L) {
  static const int mask = ab_int("AAA_CQM", kCqmC | kCqmG | kCqmDO) & 7;   // A/B: tools/gpu_ab.sh
  return frames_bwd(L, gates_f16(L.dt, L.B * L.P)) != 0 ? mask : 0;
}

}  // namespace aaa
