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
// weight gradients as long-K GEMMs over every frame.//
// This unit holds the C ABI of the whole path, the optimizer / loss / sampler
// / actor entries; the layout and state live in rt_core.hip, the forward in
// rt_forward.hip, the backward in rt_backward.hip, the component entries in
// rt_components.hip (shared declarations: rt.h).
#include "rt.h"


using namespace aaa;

extern "C" {

int aaa_abi_version(void) { return AAA_ABI_VERSION; }

#ifdef AAA_ABLATION
// Present only in the A/B library (make ablation): tells the tests and tools which build is loaded.
int aaa_ablation_build(void) { return 1; }
#endif

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
  for (auto& v : g_timers.variant) v.clear();
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

int aaa_workspace_region(const aaa_cfg* cfg, int region, size_t* offset, size_t* bytes) {
  if (!offset || !bytes) return fail(AAA_E_ARG, "workspace_region: NULL output");
  Layout L;
  if (int r = build_layout(cfg, L)) return r;
  const size_t F = L.F;
  switch (region) {
    case AAA_WS_ANSWER_HIDDEN: *offset = L.hid1; *bytes = F * 512 * 4; return AAA_OK;
    case AAA_WS_QUERY_HIDDEN0:
      if (!L.sc) break;
      *offset = L.q1s; *bytes = F * 128 * 4; return AAA_OK;
    case AAA_WS_QUERY_HIDDEN1:
      if (!L.sc) break;
      *offset = L.q2s; *bytes = F * (size_t)L.qd * 4; return AAA_OK;
    default: break;
  }
  return fail(AAA_E_ARG, "workspace_region: region %d not computed by this cfg", region);
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
  TimerScope tim(AAA_TIMER_PACK, stream, 0.0, "pack_all + fragment-order copies + query pack");
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
  if (!(cfg->flags & AAA_FLAG_DEFER_STRANDED) && (r = pair_check())) return r;
  return L.dt == AAA_BF16 ? forward_impl<__bf16>(L, io, stream, AAA_FWD_ALL)
                          : forward_impl<float>(L, io, stream, AAA_FWD_ALL);
}

int aaa_forward_phases(const aaa_cfg* cfg, const aaa_io* io, int phases, hipStream_t stream) {
  Layout L;
  int r = build_layout(cfg, L);
  if (r) return r;
  if (phases != AAA_FWD_ALL && phases != (AAA_FWD_VISION | AAA_FWD_TAIL))
    return fail(AAA_E_ARG, "forward phases %d: AAA_FWD_ALL or AAA_FWD_VISION | AAA_FWD_TAIL", phases);
  if (!(phases & AAA_FWD_CORE) && cqm_layout(L))
    return fail(AAA_E_ARG, "skipping the core: not with channel-quad-major slices (the frame-resident BPTT's)");
  if ((r = check_device())) return r;
  if ((r = check_io(L, io, false))) return r;
  if (!(cfg->flags & AAA_FLAG_DEFER_STRANDED) && (r = pair_check())) return r;
  return L.dt == AAA_BF16 ? forward_impl<__bf16>(L, io, stream, phases) : forward_impl<float>(L, io, stream, phases);
}

// The recurrence's per-step products in the workspace (rt_core.hip
// build_layout): Gt [T][M][512] (fp32, or fp16 on the bf16 path's gate
// storage), Cst [T+1][M][128] fp32 (slot t+1 = c_t), Hs [T][M][128] fp32 (= h_t;
// fp32 path only), XH [T+1][M][192] (channels 64.. of slot t+1 = h_t, in the
// operand type: the bf16 path's only copy of h_t).
static int core_xfer_check(const aaa_cfg* cfg, Layout& L, const void* ws, int t0, int n) {
  int r = build_layout(cfg, L);
  if (r) return r;
  if (cqm_layout(L)) return fail(AAA_E_ARG, "core export/import: channel-quad-major slices unsupported");
  if (!ws || t0 < 0 || n < 1 || t0 + n > L.T) return fail(AAA_E_ARG, "core export/import: steps [%d, %d) of T=%d", t0, t0 + n, L.T);
  return check_device();
}
static int core_gate_bytes(const Layout& L) { return L.dt == AAA_BF16 && gates_f16(L.dt, L.B * L.P) ? 2 : 4; }

int aaa_core_elem_bytes(const aaa_cfg* cfg, int* gate_bytes, int* h_bytes) {
  if (!gate_bytes || !h_bytes) return fail(AAA_E_ARG, "core_elem_bytes: NULL output");
  Layout L;
  if (int r = build_layout(cfg, L)) return r;
  const bool ok = !cqm_layout(L);   // channel-quad-major slices: no export / import (0 bytes)
  *gate_bytes = ok ? core_gate_bytes(L) : 0;
  *h_bytes = ok ? L.esz : 0;
  return AAA_OK;
}

int aaa_core_export(const aaa_cfg* cfg, const void* workspace, int t0, int n, void* gates, float* c, void* h,
                    hipStream_t st) {
  Layout L;
  if (int r = core_xfer_check(cfg, L, workspace, t0, n)) return r;
  const char* ws = (const char*)workspace;
  const size_t M = (size_t)L.B * L.P, ge = core_gate_bytes(L);
  if (gates) HIPCHK(hipMemcpyAsync(gates, ws + L.Gt + (size_t)t0 * M * 512 * ge, (size_t)n * M * 512 * ge, hipMemcpyDeviceToDevice, st));
  if (c) HIPCHK(hipMemcpyAsync(c, ws + L.Cst + (size_t)(t0 + 1) * M * 128 * 4, (size_t)n * M * 128 * 4, hipMemcpyDeviceToDevice, st));
  if (h && L.esz == 4)
    HIPCHK(hipMemcpyAsync(h, ws + L.Hs + (size_t)t0 * M * 128 * 4, (size_t)n * M * 128 * 4, hipMemcpyDeviceToDevice, st));
  else if (h)   // bf16: the h half of XH slots t0+1 .. t0+n (n*M consecutive 192-channel rows)
    HIPCHK(hipMemcpy2DAsync(h, 128 * 2, ws + L.XH + ((size_t)(t0 + 1) * M * 192 + 64) * 2, 192 * 2, 128 * 2, n * M,
                            hipMemcpyDeviceToDevice, st));
  return AAA_OK;
}

int aaa_core_import(const aaa_cfg* cfg, void* workspace, int t0, int n, const void* gates, const float* c,
                    const void* h, hipStream_t st) {
  Layout L;
  if (int r = core_xfer_check(cfg, L, workspace, t0, n)) return r;
  if (!gates || !c || !h) return fail(AAA_E_ARG, "core import: gates, c and h are required");
  char* ws = (char*)workspace;
  const size_t M = (size_t)L.B * L.P, ge = core_gate_bytes(L);
  HIPCHK(hipMemcpyAsync(ws + L.Gt + (size_t)t0 * M * 512 * ge, gates, (size_t)n * M * 512 * ge, hipMemcpyDeviceToDevice, st));
  HIPCHK(hipMemcpyAsync(ws + L.Cst + (size_t)(t0 + 1) * M * 128 * 4, c, (size_t)n * M * 128 * 4, hipMemcpyDeviceToDevice, st));
  if (L.esz == 4) {
    HIPCHK(hipMemcpyAsync(ws + L.Hs + (size_t)t0 * M * 128 * 4, h, (size_t)n * M * 128 * 4, hipMemcpyDeviceToDevice, st));
    // slots t0+1 .. t0+n of XH are n*M consecutive 192-channel rows: one launch
    HIPCHK(state_to_xh<float>((int)(n * M), (const float*)h, (float*)(ws + L.XH) + (size_t)(t0 + 1) * M * 192, st));
  } else {
    HIPCHK(hipMemcpy2DAsync(ws + L.XH + ((size_t)(t0 + 1) * M * 192 + 64) * 2, 192 * 2, h, 128 * 2, 128 * 2, n * M,
                            hipMemcpyDeviceToDevice, st));
  }
  return AAA_OK;
}

int aaa_backward(const aaa_cfg* cfg, const aaa_io* io, int phases, hipStream_t stream) {
  Layout L;
  int r = build_layout(cfg, L);
  if (r) return r;
  if ((r = check_device())) return r;
  if ((r = check_io(L, io, true))) return r;
  if (phases & ~AAA_BWD_ALL || !phases) return fail(AAA_E_ARG, "bad phase mask %d", phases);
  if (!(cfg->flags & AAA_FLAG_DEFER_STRANDED) && (r = pair_check())) return r;
  return L.dt == AAA_BF16 ? backward_impl<__bf16>(L, io, phases, stream)
                          : backward_impl<float>(L, io, phases, stream);
}

int aaa_pair_status(hipStream_t stream, int clear) {
  if (stream && hipStreamSynchronize(stream) != hipSuccess) return fail(AAA_E_LAUNCH, "stream synchronize failed");
  if (!stream && hipDeviceSynchronize() != hipSuccess) return fail(AAA_E_LAUNCH, "device synchronize failed");
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return fail(AAA_E_DEVICE, "no HIP device");
  return clear ? pair_take() : pair_peek();
}

int aaa_pair_flag(float* dst, hipStream_t stream) {
  if (!dst) return fail(AAA_E_ARG, "pair_flag: NULL dst");
  int r = check_device();
  if (r) return r;
  int dev = 0;
  HIPCHK(hipGetDevice(&dev));
  const int* rep = pair_report(dev);
  int* base = pair_flag_base(dev);
  if (!rep || !base) return fail(AAA_E_LAUNCH, "cannot map the partner-timeout report word");
  HIPCHK(pair_flag_launch(rep, base, dst, stream));
  return AAA_OK;
}

int aaa_pair_flag_at(float* dst, int* base, hipStream_t stream) {
  if (!dst || !base) return fail(AAA_E_ARG, "pair_flag_at: NULL dst or base");
  int r = check_device();
  if (r) return r;
  int dev = 0;
  HIPCHK(hipGetDevice(&dev));
  const int* rep = pair_report(dev);
  if (!rep) return fail(AAA_E_LAUNCH, "cannot map the partner-timeout report word");
  HIPCHK(pair_flag_launch(rep, base, dst, stream));
  return AAA_OK;
}

int aaa_adam_step(const aaa_adam_hparams* hp, long step, int ntensors, float* const* params,
                  const float* const* grads, float* const* exp_avg, float* const* exp_avg_sq,
                  float* const* max_exp_avg_sq, const size_t* numel, hipStream_t stream) {
  return aaa_adam_step_guarded(hp, step, nullptr, ntensors, params, grads, exp_avg, exp_avg_sq, max_exp_avg_sq, numel,
                               stream);
}

static int adam_impl(const aaa_adam_hparams* hp, long step, int* step_dev, const float* guard, int ntensors,
                     float* const* params, const float* const* grads, float* const* exp_avg,
                     float* const* exp_avg_sq, float* const* max_exp_avg_sq, const size_t* numel,
                     hipStream_t stream) {
  if (!hp || ntensors < 0 || (ntensors > 0 && (!params || !grads || !exp_avg || !exp_avg_sq || !numel)))
    return fail(AAA_E_ARG, "adam: NULL argument");
  if (!step_dev && step < 1) return fail(AAA_E_ARG, "adam: step must be >= 1 (got %ld)", step);
  if (hp->amsgrad && !max_exp_avg_sq) return fail(AAA_E_ARG, "adam: amsgrad needs max_exp_avg_sq");
  if (!(hp->lr >= 0.0) || !(hp->eps >= 0.0) || !(hp->beta1 >= 0.0 && hp->beta1 < 1.0) ||
      !(hp->beta2 >= 0.0 && hp->beta2 < 1.0) || !(hp->weight_decay >= 0.0))
    return fail(AAA_E_ARG, "adam: invalid hyper-parameters");
  int r = check_device();
  if (r) return r;
  AdamHost h{hp->lr, hp->beta1, hp->beta2, hp->eps, hp->weight_decay, step_dev ? 1 : step, hp->amsgrad ? 1 : 0,
             hp->maximize ? 1 : 0, guard, step_dev};
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
    HIPCHK(adam_launch(tab, nch, h, stream, t0 + kAdamMaxTensors >= ntensors));
  }
  if (ntensors == 0 && step_dev) HIPCHK(adam_launch(AdamTable{}, 0, h, stream, true));
  return AAA_OK;
}

int aaa_adam_step_guarded(const aaa_adam_hparams* hp, long step, const float* guard, int ntensors,
                          float* const* params, const float* const* grads, float* const* exp_avg,
                          float* const* exp_avg_sq, float* const* max_exp_avg_sq, const size_t* numel,
                          hipStream_t stream) {
  return adam_impl(hp, step, nullptr, guard, ntensors, params, grads, exp_avg, exp_avg_sq, max_exp_avg_sq, numel,
                   stream);
}

int aaa_adam_step_counted(const aaa_adam_hparams* hp, int* step_dev, const float* guard, int ntensors,
                          float* const* params, const float* const* grads, float* const* exp_avg,
                          float* const* exp_avg_sq, float* const* max_exp_avg_sq, const size_t* numel,
                          hipStream_t stream) {
  if (!step_dev) return fail(AAA_E_ARG, "adam: NULL step counter");
  return adam_impl(hp, 0, step_dev, guard, ntensors, params, grads, exp_avg, exp_avg_sq, max_exp_avg_sq, numel,
                   stream);
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
// Workspace: conv2 output X (B,P,64), h_t Hs (B,P,128), hid1 (B,512), AO (B,256), LH (B,256),
// the ConvLSTM's split-K partial tiles, the tile and readout counters, the attention logits,
// the readout's chunk partials and the answer row (actor.h).
static int actor_layout(const aaa_cfg* cfg, Layout& L, size_t off[10], size_t* total) {
  int r = build_layout(cfg, L);
  if (r) return r;
  if (cfg->T != 1) return fail(AAA_E_ARG, "actor_step: T must be 1 (got %d)", cfg->T);
  if (cfg->dtype != AAA_F32) return fail(AAA_E_ARG, "actor_step: fp32 weights only (bf16 agents use aaa_forward)");
  if (L.sc) return fail(AAA_E_ARG, "actor_step: the stateful policy core uses aaa_forward");
  if (cfg->B > 16) return fail(AAA_E_ARG, "actor_step: B <= 16 (got %d); larger batches use aaa_forward", cfg->B);
  if (actor_chunks(L.P) > kActMaxChunks)
    return fail(AAA_E_ARG, "actor_step: a %dx%d grid exceeds the readout's %d position chunks; use aaa_forward",
                L.h, L.w, kActMaxChunks);
  const size_t B = cfg->B, P = L.P;
  const size_t nt = 8 * (size_t)actor_pix_tiles(L.P), nch = actor_chunks(L.P), nq = L.nq;
  const size_t sz[10] = {B * P * 64 * 4, B * P * 128 * 4, B * 512 * 4, B * 256 * 4, B * 256 * 4,
                         B * nt * kActLstmKS * 4096 * 4, (B * nt + B + 1) * 4, B * P * nq * 4,
                         B * nch * nq * kAttnPart * 4, B * (size_t)L.ans_ld * 4};
  size_t o = 0;
  for (int i = 0; i < 10; ++i) { off[i] = o; o = al256(o + sz[i]); }
  *total = o;
  return AAA_OK;
}

size_t aaa_actor_workspace_bytes(const aaa_cfg* cfg) {
  Layout L;
  size_t off[10], tot = 0;
  return actor_layout(cfg, L, off, &tot) ? 0 : tot;
}

int aaa_actor_step(const aaa_cfg* cfg, const aaa_actor_io* io, hipStream_t stream) {
  Layout L;
  size_t off[10], tot = 0;
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
  p.gates = io->gates;
  p.hout = io->h_out; p.cout = io->c_out;
  p.X = (float*)(ws + off[0]); p.Hs = (float*)(ws + off[1]); p.hid1 = (float*)(ws + off[2]);
  p.AO = (float*)(ws + off[3]); p.LH = (float*)(ws + off[4]);
  p.Zp = (float*)(ws + off[5]); p.zcnt = (int*)(ws + off[6]);
  p.Lg = (float*)(ws + off[7]); p.Apart = (float*)(ws + off[8]); p.arow = (float*)(ws + off[9]);
  p.seed = io->seed; p.counter = io->counter; p.actions = io->actions; p.logp = io->logp; p.jac = io->dlogp_dlogits;
  HIPCHK(actor_launch(p, stream));
  return AAA_OK;
}

}  // extern "C"
