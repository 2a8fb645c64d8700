/*
 * aaa.h -- C ABI of the MI355X (gfx950) attention-augmented-agent learner.
 *
 * One shared library (libaaa.so, built by hipcc --offload-arch=gfx950) that
 * replaces the ATen op sequence of the reference's batched unroll: the
 * forward of Agent (reference attention.py:298-368, including
 * VisionNetwork.forward :178-181, ConvLSTMCell.forward :110-126,
 * QueryNetwork :184-198, SpatialBasis.__call__ :228-232, spatial_softmax
 * :235-243, apply_alpha :246-254) over T steps from reset() (:293-296), and
 * the backward that autograd runs for it when main_mp.py:77 calls
 * policy_loss.backward().
 *
 * Conventions
 *  - All pointers are DEVICE pointers on the caller's current HIP device,
 *    except the cfg/io structs themselves (host memory).
 *  - Ownership: the caller owns every buffer (params, packed weights,
 *    workspace, outputs).  The library never allocates or frees device
 *    memory and keeps no device state.
 *  - Streams: all work is enqueued on ``stream``; nothing synchronises.
 *  - Errors: functions return 0 on success, a negative AAA_E* code
 *    otherwise; aaa_last_error() returns a thread-local message.
 *  - Threading: re-entrant; each call only touches the buffers it is given.
 *
 * Layouts
 *  - params / grads: the 34 reference state_dict tensors, fp32, concatenated
 *    in state_dict order (reference attention.py:257-291),
 *    each tensor in its PyTorch (contiguous) layout.  aaa_param_layout()
 *    returns the offsets.  nq != 4 uses the generalised query / answer widths
 *    (query 256->128->72nq->72nq, answer 256nq+2).
 *  - frames: (T, B, H, W, 3) NHWC raw pixels, fp32 (main_mp.py:53 casts the
 *    uint8 observation to float without normalisation) or the uint8
 *    observation itself (AAA_FLAG_FRAMES_U8).
 *  - basis: (h, w, 64) fp32 spatial basis (SpatialBasis.S, attention.py:226).
 *  - logits, values: (T, B, A) fp32; attn: (T, B, h, w, nq) fp32 softmax maps.
 *  - prev_reward / prev_action: (T, B) fp32 or NULL (zeros, :303-312).
 *  - ConvLSTM state h0, c0, hT, cT, dh0, dc0, dhT, dcT: (B, h, w, 128) fp32
 *    NHWC (the reference keeps (B,128,w,h)), NULL = zero /
 *    not requested.
 */
#ifndef AAA_H
#define AAA_H

#include <stddef.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AAA_ABI_VERSION 9

enum aaa_status {
  AAA_OK = 0,
  AAA_E_ARG = -1,      /* bad shape / NULL / unsupported configuration */
  AAA_E_ALIGN = -2,    /* a buffer is not 16-byte aligned */
  AAA_E_LAUNCH = -3,   /* a HIP launch or runtime call failed */
  AAA_E_DEVICE = -4,   /* current device is not gfx950 */
  AAA_E_STRANDED = -5  /* a paired frame-resident kernel of an EARLIER call timed out
                          waiting for its partner workgroup: that call's outputs are
                          invalid (reported once, by the next call or aaa_pair_status) */
};

enum aaa_dtype {
  AAA_F32 = 0,   /* conv/ConvLSTM GEMM operands fp32 (exact v_mfma_f32_32x32x2_f32) */
  AAA_BF16 = 1   /* conv/ConvLSTM GEMM operands bf16, fp32 accumulate + gate math */
};

typedef struct aaa_cfg {
  int B;        /* sequences (batch rows)                                    */
  int T;        /* unroll length (steps since reset())                        */
  int H, W;     /* frame size, e.g. 84x84, 168x168, 210x160                    */
  int nq;       /* attention queries (reference: 4, attention.py:265)          */
  int A;        /* actions (Seaquest: 18, main_mp.py:179)                       */
  int dtype;    /* enum aaa_dtype                                             */
  int flags;    /* AAA_FLAG_* (0: the reference's reachable path)             */
} aaa_cfg;

/* Stateful policy core: the reference's `else` branch (attention.py:356-358),
 * taken when agent.prev_hidden holds a tensor -- the query is computed from
 * prev_output = h_{t-1} and the LSTMCell runs from (h_{t-1}, c_{t-1}), both
 * carried across steps (and across calls through io->core_*).  Off, the
 * reference's reachable path: zero query input, zero-state LSTMCell (Q1). */
#define AAA_FLAG_STATEFUL_CORE 1
/* io->frames holds uint8 pixels (T, B, H, W, 3) -- the environment's
 * observation (main_mp.py:49-53 casts it to float on the host); the cast is
 * fused into the kernel that lays the frames out for conv1. */
#define AAA_FLAG_FRAMES_U8 2
/* Do not consume / fail on partner-timeout reports of earlier launches at
 * entry (see aaa_pair_status): the caller checks them itself after the
 * iteration, e.g. through aaa_pair_flag and the guarded optimizer. */
#define AAA_FLAG_DEFER_STRANDED 4

typedef struct aaa_io {
  /* inputs */
  const float* params;       /* flat fp32 params (state_dict order)            */
  const void* packed;        /* aaa_pack_weights output                        */
  const float* basis;        /* (h, w, 64)                                     */
  const void* frames;        /* (T, B, H, W, 3) fp32, or uint8 with AAA_FLAG_FRAMES_U8 */
  const float* prev_reward;  /* (T, B) or NULL                                 */
  const float* prev_action;  /* (T, B) or NULL                                 */
  const float* h0;           /* (B, h, w, 128) or NULL                         */
  const float* c0;           /* (B, h, w, 128) or NULL                         */
  /* forward outputs */
  float* logits;             /* (T, B, A)                                      */
  float* values;             /* (T, B, A)                                      */
  float* attn;               /* (T, B, h, w, nq) or NULL                       */
  float* hT;                 /* (B, h, w, 128) or NULL                         */
  float* cT;                 /* (B, h, w, 128) or NULL                         */
  /* backward inputs */
  const float* dlogits;      /* (T, B, A)                                      */
  const float* dvalues;      /* (T, B, A) or NULL                              */
  const float* dhT;          /* (B, h, w, 128) or NULL                         */
  const float* dcT;          /* (B, h, w, 128) or NULL                         */
  /* backward outputs */
  float* grads;              /* flat fp32 grads, same layout as params         */
  float* dh0;                /* (B, h, w, 128) or NULL                         */
  float* dc0;                /* (B, h, w, 128) or NULL                         */
  /* scratch */
  void* workspace;           /* aaa_workspace_bytes(); activations saved by
                                aaa_forward for aaa_backward live here        */
  /* stateful policy core (AAA_FLAG_STATEFUL_CORE only; ignored otherwise):
     (B, 256) fp32 (prev_output, prev_hidden) in, out and their grads      */
  const float* core_h0;      /* or NULL (zeros: reset())                       */
  const float* core_c0;      /* or NULL                                        */
  float* core_hT;            /* or NULL                                        */
  float* core_cT;            /* or NULL                                        */
  const float* dcore_hT;     /* backward input or NULL                         */
  const float* dcore_cT;     /* backward input or NULL                         */
  float* dcore_h0;           /* backward output or NULL                        */
  float* dcore_c0;           /* backward output or NULL                        */
} aaa_io;

/* Backward phases, in execution order (DP bucket boundaries). */
enum aaa_bwd_phase {
  AAA_BWD_HEAD = 1,    /* heads, LSTMCell, answer MLP, attention, query MLP */
  AAA_BWD_CORE = 2,    /* ConvLSTM BPTT + ConvLSTM weight/bias grads         */
  AAA_BWD_VISION = 4,  /* conv2 / conv1 weight & bias grads                  */
  AAA_BWD_ALL = 7
};

int aaa_abi_version(void);
const char* aaa_last_error(void);

/* Spatial grid (h, w) the encoder produces for an H x W frame. */
int aaa_grid(int H, int W, int* h, int* w);

/* Number of fp32 params and the offset/size of each of the 34 tensors
 * (state_dict order).  offsets/sizes may be NULL. */
int aaa_param_layout(const aaa_cfg* cfg, size_t* total, size_t* offsets, size_t* sizes);

size_t aaa_packed_bytes(const aaa_cfg* cfg);
size_t aaa_workspace_bytes(const aaa_cfg* cfg);

/* Re-lay the params into the kernels' operand layouts (gate-interleaved
 * ConvLSTM / LSTMCell rows, NHWC tap-major conv weights with the
 * reference's transposed kernel orientation, bf16 when cfg->dtype says so).
 * Must run after every parameter update. */
int aaa_pack_weights(const aaa_cfg* cfg, const float* params, void* packed, hipStream_t stream);

/* T-step forward from reset(); replaces T calls of Agent.forward. */
int aaa_forward(const aaa_cfg* cfg, const aaa_io* io, hipStream_t stream);

/* Forward phases (aaa_forward_phases).  Skipping CORE leaves the ConvLSTM
 * recurrence out: its per-step products -- gate activations, c_t, h_t of
 * every step -- must already be in the workspace (aaa_core_import), as the
 * fused episode backward does with the products each per-step call of the
 * episode exported (episode.py).  VISION and TAIL always run. */
enum aaa_fwd_phase {
  AAA_FWD_VISION = 1,  /* conv1 + conv2 over all T*B frames                   */
  AAA_FWD_CORE = 2,    /* the ConvLSTM recurrence                             */
  AAA_FWD_TAIL = 4,    /* attention readout, answer MLP, LSTMCell, heads      */
  AAA_FWD_ALL = 7
};
/* aaa_forward with a phase mask: AAA_FWD_ALL, or AAA_FWD_VISION |
 * AAA_FWD_TAIL (configs whose slices are row-major: not the frame-resident
 * bf16 BPTT's channel-quad-major ones).  Replaces the recomputation half of the
 * reference's per-step graph (main_mp.py:54 -> attention.py:110-126). */
int aaa_forward_phases(const aaa_cfg* cfg, const aaa_io* io, int phases, hipStream_t stream);

/* The ConvLSTM products of steps [t0, t0+n) between an aaa_forward workspace
 * and flat buffers: gates (n, B*h*w, 512) post-activation (i, f, c~, o
 * interleaved per channel), c (n, B*h*w, 128) = c_t fp32, h (n, B*h*w, 128) =
 * h_t (pixel-major, channel fastest).  Element types (aaa_core_elem_bytes):
 * fp32 configs all fp32; bf16 configs gates in the workspace's gate storage
 * (fp16, or fp32 with AAA_GATES_F16=0) and h bf16 (the operand the next step
 * and the weight gradient read).  Export reads a workspace aaa_forward
 * filled; import writes one for aaa_forward_phases without CORE (and the h
 * half of the [x | h] operand slots).  Not for channel-quad-major slices
 * (large-batch bf16: AAA_E_ARG; aaa_core_elem_bytes reports 0 bytes for such
 * a geometry); device pointers, stream-ordered, no host sync. */
int aaa_core_elem_bytes(const aaa_cfg* cfg, int* gate_bytes, int* h_bytes);
int aaa_core_export(const aaa_cfg* cfg, const void* workspace, int t0, int n, void* gates, float* c, void* h,
                    hipStream_t stream);
int aaa_core_import(const aaa_cfg* cfg, void* workspace, int t0, int n, const void* gates, const float* c,
                    const void* h, hipStream_t stream);

/* Backward of the loss sum(logits*dlogits)+sum(values*dvalues) (+ state
 * cotangents) through the saved activations of the matching aaa_forward.
 * ``phases`` is a mask of aaa_bwd_phase; phases must run in order. grads
 * are overwritten (not accumulated) by the phases that own them. */
int aaa_backward(const aaa_cfg* cfg, const aaa_io* io, int phases, hipStream_t stream);

/* Health of the multi-workgroup frame-resident ConvLSTM kernels (two or more
 * cooperating workgroups per frame: the paired and band-mode bf16 kernels and
 * the fp32 frame-group kernels, launched as ordinary grids that fit one
 * residency wave of an idle chip).  Their partner waits are bounded by a
 * deadline on the 100-MHz real-time counter (1 s + 20 ms per step after a
 * workgroup's first wait); a wait that expires is counted in a word of
 * pinned, device-mapped host memory and the kernel proceeds on a stale
 * partner slice (later waits of that workgroup return at once, so a kernel
 * whose partner never runs ends within about one budget).  The count is
 * monotonic; its two readers keep their own snapshots of it:
 *  - the host: aaa_forward / aaa_backward consume the counts reported since
 *    the host last did and return AAA_E_STRANDED -- unless the cfg carries
 *    AAA_FLAG_DEFER_STRANDED, for a caller that must not fail mid-iteration
 *    (a data-parallel learner whose peers would wait in a collective) and
 *    checks with aaa_pair_status after it; aaa_pair_status synchronises
 *    ``stream`` (NULL: the device) and returns that count (>= 0; clear != 0
 *    consumes it);
 *  - the device: aaa_pair_flag enqueues on ``stream`` a kernel that writes
 *    into dst[0], as a float, the counts reported since the previous
 *    aaa_pair_flag on this device, in stream order.  A learner puts it beside
 *    its gradients so the gradient all-reduce carries it to every rank and
 *    aaa_adam_step_counted / _guarded skips the update of a step whose
 *    gradients came from a stranded launch, with no host sync; host-side
 *    consumption never resets what the device-side reader sees. */
int aaa_pair_status(hipStream_t stream, int clear);
int aaa_pair_flag(float* dst, hipStream_t stream);
/* aaa_pair_flag_at (ABI 9): as aaa_pair_flag, but against the caller's own
 * snapshot ``base`` (one int of device memory the caller owns; the kernel
 * reads it, writes the count past it into dst[0] and advances it), so several
 * readers on one device -- two learners, a learner and a diagnostic -- never
 * take each other's timeouts.  A new reader syncs its base to the current
 * report word with one call whose dst it discards. */
int aaa_pair_flag_at(float* dst, int* base, hipStream_t stream);

/* ---- workspace inspection (checkers, diagnostics) ----
 * Byte offset and size, inside an aaa_forward workspace laid out for ``cfg``,
 * of a forward product a checker may read after the call (the workspace is
 * caller-owned device memory; nothing here syncs or copies):
 *   AAA_WS_ANSWER_HIDDEN  (T*B, 512) fp32: relu(answer_processor.0(answer)),
 *                         attention.py:277-282 -- its > 0 pattern is the
 *                         ReLU mask the hand-written backward applies;
 *   AAA_WS_QUERY_HIDDEN0  (T*B, 128) fp32: relu(query.model.0(h_{t-1})),
 *   AAA_WS_QUERY_HIDDEN1  (T*B, 72 nq) fp32: relu(query.model.2(.)), the
 *                         stateful core's query MLP (attention.py:184-198);
 *                         AAA_FLAG_STATEFUL_CORE only.
 * Frame f = t*B + b.  AAA_E_ARG for an unknown region or one the cfg does not
 * compute.  A test reads these masks to run the oracle's backward through the
 * same ReLU on/off pattern (tests/helpers.py hip_relu_masks). */
enum aaa_ws_region { AAA_WS_ANSWER_HIDDEN = 0, AAA_WS_QUERY_HIDDEN0 = 1, AAA_WS_QUERY_HIDDEN1 = 2 };
int aaa_workspace_region(const aaa_cfg* cfg, int region, size_t* offset, size_t* bytes);

/* ---- optional kernel timing (benchmarks) ----
 * While enabled, the runtime records a hipEvent pair on the launch stream
 * around every launch of the kernel classes below.  aaa_timing_read()
 * waits for the recorded events and returns the summed device time and the
 * number of launches since the last enable/read, then clears that class. */
enum aaa_timer {
  AAA_TIMER_FWD_STEP = 0,    /* fused ConvLSTM forward step (one per t)          */
  AAA_TIMER_BPTT_STEP = 1,   /* ConvLSTM dgrad + fused gate backward (one per t) */
  AAA_TIMER_CORE_WGRAD = 2,  /* ConvLSTM weight-gradient GEMM over all frames    */
  AAA_TIMER_ATTN_FWD = 3,    /* fused spatial-softmax attention readout (HBM)    */
  AAA_TIMER_ATTN_BWD = 4,    /* its backward (HBM)                               */
  /* the rest of a learner iteration, so the classes cover the whole step
     (work in FLOP where a GEMM dominates, 0 for the latency-bound glue):     */
  AAA_TIMER_PACK = 5,        /* aaa_pack_weights (all packed layouts)            */
  AAA_TIMER_VISION_FWD = 6,  /* frames -> conv1 -> conv2 (the vision encoder)    */
  AAA_TIMER_TAIL_FWD = 7,    /* query pack, answer MLP, LSTMCell, heads          */
  AAA_TIMER_TAIL_BWD = 8,    /* their backward (HEAD phase minus the attention)  */
  AAA_TIMER_CORE_DX = 9,     /* batched conv2-output grad dx (when not fused)    */
  AAA_TIMER_VISION_BWD = 10, /* conv2 wgrad + dgrad, conv1 wgrad, grad unpack    */
  AAA_TIMER_MISC = 11,       /* state copies, memsets, bias column sums          */
  AAA_TIMER_N = 12
};
int aaa_timing_enable(int on);
int aaa_timing_read(int kind, double* total_ms, long* launches);
/* The same read with the roofline inputs the runtime knows: the summed
 * algorithmic work of those launches (FLOP for the MFMA classes 0-2 and 6-10:
 * 2*M*N*K of each GEMM; bytes for the HBM classes 3-4: the fp32 tensors each
 * frame must move; 0 for 5 and 11) and the kernel variant (tile / ring)
 * dispatched last.  A "launch" of classes 5-11 is one timed region (a group
 * of consecutive kernels of that class). */
typedef struct aaa_timer_stats {
  double total_ms;
  long launches;
  double work;
  char variant[192];
} aaa_timer_stats;
int aaa_timing_stats(int kind, aaa_timer_stats* out);

/* ---- optimizer ----
 * One fused multi-tensor Adam step with torch.optim.Adam semantics (the
 * reference's optimizer: main_mp.py:92 builds Adam(policy.parameters(),
 * lr=1e-3), main_mp.py:78 steps it).  ``step`` is the step count after this
 * update (1 on the first call).  Tensor i has numel[i] fp32 elements at
 * params[i] / grads[i] / exp_avg[i] / exp_avg_sq[i] (and max_exp_avg_sq[i]
 * when amsgrad; the array may be NULL otherwise), all updated in place on
 * ``stream``.  The pointer arrays are host memory; the tensors are device
 * memory.  A flat parameter buffer is simply ntensors = 1. */
typedef struct aaa_adam_hparams {
  double lr, beta1, beta2, eps, weight_decay;
  int amsgrad, maximize;
} aaa_adam_hparams;

int aaa_adam_step(const aaa_adam_hparams* hp, long step, int ntensors, float* const* params,
                  const float* const* grads, float* const* exp_avg, float* const* exp_avg_sq,
                  float* const* max_exp_avg_sq, const size_t* numel, hipStream_t stream);
/* The same update, skipped on the device when *guard != 0 (guard: one
 * device float, e.g. the all-reduced aaa_pair_flag slot of the gradients):
 * no parameter or moment is written and no host sync is needed. */
int aaa_adam_step_guarded(const aaa_adam_hparams* hp, long step, const float* guard, int ntensors,
                          float* const* params, const float* const* grads, float* const* exp_avg,
                          float* const* exp_avg_sq, float* const* max_exp_avg_sq, const size_t* numel,
                          hipStream_t stream);
/* The guarded update with the step count kept on the device: *step_dev (one
 * device int, 0 before the first update) is the number of updates applied so
 * far; this one runs as update *step_dev + 1 (torch's bias corrections of
 * that step, in double) and, in stream order after it, *step_dev advances
 * only if the guard let the update through -- so a skipped step leaves the
 * moments AND the bias corrections exactly where they were. */
int aaa_adam_step_counted(const aaa_adam_hparams* hp, int* step_dev, const float* guard, int ntensors,
                          float* const* params, const float* const* grads, float* const* exp_avg,
                          float* const* exp_avg_sq, float* const* max_exp_avg_sq, const size_t* numel,
                          hipStream_t stream);

/* ---- REINFORCE loss ----
 * finish_episode's loss (reference main_mp.py:62-77) for B independent
 * episodes of T steps, on device: discounted returns R_t = r_t + gamma R_{t+1}
 * (double, then fp32), normalised (R - mean) / (std_unbiased + FLT_EPSILON)
 * into returns_norm (T, B); loss[b] = sum_t -log pi(a_t) R^_t with pi =
 * Categorical(softmax(logits_t)) and its probability clamp to [eps, 1-eps]
 * (main_mp.py:55-58); dlogits (T, B, A) = d(sum_b loss[b]) / d logits, the
 * cotangent aaa_backward takes.  logits (T, B, A) fp32, actions (T, B) int32
 * in [0, A), rewards (T, B) fp32; every pointer is device memory. */
int aaa_reinforce(int T, int B, int A, const float* logits, const int* actions, const float* rewards, double gamma,
                  float* loss, float* returns_norm, float* dlogits, hipStream_t stream);

/* ---- actor: action sampling ----
 * Policy.forward's draw (reference main_mp.py:54-58: F.softmax over the
 * logits, Categorical(probs).sample(), .log_prob(action)) for B rows of
 * logits (B, A) fp32, on device and without a host round trip: actions (B)
 * int32 by inverse-CDF sampling of softmax(logits) with a counter-based
 * uniform u = rng(seed, *counter, row) (splitmix64 finaliser, 24-bit);
 * logp (B) = log(clamp(p_a, FLT_EPSILON, 1 - FLT_EPSILON)) as Categorical
 * computes it; dlogp_dlogits (B, A) = 1[k == a] - p_k (0 where the clamp is
 * active), or NULL.  ``counter`` is a device uint64 advanced by one per call
 * (NULL = draw index 0), so a captured hipGraph replays fresh draws.  The
 * draws are not torch's multinomial stream; the distribution is the same. */
int aaa_sample_actions(int B, int A, const float* logits, unsigned long long seed, unsigned long long* counter,
                       int* actions, float* logp, float* dlogp_dlogits, hipStream_t stream);

/* ---- actor: one environment step ----
 * The acting half of the reference's loop -- Policy.forward (main_mp.py:49-59)
 * = Agent.forward (attention.py:298-368) on one observation per row, with the
 * ConvLSTM state carried (attention.py:125, 142-149), then the draw of
 * aaa_sample_actions -- for B <= 16 rows, as a chain of six launches sized for
 * small B (vision, ConvLSTM step, attention + answer layer 0, answer layer 2,
 * LSTMCell, heads + draw) instead of aaa_forward's whole-batch kernels.
 * Results equal aaa_forward with T = 1, h0 = *h, c0 = *c up to fp32
 * summation order; the draw is bit-identical to aaa_sample_actions on those
 * logits.  cfg: T = 1, dtype AAA_F32, no AAA_FLAG_STATEFUL_CORE (those use
 * aaa_forward); ``packed`` from aaa_pack_weights with the same cfg.  h, c
 * (B, h, w, 128) are read and overwritten with the step's state (zero them for
 * reset()).  actions == NULL skips the draw (seed/counter/logp/dlogp ignored). */
typedef struct aaa_actor_io {
  const float* params;       /* flat fp32 params                               */
  const void* packed;        /* aaa_pack_weights output (same cfg)             */
  const float* basis;        /* (h, w, 64)                                     */
  const void* frames;        /* (B, H, W, 3) fp32, or uint8 with AAA_FLAG_FRAMES_U8 */
  const float* prev_reward;  /* (B) or NULL                                    */
  const float* prev_action;  /* (B) or NULL                                    */
  float* h;                  /* (B, h, w, 128) ConvLSTM state, in/out          */
  float* c;                  /* (B, h, w, 128) cell state, in/out              */
  float* logits;             /* (B, A)                                         */
  float* values;             /* (B, A)                                         */
  float* attn;               /* (B, h, w, nq) or NULL                          */
  void* workspace;           /* aaa_actor_workspace_bytes()                    */
  unsigned long long seed;   /* action draw: as aaa_sample_actions             */
  unsigned long long* counter;
  int* actions;              /* (B) or NULL (no draw)                          */
  float* logp;               /* (B) or NULL                                    */
  float* dlogp_dlogits;      /* (B, A) or NULL                                 */
  float* gates;              /* (B, h, w, 512) or NULL: the ConvLSTM step's gate
                                activations (i, f, c~, o), row 4*ch + gate -- the
                                products a fused episode backward imports
                                (aaa_core_import) instead of re-running the step */
  float* h_out;              /* (B, h, w, 128) or NULL: h_t written here instead of
                                over ``h`` (which is then only read)         */
  float* c_out;              /* (B, h, w, 128) or NULL: likewise c_t           */
} aaa_actor_io;
size_t aaa_actor_workspace_bytes(const aaa_cfg* cfg);
int aaa_actor_step(const aaa_cfg* cfg, const aaa_actor_io* io, hipStream_t stream);

/* ---- single-kernel entry points (unit tests against PyTorch fp32) ---- */

/* NHWC convolution y[n,oy,ox,co] = b[co] + sum w[co,ky,kx,ci] x[n,iy,ix,ci]
 * (weights in [Cout][KH][KW][Cin] order, i.e. torch weight.permute(0,2,3,1)).
 * dtype selects the MFMA operand type.  bias may be NULL. */
typedef struct aaa_conv_desc {
  int N, Hin, Win, Cin, Hout, Wout, Cout, KH, KW, stride, pad, dtype;
} aaa_conv_desc;

int aaa_conv2d_nhwc(const aaa_conv_desc* d, const float* x, const float* w, const float* bias,
                    float* y, hipStream_t stream);
/* dx = conv2d_input(dy, w) (NHWC) */
int aaa_conv2d_nhwc_dgrad(const aaa_conv_desc* d, const float* dy, const float* w, float* dx,
                          hipStream_t stream);
/* dw[co][ky][kx][ci] = conv2d_weight(x, dy), overwritten */
int aaa_conv2d_nhwc_wgrad(const aaa_conv_desc* d, const float* x, const float* dy, float* dw,
                          hipStream_t stream);

/* C[m][n] = sum_k A[m][k] * Bw[n][k] (+ bias[n]) -- torch.nn.functional.linear */
int aaa_linear(int M, int N, int K, const float* x, const float* w, const float* bias, float* y,
               hipStream_t stream);

/* ---- component entry points ----
 * One reference module each, on caller-owned buffers, through the kernels
 * aaa_forward / aaa_backward run for that module.  They back the drop-in's
 * standalone ConvLSTMCell.forward / VisionNetwork.forward and let each piece
 * be checked in isolation.  Layout convention (Q3): the reference's NCHW
 * tensors (B, C, a, b) of the vision core are passed NHWC as
 * x.permute(0, 3, 2, 1) = (B, b, a, C); for the Agent's vision core that is
 * (B, h, w, C) with (h, w) the grid of an H x W frame. */

/* ConvLSTMCell(64, 128, 3) at one step (attention.py:110-126, zero
 * peepholes :132-141).  cell_params: the cell's 12 state_dict tensors fp32,
 * concatenated in state_dict order (W{x,h}{i,f,c,o} as in attention.py:39-102:
 * Wxi.weight, Wxi.bias, Whi.weight, Wxf.weight, ...; 885,248 floats) -- a
 * contiguous slice of aaa_param_layout's params.  x (B,h,w,64); h0, c0, h1,
 * c1 (B,h,w,128); h0/c0 NULL = the zero state of init_hidden (:142-149).
 * The workspace keeps the step's activations for aaa_convlstm_cell_bwd. */
typedef struct aaa_cell_desc {
  int B, h, w, dtype;
} aaa_cell_desc;
size_t aaa_convlstm_packed_bytes(const aaa_cell_desc* d);
size_t aaa_convlstm_workspace_bytes(const aaa_cell_desc* d);
int aaa_convlstm_pack(const aaa_cell_desc* d, const float* cell_params, void* packed, hipStream_t stream);
int aaa_convlstm_cell_fwd(const aaa_cell_desc* d, const void* packed, const float* x, const float* h0,
                          const float* c0, float* h1, float* c1, void* workspace, hipStream_t stream);
/* Backward through the matching forward's workspace: dh1/dc1 (NULL = 0) ->
 * dx (B,h,w,64), dh0, dc0 (each NULL = not wanted) and, when cell_grads is
 * set, the 12 parameter gradients (overwritten) in cell_params' layout. */
int aaa_convlstm_cell_bwd(const aaa_cell_desc* d, const void* packed, const float* dh1, const float* dc1, float* dx,
                          float* dh0, float* dc0, float* cell_grads, void* workspace, hipStream_t stream);

/* VisionNetwork.vision_cnn (attention.py:155-170) applied to X.transpose(1,3)
 * (:179): frames (N,H,W,3) fp32 -> y2 (N,h,w,64) (= the reference's output
 * permuted (0,3,2,1)), y1 (N,H1,W1,32) the conv1 output (NULL = not wanted).
 * cnn_params: vision_cnn.{0,1}.{weight,bias} fp32 in state_dict order (39,008
 * floats, the head of aaa_param_layout's params). */
typedef struct aaa_cnn_desc {
  int N, H, W, dtype;
} aaa_cnn_desc;
size_t aaa_vision_cnn_packed_bytes(const aaa_cnn_desc* d);
size_t aaa_vision_cnn_workspace_bytes(const aaa_cnn_desc* d);
int aaa_vision_cnn_pack(const aaa_cnn_desc* d, const float* cnn_params, void* packed, hipStream_t stream);
int aaa_vision_cnn_fwd(const aaa_cnn_desc* d, const float* cnn_params, const void* packed, const float* frames,
                       float* y1, float* y2, void* workspace, hipStream_t stream);
/* dy2 (N,h,w,64) -> the four parameter gradients (overwritten, cnn_params'
 * layout) and dy1 (N,H1,W1,32) (NULL = not wanted); frames get no gradient. */
int aaa_vision_cnn_bwd(const aaa_cnn_desc* d, const void* packed, const float* dy2, float* dy1, float* cnn_grads,
                       void* workspace, hipStream_t stream);

/* Attention readout of F frames (attention.py:319-348: K/V split + spatial
 * basis, logits K.Q, spatial_softmax :235-243, apply_alpha :246-254, answer
 * assembly): O (F,h,w,128) the vision output, S (h,w,64), Q (nq,72) shared by
 * every frame (q_stride 0, the reference's constant query) or (F,nq,72)
 * (q_stride nq*72), prev_reward/prev_action (F) or NULL (zeros) ->
 * attn (F,h,w,nq) and answer (F, 256nq+2) = [a_0..a_{nq-1} (184 each) |
 * Q_0..Q_{nq-1} (72 each) | r | a_prev], the reference's ``answer`` before
 * answer_processor. */
int aaa_attn_fwd(int F, int h, int w, int nq, const float* O, const float* S, const float* Q, int q_stride,
                 const float* prev_reward, const float* prev_action, float* attn, float* answer, hipStream_t stream);
/* Its backward from danswer (F, 256nq+2): dO (F,h,w,128) and dQ (F,nq,72) per
 * frame (logits path + the answer's Q columns; sum over F for a shared Q). */
int aaa_attn_bwd(int F, int h, int w, int nq, const float* O, const float* S, const float* Q, int q_stride,
                 const float* attn, const float* danswer, float* dO, float* dQ, hipStream_t stream);

/* ---- index-arithmetic self-checks (host only, no device needed) ----
 * Every pixel / tap / tile index in the kernels is divided by a runtime
 * constant through one multiply-shift divider (csrc/common.h FastDiv).
 * aaa_fastdiv_check runs the divider for d on every dividend n in [lo, hi)
 * (hi <= 2^31, the divider's whole domain) against the exact quotient and
 * returns the number of mismatches in *mismatches.  aaa_divisor_log(1, ...)
 * starts recording every divisor the runtime builds for its launches;
 * aaa_divisor_log(-1, out, cap) copies them out; aaa_divisor_log(0, ...)
 * copies, stops and clears.  Returns the number recorded. */
int aaa_fastdiv_check(unsigned d, unsigned lo, unsigned hi, unsigned long long* mismatches);
int aaa_divisor_log(int enable, unsigned* out, int cap);

#ifdef __cplusplus
}
#endif
#endif /* AAA_H */
