"""CPU oracle for the attention-agent unroll.  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module, and only as the checker / the timed CPU baseline.  The product
path (the HIP library behind the drop-in ``attention`` module) never calls it.

What it is: a functional plain-PyTorch (fp32, CPU) restatement of the
reference hot path, op for op, so its numbers are the reference's numbers:

  * vision encoder + ConvLSTM step ........ attention.py:110-126, 152-181
  * spatial basis ......................... attention.py:201-232
  * query MLP on the (always zero) prev_output  attention.py:184-198, 325-331
  * logits / spatial softmax / readout .... attention.py:235-254, 336-340
  * answer assembly, answer MLP, LSTMCell,
    heads ................................. attention.py:343-368
  * REINFORCE loss (finish_episode) ........ main_mp.py:62-77

Behavioural quirks Q1-Q6 of SURVEY.md §3 are reproduced: zero peepholes
(c*0 terms kept), zero-state LSTMCell every step, constant query from a zero
input, transposed image orientation (X.transpose(1,3)), 4 chunks of the answer
generalised to ``nq`` queries (identical at nq=4).

Parity pinning: tests/test_oracle_golden.py checks this restatement against
fixtures produced by importing the reference itself (tests/golden/gen_golden.py).

``conv_mode='bf16'`` is the bf16-emulated oracle (SURVEY.md §8c G7 analogue):
the attention readout reads h_t rounded to bf16 (``h_store``, as the HIP
bf16 path does since round 4), and
every convolution rounds its GEMM operands to bf16 where the HIP kernels do
(forward: activation and weight; dgrad: output-gradient and weight; wgrad:
activation and output-gradient) and accumulates in fp32, and the ConvLSTM
backward reads the gate activations rounded to fp16, as the HIP bf16 path
stores them (``gate_store``).  What it does not emulate: the order of the fp32
accumulations (MFMA tiles, split-K atomics) and the HIP path's bf16 rounding
of conv1's bordered input image (exact for raw 0..255 pixels) -- so the HIP
bf16 path matches it to ~1e-3, well inside the 2e-2 criterion, not bit for bit.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

__all__ = ["spatial_basis", "unroll", "reinforce_loss", "grid_of", "tensor_params", "vision_cnn", "convlstm_cell",
           "attention_readout"]


def grid_of(H: int, W: int):
    """Spatial grid (h, w) after conv 8/4/1 then conv 4/2/2 (attention.py:155-170)."""
    def out(n, k, s, p):
        return (n + 2 * p - k) // s + 1
    return out(out(H, 8, 4, 1), 4, 2, 2), out(out(W, 8, 4, 1), 4, 2, 2)


def spatial_basis(h: int, w: int, channels: int = 64) -> torch.Tensor:
    """(h, w, channels) cosine basis, attention.py:208-226, same fp32 ops."""
    nb = int(round(math.sqrt(channels)))
    iy = torch.arange(1, h + 1).unsqueeze(1).float().mul(torch.ones(1, w)).mul(math.pi / h)
    ix = torch.ones(h, 1).mul(torch.arange(1, w + 1).unsqueeze(0).float()).mul(math.pi / w)
    freq = torch.arange(1, nb + 1).unsqueeze(0).float()
    cy = torch.cos(iy.unsqueeze(2) * freq)          # (h, w, nb)
    cx = torch.cos(ix.unsqueeze(2) * freq)
    return (cy.unsqueeze(3) * cx.unsqueeze(2)).reshape(h, w, nb * nb)


def tensor_params(params: dict, requires_grad: bool = True, dtype=torch.float32):
    out = {}
    for k, v in params.items():
        t = torch.as_tensor(np.ascontiguousarray(v)).to(dtype).clone()
        t.requires_grad_(requires_grad)
        out[k] = t
    return out


def _bf(t):
    return t.to(torch.bfloat16).to(t.dtype)


class _Bf16Conv(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, stride, pad):
        xr, wr = _bf(x), _bf(w)
        ctx.save_for_backward(xr, wr)
        ctx.conf = (stride, pad, x.shape, w.shape, b is not None)
        return F.conv2d(xr, wr, b, stride=stride, padding=pad)

    @staticmethod
    def backward(ctx, g):
        xr, wr = ctx.saved_tensors
        stride, pad, xs, ws, hasb = ctx.conf
        gr = _bf(g)
        dx = torch.nn.grad.conv2d_input(xs, wr, gr, stride=stride, padding=pad)
        dw = torch.nn.grad.conv2d_weight(xr, ws, gr, stride=stride, padding=pad)
        db = g.sum((0, 2, 3)) if hasb else None
        return dx, dw, db, None, None


def _conv(mode, x, w, b, stride, pad):
    if mode == "bf16":
        return _Bf16Conv.apply(x, w, b, stride, pad)
    return F.conv2d(x, w, b, stride=stride, padding=pad)


def vision_cnn(P, X_t, mode="fp32"):
    """VisionNetwork.vision_cnn on X.transpose(1,3) (attention.py:155-170, 179):
    frames (B,H,W,3) -> (B,64,w,h) in the reference's transposed orientation."""
    x = X_t.transpose(1, 3)                                            # attention.py:179
    y = _conv(mode, x, P["vision.vision_cnn.0.weight"], P["vision.vision_cnn.0.bias"], 4, 1)
    return _conv(mode, y, P["vision.vision_cnn.1.weight"], P["vision.vision_cnn.1.bias"], 2, 2)


class _GateCellF16(torch.autograd.Function):
    """Cell update of attention.py:119-123 (zero peepholes) whose backward reads
    the gate activations rounded to fp16 -- the HIP bf16 path stores them so
    (csrc/epilogues.h store_gates / gate_bwd); the forward and the cell state
    stay fp32, and tanh(c) is recomputed from the fp32 c, as there."""

    @staticmethod
    def forward(ctx, zi, zf, zc, zo, c):
        gi, gf, gc, go = torch.sigmoid(zi), torch.sigmoid(zf), torch.tanh(zc), torch.sigmoid(zo)
        c_new = gf * c + gi * gc
        h_new = go * torch.tanh(c_new)
        r = [g.to(torch.float16).to(g.dtype) for g in (gi, gf, gc, go)]
        ctx.save_for_backward(*r, c, c_new)
        return h_new, c_new

    @staticmethod
    def backward(ctx, dh, dc):
        gi, gf, gc, go, c, c_new = ctx.saved_tensors
        tc = torch.tanh(c_new)
        dcc = dc + dh * go * (1 - tc * tc)
        return (dcc * gc * (1 - gi) * gi, dcc * c * (1 - gf) * gf, dcc * gi * (1 - gc * gc),
                dh * tc * (1 - go) * go, dcc * gf)


def convlstm_cell(P, x, state, mode="fp32", peep=None, gate_store="fp32"):
    """One ConvLSTMCell step (attention.py:110-126) on the reference's NCHW input
    x (B,64,a,b); state (h, c) (B,128,a,b) or None (zeros, :111-115, 142-149).
    Returns (h, c, peep).  gate_store="fp16" (bf16 mode only) emulates the HIP
    bf16 path's fp16 storage of the gate activations for the backward."""
    if state is None:
        B, _, a, b = x.shape
        h = torch.zeros(B, 128, a, b, dtype=x.dtype)
        c = torch.zeros(B, 128, a, b, dtype=x.dtype)
    else:
        h, c = state
    if peep is None:                                                     # Q2: zero, lazily sized
        peep = torch.zeros(1, 128, x.shape[2], x.shape[3], dtype=x.dtype)

    def gate(g):
        L = "vision.vision_lstm."
        return (_conv(mode, x, P[L + f"Wx{g}.weight"], P[L + f"Wx{g}.bias"], 1, 1)
                + _conv(mode, h, P[L + f"Wh{g}.weight"], None, 1, 1))

    if gate_store == "fp16":
        assert not bool(peep.count_nonzero()), "fp16 gate emulation assumes the reference's zero peepholes"
        h_new, c_new = _GateCellF16.apply(gate("i"), gate("f"), gate("c"), gate("o"), c)
        return h_new, c_new, peep
    gi = torch.sigmoid(gate("i") + c * peep)                            # attention.py:119
    gf = torch.sigmoid(gate("f") + c * peep)                            # :120
    c_new = gf * c + gi * torch.tanh(gate("c"))                         # :121
    go = torch.sigmoid(gate("o") + c_new * peep)                        # :122
    h_new = go * torch.tanh(c_new)                                      # :123
    return h_new, c_new, peep


class _RoundBf16(torch.autograd.Function):
    """h_t as the HIP bf16 path hands it to the attention readout: rounded to
    bf16 (it reads the bf16 copy the recurrence keeps for the next step's
    h-conv and the weight gradient, csrc/recur.h), gradient straight through
    (the readout's dO is added to dh of the fp32 h_t, csrc/recur_bwd.h)."""

    @staticmethod
    def forward(ctx, h):
        return _bf(h)

    @staticmethod
    def backward(ctx, g):
        return g


def _vision_step(P, X_t, state, mode, peep, gate_store="fp32"):
    """Encoder + one ConvLSTM step in the reference's transposed orientation."""
    return convlstm_cell(P, vision_cnn(P, X_t, mode), state, mode, peep, gate_store)


def _relu(x, probe):
    return F.relu(x) if probe is None else _ProbedReLU.apply(x, probe, len(probe.pre))


def _query(P, B, nq, hidden=256, prev_output=None, probe=None):
    """QueryNetwork on prev_output (attention.py:184-198,325-331): the zero
    tensor in the reference's reachable path (Q1), h_{t-1} in the stateful core."""
    z = prev_output if prev_output is not None else torch.zeros(B, hidden, dtype=P["query.model.0.weight"].dtype)
    if prev_output is None:
        probe = None          # a constant query: no kink moves
    q = _relu(F.linear(z, P["query.model.0.weight"], P["query.model.0.bias"]), probe)
    q = _relu(F.linear(q, P["query.model.2.weight"], P["query.model.2.bias"]), probe)
    q = F.linear(q, P["query.model.4.weight"], P["query.model.4.bias"])
    return q.reshape(-1, nq, 72)


def attention_readout(O, S, Q, prev_reward=None, prev_action=None):
    """K/V split + spatial basis, logits, spatial_softmax, apply_alpha and the
    answer assembly (attention.py:319-348, 235-254) for one frame batch:
    O (B,h,w,128), S (h,w,64), Q (B,nq,72) -> A (B,h,w,nq), answer (B, 256nq+2)."""
    B, h, w, _ = O.shape
    nq = Q.shape[1]
    K, V = O.split([8, 120], dim=3)                                     # attention.py:319
    Sb = torch.stack([S.to(O.dtype)] * B)
    K, V = torch.cat([K, Sb], dim=3), torch.cat([V, Sb], dim=3)         # :231-232
    A = torch.matmul(K, Q.transpose(2, 1).unsqueeze(1))                  # :336
    A = F.softmax(A.reshape(B, h * w, nq), dim=1).reshape(B, h, w, nq)  # :235-243
    a = torch.matmul(A.reshape(B, h * w, nq).transpose(1, 2),
                     V.reshape(B, h * w, V.shape[3]))                   # :246-254
    if prev_reward is None:
        r = torch.zeros(B, 1, 1, dtype=O.dtype)
    else:
        r = prev_reward.to(O.dtype).reshape(B, 1, 1)
    if prev_action is None:
        act = torch.zeros(B, 1, 1, dtype=O.dtype)
    else:
        act = prev_action.to(O.dtype).reshape(B, 1, 1)
    answer = torch.cat(torch.chunk(a, nq, dim=1) + torch.chunk(Q, nq, dim=1) + (r, act),
                       dim=2).squeeze(1)                                 # :343-348
    return A, answer


class KinkProbe:
    """The answer MLP's ReLU (attention.py:277-282) -- and, in the stateful
    core, the query MLP's two (attention.py:184-198) -- as a probe of the
    gradient's kinks.  The reference's gradient is discontinuous where a
    pre-activation of answer_processor.0 crosses zero: a unit within a few
    1e-6 of zero switches its whole frame's cotangent path on or off under
    perturbations far below bf16's rounding (one such unit moves a T=20, B=3
    ConvLSTM weight gradient by ~2% norm-relative -- measured on this oracle
    by perturbing h_t by 1e-6 before its bf16 rounding).  ``unroll(...,
    kinks=probe)`` records every probed pre-activation (in call order) and
    lets the backward flip one unit's mask (``flip = (call, flat index)``):
    ``near(eps)`` lists the units within eps of zero, so a test can bound the
    gradient over every on/off choice of those units (tests/helpers.py
    kink_envelope).

    ``masks`` (call index -> bool tensor of the pre-activation's shape): run
    those ReLUs with the given on/off pattern instead of ``pre > 0``, forward
    (x * mask) and backward (g * mask) -- the mask-matched oracle: the HIP
    path's own masks (aaa_workspace_region, tests/helpers.py hip_relu_masks)
    put the oracle's gradient on the same side of every kink as the kernels',
    so a bf16 comparison needs no kink allowance.  ``mismatch`` counts, per
    call, the units where the given mask disagrees with the oracle's own sign."""

    def __init__(self, masks=None):
        self.pre = []
        self.flip = None
        self.masks = masks
        self.mismatch = {}
        self.mismatch_pre = {}   # call -> largest |pre-activation| among the disagreeing units
        self.units = {}          # call -> units compared (the denominator of mismatch)

    def near(self, eps, limit=8):
        """(t, flat index, |pre|) of the units with |pre| < eps, nearest first."""
        out = []
        for t, x in enumerate(self.pre):
            a = x.reshape(-1).abs()
            for i in torch.nonzero(a < eps).reshape(-1).tolist():
                out.append((t, i, float(a[i])))
        return sorted(out, key=lambda u: u[2])[:limit]


class _ProbedReLU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, probe, t):
        ctx.probe, ctx.t = probe, t
        probe.pre.append(x.detach().clone())
        given = probe.masks.get(t) if probe.masks is not None else None
        if given is None:
            ctx.save_for_backward(x > 0)
            return x.clamp_min(0)
        given = given.reshape(x.shape).to(torch.bool)
        dis = given != (x > 0)
        probe.mismatch[t] = int(dis.sum())
        probe.units[t] = int(dis.numel())
        probe.mismatch_pre[t] = float(x.detach().abs()[dis].max()) if bool(dis.any()) else 0.0
        ctx.save_for_backward(given)
        return x * given.to(x.dtype)

    @staticmethod
    def backward(ctx, g):
        (mb,) = ctx.saved_tensors
        m = mb.to(g.dtype)
        f = ctx.probe.flip
        if f is not None and f[0] == ctx.t:
            m.view(-1)[f[1]] = 1.0 - m.view(-1)[f[1]]
        return g * m, None, None


def _head(P, O, S, nq, prev_reward, prev_action, core=None, probe=None):
    """Attention readout + answer MLP + LSTMCell + heads (one frame batch).

    core=None: the reference's reachable path, zero-state LSTMCell and a query
    of zeros (Q1).  core=(h, c): the stateful core -- the reference's own
    ``else`` branch (attention.py:356-358), reached when ``agent.prev_hidden``
    holds a tensor: Q = query(h), LSTMCell from (h, c); returns the new (h, c).
    """
    B = O.shape[0]
    Q = _query(P, B, nq, prev_output=None if core is None else core[0], probe=probe)
    A, answer = attention_readout(O, S, Q, prev_reward, prev_action)
    x = _relu(F.linear(answer, P["answer_processor.0.weight"], P["answer_processor.0.bias"]), probe)
    x = F.linear(x, P["answer_processor.2.weight"], P["answer_processor.2.bias"])
    if core is None:
        zeros = torch.zeros(B, P["policy_core.weight_hh"].shape[1], dtype=O.dtype)
        state = (zeros, zeros)                                          # :354-355 (Q1)
    else:
        state = core                                                    # :356-358
    hc, cc = torch._VF.lstm_cell(x, state, P["policy_core.weight_ih"],
                                 P["policy_core.weight_hh"], P["policy_core.bias_ih"],
                                 P["policy_core.bias_hh"])
    logits = F.linear(hc, P["policy_head.0.weight"], P["policy_head.0.bias"])
    values = F.linear(hc, P["values_head.0.weight"], P["values_head.0.bias"])
    if core is not None:
        return logits, values, A, (hc, cc)
    return logits, values, A


def unroll(P: dict, X: torch.Tensor, nq: int = 4, prev_reward=None, prev_action=None,
           state=None, S=None, conv_mode: str = "fp32", return_state: bool = False,
           stateful_core: bool = False, core_state=None, gate_store=None, h_store=None,
           kinks: "KinkProbe | None" = None):
    """T-step unroll from ``reset()``: X is (T, B, H, W, 3) fp32 raw pixels.

    Returns logits (T,B,A), values (T,B,A), attention maps (T,B,h,w,nq)
    [, (h_T, c_T) in the reference's (B,128,w,h) layout].  With
    ``stateful_core`` the policy core carries (prev_output, prev_hidden) --
    the reference with ``agent.prev_hidden`` set to zeros after ``reset()``
    (attention.py:324-331, 356-358); ``core_state`` = (h, c) (B, 256) to
    continue from, and return_state then returns ((h_T, c_T), (core_h, core_c)).
    """
    T, B = X.shape[0], X.shape[1]
    if gate_store is None:   # the HIP path's default: fp16 gate activations on the bf16 path
        gate_store = "fp16" if conv_mode == "bf16" else "fp32"
    if h_store is None:      # the HIP bf16 path's readout reads its bf16 copy of h_t (_RoundBf16)
        h_store = "bf16" if conv_mode == "bf16" else "fp32"
    if S is None:
        S = spatial_basis(*grid_of(X.shape[2], X.shape[3]))
    peep = None
    L, Vv, Am = [], [], []
    core = None
    if stateful_core:
        dt = P["policy_core.weight_hh"].dtype
        core = core_state if core_state is not None else (torch.zeros(B, 256, dtype=dt), torch.zeros(B, 256, dtype=dt))
    for t in range(T):
        hN, cN, peep = _vision_step(P, X[t], state, conv_mode, peep, gate_store)
        state = (hN, cN)
        O = (_RoundBf16.apply(hN) if h_store == "bf16" else hN).transpose(1, 3)   # attention.py:181
        r = None if prev_reward is None else prev_reward[t]
        a = None if prev_action is None else prev_action[t]
        if stateful_core:
            lg, vl, A, core = _head(P, O, S, nq, r, a, core, probe=kinks)
        else:
            lg, vl, A = _head(P, O, S, nq, r, a, probe=kinks)
        L.append(lg), Vv.append(vl), Am.append(A)
    out = (torch.stack(L), torch.stack(Vv), torch.stack(Am))
    if return_state:
        return out + (((state, core) if stateful_core else state),)
    return out


def reinforce_loss(logits: torch.Tensor, actions, rewards, gamma: float = 0.99):
    """finish_episode's loss (main_mp.py:62-77) given per-step logits (T,1,A)."""
    eps = np.finfo(np.float32).eps.item()
    R, returns = 0, []
    for r in list(rewards)[::-1]:
        R = r + gamma * R
        returns.insert(0, R)
    returns = torch.tensor(returns)
    returns = (returns - returns.mean()) / (returns.std() + eps)
    terms = []
    for t, (a, Rt) in enumerate(zip(actions, returns)):
        probs = F.softmax(logits[t], dim=-1)
        lp = torch.distributions.Categorical(probs).log_prob(torch.tensor([int(a)]))
        terms.append(-lp * Rt)
    return torch.cat(terms).sum()


# ---------------------------------------------------------------- actor ----
# Policy.forward's draw (main_mp.py:54-58): softmax -> Categorical -> sample ->
# log_prob.  The HIP sampler (aaa_sample_actions, csrc/loss.hip) replaces
# torch's multinomial stream with a counter-based uniform; this restates that
# generator and the inverse-CDF draw in plain Python/numpy so the device draws
# can be checked action for action.  log_prob follows Categorical(probs):
# probs normalised, then log(clamp(p, eps, 1 - eps)).
_M64 = (1 << 64) - 1


def _mix64(z: int) -> int:
    z = (z + 0x9E3779B97F4A7C15) & _M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
    return z ^ (z >> 31)


def sample_uniform(seed: int, counter: int, row: int) -> float:
    """u in [0, 1) with 24 bits, exactly the kernel's sample_uniform()."""
    x = _mix64(_mix64(seed & _M64) ^ ((counter * 0xD1B54A32D192ED03 + row) & _M64))
    return float(np.float32(x >> 40) * np.float32(1.0 / 16777216.0))


def sample_actions(logits, seed: int, counter: int):
    """Inverse-CDF draw of one action per row of logits (B, A).

    Returns (actions int64 (B,), log_prob float32 (B,), margin (B,)): margin is
    the distance of u*Z from the nearest CDF boundary, relative to Z -- draws
    within fp32 rounding of a boundary may legitimately differ from the kernel.
    """
    l = np.asarray(logits, dtype=np.float32)
    B, A = l.shape
    acts = np.zeros(B, np.int64)
    logp = np.zeros(B, np.float32)
    margin = np.zeros(B, np.float64)
    eps = np.float32(np.finfo(np.float32).eps)
    for b in range(B):
        e = np.exp(l[b] - l[b].max()).astype(np.float32)
        z = np.float32(e.sum(dtype=np.float32))
        cum = np.cumsum(e, dtype=np.float32)
        target = np.float32(sample_uniform(seed, counter, b)) * z
        hit = np.nonzero(cum > target)[0]
        a = int(hit[0]) if hit.size else int(np.nonzero(e > 0)[0][-1])
        acts[b] = a
        pa = np.float32(e[a] / z)
        logp[b] = np.log(np.clip(pa, eps, np.float32(1) - eps))
        margin[b] = float(np.min(np.abs(cum.astype(np.float64) - float(target)))) / float(z)
    return acts, logp, margin
