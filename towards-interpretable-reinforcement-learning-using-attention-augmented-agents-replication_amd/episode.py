"""Fused episode backward for the reference's per-step call pattern.

main_mp.py calls ``policy(observation)`` -> ``agent(state)`` once per
environment step (main_mp.py:49-59, :111) and, when the episode ends,
``policy_loss.backward()`` once through every step's graph (:76-77).  Run
naively that is T separate T=1 backward calls, each with its own saved T=1
workspace (12.6 MB per step at 210x160): the backward is launch- and
latency-bound (0.5 ms per step) and a 10,000-step episode (:151) would hold
126 GB of autograd graph.

Here the per-step ``Agent.forward`` calls of one episode record into an
``Episode``:

* each step runs the T=1 forward (its logits drive the action draw at once)
  on one reused workspace, and keeps only what the BPTT needs to redo it:
  the step's frames (a reference to the caller's tensor, version-checked),
  prev_reward / prev_action, and the ConvLSTM state at every ``seg``-th step;
* every step's autograd node takes the episode's *anchor* -- a scalar output
  of one node whose inputs are the 34 parameters and the episode's initial
  ConvLSTM state -- so autograd runs the anchor's backward only after every
  step node reached by the loss has delivered its cotangents;
* the step nodes only stash (dlogits, dvalues) (and a state cotangent on the
  last step, when a later call continued from it); the anchor's backward then
  re-runs the episode as multi-step unrolls of ``seg`` steps from the
  checkpointed states and back-propagates each with one hand-written BPTT
  call (``aaa_forward`` / ``aaa_backward``, T = seg), last segment first,
  carrying dh/dc between segments, and returns the summed parameter grads
  (and the initial state's grads) in one go.

The result is the gradient of the same loss through the same op sequence
(the recomputed forward runs the same kernels as the per-step one at this
batch, up to summation order).  The memory kept per step is the frames plus
``2 * B*h*w*128*4 / seg`` bytes of state.

fp32 agents also keep each step's ConvLSTM products (gate activations, c_t,
h_t: ``B*h*w*768*4`` bytes, 1.66 MB at 210x160) exported from the per-step
workspace (``aaa_core_export``); the segment's re-run then imports them and
skips the recurrence (``aaa_forward_phases`` without CORE) -- the 64
sequential step launches that dominated the recomputation -- and runs only
the batched vision encoder and tail.  AAA_EPISODE_STORE=0 recomputes instead.
"""
from __future__ import annotations

import os

import torch

from . import _native as N

__all__ = ["Episode", "EPISODE_SEGMENT"]

# Steps per recomputed segment (memory of one segment's workspace is live
# only inside the anchor's backward; the state is checkpointed every EPISODE_SEGMENT steps).
EPISODE_SEGMENT = 64
# Steps per block of the kept ConvLSTM products (allocated as the episode
# grows; one aaa_core_import per block in the backward).
STORE_BLOCK = 16


class _EpisodeAnchorFn(torch.autograd.Function):
    """Scalar node whose backward is the whole episode's BPTT."""

    @staticmethod
    def forward(ctx, ep, h0, c0, *params):
        ctx.ep = ep
        ctx.shapes = [p.shape for p in params]
        ctx.has_state = (h0 is not None, c0 is not None)
        return torch.zeros((), device=ep.device)

    @staticmethod
    def backward(ctx, _g):
        need = ctx.needs_input_grad
        want_state = bool((need[1] and ctx.has_state[0]) or (need[2] and ctx.has_state[1]))
        grads, dh0, dc0 = ctx.ep.backward_all(want_state)
        views = [g.view(s) for g, s in zip(grads.split(ctx.ep.runner.sizes), ctx.shapes)]
        return (None, dh0 if need[1] else None, dc0 if need[2] else None, *views)


class _EpisodeStepFn(torch.autograd.Function):
    """One per-step forward of an episode; its backward only stashes cotangents."""

    @staticmethod
    def forward(ctx, ep, t, anchor):
        ctx.set_materialize_grads(False)
        ctx.ep, ctx.t = ep, t
        logits, values, attn, hT, cT = ep.forward_step(t)
        ctx.mark_non_differentiable(attn)
        return logits, values, attn, hT, cT

    @staticmethod
    def backward(ctx, dl, dv, _dattn, dh, dc):
        ctx.ep.stash(ctx.t, dl, dv, dh, dc)
        # no cotangent for the anchor: the edge alone orders its backward after
        # this node (a zeros() here cost a fill + an accumulate launch per step)
        return None, None, None


class _EpisodeActFn(torch.autograd.Function):
    """_EpisodeStepFn plus Policy.act's draw (policy.py): one node per step
    instead of two.  The log-prob's cotangent is stashed with the draw's
    Jacobian and folded into dlogits per segment in one batched product
    (backward_all), instead of one sampler backward launch per step."""

    @staticmethod
    def forward(ctx, ep, t, anchor, sampler):
        from .policy import _sample_raw
        ctx.set_materialize_grads(False)
        ctx.ep, ctx.t = ep, t
        logits, values, attn, hT, cT = ep.forward_step(t)
        action, logp, jac = _sample_raw(logits[0], sampler.seed, sampler.counter)
        ep.jac[t] = jac
        ctx.mark_non_differentiable(attn, action)
        return logits, values, attn, hT, cT, action, logp

    @staticmethod
    def backward(ctx, dl, dv, _dattn, dh, dc, _daction, dlogp):
        ctx.ep.stash(ctx.t, dl, dv, dh, dc, dlogp)
        return None, None, None, None


class Episode:
    """The per-step calls of one episode (from reset(), a carried state or a
    parameter change) of one Agent geometry and parameter version."""

    def __init__(self, agent, runner, flat, packed, key, basis, h0, c0, seg: int | None = None):
        self.agent, self.runner, self.flat, self.packed, self.key, self.basis = agent, runner, flat, packed, key, basis
        self.device = runner.device
        self.seg = max(1, int(EPISODE_SEGMENT if seg is None else seg))
        self.ws = runner.new_workspace()          # per-step scratch, reused: nothing of it is kept
        self.steps = []                            # (frames (1,B,H,W,3), version, pr, pa)
        h = None if h0 is None else h0.detach().contiguous()
        c = None if c0 is None else c0.detach().contiguous()
        self.ckpt = {0: (h, c)}                    # segment start -> ConvLSTM state entering it
        self.cur = (h, c)
        self.cot, self.ext = {}, {}
        self.cotp, self.jac = {}, {}               # log-prob cotangents / draw Jacobians (_EpisodeActFn)
        # step block t // STORE_BLOCK -> (gates, c, h) of its steps (fp32: aaa_core_export), or None (recompute)
        self.store = {} if (runner.cfg.dtype == N.F32 and os.environ.get("AAA_EPISODE_STORE", "1") != "0") else None
        self.blk = max(1, min(self.seg, STORE_BLOCK))
        while self.seg % self.blk:   # blocks never straddle a segment
            self.blk -= 1
        self.state_ref = None                      # the prev_hidden tuple this episode last set
        self.anchor = None

    # -- forward --------------------------------------------------------------
    def record(self, X, pr, pa):
        self.steps.append((X, X._version, pr, pa))
        return len(self.steps) - 1

    def forward_step(self, t):
        X, _, pr, pa = self.steps[t]
        h, c = self.cur
        r = self.runner
        logits, values, attn, hT, cT = r.forward(self.flat, self.packed, self.basis, X, self.ws, pr, pa, h, c,
                                                 want_attn=True, want_state=True)
        if getattr(r, "relu_trace", None) is not None:   # inspection hook (Agent.relu_trace)
            r.relu_trace.append(r.relu_masks(self.ws))
        self.cur = (hT, cT)
        if (t + 1) % self.seg == 0:
            self.ckpt[t + 1] = (hT, cT)
        if self.store is not None:
            k, i = divmod(t, self.blk)
            if k not in self.store:
                self.store[k] = tuple(torch.empty(s, device=self.device) for s in r.core_shapes(self.blk))
            g, c, h = self.store[k]
            r.core_export(self.ws, 0, 1, g[i:i + 1], c[i:i + 1], h[i:i + 1])
        return logits, values, attn, hT, cT

    # -- backward -------------------------------------------------------------
    def stash(self, t, dl, dv, dh, dc, dlogp=None):
        if dlogp is not None:
            self.cotp[t] = _add(self.cotp.get(t), dlogp)
        if dl is not None or dv is not None:
            pl, pv = self.cot.get(t, (None, None))
            self.cot[t] = (_add(pl, dl), _add(pv, dv))
        if dh is not None or dc is not None:
            ph, pc = self.ext.get(t, (None, None))
            self.ext[t] = (_add(ph, dh), _add(pc, dc))

    def backward_all(self, want_state: bool):
        """Every recorded step's cotangents -> (flat param grads, dh0, dc0)."""
        n = len(self.steps)
        r = self.runner
        for t, (X, ver, pr, pa) in enumerate(self.steps):
            if X._version != ver:
                raise RuntimeError(f"aaa: the frames of episode step {t} were modified in place after the forward; "
                                   f"the fused episode backward needs them unchanged (as autograd would)")
        bad = [t for t in self.ext if t != n - 1]
        if bad:
            raise NotImplementedError(f"aaa: a gradient reached the ConvLSTM state of episode step {bad[0]} (not the "
                                      f"last); the fused episode backward takes state cotangents on the last step "
                                      f"only -- set agent.fuse_episode_backward = False for this pattern")
        total = torch.zeros(r.n_params, device=self.device)
        dh, dc = self.ext.get(n - 1, (None, None))
        starts = list(range(0, n, self.seg))
        A, B = r.A, r.B
        for k, t0 in reversed(list(enumerate(starts))):
            t1 = min(n, t0 + self.seg)
            live = any(t in self.cot or t in self.cotp for t in range(t0, t1)) or dh is not None or dc is not None
            need_state = k > 0 or want_state
            if not live:                  # no cotangent reaches this segment or anything before it through it
                dh = dc = None
                continue
            L = t1 - t0
            ru = self.agent._runner(B, L, r.H, r.W, self.device, False, r.frames_u8)
            ru.relu_trace = None             # the re-run is not a forward call of the caller's
            assert ru.pk_bytes == r.pk_bytes   # packed layouts do not depend on B or T
            frames = torch.cat([self.steps[t][0] for t in range(t0, t1)]) if L > 1 else self.steps[t0][0]
            pr = _stack([self.steps[t][2] for t in range(t0, t1)], (1, B), self.device)
            pa = _stack([self.steps[t][3] for t in range(t0, t1)], (1, B), self.device)
            dl = _stack([self.cot.get(t, (None, None))[0] for t in range(t0, t1)], (1, B, A), self.device, zero=True)
            dv = _stack([self.cot.get(t, (None, None))[1] for t in range(t0, t1)], (1, B, A), self.device, zero=True)
            if any(t in self.cotp for t in range(t0, t1)):   # dlogits += jac * dlogp, all steps at once
                J = torch.stack([self.jac[t] for t in range(t0, t1)])
                G = _stack([self.cotp.get(t) for t in range(t0, t1)], (1, B), self.device, zero=True)
                dl = torch.addcmul(dl, J, G.unsqueeze(-1))
            h0, c0 = self.ckpt[t0]
            ws = ru.new_workspace()
            if self.store is not None:   # the recorded products: no recurrence re-run
                for b0 in range(t0, t1, self.blk):
                    nb = min(self.blk, t1 - b0)
                    sg, sc, sh = self.store[b0 // self.blk]
                    ru.core_import(ws, b0 - t0, nb, sg[:nb], sc[:nb], sh[:nb])
                ru.forward(self.flat, self.packed, self.basis, frames, ws, pr, pa, h0, c0, want_attn=False,
                           phases=N.FWD_VISION | N.FWD_TAIL)
            else:
                ru.forward(self.flat, self.packed, self.basis, frames, ws, pr, pa, h0, c0, want_attn=False)
            g, dh, dc = ru.backward(self.flat, self.packed, self.basis, frames, ws, dl, dv, dh, dc,
                                    want_state_grads=need_state)
            total += g
            del ws
        self.cot.clear()
        self.ext.clear()
        self.cotp.clear()
        return total, dh, dc


def _add(a, b):
    if a is None:
        return b
    if b is None:
        return a
    return a + b


def _stack(items, shape, device, zero=False):
    """Concatenate per-step tensors of ``shape`` (leading dim 1) into
    (L, *shape[1:]); None entries become zeros, and all-None gives None
    (zeros with ``zero``)."""
    if all(x is None for x in items):
        return torch.zeros((len(items), *shape[1:]), device=device) if zero else None
    n = 1
    for d in shape:
        n *= d
    d0 = items[0].dim() if items[0] is not None else -1
    if all(x is not None and x.numel() == n and x.dtype == torch.float32 and x.dim() == d0 for x in items):
        return torch.cat(items).reshape((len(items), *shape[1:]))   # one launch, no per-item ops
    out = [torch.zeros(shape, device=device) if x is None else x.reshape(shape).float() for x in items]
    return torch.cat(out) if len(out) > 1 else out[0]
