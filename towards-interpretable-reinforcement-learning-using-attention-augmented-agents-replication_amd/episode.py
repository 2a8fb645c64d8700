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

* each step runs the agent step (its logits drive the action draw at once)
  and keeps only what the BPTT needs to redo it: the step's frames (a
  reference to the caller's tensor, version-checked), prev_reward /
  prev_action, the ConvLSTM state at every ``seg``-th step, and -- the
  episode *store* -- the step's ConvLSTM products (gate activations, c_t, h_t:
  ``B*h*w*768*4`` bytes, 1.66 MB at 210x160, up to a byte budget);
* fp32 agents with the reference's zero-state policy core and B <= 16 record
  on the actor chain (aaa_actor_step: six launches sized for small B, its
  ConvLSTM step writing the gate activations straight into the store, the
  action drawn in the same call); other agents on the learner's T=1 forward
  (aaa_forward), whose products are exported into the store
  (aaa_core_export; fp32 runners);
* every step's autograd node takes the episode's *anchor* -- a scalar output
  of one node whose inputs are the 34 parameters and the episode's initial
  ConvLSTM state -- so autograd runs the anchor's backward only after every
  step node reached by the loss has delivered its cotangents;
* the step nodes only stash (dlogits, dvalues), a log-prob cotangent, and a
  cotangent of the step's output state (h_t, c_t: the ``prev_hidden`` the
  reference keeps live after every step, attention.py:125); the anchor's
  backward then re-runs the episode as multi-step unrolls -- segments of at
  most ``seg`` steps, additionally cut after every step whose state received a
  cotangent -- from checkpointed or stored states, back-propagates each with one
  hand-written BPTT call (T = its length), last segment first, carrying dh/dc
  between segments and adding each cut's state cotangent to the carry, and
  returns the summed parameter grads (and the initial state's grads) in one go.
  Where the store holds a segment's products the re-run imports them
  (aaa_core_import) and runs only the batched vision encoder and tail
  (aaa_forward_phases without CORE); elsewhere it recomputes the recurrence.

The result is the gradient of the same loss through the same op sequence
(the re-run uses the recorded products, or the same kernels as the per-step
forward at this batch, up to summation order).

Memory: the frames, ``2 * B*h*w*128*4 / seg`` bytes of checkpointed state per
step, and the store: ``B*h*w*768*4`` bytes per step up to AAA_EPISODE_STORE_MB
(default 4096 MB: 2,470 steps at 210x160, B = 1), past which the steps are
recomputed.  AAA_EPISODE_STORE=0 keeps no store (and records on aaa_forward).
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
        ctx.set_materialize_grads(False)
        ctx.ep, ctx.t = ep, t
        logits, values, attn, hT, cT, action, logp, jac = ep.forward_step(t, sampler)
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
        self.steps = []                            # (frames (1,B,H,W,3), version, pr, pa)
        h = None if h0 is None else h0.detach().contiguous()
        c = None if c0 is None else c0.detach().contiguous()
        self.ckpt = {0: (h, c)}                    # step -> ConvLSTM state entering it (segment starts)
        self.cur = (h, c)
        self.cot, self.ext = {}, {}
        self.cotp, self.jac = {}, {}               # log-prob cotangents / draw Jacobians (_EpisodeActFn)
        # step block t // STORE_BLOCK -> (gates, c, h) of its steps, up to the byte budget; bf16 runners
        # keep their own element types (fp16 gates, bf16 h), not the channel-quad-major slices of
        # the large-batch frame-resident BPTT (no episode runs at such batches)
        # (not for the channel-quad-major slices of large-batch bf16 geometries: their products
        # stay in the frame-resident layout, core_dtypes() is None, and the backward recomputes)
        store_on = os.environ.get("AAA_EPISODE_STORE", "1") != "0" and runner.core_dtypes() is not None
        self.store = {} if store_on else None
        self._slots = {}
        self.store_budget = int(float(os.environ.get("AAA_EPISODE_STORE_MB", "4096")) * 2**20)
        self.store_bytes = 0
        self.blk = max(1, min(self.seg, STORE_BLOCK))
        self.state_ref = None                      # the prev_hidden tuple this episode last set
        self.anchor = None
        # the recording step: the actor chain (aaa_actor_step) where it applies, else aaa_forward T=1
        self.actor = None
        if store_on and runner.cfg.dtype == N.F32 and runner.B <= 16 and os.environ.get("AAA_EPISODE_ACTOR", "1") != "0":
            from .policy import _actor_chain_fits
            if _actor_chain_fits(runner.B, runner.H, runner.W, runner.nq, runner.A):
                from .runtime import ActorRunner
                cache = agent.__dict__.setdefault("_episode_actors", {})   # one per geometry, kept across episodes
                key = (runner.B, runner.H, runner.W, str(self.device), runner.frames_u8)
                if key not in cache:
                    ar = ActorRunner(runner.B, runner.H, runner.W, runner.nq, runner.A, self.device,
                                     frames_u8=runner.frames_u8)
                    cache[key] = (ar, ar.new_workspace())
                self.actor, self.ws = cache[key]
        if self.actor is not None:   # one aaa_actor_io for the episode: the fixed pointers set once
            import ctypes
            self._io = N.ActorIO()
            self._io.params, self._io.packed = flat.data_ptr(), packed.data_ptr()
            self._io.basis, self._io.workspace = basis.data_ptr(), self.ws.data_ptr()
            self._io_ref, self._cfg_ref = ctypes.byref(self._io), ctypes.byref(self.actor.cfg)
            self._lib = N.load()
        if self.actor is not None and h is None:   # the actor chain reads a state tensor: zeros
            shp = runner.state_shape()
            self.hbuf, self.cbuf = torch.zeros(shp, device=self.device), torch.zeros(shp, device=self.device)
        elif self.actor is None:
            self.ws = runner.new_workspace()      # per-step scratch, reused: nothing of it is kept

    # -- forward --------------------------------------------------------------
    def record(self, X, pr, pa):
        self.steps.append((X, X._version, pr, pa))
        return len(self.steps) - 1

    def _slot(self, t):
        """(gates, c, h) store rows of step t ((1, M, 512), (1, M, 128) x 2) and its c / h rows as
        state-shaped views, or None past the budget.  A block's row views are made once, with the block."""
        if self.store is None:
            return None
        k, i = divmod(t, self.blk)
        views = self._slots.get(k)
        if views is None:
            shapes, dts = self.runner.core_shapes(self.blk), self.runner.core_dtypes()
            nbytes = sum(a * b * c * torch.empty((), dtype=dt).element_size() for (a, b, c), dt in zip(shapes, dts))
            if self.store_bytes + nbytes > self.store_budget:
                return None
            self.store[k] = g, c, h = tuple(torch.empty(s, dtype=dt, device=self.device) for s, dt in zip(shapes, dts))
            self.store_bytes += nbytes
            shp = self.runner.state_shape()
            self._slots[k] = views = [(g[j:j + 1], c[j:j + 1], h[j:j + 1], c[j].view(shp), h[j].view(shp))
                                      for j in range(self.blk)]
        return views[i]

    def forward_step(self, t, sampler=None):
        """Run step t: (logits, values, attn, hT, cT) -- plus (action, logp, jac)
        with a ``sampler`` (the draw of Policy.act)."""
        X, _, pr, pa = self.steps[t]
        r = self.runner
        slot = self._slot(t)
        if self.actor is not None:
            if getattr(r, "relu_trace", None) is not None:
                raise RuntimeError("Agent.relu_trace: the actor-chain recording keeps no learner workspace; "
                                   "set AAA_EPISODE_ACTOR=0 to trace an episode")
            B, A, dev = r.B, r.A, self.device
            logits = torch.empty(1, B, A, device=dev)
            values = torch.empty(1, B, A, device=dev)
            attn = torch.empty(1, B, r.h, r.w, r.nq, device=dev)
            h, c = self.cur
            if h is None:   # zero state entering the episode
                h, c = self.hbuf, self.cbuf
            if slot is not None:   # h_t, c_t straight into the store rows (written by the kernels, so no
                # in-place op on the store's blocks: these views are handed out as prev_hidden)
                cT, hT = slot[3], slot[4]
            else:
                shp = r.state_shape()
                hT, cT = torch.empty(shp, device=dev), torch.empty(shp, device=dev)
            # aaa_actor_step with the episode's io (the recorded frames, states and store rows are
            # contiguous tensors of the runner's geometry by construction: ActorRunner.step's checks
            # are not repeated per step)
            io = self._io
            io.frames, io.h, io.c, io.h_out, io.c_out = X.data_ptr(), h.data_ptr(), c.data_ptr(), hT.data_ptr(), \
                cT.data_ptr()
            io.logits, io.values, io.attn = logits.data_ptr(), values.data_ptr(), attn.data_ptr()
            io.gates = slot[0].data_ptr() if slot is not None else None
            prf = None if pr is None else pr.reshape(-1).to(dev, torch.float32).contiguous()
            paf = None if pa is None else pa.reshape(-1).to(dev, torch.float32).contiguous()
            io.prev_reward = None if prf is None else prf.data_ptr()
            io.prev_action = None if paf is None else paf.data_ptr()
            draw = ()
            if sampler is not None:
                draw = (torch.empty(B, dtype=torch.int32, device=dev), torch.empty(B, device=dev),
                        torch.empty(B, A, device=dev))
                io.seed = sampler.seed & (2**64 - 1)
                io.counter = sampler.counter.data_ptr()
                io.actions, io.logp, io.dlogp_dlogits = draw[0].data_ptr(), draw[1].data_ptr(), draw[2].data_ptr()
            else:
                io.seed, io.counter, io.actions, io.logp, io.dlogp_dlogits = 0, None, None, None, None
            N.check(self._lib.aaa_actor_step(self._cfg_ref, self._io_ref, N.stream_ptr(dev)), "actor_step")
            self.cur = (hT, cT)
            if (t + 1) % self.seg == 0:
                self.ckpt[t + 1] = (hT, cT)
            return (logits, values, attn, hT, cT) + draw
        h, c = self.cur
        logits, values, attn, hT, cT = r.forward(self.flat, self.packed, self.basis, X, self.ws, pr, pa, h, c,
                                                 want_attn=True, want_state=True)
        if getattr(r, "relu_trace", None) is not None:   # inspection hook (Agent.relu_trace)
            r.relu_trace.append(r.relu_masks(self.ws))
        self.cur = (hT, cT)
        if (t + 1) % self.seg == 0:
            self.ckpt[t + 1] = (hT, cT)
        if slot is not None:
            r.core_export(self.ws, 0, 1, *slot[:3])
        if sampler is not None:
            from .policy import _sample_raw
            return (logits, values, attn, hT, cT) + _sample_raw(logits[0], sampler.seed, sampler.counter)
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

    def _stored(self, t0, t1):
        """Whether the store holds every step of [t0, t1)."""
        return self.store is not None and all((t // self.blk) in self.store for t in range(t0, t1))

    def _state_entering(self, b):
        """(h, c) entering step b: a checkpoint, the store's h_{b-1} / c_{b-1}, or a
        forward re-run of the steps since the last checkpoint before b."""
        if b in self.ckpt:
            return self.ckpt[b]
        r = self.runner
        shp = r.state_shape()
        if self._stored(b - 1, b):
            g, c, h = self.store[(b - 1) // self.blk]
            i = (b - 1) % self.blk
            return h[i].view(shp).float(), c[i].view(shp)
        a = max(k for k in self.ckpt if k < b)
        h0, c0 = self.ckpt[a]
        ru = self.agent._runner(r.B, b - a, r.H, r.W, self.device, False, r.frames_u8)
        ru.relu_trace = None
        frames = torch.cat([self.steps[t][0] for t in range(a, b)])
        pr = _stack([self.steps[t][2] for t in range(a, b)], (1, r.B), self.device)
        pa = _stack([self.steps[t][3] for t in range(a, b)], (1, r.B), self.device)
        _, _, _, hT, cT = ru.forward(self.flat, self.packed, self.basis, frames, ru.new_workspace(), pr, pa, h0, c0,
                                     want_attn=False, want_state=True)
        return hT, cT

    def backward_all(self, want_state: bool):
        """Every recorded step's cotangents -> (flat param grads, dh0, dc0)."""
        n = len(self.steps)
        r = self.runner
        for t, (X, ver, pr, pa) in enumerate(self.steps):
            if X._version != ver:
                raise RuntimeError(f"aaa: the frames of episode step {t} were modified in place after the forward; "
                                   f"the fused episode backward needs them unchanged (as autograd would)")
        total = torch.zeros(r.n_params, device=self.device)
        # segments: every seg-th step, and a cut after each step whose output state has a cotangent
        cuts = sorted(set(range(0, n, self.seg)) | {t + 1 for t in self.ext if t + 1 < n})
        bounds = list(zip(cuts, cuts[1:] + [n]))
        A, B = r.A, r.B
        dh = dc = None
        for t0, t1 in reversed(bounds):
            if (t1 - 1) in self.ext:   # the cotangent of the state leaving this segment joins the carry
                eh, ec = self.ext[t1 - 1]
                dh, dc = _add(dh, eh), _add(dc, ec)
            live = any(t in self.cot or t in self.cotp for t in range(t0, t1)) or dh is not None or dc is not None
            need_state = t0 > 0 or want_state
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
                zj = torch.zeros(B, A, device=self.device)   # steps recorded by plain forward calls: no draw
                J = torch.stack([self.jac.get(t, zj) for t in range(t0, t1)])
                G = _stack([self.cotp.get(t) for t in range(t0, t1)], (1, B), self.device, zero=True)
                dl = torch.addcmul(dl, J, G.unsqueeze(-1))
            h0, c0 = self._state_entering(t0)
            ws = ru.new_workspace()
            if self._stored(t0, t1):   # the recorded products: no recurrence re-run
                t = t0
                while t < t1:
                    k, i = divmod(t, self.blk)
                    nb = min(self.blk - i, t1 - t)
                    sg, sc, sh = self.store[k]
                    ru.core_import(ws, t - t0, nb, sg[i:i + nb], sc[i:i + nb], sh[i:i + nb])
                    t += nb
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
