"""Actor path on the device: the reference's ``Policy``.

``Policy`` mirrors main_mp.py:40-59 -- same constructor, attributes
(``agent``, ``saved_log_probs``, ``rewards``) and ``forward(observation, ts=0)
-> int`` -- so ``train``/``finish_episode`` (main_mp.py:62-80, 95-150) and
test_model.py:42-73 run unchanged with it.  What changes underneath:

* the observation goes to the GPU as uint8 (1/4 of the float bytes the
  reference copies at main_mp.py:53) and is cast inside the kernel that lays
  the frames out for conv1 (AAA_FLAG_FRAMES_U8);
* the agent step is the HIP forward (``Agent.forward``, T=1), whose packed
  weights are cached between parameter updates (``Agent._packed_params``);
* softmax, the Categorical draw and its log-prob are one kernel
  (``aaa_sample_actions``, csrc/loss.hip) with a device-side draw counter, so
  ``act()`` returns the action as a device tensor without a host sync; only
  ``forward`` calls ``.item()``, as the reference does at main_mp.py:59.

The saved log-probs are differentiable through the per-step agent graph, so
``torch.cat(policy.saved_log_probs)`` in finish_episode back-propagates into
the hand-written BPTT exactly like the reference's Categorical objects.
Sampling uses its own counter-based generator (not torch's multinomial
stream): the same distribution, different draws.
"""
from __future__ import annotations

import numpy as np
import torch
from torch import nn

from . import _native as N

__all__ = ["Policy", "sample_actions", "ActionSampler", "GraphActor"]


def _sample_raw(logits, seed, counter):
    """aaa_sample_actions on (B, A) fp32 logits -> (actions int32 (B,), log_prob (B,),
    jac (B, A) = d log_prob / d logits); no autograd."""
    B, A = logits.shape
    lg = logits.detach().contiguous()
    actions = torch.empty(B, dtype=torch.int32, device=lg.device)
    logp = torch.empty(B, dtype=torch.float32, device=lg.device)
    jac = torch.empty(B, A, dtype=torch.float32, device=lg.device)
    N.check(N.load().aaa_sample_actions(B, A, lg.data_ptr(), int(seed) & (2**64 - 1),
                                        None if counter is None else counter.data_ptr(),
                                        actions.data_ptr(), logp.data_ptr(), jac.data_ptr(),
                                        N.stream_ptr(lg.device)), "sample_actions")
    return actions, logp, jac


class _SampleFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, seed, counter):
        actions, logp, jac = _sample_raw(logits, seed, counter)
        ctx.save_for_backward(jac)
        ctx.mark_non_differentiable(actions)
        return actions, logp

    @staticmethod
    def backward(ctx, _g_actions, g_logp):
        (jac,) = ctx.saved_tensors
        return jac * g_logp.unsqueeze(1), None, None


def sample_actions(logits: torch.Tensor, seed: int = 0, counter: torch.Tensor | None = None):
    """Draw one action per row of ``logits`` (B, A) from softmax(logits).

    Returns ``(actions int32 (B,), log_prob (B,))``; ``log_prob`` is
    differentiable w.r.t. ``logits`` (d/dl_k = 1[k = a] - p_k).  ``counter``
    is a device int64 scalar tensor advanced by one per call (None: draw 0).
    """
    if logits.dim() != 2:
        raise ValueError(f"logits must be (B, A), got {tuple(logits.shape)}")
    if not logits.is_cuda or logits.dtype != torch.float32:
        raise RuntimeError("sample_actions: logits must be fp32 on the gfx950 device (there is no CPU fallback)")
    if counter is not None and (counter.dtype != torch.int64 or counter.numel() != 1 or
                                counter.device != logits.device):
        raise ValueError("counter must be a one-element int64 tensor on the logits' device")
    return _SampleFn.apply(logits, seed, counter)


class ActionSampler:
    """A seeded draw stream on one device: ``sampler(logits) -> (actions, log_prob)``."""

    def __init__(self, seed: int = 0, device=None):
        self.seed = int(seed)
        self.counter = torch.zeros(1, dtype=torch.int64, device=device if device is not None else "cuda")

    def __call__(self, logits):
        if self.counter.device != logits.device:
            self.counter = self.counter.to(logits.device)
        return sample_actions(logits, self.seed, self.counter)


class Policy(nn.Module):
    """main_mp.py:40-59 on the gfx950 path (see the module docstring)."""

    def __init__(self, agent, seed: int | None = None):
        super().__init__()
        self.agent = agent
        self.saved_log_probs = []
        self.rewards = []
        if seed is None:   # follow torch.manual_seed(config.seed + rank) (main_mp.py:87) like the reference's draws
            seed = int(torch.initial_seed())
        self._sampler = None
        self._seed = seed
        self._frames = []      # ring of (pinned uint8 staging buffer, copy-done event)
        self._slot = 0

    def _device(self):
        # the agent's cached parameter list as last validated (the device of its first
        # parameter: .to() moves parameters in place), without re-validating it -- the
        # step's _episode_params does that once per step
        c = getattr(self.agent, "__dict__", {}).get("_plist")
        if c is not None and c[3]:
            return c[3][0].device
        pl = getattr(self.agent, "_param_list", None)
        return pl()[0].device if pl is not None else next(self.agent.parameters()).device

    def _upload(self, observation):
        dev = self._device()
        if isinstance(observation, torch.Tensor):
            x = observation.to(dev, non_blocking=True)
        else:
            obs = np.ascontiguousarray(observation)
            src = torch.from_numpy(obs)
            if obs.dtype == np.uint8:   # stage through pinned memory: async H2D of 1 B/pixel
                if not self._frames or self._frames[0][0].shape != src.shape:
                    self._frames = [(torch.empty(src.shape, dtype=torch.uint8, pin_memory=True),
                                     torch.cuda.Event()) for _ in range(4)]
                buf, done = self._frames[self._slot]
                self._slot = (self._slot + 1) % len(self._frames)
                done.synchronize()      # the copy that last read this buffer (4 steps ago) has finished
                buf.copy_(src)
                x = buf.to(dev, non_blocking=True)
                done.record(torch.cuda.current_stream(dev))
                return x.unsqueeze(0)           # uint8: cast inside the frame-layout kernel
            x = src.to(dev)
        return (x if x.dtype == torch.uint8 else x.float()).unsqueeze(0)

    def act(self, observation, ts: int = 0):
        """One step without a host sync: returns (action int32 (1,), log_prob (1,)) on the device."""
        state = self._upload(observation)
        dev = state.device
        if self._sampler is None or self._sampler.counter.device != dev:
            self._sampler = ActionSampler(self._seed, dev)
        act_episode = getattr(self.agent, "act_episode", None)
        out = act_episode(state, self._sampler, ts=ts) if act_episode is not None else None
        if out is not None:   # the step and its draw as ONE episode node (episode.py _EpisodeActFn)
            action, logp = out
        else:
            logits, _ = self.agent(state, ts=ts)
            action, logp = self._sampler(logits)
        self.saved_log_probs.append(logp)
        return action, logp

    def forward(self, observation, ts: int = 0):
        """Sample an action from the agent's output distribution (main_mp.py:48-59)."""
        action, _ = self.act(observation, ts)
        return int(action.item())


def _actor_chain_fits(B, H, W, nq, A) -> bool:
    """Whether aaa_actor_step accepts this geometry: its layout query returns 0
    bytes (AAA_E_ARG) for what it refuses, e.g. a grid whose readout exceeds
    the kernel's LDS; no device call."""
    import ctypes
    cfg = N.Cfg(B, 1, H, W, nq, A, N.F32, N.FLAG_FRAMES_U8)
    return N.load().aaa_actor_workspace_bytes(ctypes.byref(cfg)) > 0


class GraphActor:
    """One B-row environment step of the agent + action draw, captured once as
    a HIP graph and replayed per step (inference: test_model.py rollouts, or
    the acting half of an actor/learner split whose learner re-runs the
    episode with ``Agent.unroll`` + ``reinforce_loss``).

    ``step(observation)`` -> action int32 (B,) device tensor (the draw of
    Policy.forward, main_mp.py:54-57), with ``logits``, ``values``,
    ``log_prob`` and ``attention`` left in static device buffers.  The
    ConvLSTM state carries between steps inside the graph (``reset()`` zeroes
    it, attention.py:293-296).  Weights are re-packed into the graph's own
    buffers whenever a parameter of ``agent`` changed (storage or in-place
    version), so optimizer steps between episodes are picked up.

    ``chain`` selects the step: the actor chain (``aaa_actor_step``: six
    launches sized for small B; fp32 agents with the reference's zero-state
    policy core, B <= 16) or the learner's T=1 forward (``aaa_forward`` +
    ``aaa_sample_actions``); None picks the chain whenever it applies.
    """

    def __init__(self, agent, H: int, W: int, B: int = 1, seed: int = 0, chain: bool | None = None):
        from .runtime import ActorRunner, UnrollRunner
        self.agent = agent
        dev = next(agent.parameters()).device
        if dev.type != "cuda":
            raise RuntimeError("GraphActor needs the agent on the gfx950 device (there is no CPU fallback)")
        self.device, self.B, self.H, self.W = dev, B, H, W
        eligible = agent.conv_dtype == "fp32" and not getattr(agent, "stateful_core", False) and B <= 16
        if chain and not eligible:
            raise ValueError("the actor chain needs an fp32 agent with the zero-state policy core and B <= 16")
        self.chain = eligible if chain is None else bool(chain)
        if self.chain and chain is None and not _actor_chain_fits(B, H, W, agent.num_queries, agent.num_actions):
            self.chain = False   # the geometry the chain refuses (its readout LDS): the learner's T=1 forward
        if self.chain:   # any failure here (asked for, or a real HIP error) propagates
            r = ActorRunner(B, H, W, agent.num_queries, agent.num_actions, dev, frames_u8=True)
        if self.chain:
            self.runner = r
            self._ws = r.new_workspace()
            A = agent.num_actions
            self._logits = torch.empty(B, A, device=dev)
            self._values = torch.empty(B, A, device=dev)
            self._attn = torch.empty(B, r.h, r.w, agent.num_queries, device=dev)
            self._actions = torch.empty(B, dtype=torch.int32, device=dev)
            self._logp = torch.empty(B, device=dev)
        else:
            r = UnrollRunner(B, 1, H, W, agent.num_queries, agent.num_actions, agent.conv_dtype, dev,
                             frames_u8=True)
            self.runner = r
        self.S = agent._basis_for(r.h, r.w, H, W, dev)
        self.params = list(agent.parameters())
        self.flat = torch.empty(r.n_params, device=dev)
        self.packed = r.new_packed()
        self._key = None
        self.frame_u8 = torch.zeros(1, B, H, W, 3, dtype=torch.uint8, device=dev)
        self.h = torch.zeros(r.state_shape(), device=dev)
        self.c = torch.zeros(r.state_shape(), device=dev)
        self.sampler = ActionSampler(seed, dev)
        self._host = [(torch.empty(B, H, W, 3, dtype=torch.uint8, pin_memory=True), torch.cuda.Event())
                      for _ in range(4)]
        self._slot = 0
        self._refresh()
        stream = torch.cuda.Stream(dev)
        stream.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(stream), torch.no_grad():
            for _ in range(2):      # warm-up outside the capture (lazy library init, allocator)
                self._body()
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph, stream=stream):
                self._outs = self._body()
        torch.cuda.current_stream(dev).wait_stream(stream)
        self.sampler.counter.zero_()   # the warm-up draws do not count: step k uses draw index k
        self.reset()

    def _body(self):
        r = self.runner
        if self.chain:
            s = self.sampler
            r.step(self.flat, self.packed, self.S, self.frame_u8, self._ws, self.h, self.c, self._logits,
                   self._values, attn=self._attn, seed=s.seed, counter=s.counter, actions=self._actions,
                   logp=self._logp)
            return self._actions, self._logp, self._logits, self._values, self._attn
        X = self.frame_u8                  # uint8, cast in-kernel (AAA_FLAG_FRAMES_U8)
        ws = r.new_workspace()
        logits, values, attn, hT, cT = r.forward(self.flat, self.packed, self.S, X, ws, h0=self.h, c0=self.c,
                                                 want_attn=True, want_state=True)
        action, logp = self.sampler(logits[0])
        self.h.copy_(hT)
        self.c.copy_(cT)
        return action, logp, logits[0], values[0], attn[0]

    def _refresh(self):
        key = tuple((p.data_ptr(), p._version) for p in self.params)
        if key != self._key:
            with torch.no_grad():
                torch.cat([p.detach().reshape(-1) for p in self.params], out=self.flat)
                self.runner.pack(self.flat, self.packed)
            self._key = key

    def reset(self):
        self.h.zero_()
        self.c.zero_()

    @property
    def logits(self):
        return self._outs[2]

    @property
    def values(self):
        return self._outs[3]

    @property
    def log_prob(self):
        return self._outs[1]

    @property
    def attention(self):
        return self._outs[4]

    def step(self, observation):
        """observation: uint8 (H, W, 3) / (B, H, W, 3) numpy array or tensor."""
        self._refresh()
        if isinstance(observation, torch.Tensor) and observation.is_cuda:
            self.frame_u8.view(self.B, self.H, self.W, 3).copy_(observation.reshape(self.B, self.H, self.W, 3))
        else:
            src = torch.as_tensor(np.ascontiguousarray(observation)).reshape(self.B, self.H, self.W, 3)
            buf, done = self._host[self._slot]
            self._slot = (self._slot + 1) % len(self._host)
            done.synchronize()   # the H2D copy that read this buffer 4 steps ago has run
            buf.copy_(src)
            self.frame_u8.view(self.B, self.H, self.W, 3).copy_(buf, non_blocking=True)
            done.record(torch.cuda.current_stream(self.device))
        self.graph.replay()
        return self._outs[0]
