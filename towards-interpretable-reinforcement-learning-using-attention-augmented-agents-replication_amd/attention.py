"""Drop-in ``attention`` module: the reference's nn.Module API on the HIP path.

Same class names, constructor signatures, attributes and state_dict keys as
the reference ``attention.py``, so ``main_mp.py`` /
``test_model.py`` and saved checkpoints work unchanged:

  ConvLSTMCell   attention.py:7-149      (aaa_convlstm_cell_fwd/bwd; fused into Agent's unroll)
  VisionNetwork  attention.py:152-181    (aaa_vision_cnn_fwd/bwd + the cell; fused into Agent's unroll)
  QueryNetwork   attention.py:184-198
  SpatialBasis   attention.py:201-232
  spatial_softmax / apply_alpha  attention.py:235-254
  Agent          attention.py:257-368

``Agent.forward`` (one step, state carried in ``vision.vision_lstm.prev_hidden`` in
the reference's (B, 128, w, h) layout -- a permuted view of the kernels' NHWC state)
and the added ``Agent.unroll`` (T steps in one call) run entirely in the gfx950
kernels of libaaa.so through one ``torch.autograd.Function`` per call; the
Function's backward is the hand-written BPTT, and consecutive per-step calls
chain through the ConvLSTM state so ``loss.backward()`` after an episode
(main_mp.py:77) back-propagates through every step exactly like the reference.
There is no CPU fallback: calling the Agent with CPU tensors raises.

Added (optional) surface: ``Agent(..., grid=None | (h, w) | "auto",
conv_dtype="fp32" | "bf16", stateful_core=False)`` and ``Agent.unroll``.
``stateful_core`` (or a tensor placed in ``agent.prev_hidden``, as the
reference itself reacts to) runs the reference's otherwise unreachable else
branch (attention.py:356-358): the query reads prev_output = h_{t-1} and the
LSTMCell carries (prev_output, prev_hidden) across steps and calls.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F
from torch import nn

from .runtime import UnrollRunner

__all__ = ["ConvLSTMCell", "VisionNetwork", "QueryNetwork", "SpatialBasis", "spatial_softmax",
           "apply_alpha", "Agent"]


# Generation of the process's module structure: bumped whenever any module
# registers a parameter or a submodule (torch's global registration hooks), so
# a cached parameter list is re-made after such a change (Agent._param_list).
_STRUCT_GEN = [0]


def _bump_struct(*_):
    _STRUCT_GEN[0] += 1


torch.nn.modules.module.register_module_parameter_registration_hook(_bump_struct)
torch.nn.modules.module.register_module_module_registration_hook(_bump_struct)


def _no_cpu(t, what):
    if not t.is_cuda:
        raise RuntimeError(f"aaa: {what} runs only on the MI355X HIP path; move it and its inputs to a ROCm GPU "
                           f"(there is no CPU fallback)")


def _packed_cache(owner, params, dtype, pack):
    """(flat fp32 params, packed operands) of ``params``, re-made only when a
    parameter changed (storage or in-place version: optimizer steps,
    load_state_dict, .to()).  The cached tensors are never written again."""
    key = (dtype,) + tuple((p.data_ptr(), p._version) for p in params)
    cached = getattr(owner, "_pack_cache", None)
    if cached is not None and cached[0] == key:
        return cached[1], cached[2]
    with torch.no_grad():
        flat = torch.cat([p.detach().reshape(-1) for p in params])
        packed = pack(flat)
    owner._pack_cache = (key, flat, packed)
    return flat, packed


class _CellFn(torch.autograd.Function):
    """One ConvLSTM step (aaa_convlstm_cell_fwd); backward = aaa_convlstm_cell_bwd."""

    @staticmethod
    def forward(ctx, runner, packed, x, h0, c0, *params):
        h1, c1, ws = runner.forward(packed, x, h0, c0)
        ctx.runner, ctx.packed, ctx.ws = runner, packed, ws
        ctx.shapes = [p.shape for p in params]
        ctx.has_state = (h0 is not None, c0 is not None)
        return h1, c1

    @staticmethod
    def backward(ctx, dh1, dc1):
        need = ctx.needs_input_grad
        dx, dh0, dc0, grads = ctx.runner.backward(
            ctx.packed, ctx.ws, dh1, dc1, want_dx=need[2], want_dh0=need[3] and ctx.has_state[0],
            want_dc0=need[4] and ctx.has_state[1], want_grads=any(need[5:]))
        ctx.ws = None
        views = ([g.view(s) for g, s in zip(grads.split([int(torch.Size(s).numel()) for s in ctx.shapes]),
                                            ctx.shapes)] if grads is not None else [None] * len(ctx.shapes))
        return (None, None, dx, dh0, dc0, *views)


class _CnnFn(torch.autograd.Function):
    """VisionNetwork.vision_cnn over N frames (aaa_vision_cnn_fwd / _bwd)."""

    @staticmethod
    def forward(ctx, runner, flat, packed, X, *params):
        y2, _, ws = runner.forward(flat, packed, X)
        ctx.runner, ctx.packed, ctx.ws = runner, packed, ws
        ctx.shapes = [p.shape for p in params]
        return y2

    @staticmethod
    def backward(ctx, dy2):
        grads, _ = ctx.runner.backward(ctx.packed, ctx.ws, dy2)
        ctx.ws = None
        views = [g.view(s) for g, s in zip(grads.split([int(torch.Size(s).numel()) for s in ctx.shapes]), ctx.shapes)]
        return (None, None, None, None, *views)


class ConvLSTMCell(nn.Module):
    """Zero-peephole ConvLSTM cell (attention.py:7-149) on the HIP path.

    ``forward(x)`` takes the reference's (B, C, a, b) input and returns
    ``(h, c)`` (B, hidden, a, b), carrying them in ``prev_hidden`` exactly as
    attention.py:110-126 does (``reset()`` clears it; the zero peepholes
    ``Wci/Wcf/Wco`` are created on the first zero-state step, :132-141, and
    are not parameters).  The eight gate convs, the gate math and the cell
    update are one MFMA implicit-GEMM launch with a fused epilogue
    (aaa_convlstm_cell_fwd); the backward is aaa_convlstm_cell_bwd.  Inside
    ``Agent`` the same kernels run fused over the whole unroll.
    """

    conv_dtype = "fp32"

    def __init__(self, input_channels, hidden_channels, kernel_size):
        super().__init__()
        assert hidden_channels % 2 == 0
        self.input_channels = input_channels
        self.hidden_channels = hidden_channels
        self.kernel_size = kernel_size
        self.num_features = 4
        self.padding = int((kernel_size - 1) / 2)
        k, p = kernel_size, self.padding
        # registration order == reference state_dict order
        for g in "ifco":
            setattr(self, f"Wx{g}", nn.Conv2d(input_channels, hidden_channels, k, 1, p, bias=True))
            setattr(self, f"Wh{g}", nn.Conv2d(hidden_channels, hidden_channels, k, 1, p, bias=False))
        self.Wci = None
        self.Wcf = None
        self.Wco = None
        self.prev_hidden = None
        self._runners = {}
        self._own_peepholes = None

    def forward(self, x):
        _no_cpu(x, "ConvLSTMCell")
        if x.dim() != 4 or x.shape[1] != self.input_channels:
            raise ValueError(f"ConvLSTMCell expects (B, {self.input_channels}, H, W), got {tuple(x.shape)}")
        h, c = self.step_nhwc(x.permute(0, 3, 2, 1))
        return h.permute(0, 3, 2, 1), c.permute(0, 3, 2, 1)

    def step_nhwc(self, x):
        """One step on x (B, b, a, C) = the reference input permuted (0, 3, 2, 1);
        returns (h, c) in that layout and keeps prev_hidden in the reference's."""
        if (self.input_channels, self.hidden_channels, self.kernel_size) != (64, 128, 3):
            raise NotImplementedError("the HIP cell implements ConvLSTMCell(64, 128, 3), the reference's only "
                                      "instance (attention.py:171-173)")
        B, b, a, _ = x.shape
        if self.prev_hidden is None:
            h0 = c0 = None                       # init_hidden: zeros (attention.py:111-115, 142-149)
            self._peepholes(a, b, x.device)
        else:
            h, c = self.prev_hidden
            if tuple(h.shape) != (B, self.hidden_channels, a, b) or tuple(c.shape) != tuple(h.shape):
                raise RuntimeError(f"prev_hidden is {tuple(h.shape)}, this input needs "
                                   f"{(B, self.hidden_channels, a, b)}; call reset()")
            h0, c0 = h.permute(0, 3, 2, 1), c.permute(0, 3, 2, 1)
        self._check_peepholes(a, b)
        params = list(self.parameters())
        r = self._runner(B, b, a, x.device)
        _, packed = _packed_cache(self, params, self.conv_dtype, r.pack)
        h1, c1 = _CellFn.apply(r, packed, x.float().contiguous(), h0, c0, *params)
        self.prev_hidden = (h1.permute(0, 3, 2, 1), c1.permute(0, 3, 2, 1))
        return h1, c1

    def reset(self):
        self.prev_hidden = None

    def init_hidden(self, batch_size, hidden, height, width, device):
        """The reference's zero state (attention.py:131-149), (B, hidden, height, width)."""
        self._peepholes(height, width, device)
        z = torch.zeros(batch_size, hidden, height, width, device=device)
        return z, z.clone()

    # -- internals ----------------------------------------------------------
    def _runner(self, B, h, w, device):
        from .runtime import CellRunner
        key = (B, h, w, str(device), self.conv_dtype)
        r = self._runners.get(key)
        if r is None:
            r = self._runners[key] = CellRunner(B, h, w, self.conv_dtype, device)
        return r

    def _peepholes(self, height, width, device):
        if self.Wci is None:   # created once, sized by the first input; never cleared (Q2)
            self.Wci, self.Wcf, self.Wco = (torch.zeros(1, self.hidden_channels, height, width, device=device)
                                            for _ in range(3))
            self._own_peepholes = (self.Wci, self.Wcf, self.Wco)

    def _check_peepholes(self, a, b):
        """The kernels drop the c * W_c* terms, exact for the reference's zero
        peepholes; a later input of another size fails there as in the
        reference (``c * self.Wci`` does not broadcast)."""
        if self.Wci is None:
            return
        if tuple(self.Wci.shape[2:]) != (a, b):
            raise RuntimeError(f"The size of tensor a ({b}) must match the size of tensor b ({self.Wci.shape[3]}) "
                               f"at non-singleton dimension 3 (the zero peepholes Wci/Wcf/Wco were sized "
                               f"{tuple(self.Wci.shape[2:])} by the first input, attention.py:132-141)")
        if self._own_peepholes is None or any(p is not q for p, q in zip((self.Wci, self.Wcf, self.Wco),
                                                                           self._own_peepholes)):
            if any(bool(p.count_nonzero()) for p in (self.Wci, self.Wcf, self.Wco)):
                raise NotImplementedError("non-zero peepholes: the reference's are constant zeros (attention.py:"
                                          "132-141) and the HIP cell drops the c * W_c* terms")
            self._own_peepholes = (self.Wci, self.Wcf, self.Wco)


class VisionNetwork(nn.Module):
    """conv 8/4/1 -> conv 4/2/2 (no activation) -> ConvLSTM (attention.py:152-181).

    ``forward(X)`` (B, H, W, 3) -> O (B, h, w, 128), the reference's
    ``O.transpose(1, 3)``, with the cell state carried in
    ``vision_lstm.prev_hidden``: the encoder is aaa_vision_cnn_fwd, the cell
    aaa_convlstm_cell_fwd (both with hand-written backwards).
    """

    conv_dtype = "fp32"

    def __init__(self):
        super().__init__()
        self.vision_cnn = nn.Sequential(
            nn.Conv2d(in_channels=3, out_channels=32, kernel_size=(8, 8), stride=4, padding=1),
            nn.Conv2d(in_channels=32, out_channels=64, kernel_size=(4, 4), stride=2, padding=2),
        )
        self.vision_lstm = ConvLSTMCell(input_channels=64, hidden_channels=128, kernel_size=3)
        self._runners = {}

    def reset(self):
        self.vision_lstm.reset()

    def forward(self, X):
        _no_cpu(X, "VisionNetwork")
        if X.dim() != 4 or X.shape[3] != 3:
            raise ValueError(f"VisionNetwork expects (B, H, W, 3) frames, got {tuple(X.shape)}")
        if X.requires_grad:
            raise NotImplementedError("frame gradients are not computed on the HIP path (the reference's frames "
                                      "are data, main_mp.py:53)")
        B, H, W, _ = X.shape
        from .runtime import CnnRunner
        key = (B, H, W, str(X.device), self.conv_dtype)
        r = self._runners.get(key)
        if r is None:
            r = self._runners[key] = CnnRunner(B, H, W, self.conv_dtype, X.device)
        params = list(self.vision_cnn.parameters())
        flat, packed = _packed_cache(self, params, self.conv_dtype, r.pack)
        y = _CnnFn.apply(r, flat, packed, X.float().contiguous(), *params)   # (B, h, w, 64)
        self.vision_lstm.conv_dtype = self.conv_dtype
        O, _ = self.vision_lstm.step_nhwc(y)
        return O


class QueryNetwork(nn.Module):
    """256 -> 128 -> 72*nq -> 72*nq MLP (attention.py:184-198; nq=4 in the reference)."""

    def __init__(self, num_queries: int = 4):
        super().__init__()
        self.num_queries = num_queries
        qd = 72 * num_queries
        self.model = nn.Sequential(nn.Linear(256, 128), nn.ReLU(), nn.Linear(128, qd), nn.ReLU(),
                                   nn.Linear(qd, qd))

    def forward(self, query):
        return self.model(query).reshape(-1, self.num_queries, 72)


class SpatialBasis:
    """Constant (h, w, channels) cosine basis (attention.py:201-232).

    S[i, j, 8u + v] = cos((i+1)*pi/h * (u+1)) * cos((j+1)*pi/w * (v+1)), built
    with the same fp32 ops as the reference so it is bit-identical.
    """

    def __init__(self, height=27, width=20, channels=64):
        nb = int(round(math.sqrt(channels)))
        rows = torch.arange(1, height + 1).unsqueeze(1).float().mul(torch.ones(1, width)).mul(math.pi / height)
        cols = torch.ones(height, 1).mul(torch.arange(1, width + 1).unsqueeze(0).float()).mul(math.pi / width)
        freq = torch.arange(1, nb + 1).unsqueeze(0).float()
        cy = torch.cos(rows.unsqueeze(2) * freq)
        cx = torch.cos(cols.unsqueeze(2) * freq)
        self.S = (cy.unsqueeze(3) * cx.unsqueeze(2)).reshape(height, width, nb * nb)

    def __call__(self, X):
        S = self.S.to(X.device).unsqueeze(0).expand(X.shape[0], -1, -1, -1)
        return torch.cat([X, S], dim=3)


def spatial_softmax(A):
    """Softmax over the h*w grid for each query (attention.py:235-243)."""
    b, h, w, d = A.size()
    return F.softmax(A.reshape(b, h * w, d), dim=1).reshape(b, h, w, d)


def apply_alpha(A, V):
    """Attention-weighted readout sum_p A[p, q] V[p] (attention.py:246-254)."""
    b, h, w, c = A.size()
    return torch.matmul(A.reshape(b, h * w, c).transpose(1, 2), V.reshape(b, h * w, V.size(3)))


class _UnrollFn(torch.autograd.Function):
    """One library forward over T steps; its backward is the hand-written BPTT."""

    @staticmethod
    def forward(ctx, runner, flat, packed, S, X, pr, pa, h0, c0, ch0, cc0, *params):
        ws = runner.new_workspace()
        out = runner.forward(flat, packed, S, X, ws, pr, pa, h0, c0, want_attn=True, want_state=True,
                             core=(ch0, cc0) if runner.stateful_core else None)
        if getattr(runner, "relu_trace", None) is not None:   # inspection hook (Agent.relu_trace)
            runner.relu_trace.append(runner.relu_masks(ws))
        logits, values, attn, hT, cT = out[:5]
        chT, ccT = out[5:] if runner.stateful_core else (None, None)
        ctx.runner, ctx.flat, ctx.packed, ctx.ws, ctx.S, ctx.X = runner, flat, packed, ws, S, X
        ctx.Xv = X._version   # the backward rebuilds conv1's operand from these frames
        ctx.shapes = [p.shape for p in params]
        ctx.mark_non_differentiable(attn)
        return logits, values, attn, hT, cT, chT, ccT

    @staticmethod
    def backward(ctx, dl, dv, _dattn, dhT, dcT, dchT=None, dccT=None):
        r = ctx.runner
        if ctx.X._version != ctx.Xv:
            raise RuntimeError("aaa: the frames of this unroll were modified by an inplace operation after the "
                               "forward; the backward reads them again (conv1's weight gradient), as autograd "
                               "would need them unchanged")
        want_state = bool(ctx.needs_input_grad[7] or ctx.needs_input_grad[8])
        if r.stateful_core:
            want_core = bool(ctx.needs_input_grad[9] or ctx.needs_input_grad[10])
            grads, dh0, dc0, dch0, dcc0 = r.backward(ctx.flat, ctx.packed, ctx.S, ctx.X, ctx.ws, dl, dv, dhT, dcT,
                                                     want_state_grads=want_state, dcore=(dchT, dccT),
                                                     want_core_grads=want_core)
        else:
            grads, dh0, dc0 = r.backward(ctx.flat, ctx.packed, ctx.S, ctx.X, ctx.ws, dl, dv, dhT, dcT,
                                         want_state_grads=want_state)
            dch0 = dcc0 = None
        ctx.ws = None
        views = [g.view(s) for g, s in zip(grads.split(r.sizes), ctx.shapes)]
        return (None, None, None, None, None, None, None, dh0, dc0, dch0, dcc0, *views)


class Agent(nn.Module):
    """Attention-augmented agent (attention.py:257-368) on the gfx950 HIP path."""

    def __init__(self, num_actions, hidden_size: int = 256, c_v: int = 120, c_k: int = 8, c_s: int = 64,
                 num_queries: int = 4, *, grid=None, conv_dtype: str = "fp32", stateful_core: bool = False):
        super().__init__()
        if (hidden_size, c_v, c_k, c_s) != (256, 120, 8, 64):
            raise ValueError("hidden_size/c_v/c_k/c_s are hard-coded elsewhere in the reference "
                             "(attention.py:171-198, SURVEY.md Q6); only the defaults are supported")
        if num_queries not in (4, 8):
            raise ValueError("num_queries must be 4 (reference) or 8 (generalised, SURVEY.md Q5)")
        if conv_dtype not in ("fp32", "bf16"):
            raise ValueError("conv_dtype must be 'fp32' or 'bf16'")
        self.hidden_size = hidden_size
        self.c_v, self.c_k, self.c_s, self.num_queries = c_v, c_k, c_s, num_queries
        self.num_actions = num_actions
        self.conv_dtype = conv_dtype
        # the reference's else branch (attention.py:356-358): also taken whenever
        # a caller puts a tensor in ``prev_hidden``, exactly as the reference does
        self.stateful_core = bool(stateful_core)
        self.vision = VisionNetwork()
        self.vision.conv_dtype = self.vision.vision_lstm.conv_dtype = conv_dtype
        self.query = QueryNetwork(num_queries)
        self._auto_grid = grid == "auto"
        self.spatial = SpatialBasis(*grid) if isinstance(grid, (tuple, list)) else SpatialBasis()
        self.answer_processor = nn.Sequential(
            nn.Linear((c_v + c_s) * num_queries + (c_k + c_s) * num_queries + 1 + 1, 512),
            nn.ReLU(),
            nn.Linear(512, hidden_size),
        )
        self.policy_core = nn.LSTMCell(hidden_size, hidden_size)
        self.prev_output = None
        self.prev_hidden = None
        self.policy_head = nn.Sequential(nn.Linear(hidden_size, num_actions))
        self.values_head = nn.Sequential(nn.Linear(hidden_size, num_actions))
        self._runners = {}
        self._basis = None
        self.last_attention = None
        self._episode = None

    # Per-step forward calls with autograd on record into one episode whose
    # backward runs as multi-step BPTT calls (episode.py); False: one T=1
    # autograd node with its own saved workspace per call.
    fuse_episode_backward = True
    # Inspection hook for checkers (None: off): a list that every forward call of
    # this agent appends its ReLU masks to (UnrollRunner.relu_masks), in call
    # order -- what the mask-matched oracle runs its backward through
    # (tests/helpers.py oracle_masks).  Costs a host copy per call.
    relu_trace = None

    # -- reference API --------------------------------------------------------
    def reset(self):
        self.vision.reset()
        self.prev_output = None
        self.prev_hidden = None
        self._episode = None

    def forward(self, X, prev_reward=None, prev_action=None, ts=0):
        """One step (attention.py:298-368): X (B, H, W, 3) -> logits, values (B, A)."""
        pr = None if prev_reward is None else prev_reward.reshape(1, -1)
        pa = None if prev_action is None else prev_action.reshape(1, -1)
        params = self._episode_params(X)
        if params is not None:
            logits, values, attn = self._episode_step(X, pr, pa, params)
        else:
            logits, values, attn = self._step(X.unsqueeze(0), pr, pa)
        self.last_attention = attn[0]
        # squeeze, not [0]: the same (B, A) view, but its backward is a view too
        # (select_backward allocates zeros and copies: two launches per step)
        return logits.squeeze(0), values.squeeze(0)

    def act_episode(self, X, sampler, ts=0):
        """Policy.act's step (forward + action draw, policy.py) as one node of the
        open episode when the fused episode backward applies: (action, log_prob),
        else None (the caller then runs forward() and samples itself)."""
        params = self._episode_params(X)
        if params is None:
            return None
        logits, values, attn, action, logp = self._episode_step(X, None, None, params, sampler)
        self.last_attention = attn[0]
        return action, logp

    # -- added API ----------------------------------------------------------
    def unroll(self, X, prev_reward=None, prev_action=None):
        """T steps in one call: X (T, B, H, W, 3) -> logits, values (T, B, A), attn (T, B, h, w, nq).

        Continues from the current ConvLSTM state (zero after ``reset()``) and
        leaves the final state in ``vision.vision_lstm.prev_hidden``.
        """
        logits, values, attn = self._step(X, prev_reward, prev_action)
        self.last_attention = attn
        return logits, values, attn

    # -- internals ----------------------------------------------------------
    def _param_list(self):
        """``list(self.parameters())`` without walking the module tree per call
        (~60 us of Python per walk; an actor pays it every step).  The list is
        re-made after any parameter or submodule registration (_STRUCT_GEN)
        and whenever a module's parameter or child count changed (deletions
        register nothing), and whenever a cached entry is no longer the object its
        module holds: a Parameter replaced without a registration hook or a count
        change -- ``.to()`` under torch.__future__'s overwrite-on-conversion flag,
        or a direct ``_parameters[k] = ...`` -- so gradients never
        land on tensors the optimizer no longer holds.  In-place changes keep the
        same Parameter objects."""
        c = self.__dict__.get("_plist")
        if c is not None and c[0] == _STRUCT_GEN[0]:
            n = 0
            for m in c[1]:
                n += len(m._parameters) + len(m._modules)
            if n == c[2]:
                ps = c[3]
                for (d, k), p in zip(c[4], ps):
                    if d.get(k) is not p:
                        break
                else:
                    return ps
        mods = list(self.modules())
        n = sum(len(m._parameters) + len(m._modules) for m in mods)
        slots, ps, seen = [], [], set()
        for m in mods:   # the order of self.parameters(): modules in order, each one's own parameters
            for k, p in m._parameters.items():
                if p is not None and id(p) not in seen:
                    seen.add(id(p))
                    slots.append((m._parameters, k))
                    ps.append(p)
        self.__dict__["_plist"] = (_STRUCT_GEN[0], mods, n, ps, slots)
        return ps

    def _check_devices(self, params, device):
        for p in params:
            if p.device != device:
                raise RuntimeError(f"agent parameters are on {p.device} but frames are on {device}; "
                                   f"call agent.to({device})")

    def _episode_params(self, X):
        """The parameter list when this per-step call records into an episode, else None."""
        if not (self.fuse_episode_backward and X.is_cuda and X.dim() == 4 and torch.is_grad_enabled()
                and not (self.stateful_core or self.prev_hidden is not None)):
            return None
        params = self._param_list()
        return params if any(p.requires_grad for p in params) else None

    def _episode_step(self, X, pr, pa, params, sampler=None):
        """One per-step call recorded into the open episode (episode.py): a new
        episode after reset(), a parameter change, another geometry, or a
        prev_hidden the episode did not set itself."""
        from .episode import Episode, _EpisodeActFn, _EpisodeAnchorFn, _EpisodeStepFn
        B, H, W, C = X.shape
        if C != 3:
            raise ValueError(f"frames must be (..., H, W, 3), got {tuple(X.shape)}")
        u8 = X.dtype == torch.uint8
        runner = self._runner(B, 1, H, W, X.device, False, u8)
        runner.relu_trace = self.relu_trace
        S = self._basis_for(runner.h, runner.w, H, W, X.device)
        flat, packed = self._packed_params(runner, params, self)
        key = runner._pack_cache[0]
        cell = self.vision.vision_lstm
        ep = self._episode
        if ep is None or ep.runner is not runner or ep.key != key or cell.prev_hidden is not ep.state_ref:
            if cell.prev_hidden is None:
                h0 = c0 = None
                cell._peepholes(runner.w, runner.h, X.device)      # init_hidden's lazy zero peepholes (Q2)
            else:
                h0, c0 = (s.permute(0, 3, 2, 1) for s in cell.prev_hidden)
                if tuple(h0.shape) != runner.state_shape() or tuple(c0.shape) != runner.state_shape():
                    raise RuntimeError(f"carried ConvLSTM state {tuple(cell.prev_hidden[0].shape)} does not match "
                                       f"this batch {(B, 128, runner.w, runner.h)}; call agent.reset()")
            cell._check_peepholes(runner.w, runner.h)
            ep = Episode(self, runner, flat, packed, key, S, h0, c0)
            ep.anchor = _EpisodeAnchorFn.apply(ep, h0, c0, *params)
            self._episode = ep
        t = ep.record((X if u8 else X.float()).unsqueeze(0).contiguous(), pr, pa)
        if sampler is None:
            logits, values, attn, hT, cT = _EpisodeStepFn.apply(ep, t, ep.anchor)
        else:
            logits, values, attn, hT, cT, action, logp = _EpisodeActFn.apply(ep, t, ep.anchor, sampler)
        cell.prev_hidden = (hT.permute(0, 3, 2, 1), cT.permute(0, 3, 2, 1))
        ep.state_ref = cell.prev_hidden
        if self.prev_output is None:   # Q1: the query input is created once and never updated
            self.prev_output = torch.zeros(B, self.hidden_size, device=X.device)
        if sampler is not None:
            return logits, values, attn, action, logp
        return logits, values, attn

    def _step(self, X, pr, pa):
        if not X.is_cuda:
            raise RuntimeError("aaa: Agent runs only on the MI355X HIP path; move the agent and its "
                               "inputs to a ROCm GPU (there is no CPU fallback)")
        T, B, H, W, C = X.shape
        if C != 3:
            raise ValueError(f"frames must be (..., H, W, 3), got {tuple(X.shape)}")
        params = self._param_list()
        stateful = self.stateful_core or self.prev_hidden is not None
        u8 = X.dtype == torch.uint8      # the environment's observation: cast in-kernel (AAA_FLAG_FRAMES_U8)
        runner = self._runner(B, T, H, W, X.device, stateful, u8)
        runner.relu_trace = self.relu_trace
        S = self._basis_for(runner.h, runner.w, H, W, X.device)
        cell = self.vision.vision_lstm
        # prev_hidden holds the reference's (B, 128, w, h) tensors (attention.py:125); the
        # kernels' NHWC (B, h, w, 128) is their permute(0, 3, 2, 1) -- a view, no copy
        if cell.prev_hidden is None:
            h0 = c0 = None
            cell._peepholes(runner.w, runner.h, X.device)      # init_hidden's lazy zero peepholes (Q2)
        else:
            h0, c0 = (s.permute(0, 3, 2, 1) for s in cell.prev_hidden)
            if tuple(h0.shape) != runner.state_shape() or tuple(c0.shape) != runner.state_shape():
                raise RuntimeError(f"carried ConvLSTM state {tuple(cell.prev_hidden[0].shape)} does not match this "
                                   f"batch {(B, 128, runner.w, runner.h)}; call agent.reset()")
        cell._check_peepholes(runner.w, runner.h)
        ch0 = cc0 = None
        if stateful:   # (prev_output, prev_hidden) of the policy core, zeros after reset()
            ch0, cc0 = self.prev_output, self.prev_hidden
            for name, v in (("prev_output", ch0), ("prev_hidden", cc0)):
                if v is not None and tuple(v.shape) != (B, self.hidden_size):
                    raise RuntimeError(f"{name} has shape {tuple(v.shape)}, expected {(B, self.hidden_size)}")
        Xf = X.contiguous() if u8 else X.float().contiguous()
        flat, packed = self._packed_params(runner, params, self)
        logits, values, attn, hT, cT, chT, ccT = _UnrollFn.apply(runner, flat, packed, S, Xf, pr, pa, h0, c0,
                                                                 ch0, cc0, *params)
        cell.prev_hidden = (hT.permute(0, 3, 2, 1), cT.permute(0, 3, 2, 1))
        if stateful:
            self.prev_output, self.prev_hidden = chT, ccT
        elif self.prev_output is None:   # Q1: the query input is created once and never updated
            self.prev_output = torch.zeros(B, self.hidden_size, device=X.device)
        return logits, values, attn

    @staticmethod
    def _packed_params(runner, params, agent=None):
        """Flat fp32 params + their packed operand layout, re-made only when a
        parameter changed (its storage or in-place version counter: optimizer
        steps, load_state_dict, .to()).  An actor stepping one frame at a time
        (main_mp.py:100, test_model.py:44) then pays no per-step re-pack.  The
        cached tensors are never written again, so graphs that saved them stay valid.
        A re-pack first checks that every parameter is on the runner's device (a
        cache hit means the same storages, so the same devices, as that check)."""
        key = tuple((p.data_ptr(), p._version) for p in params)
        cached = getattr(runner, "_pack_cache", None)
        if cached is not None and cached[0] == key:
            return cached[1], cached[2]
        if agent is not None:
            agent._check_devices(params, runner.device)
        with torch.no_grad():
            flat = torch.cat([p.detach().reshape(-1) for p in params])
            packed = runner.new_packed()
            runner.pack(flat, packed)
        runner._pack_cache = (key, flat, packed)
        return flat, packed

    def _runner(self, B, T, H, W, device, stateful=False, frames_u8=False):
        key = (B, T, H, W, str(device), self.conv_dtype, bool(stateful), bool(frames_u8))
        r = self._runners.get(key)
        if r is None:
            r = UnrollRunner(B, T, H, W, self.num_queries, self.num_actions, self.conv_dtype, device,
                             stateful_core=stateful, frames_u8=frames_u8)
            self._runners[key] = r
        return r

    def _basis_for(self, h, w, H, W, device):
        if self._auto_grid and tuple(self.spatial.S.shape[:2]) != (h, w):
            self.spatial = SpatialBasis(h, w)
        S = self.spatial.S
        if tuple(S.shape) != (h, w, 64):
            raise RuntimeError(
                f"Sizes of tensors must match: the spatial basis is {tuple(S.shape[:2])} but {H}x{W} frames "
                f"give a {h}x{w} grid; set agent.spatial = SpatialBasis({h}, {w}) (the reference hard-codes "
                f"27x20 at attention.py:208,275)")
        cached = self._basis
        if cached is None or cached[0] is not S or cached[1] != str(device):
            self._basis = (S, str(device), S.to(device=device, dtype=torch.float32).contiguous())
        return self._basis[2]
