"""REINFORCE loss on the device.

``finish_episode`` in the reference (main_mp.py:62-77) builds the discounted
returns in a Python loop, normalises them, and sums ``-log_prob * R`` over
the per-step ``Categorical`` objects saved by ``Policy.forward``
(main_mp.py:55-58).  ``reinforce_loss`` computes the same loss for B
episodes at once from the unrolled logits, in one kernel (csrc/loss.hip, C
ABI ``aaa_reinforce``) that also writes d loss / d logits, so
``loss.backward()`` hands the cotangent straight to the hand-written BPTT.
There is no CPU fallback.
"""
from __future__ import annotations

import torch

from . import _native as N

__all__ = ["reinforce_loss", "finish_episode_returns"]


class _ReinforceFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, actions, rewards, gamma):
        T, B, A = logits.shape
        lg = logits.detach().contiguous()
        act = actions.to(device=lg.device, dtype=torch.int32).contiguous()
        rew = rewards.to(device=lg.device, dtype=torch.float32).contiguous()
        loss = torch.empty(B, device=lg.device, dtype=torch.float32)
        rn = torch.empty(T, B, device=lg.device, dtype=torch.float32)
        dl = torch.empty_like(lg)
        N.check(N.load().aaa_reinforce(T, B, A, lg.data_ptr(), act.data_ptr(), rew.data_ptr(), float(gamma),
                                       loss.data_ptr(), rn.data_ptr(), dl.data_ptr(), N.stream_ptr(lg.device)),
                "reinforce")
        ctx.save_for_backward(dl)
        ctx.mark_non_differentiable(rn)
        return loss.sum(), rn

    @staticmethod
    def backward(ctx, g_loss, g_rn):
        (dl,) = ctx.saved_tensors
        return dl * g_loss, None, None, None


def reinforce_loss(logits: torch.Tensor, actions, rewards, gamma: float = 0.99, return_returns: bool = False):
    """Sum over episodes of finish_episode's policy loss.

    logits (T, B, A) fp32 on the gfx950 device (e.g. from ``Agent.unroll``),
    actions (T, B) ints in [0, A), rewards (T, B).  With B = 1 this is exactly
    the reference's ``policy_loss`` for one episode.  Returns the scalar loss
    (and the normalised returns (T, B) when ``return_returns``).
    """
    if logits.dim() != 3:
        raise ValueError(f"logits must be (T, B, A), got {tuple(logits.shape)}")
    if not logits.is_cuda or logits.dtype != torch.float32:
        raise RuntimeError("reinforce_loss: logits must be fp32 on the gfx950 device (there is no CPU fallback)")
    T, B, A = logits.shape
    actions = torch.as_tensor(actions).reshape(T, B)
    rewards = torch.as_tensor(rewards, dtype=torch.float32).reshape(T, B)
    if actions.numel() and (int(actions.min()) < 0 or int(actions.max()) >= A):
        raise ValueError(f"actions must lie in [0, {A})")
    loss, rn = _ReinforceFn.apply(logits, actions, rewards, gamma)
    return (loss, rn) if return_returns else loss


def finish_episode_returns(rewards, gamma: float = 0.99) -> list:
    """The reference's discounted-return loop (main_mp.py:66-68), for callers that log returns."""
    R, out = 0.0, []
    for r in list(rewards)[::-1]:
        R = r + gamma * R
        out.insert(0, R)
    return out
