"""Drop-in fused Adam for the learner.

The reference trains with ``optim.Adam(policy.parameters(), lr=1e-3)``
(main_mp.py:92) and calls ``optimizer.step()`` after every episode's backward
(main_mp.py:78).  ``aaa_amd.optim.Adam`` takes the same constructor arguments
and keeps the same per-parameter state (``step``, ``exp_avg``,
``exp_avg_sq`` [, ``max_exp_avg_sq``]) so a torch.optim.Adam state_dict loads
into it and back; ``step()`` is ONE fused multi-tensor HIP launch
(csrc/optim.hip, C ABI ``aaa_adam_step``) instead of torch's seven foreach
passes.  There is no CPU fallback: parameters must be fp32 tensors on the
gfx950 device.
"""
from __future__ import annotations

from collections import defaultdict

import torch
from torch.autograd.graph import increment_version

from . import _native as N

__all__ = ["Adam", "adam_flat_"]


class Adam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0, amsgrad=False, *,
                 maximize: bool = False, foreach=None, capturable: bool = False, differentiable: bool = False,
                 fused=None):
        if not 0.0 <= float(lr):
            raise ValueError(f"Invalid learning rate: {lr}")
        if not 0.0 <= eps:
            raise ValueError(f"Invalid epsilon value: {eps}")
        if not 0.0 <= betas[0] < 1.0:
            raise ValueError(f"Invalid beta parameter at index 0: {betas[0]}")
        if not 0.0 <= betas[1] < 1.0:
            raise ValueError(f"Invalid beta parameter at index 1: {betas[1]}")
        if not 0.0 <= weight_decay:
            raise ValueError(f"Invalid weight_decay value: {weight_decay}")
        if differentiable:
            raise RuntimeError("aaa_amd.optim.Adam: differentiable=True is not supported by the fused kernel")
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=amsgrad, maximize=maximize,
                        foreach=foreach, capturable=capturable, differentiable=differentiable, fused=fused)
        super().__init__(params, defaults)

    @staticmethod
    def _hp(group) -> N.AdamHP:
        b1, b2 = group["betas"]
        return N.AdamHP(float(group["lr"]), float(b1), float(b2), float(group["eps"]),
                        float(group["weight_decay"]), 1 if group["amsgrad"] else 0, 1 if group["maximize"] else 0)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            amsgrad = group["amsgrad"]
            by_step = defaultdict(lambda: ([], [], [], [], []))
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.grad.is_sparse:
                    raise RuntimeError("Adam does not support sparse gradients")
                if not p.is_cuda or p.dtype != torch.float32 or not p.is_contiguous():
                    raise RuntimeError("aaa_amd.optim.Adam: parameters must be contiguous fp32 tensors on the "
                                       "gfx950 device (there is no CPU fallback)")
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = torch.tensor(0.0, dtype=torch.float32)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    if amsgrad:
                        st["max_exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["step"] += 1
                lists = by_step[int(st["step"].item())]
                lists[0].append(p)
                lists[1].append(p.grad.contiguous())
                lists[2].append(st["exp_avg"])
                lists[3].append(st["exp_avg_sq"])
                if amsgrad:
                    lists[4].append(st["max_exp_avg_sq"])
            hp = self._hp(group)
            for step, (ps, gs, ms, vs, xs) in by_step.items():
                N.adam_step(hp, step, ps, gs, ms, vs, xs if amsgrad else None,
                            stream=N.stream_ptr(ps[0].device))
                _bump_versions(ps)
        return loss


def _bump_versions(ps) -> None:
    """The kernel writes the parameters through raw pointers, which autograd's
    version counters do not see; bump them as an in-place torch op would, so
    every cache keyed on (data_ptr, _version) -- Agent's packed weights,
    GraphActor's re-pack check -- sees the update (and autograd still catches
    a stale saved parameter)."""
    for p in ps:
        increment_version(p)


def adam_flat_(params: torch.Tensor, grads: torch.Tensor, exp_avg: torch.Tensor, exp_avg_sq: torch.Tensor,
               step: int, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0,
               guard: torch.Tensor | None = None, step_dev: torch.Tensor | None = None) -> None:
    """Adam over one flat fp32 buffer (the Learner's state_dict-ordered params): one launch.
    ``guard`` (one fp32 device element): skip the update on the device when it is non-zero.
    ``step_dev`` (one int32 device element, updates applied so far): use it instead of
    ``step`` and advance it on the device only when the update ran."""
    hp = N.AdamHP(float(lr), float(betas[0]), float(betas[1]), float(eps), float(weight_decay), 0, 0)
    N.adam_step(hp, step, [params], [grads], [exp_avg], [exp_avg_sq], None, stream=N.stream_ptr(params.device),
                guard=guard, step_dev=step_dev)
    _bump_versions([params])
