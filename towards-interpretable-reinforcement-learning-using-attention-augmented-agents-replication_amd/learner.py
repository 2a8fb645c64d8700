"""One synchronous learner iteration on the HIP path (bench / DP driver).

step():  pack weights -> T-step forward -> backward (3 phases) with each
phase's gradient bucket all-reduced (RCCL) while the next phase runs.
train_step(): step() followed by the fused Adam update of the flat params
(main_mp.py:78; csrc/optim.hip), i.e. one complete learner iteration.
Weights live in one flat fp32 buffer in state_dict order, grads likewise, so
a bucket is a contiguous slice and no flatten/unflatten copies are needed.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

from . import _native as N
from . import detinit
from .attention import SpatialBasis
from .optim import adam_flat_
from .parallel import allreduce_buckets, bucket_bounds
from .runtime import UnrollRunner


class Learner:
    def __init__(self, B: int, T: int, H: int = 84, W: int = 84, nq: int = 4, A: int = 18,
                 dtype: str = "fp32", device=None, seed: int = 0, group=None, lr: float = 1e-3):
        self.runner = r = UnrollRunner(B, T, H, W, nq, A, dtype, device)
        self.device = r.device
        params = detinit.deterministic_params(seed, A, nq)
        self.flat = torch.from_numpy(np.concatenate([v.reshape(-1) for v in params.values()])).to(self.device)
        assert self.flat.numel() == r.n_params
        self.packed = r.new_packed()
        self.ws = r.new_workspace()
        self.grads = torch.zeros(r.n_params, device=self.device)
        self.lr = lr
        self.exp_avg = torch.zeros_like(self.grads)
        self.exp_avg_sq = torch.zeros_like(self.grads)
        self.opt_steps = 0
        self.basis = SpatialBasis(r.h, r.w).S.to(self.device).contiguous()
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
        self.bounds = bucket_bounds(r.offsets, r.n_params)
        if self.world > 1:   # identical weights on every rank (they are seeded, but be explicit)
            dist.broadcast(self.flat, src=0, group=group)

    def step(self, frames, dlogits, dvalues, overlap: bool = True):
        r = self.runner
        r.pack(self.flat, self.packed)
        logits, values, _, _, _ = r.forward(self.flat, self.packed, self.basis, frames, self.ws, want_attn=False)
        if self.world == 1:
            r.backward(self.flat, self.packed, self.basis, frames, self.ws, dlogits, dvalues, grads=self.grads)
            return logits, values
        works = []
        for phase, bnd in zip((N.BWD_HEAD, N.BWD_CORE, N.BWD_VISION), self.bounds):
            r.backward(self.flat, self.packed, self.basis, frames, self.ws, dlogits, dvalues, grads=self.grads,
                       phases=phase)
            if overlap:
                works += allreduce_buckets(self.grads, [bnd], self.group)
        if not overlap:
            works = allreduce_buckets(self.grads, self.bounds, self.group)
        for w in works:
            w.wait()
        return logits, values

    def optimizer_step(self):
        """Adam (lr=1e-3, torch defaults; main_mp.py:92) on the flat params, one launch."""
        self.opt_steps += 1
        adam_flat_(self.flat, self.grads, self.exp_avg, self.exp_avg_sq, self.opt_steps, lr=self.lr)

    def train_step(self, frames, dlogits, dvalues, overlap: bool = True):
        out = self.step(frames, dlogits, dvalues, overlap=overlap)
        self.optimizer_step()
        return out
