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
                 dtype: str = "fp32", device=None, seed: int = 0, group=None, lr: float = 1e-3,
                 frames_u8: bool = False):
        self.runner = r = UnrollRunner(B, T, H, W, nq, A, dtype, device, frames_u8=frames_u8)
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
        # Phase -> bucket disjointness (checked by tools/dp_check.py): a backward
        # phase writes no bucket whose all-reduce an EARLIER phase has already
        # issued -- CORE may write conv2's bias grad (VISION bucket, reduced after
        # it), never a HEAD tensor; VISION writes neither HEAD nor CORE.
        if self.world > 1:   # identical weights on every rank (they are seeded, but be explicit)
            dist.broadcast(self.flat, src=0, group=group)
            self.comm = torch.cuda.Stream(self.device)   # the gradient all-reduces (RCCL) run here

    def step(self, frames, dlogits, dvalues, overlap: bool = True, comm_timing: bool = False):
        """One learner iteration; returns (logits, values).  With N > 1 ranks the
        gradient buckets are SUM-all-reduced over RCCL on a side stream, each
        issued as soon as its backward phase is enqueued (the side stream waits
        on an event recorded after that phase), so HEAD's all-reduce overlaps
        the ConvLSTM BPTT and CORE's the vision backward.  ``comm_timing``
        records per-bucket events; read them with comm_stats() after a sync."""
        r = self.runner
        r.pack(self.flat, self.packed)
        logits, values, _, _, _ = r.forward(self.flat, self.packed, self.basis, frames, self.ws, want_attn=False)
        if self.world == 1:
            r.backward(self.flat, self.packed, self.basis, frames, self.ws, dlogits, dvalues, grads=self.grads)
            return logits, values
        main = torch.cuda.current_stream(self.device)
        self._events = [] if comm_timing else None
        phases = list(zip((N.BWD_HEAD, N.BWD_CORE, N.BWD_VISION), self.bounds))
        for i, (phase, bnd) in enumerate(phases):
            r.backward(self.flat, self.packed, self.basis, frames, self.ws, dlogits, dvalues, grads=self.grads,
                       phases=phase)
            if overlap or i == len(phases) - 1:
                self._allreduce(main, [bnd] if overlap else self.bounds, comm_timing)
        if comm_timing:
            self._compute_done = torch.cuda.Event(enable_timing=True)
            self._compute_done.record(main)
        main.wait_stream(self.comm)
        return logits, values

    def _allreduce(self, main, bounds, timing):
        ready = torch.cuda.Event(enable_timing=timing)
        ready.record(main)                          # everything the phase enqueued
        with torch.cuda.stream(self.comm):
            self.comm.wait_event(ready)
            for lo, hi in bounds:
                t0 = torch.cuda.Event(enable_timing=True) if timing else None
                if timing:
                    t0.record(self.comm)
                allreduce_buckets(self.grads, [(lo, hi)], self.group, async_op=False)
                if timing:
                    t1 = torch.cuda.Event(enable_timing=True)
                    t1.record(self.comm)
                    self._events.append((lo, hi, ready, t0, t1))

    def comm_stats(self):
        """Per-bucket all-reduce time (ms) and the communication left exposed
        after the last backward phase (ms) of the last timed step()."""
        if not getattr(self, "_events", None):
            raise RuntimeError("comm_stats(): the last step() ran without comm_timing=True (or on one rank)")
        buckets = []
        for (lo, hi, ready, t0, t1), name in zip(self._events, ("HEAD", "CORE", "VISION")):
            buckets.append({"bucket": name, "bytes": 4 * (hi - lo), "allreduce_ms": round(t0.elapsed_time(t1), 4),
                            "queued_after_phase_ms": round(ready.elapsed_time(t0), 4)})
        last = self._events[-1][4]
        exposed = max(0.0, self._compute_done.elapsed_time(last))
        return {"buckets": buckets, "exposed_ms": round(exposed, 4)}

    def optimizer_step(self):
        """Adam (lr=1e-3, torch defaults; main_mp.py:92) on the flat params, one launch."""
        self.opt_steps += 1
        adam_flat_(self.flat, self.grads, self.exp_avg, self.exp_avg_sq, self.opt_steps, lr=self.lr)

    def train_step(self, frames, dlogits, dvalues, overlap: bool = True):
        out = self.step(frames, dlogits, dvalues, overlap=overlap)
        self.optimizer_step()
        return out
