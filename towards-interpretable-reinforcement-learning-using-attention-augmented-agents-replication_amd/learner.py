"""One synchronous learner iteration on the HIP path (bench / DP driver).

step():  pack weights -> T-step forward -> backward (3 phases) with the
gradient buckets all-reduced (RCCL) on a side stream while later work runs.
train_step(): step() followed by the fused Adam update of the flat params
(main_mp.py:78; csrc/optim.hip), i.e. one complete learner iteration.
Weights live in one flat fp32 buffer in state_dict order, grads likewise, so
a bucket is a contiguous slice and no flatten/unflatten copies are needed.

Co-residency policy: the ConvLSTM recurrence runs as
multi-workgroup frame-resident launches whose partners must all be resident
at once (csrc/common.h launch_resident).  A collective kernel holding CUs
beside them would make partners wait for it, so no all-reduce is in flight
while a forward or a CORE phase is: HEAD's and CORE's buckets are reduced
together once CORE is enqueued (overlapping the VISION phase), VISION's at
the end, and the next step's forward waits for the comm stream.

Stranded-launch guard: one extra fp32 slot after the gradients receives the
device's pending partner-timeout count (aaa_pair_flag) after the CORE phase;
it rides in the HEAD+CORE all-reduce, so every rank sees any rank's timeout,
and the fused Adam skips the update on the device when it is non-zero
(aaa_adam_step_guarded) -- gradients of a stranded launch never reach the
parameters, with no host sync.  ``check_health()`` raises on it.
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
        # gradients + the stranded-launch guard slot (4 floats: 16-B aligned end)
        self._gbuf = torch.zeros(r.n_params + 4, device=self.device)
        self.grads = self._gbuf[:r.n_params]
        self.guard = self._gbuf[r.n_params:r.n_params + 1]
        self.lr = lr
        self.exp_avg = torch.zeros_like(self.grads)
        self.exp_avg_sq = torch.zeros_like(self.grads)
        self.opt_steps = 0
        self.basis = SpatialBasis(r.h, r.w).S.to(self.device).contiguous()
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
        # per-phase gradient ownership (HEAD, CORE, VISION; tools/dp_check.py checks
        # that a phase never writes a range already handed to the all-reduce)
        self.bounds = bucket_bounds(r.offsets, r.n_params)
        n, o_core = r.n_params, self.bounds[1][0]
        # all-reduce schedule: (phase after which it is issued, element ranges of _gbuf)
        self.schedule = {True: [(N.BWD_CORE, [(o_core, n + 1)]), (N.BWD_VISION, [(0, o_core)])],
                         False: [(N.BWD_VISION, [(0, n + 1)])]}
        if self.world > 1:   # identical weights on every rank (they are seeded, but be explicit)
            dist.broadcast(self.flat, src=0, group=group)
            self.comm = torch.cuda.Stream(self.device)   # the gradient all-reduces (RCCL) run here

    def step(self, frames, dlogits, dvalues, overlap: bool = True, comm_timing: bool = False):
        """One learner iteration; returns (logits, values).  With N > 1 ranks the
        gradients are SUM-all-reduced over RCCL on a side stream, issued after
        the CORE and VISION phases (``schedule``): the HEAD+CORE reduction
        overlaps the vision backward and never runs beside a frame-resident
        launch.  ``comm_timing`` records per-bucket events; read them with
        comm_stats() after a sync."""
        r = self.runner
        r.pack(self.flat, self.packed)
        logits, values, _, _, _ = r.forward(self.flat, self.packed, self.basis, frames, self.ws, want_attn=False)
        if self.world == 1:
            r.backward(self.flat, self.packed, self.basis, frames, self.ws, dlogits, dvalues, grads=self.grads)
            N.pair_flag(self.guard)
            return logits, values
        main = torch.cuda.current_stream(self.device)
        self._events = [] if comm_timing else None
        issue = dict(self.schedule[bool(overlap)])
        for phase in (N.BWD_HEAD, N.BWD_CORE, N.BWD_VISION):
            r.backward(self.flat, self.packed, self.basis, frames, self.ws, dlogits, dvalues, grads=self.grads,
                       phases=phase)
            if phase == N.BWD_CORE:   # every resident launch of this step is enqueued by now
                N.pair_flag(self.guard)
            if phase in issue:
                self._allreduce(main, issue[phase], comm_timing)
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
                allreduce_buckets(self._gbuf, [(lo, hi)], self.group, async_op=False)
                if timing:
                    t1 = torch.cuda.Event(enable_timing=True)
                    t1.record(self.comm)
                    self._events.append((lo, hi, ready, t0, t1))

    def comm_stats(self):
        """Per-bucket all-reduce time (ms) and the communication left exposed
        after the last backward phase (ms) of the last timed step()."""
        if not getattr(self, "_events", None):
            raise RuntimeError("comm_stats(): the last step() ran without comm_timing=True (or on one rank)")
        o_core, n = self.bounds[1][0], self.runner.n_params
        names = {(o_core, n + 1): "HEAD+CORE (+guard)", (0, o_core): "VISION", (0, n + 1): "ALL (+guard)"}
        buckets = []
        for lo, hi, ready, t0, t1 in self._events:
            buckets.append({"bucket": names.get((lo, hi), f"[{lo},{hi})"), "bytes": 4 * (hi - lo),
                            "allreduce_ms": round(t0.elapsed_time(t1), 4),
                            "queued_after_phase_ms": round(ready.elapsed_time(t0), 4)})
        last = self._events[-1][4]
        exposed = max(0.0, self._compute_done.elapsed_time(last))
        return {"buckets": buckets, "exposed_ms": round(exposed, 4),
                "policy": "no collective beside a frame-resident launch: HEAD+CORE reduced after CORE, VISION last"}

    def check_health(self):
        """Raise if a frame-resident launch of this rank timed out waiting for a
        partner since the last check (syncs the stream; the guarded Adam has
        already refused such a step's update on every rank)."""
        n = N.pair_status(clear=True)
        if n:
            raise RuntimeError(f"aaa: {n} partner wait(s) of a frame-resident launch timed out; the affected "
                               f"step's optimizer update was skipped on every rank")

    def optimizer_step(self):
        """Adam (lr=1e-3, torch defaults; main_mp.py:92) on the flat params, one
        launch, skipped on the device when the guard slot is non-zero."""
        self.opt_steps += 1
        adam_flat_(self.flat, self.grads, self.exp_avg, self.exp_avg_sq, self.opt_steps, lr=self.lr, guard=self.guard)

    def train_step(self, frames, dlogits, dvalues, overlap: bool = True):
        out = self.step(frames, dlogits, dvalues, overlap=overlap)
        self.optimizer_step()
        return out
