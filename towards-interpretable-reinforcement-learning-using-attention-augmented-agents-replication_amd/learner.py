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
partner timeouts reported on this device since the previous step
(aaa_pair_flag: a device-side snapshot of a monotonic word, so no host call
can consume them first) after the CORE phase; it rides in the HEAD+CORE
all-reduce, so every rank sees any rank's timeout, and the fused Adam skips
the update on the device when it is non-zero -- gradients of a stranded
launch never reach the parameters, with no host sync.  The Adam step count
lives on the device too (aaa_adam_step_counted), advanced only by an applied
update, so a skipped step leaves the bias corrections where they were.  The
learner's runner defers the API's own stranded check (AAA_FLAG_DEFER_STRANDED):
no rank can raise between its collectives and leave its peers waiting in an
unmatched all-reduce; ``check_health()`` raises after the step instead.
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
        self.runner = r = UnrollRunner(B, T, H, W, nq, A, dtype, device, frames_u8=frames_u8, defer_stranded=True)
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
        # this learner's own snapshot of the device's partner-timeout word (aaa_pair_flag_at): no
        # other reader on the device (another learner, a bench, a diagnostic) can take its timeouts;
        # synced to the current word now, so timeouts from before this learner existed are not its own
        self._pair_base = torch.zeros(1, dtype=torch.int32, device=self.device)
        N.pair_flag(self.guard, base=self._pair_base)
        self._gbuf.zero_()
        self.lr = lr
        self.exp_avg = torch.zeros_like(self.grads)
        self.exp_avg_sq = torch.zeros_like(self.grads)
        self.step_dev = torch.zeros(1, dtype=torch.int32, device=self.device)   # Adam updates applied
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
            N.pair_flag(self.guard, base=self._pair_base)
            return logits, values
        main = torch.cuda.current_stream(self.device)
        self._events = [] if comm_timing else None
        issue = dict(self.schedule[bool(overlap)])
        for phase in (N.BWD_HEAD, N.BWD_CORE, N.BWD_VISION):
            r.backward(self.flat, self.packed, self.basis, frames, self.ws, dlogits, dvalues, grads=self.grads,
                       phases=phase)
            if phase == N.BWD_CORE:   # every resident launch of this step is enqueued by now
                N.pair_flag(self.guard, base=self._pair_base)
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

    @property
    def opt_steps(self) -> int:
        """Adam updates applied so far (reads the device counter: syncs)."""
        return int(self.step_dev.item())

    def check_health(self):
        """Raise if a frame-resident launch of ANY rank timed out waiting for a
        partner in the last step (syncs the stream).  The decision is the guard
        slot, which the HEAD+CORE all-reduce summed over the ranks, so every rank
        sees the same value and all ranks raise together -- none goes on into the
        next step's collective while a peer has left.  The host-side
        count is consumed too (it would otherwise fail the next API call of this
        process); the guarded Adam has already refused the step's update."""
        g = float(self.guard.item())
        n = N.pair_status(clear=True)
        if g != 0.0 or n:
            raise RuntimeError(f"aaa: {int(g)} partner wait(s) of a frame-resident launch timed out on the "
                               f"ranks ({n} on this one); the step's optimizer update was skipped on every rank")

    def optimizer_step(self):
        """Adam (lr=1e-3, torch defaults; main_mp.py:92) on the flat params, one
        launch, skipped on the device when the guard slot is non-zero (and then
        not counted: the device step counter advances only on an update)."""
        adam_flat_(self.flat, self.grads, self.exp_avg, self.exp_avg_sq, 0, lr=self.lr, guard=self.guard,
                   step_dev=self.step_dev)

    def train_step(self, frames, dlogits, dvalues, overlap: bool = True):
        out = self.step(frames, dlogits, dvalues, overlap=overlap)
        self.optimizer_step()
        return out
