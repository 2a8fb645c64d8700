"""Data-parallel learner self-check on ONE GPU (tests/test_gpu_dp.py launches it).

Launched by torch.distributed.run with N ranks that all use cuda:0 and the
gloo backend (RCCL refuses two ranks on one device; the driver's N-GPU runs
use RCCL with one rank per GPU).  Each rank runs aaa_amd.learner.Learner.step
on its B rows -- the three backward phases with each gradient bucket
all-reduced while the next phase runs -- and rank 0 checks the summed
gradient (SUM; it replaces main_mp.py:182-184's Hogwild)
against
  (1) a single-process backward of the full batch on the same kernels, and
  (2) the CPU oracle (oracle/ref_cpu.py) on the full batch: fp32 at 1e-4,
      bf16 at 2e-2 against the bf16-emulated oracle,
and that no backward phase writes a gradient range whose all-reduce the
learner's schedule (Learner.schedule: HEAD+CORE after CORE, VISION last)
has already issued.

Environment: AAA_DP_DTYPE fp32|bf16, AAA_DP_B rows per rank (bf16 at 32..128
selects the paired frame-resident kernels, >= 160 the one-workgroup ones on a
256-CU part; fp32 at 16..32 the frame-group kernels), AAA_DP_T unroll length,
AAA_DP_H frame side (168: the band-mode kernels for bf16), AAA_DP_NQ heads.  Prints one JSON line on rank 0; exit
status 1 on a mismatch.

AAA_DP_STRAND=1 instead checks the stranded-launch path across ranks (ADVICE
r04): the LAST rank holds most CUs with a filler past the partner-wait budget
while every rank runs Learner.train_step, so a frame-resident launch times
out.  Every rank must finish the step (no rank raises between its
collectives: the learner defers the API's stranded check), no rank's
parameters or Adam step count may change (the guard slot rides in the
HEAD+CORE all-reduce), check_health() must raise on a stranded rank, and a
clean step afterwards must update every rank identically.
"""
import json
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import attention  # noqa: E402,F401
from aaa_amd import _native as N, detinit  # noqa: E402
from aaa_amd.learner import Learner  # noqa: E402
from aaa_amd.runtime import UnrollRunner  # noqa: E402


def rel(a, b):
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


def oracle_grads(X, Gl, Gv, dtype, A, nq):
    """Per-tensor gradients of the CPU oracle on the full batch (fp32 reference
    op sequence, or its bf16-emulated form for the bf16 path)."""
    from oracle import ref_cpu
    torch.set_num_threads(int(os.environ.get("AAA_DP_ORACLE_THREADS", "16")))
    P = ref_cpu.tensor_params(detinit.deterministic_params(0, A, nq))
    lg, vl, _ = ref_cpu.unroll(P, X, nq=nq, conv_mode="bf16" if dtype == "bf16" else "fp32")
    ((lg * Gl).sum() + (vl * Gv).sum()).backward()
    return {n: (p.grad if p.grad is not None else torch.zeros_like(p)) for n, p in P.items()}


def strand_check(rank, world, dev):
    import ctypes
    import time
    dtype, b, T, H, nq, A = "bf16", int(os.environ.get("AAA_DP_B", "32")), 20, 84, 4, 18
    lr = Learner(b, T, H, H, nq, A, dtype, dev, frames_u8=True)
    X = torch.from_numpy(detinit.frames_u8(1234 + rank, (T, b, H, H, 3))).to(dev)
    Gl = torch.from_numpy(detinit.normal(2 + rank, (T, b, A))).to(dev)
    Gv = torch.from_numpy(detinit.normal(3 + rank, (T, b, A))).to(dev)
    lr.step(X, Gl, Gv)                 # clean step: settles the guard's snapshot
    torch.cuda.synchronize()
    N.pair_status(clear=True)
    before = lr.flat.clone()
    res = {"mode": "strand", "world": world, "B_per_rank": b}
    dist.barrier()
    stranded_rank = world - 1
    if rank == stranded_rank:
        lib = ctypes.CDLL(os.path.join(ROOT, "tests", "native", "libaaa_filler.so"))
        lib.aaa_test_filler.argtypes = [ctypes.c_int, ctypes.c_long, ctypes.c_void_p, ctypes.c_void_p]
        side = torch.cuda.Stream(dev)
        sink = torch.zeros(4096, device=dev)
        # 200 of 256 CUs: the ranks' two paired grids (2 * b workgroups each) cannot all be placed
        assert lib.aaa_test_filler(200, 1_900_000, sink.data_ptr(), side.cuda_stream) == 0
        time.sleep(0.005)
    raised = None
    try:
        lr.train_step(X, Gl, Gv)
    except RuntimeError as e:       # the property under test: this must not happen
        raised = str(e)
    torch.cuda.synchronize()
    unchanged = bool(torch.equal(lr.flat, before))
    steps = lr.opt_steps
    try:
        lr.check_health()
        health = "quiet"
    except RuntimeError:
        health = "raised"
    # ranks share one GPU here, so the filler may strand any rank's launch; check_health() decides
    # from the all-reduced guard slot, so when one rank raises EVERY rank must (a rank
    # that stays quiet would wait forever in the next step's all-reduce for the one that left)
    hv = torch.tensor([1.0 if health == "raised" else 0.0])
    anyh, allh = hv.clone(), hv.clone()
    dist.all_reduce(anyh, op=dist.ReduceOp.MAX)
    dist.all_reduce(allh, op=dist.ReduceOp.MIN)
    # the premise: the filler stranded some rank's launch (it need not: placement on an idle box
    # can leave every partner co-resident) -- otherwise the step was an ordinary one everywhere
    stranded = anyh.item() == 1.0
    res["health_all_ranks_agree"] = anyh.item() == allh.item()
    ok = raised is None and unchanged and steps == 0 and stranded and res["health_all_ranks_agree"]
    lr.train_step(X, Gl, Gv)           # clean: every rank updates, identically
    torch.cuda.synchronize()
    lr.check_health()
    moved = not torch.equal(lr.flat, before)
    digest = torch.tensor([float(lr.flat.double().sum()), float(lr.opt_steps)], dtype=torch.float64)
    allv = [torch.zeros_like(digest) for _ in range(world)]
    dist.all_gather(allv, digest)
    same = all(torch.equal(allv[0], v) for v in allv)
    if stranded:
        ok = ok and moved and same and lr.opt_steps == 1
    else:   # nothing stranded: both steps ordinary, still identical on every rank
        ok = raised is None and moved and same and lr.opt_steps == 2
    res["stranded"] = stranded
    flags = torch.tensor([1.0 if ok else 0.0])
    dist.all_reduce(flags, op=dist.ReduceOp.MIN)
    res.update({"raised_mid_step": raised, "params_unchanged_after_stranded_step": unchanged,
                "adam_steps_after_stranded_step": steps, "health_rank": health, "clean_step_moved": moved,
                "ranks_identical_after_clean_step": same, "ok": bool(flags.item() == 1.0)})
    if rank == 0 or not ok:
        print(json.dumps({"rank": rank, **res}), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    if not res["ok"]:
        sys.exit(1)


def main():
    dist.init_process_group(os.environ.get("AAA_DP_BACKEND", "gloo"))
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    if os.environ.get("AAA_DP_STRAND") == "1":
        return strand_check(rank, world, dev)
    dtype = os.environ.get("AAA_DP_DTYPE", "fp32")
    b = int(os.environ.get("AAA_DP_B", "2"))
    T = int(os.environ.get("AAA_DP_T", "3"))
    H = int(os.environ.get("AAA_DP_H", "84"))       # square frames: 84 (11x11 grid) or 168 (21x21, band mode)
    nq = int(os.environ.get("AAA_DP_NQ", "4"))
    A, Bt = 18, b * world
    tol = 2e-2 if dtype == "bf16" else 1e-4
    X = torch.from_numpy(detinit.frames_u8(1234, (T, Bt, H, H, 3)).astype(np.float32))
    Gl = torch.from_numpy(detinit.normal(2, (T, Bt, A)))
    Gv = torch.from_numpy(detinit.normal(3, (T, Bt, A)))
    rows = slice(rank * b, (rank + 1) * b)
    res = {"world": world, "backend": dist.get_backend(), "dtype": dtype, "B_per_rank": b, "T": T, "H": H, "nq": nq}
    ok = True
    grads_dp = None
    for overlap in (True, False):
        lr = Learner(b, T, H, H, nq, A, dtype, dev)
        N.timing_enable(True)
        lr.step(X[:, rows].contiguous().to(dev), Gl[:, rows].contiguous().to(dev), Gv[:, rows].contiguous().to(dev),
                overlap=overlap, comm_timing=True)
        torch.cuda.synchronize()
        variants = {k: N.timing_stats(k)["variant"] for k in (N.TIMER_FWD_STEP, N.TIMER_BPTT_STEP)}
        N.timing_enable(False)
        cs = lr.comm_stats()
        assert len(cs["buckets"]) == len(lr.schedule[overlap]) and all(x["allreduce_ms"] >= 0 for x in cs["buckets"]), cs
        assert N.pair_status(clear=True) == 0, "a paired kernel's partner wait timed out"
        if rank == 0:   # (1) single-process full batch, same weights
            r = UnrollRunner(Bt, T, H, H, nq, A, dtype, dev)
            pk, ws = r.new_packed(), r.new_workspace()
            r.pack(lr.flat, pk)
            r.forward(lr.flat, pk, lr.basis, X.to(dev), ws, want_attn=False)
            g, _, _ = r.backward(lr.flat, pk, lr.basis, X.to(dev), ws, Gl.to(dev), Gv.to(dev))
            torch.cuda.synchronize()
            err = rel(lr.grads, g)
            res[f"vs_single_process(overlap={overlap})"] = err
            ok &= err <= (5e-3 if dtype == "bf16" else 1e-5)
            res["variants_per_rank"] = variants
            grads_dp = lr.grads.detach().cpu()
            layout = (r.offsets, r.sizes)
        dist.barrier()
    if rank == 0:   # (2) the oracle on the full batch
        ref = oracle_grads(X, Gl, Gv, dtype, A, nq)
        offs, sizes = layout
        worst = 0.0
        for (name, shape), o, n in zip(detinit.param_shapes(A, nq), offs, sizes):
            gr = ref[name].reshape(-1).float()
            gd = grads_dp[o:o + n]
            if float(gr.norm()) == 0.0:
                ok &= float(gd.abs().max()) == 0.0
                continue
            worst = max(worst, rel(gd, gr))
        res["vs_oracle_worst_rel"] = worst
        ok &= worst <= tol
        # (3) phase -> bucket write disjointness: poison the grads, run each
        # phase alone, and check that it changed nothing outside its bucket
        r = UnrollRunner(b, T, H, H, nq, A, dtype, dev)   # (lr: the last learner; no new collective here)
        pk, ws = r.new_packed(), r.new_workspace()
        r.pack(lr.flat, pk)
        Xr = X[:, rows].contiguous().to(dev)
        r.forward(lr.flat, pk, lr.basis, Xr, ws, want_attn=False)
        gbuf = torch.full((r.n_params,), float("nan"), device=dev)
        issued = []   # ranges whose all-reduce the schedule has already started
        sched = dict(lr.schedule[True])
        for phase in (N.BWD_HEAD, N.BWD_CORE, N.BWD_VISION):
            before = gbuf.clone()
            r.backward(lr.flat, pk, lr.basis, Xr, ws, Gl[:, rows].contiguous().to(dev),
                       Gv[:, rows].contiguous().to(dev), grads=gbuf, phases=phase)
            torch.cuda.synchronize()
            changed = ~((gbuf == before) | (torch.isnan(gbuf) & torch.isnan(before)))
            bad = sum(int(changed[a:z].sum()) for a, z in issued)
            res[f"phase{phase}_writes_into_issued_buckets"] = bad
            ok &= bad == 0
            issued += sched.get(phase, [])
        res["ok"] = bool(ok)
        print(json.dumps(res), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    if rank == 0 and not ok:
        sys.exit(1)


if __name__ == "__main__":
    main()
