#!/usr/bin/env python
"""Learner-throughput benchmark (BASELINE.json metric).

One step = pack weights -> T-step unroll forward -> loss cotangents ->
backward with all 34 parameter gradients ready (and SUM-all-reduced over
ranks when N > 1).  The optimizer is excluded, as the metric defines.
value = frames (B*T per rank, all ranks) / max-over-ranks wall time of K steps.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c4|c5]

N > 1 is launched by the driver with torch.distributed.run (one rank per GPU,
RCCL).  Rank 0 prints ONE JSON line.  Inputs are synthetic (seeded uint8
frames cast to fp32, seeded weights of the reference architecture).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "learner frames/sec (fwd+bwd, T=20 unroll) at 1/2/4/8 MI355X + % roofline"
PEAK_TFLOPS = {"fp32": 157.3, "bf16": 2500.0}   # MI355X dense MFMA (MI355X_MICROARCH.md)
# The fp32 path's GEMMs run on the bf16 MFMA with each fp32 operand split into three bf16 parts and
# six products per fp32 product (gemm.h SPLIT6, AAA_F32_SPLIT6, default on): their ceiling is the
# bf16 dense peak / 6 in fp32-product FLOP/s, not the fp32 MFMA's 157.3.
SPLIT6_PEAK = 2500.0 / 6


def split6_on(dtype):
    return dtype == "fp32" and os.environ.get("AAA_F32_SPLIT6", "1") != "0"
CONFIGS = {
    "c2": dict(B=32, T=20, H=84, W=84, nq=4, dtype="fp32",
               desc="C2 (BASELINE.json configs[1]): B=32 per GPU x T=20 unroll, 84x84, 4 heads, fp32"),
    "c3": dict(B=256, T=20, H=84, W=84, nq=4, dtype="bf16",
               desc="C3: B=256 per GPU x T=20, 84x84, 4 heads, bf16 conv/ConvLSTM operands"),
    "c4": dict(B=128, T=20, H=84, W=84, nq=4, dtype="bf16",
               desc="C4: B=128 per GPU (1024 over 8) x T=20, 84x84, 4 heads, bf16"),
    "c5": dict(B=64, T=50, H=168, W=168, nq=8, dtype="bf16",
               desc="C5: B=64 per GPU (512 over 8) x T=50, 168x168, 8 heads, bf16"),
}
# Dense algorithmic FLOP per frame, fwd+bwd (SURVEY.md §8d / BASELINE.md).
FLOP_PER_FRAME = {(84, 4): 684.7e6, (168, 8): 2487.4e6}


def log(msg):
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def flop_per_frame(H, W, nq, A=18):
    if (H, nq) in FLOP_PER_FRAME and H == W:
        return FLOP_PER_FRAME[(H, nq)]
    def o(n, k, s, p):
        return (n + 2 * p - k) // s + 1
    H1, W1 = o(H, 8, 4, 1), o(W, 8, 4, 1)
    P1, P = H1 * W1, o(H1, 4, 2, 2) * o(W1, 4, 2, 2)
    c1 = 2 * P1 * 32 * 192
    fwd = (c1 + 2 * P * 64 * 512 + 2 * P * 512 * 1728 + 2 * P * nq * (72 + 184)
           + 2 * ((256 * nq + 2) * 512 + 512 * 256) + 2 * 256 * 1024 + 2 * 256 * 2 * A)
    return 3 * fwd - c1


def attention_hbm(ka):
    """Achieved HBM GB/s of the fused attention readout kernels:
    the library's algorithmic bytes of each launch (forward reads the ConvLSTM
    output O and writes the attention map and answer row; backward reads O, the
    map and the answer grad, writes dO and dQ) over its event-timed duration."""
    from aaa_amd import _native as N
    names = {N.TIMER_ATTN_FWD: "attention readout fwd (softmax over P, fused)",
             N.TIMER_ATTN_BWD: "attention readout bwd"}
    out = {}
    for k, v in ka.items():
        if v["launches"] == 0:
            continue
        per_launch = v["work"] / v["launches"]
        avg_s = v["ms"] / v["launches"] * 1e-3
        gbps = per_launch / avg_s / 1e9
        out[names[k]] = {"avg_us": round(avg_s * 1e6, 2), "launches": v["launches"], "bytes_per_launch": round(per_launch),
                         "achieved_GBps": round(gbps, 1), "peak_GBps": 8000.0, "frac": round(gbps / 8000.0, 4),
                         "variant": v["variant"]}
    return out


def _cpu_threads():
    """Host threads for the CPU baseline: every CPU in this process's affinity
    mask, capped by OMP_NUM_THREADS when the box sets it (the
    GPU box's CPU share is 16 threads per GPU; its affinity mask shows the
    whole machine)."""
    aff = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS")
    return (min(aff, int(omp)) if omp and omp.isdigit() and int(omp) > 0 else aff), aff


def cpu_baseline(cfg):
    """Time the CPU oracle (the reference op sequence, oracle/ref_cpu.py) on the
    host: the bench config's shape (B capped at 32) for ~10 s of whole
    iterations, and config 1 (BASELINE.json configs[0]: B=1, T=20) for ~5 s."""
    import numpy as np
    import torch
    from oracle import ref_cpu
    from aaa_amd import detinit
    cores, aff = _cpu_threads()
    torch.set_num_threads(cores)
    T, nq = cfg["T"], cfg["nq"]
    B = min(cfg["B"], 32)
    H, W = cfg["H"], cfg["W"]
    # the reference's CPU path is fp32 whatever the GPU config computes in
    # (SURVEY.md §8d): never the bf16-emulated oracle
    mode = "fp32"
    P = ref_cpu.tensor_params(detinit.deterministic_params(0, 18, nq))

    def it(Tn, Bn, Hn, Wn, md):
        for p in P.values():
            p.grad = None
        X = torch.from_numpy(detinit.frames_u8(1234, (Tn, Bn, Hn, Wn, 3)).astype(np.float32))
        lg, vl, _ = ref_cpu.unroll(P, X, nq=nq, conv_mode=md)
        Gl = torch.from_numpy(detinit.normal(2, tuple(lg.shape)))
        Gv = torch.from_numpy(detinit.normal(3, tuple(vl.shape)))
        ((lg * Gl).sum() + (vl * Gv).sum()).backward()

    def timed(Tn, Bn, Hn, Wn, md, budget):
        n, t0 = 0, time.perf_counter()
        while True:                      # bounded sample of whole iterations
            it(Tn, Bn, Hn, Wn, md)
            n += 1
            dt = time.perf_counter() - t0
            if dt >= budget or n >= 50:
                return n, dt

    it(2, 2, H, W, mode)   # warm-up
    n, dt = timed(T, B, H, W, mode, 10.0)
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            model = next((l.split(":", 1)[1].strip() for l in f if l.startswith("model name")), "")
    except OSError:
        pass
    out = {"value": round(n * B * T / dt, 3), "unit": "frames/s", "cores": cores, "kind": "port",
           "sample": f"{n} iterations of oracle/ref_cpu.py (the reference's fp32 op sequence, torch CPU {mode}), "
                     f"B={B} x T={T}, {H}x{W}, nq={nq}, {dt:.1f} s on {cores} threads ({model}; "
                     f"affinity mask {aff} CPUs, OMP_NUM_THREADS={os.environ.get('OMP_NUM_THREADS', 'unset')})"}
    if nq == 4:   # config 1 (BASELINE.json configs[0]): the reference's CPU-runnable case, fp32
        it(2, 1, 84, 84, "fp32")
        n1, dt1 = timed(20, 1, 84, 84, "fp32", 5.0)
        out["c1"] = {"value": round(n1 * 20 / dt1, 3), "unit": "frames/s", "ms_per_iteration": round(dt1 / n1 * 1e3, 1),
                     "sample": f"{n1} iterations of B=1 x T=20, 84x84, fp32, fwd+bwd, {dt1:.1f} s on {cores} threads"}
    return out


def dropin_api(cfg, dev, frames, dl, dv, steps, flat):
    """The same iteration through the public drop-in API (what a reference user
    runs): ``attention.Agent.unroll`` -> loss -> ``loss.backward()`` into the
    parameters' ``.grad`` (autograd Function, per-call workspace, weight
    re-pack only when a parameter changed), timed like the main line."""
    import torch
    import attention
    B, T, H, W, nq = cfg["B"], cfg["T"], cfg["H"], cfg["W"], cfg["nq"]
    h, w = (((H + 2 - 8) // 4 + 1) + 4 - 4) // 2 + 1, (((W + 2 - 8) // 4 + 1) + 4 - 4) // 2 + 1
    agent = attention.Agent(18, num_queries=nq, grid=(h, w), conv_dtype=cfg["dtype"]).to(dev)
    with torch.no_grad():
        off = 0
        for p in agent.parameters():
            p.copy_(flat[off:off + p.numel()].view_as(p))
            off += p.numel()

    def it():
        agent.reset()
        agent.zero_grad(set_to_none=True)
        lg, vl, _ = agent.unroll(frames)
        ((lg * dl).sum() + (vl * dv).sum()).backward()

    for _ in range(2):
        it()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        it()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return {"value": round(B * T * steps / dt, 2), "unit": "frames/s", "ms_per_step": round(dt / steps * 1e3, 3),
            "path": "attention.Agent.unroll + loss.backward() (autograd .grad), same frames and weights"}


def episode_leg(dev, T_ep=64, H=210, W=160, cpu=True, per_step=True):
    """The reference's own call pattern (main_mp.py:49-59, 62-80): one episode of
    T_ep per-step ``Policy.forward(observation)`` calls -- B = 1, Seaquest's
    210x160 frames, the default 27x20 spatial basis, the ``.item()`` host sync
    every step -- then finish_episode's discounted-return loss and ONE
    ``loss.backward()`` through all T_ep per-step graphs (T_ep separate T=1
    backward calls of the hand-written BPTT).  Reports the host wall time per
    step, the device-side backward, the memory the episode's graph keeps alive
    per step (each step's saved workspace), and the CPU oracle on the same
    episode.  Bounded: T_ep = 64 (main_mp.py:151 allows 10,000 steps; the memory
    column says what that would hold)."""
    import numpy as np
    import torch
    import attention
    from aaa_amd import detinit
    from aaa_amd.policy import Policy
    agent = attention.Agent(18).to(dev)          # default SpatialBasis(27, 20): 210x160 frames (Q4)
    detinit.load_into(agent, detinit.deterministic_params(0, 18))
    agent.to(dev)
    policy = Policy(agent, seed=0)
    obs = detinit.frames_u8(4321, (T_ep, H, W, 3))
    rewards = (detinit.frames_u8(4322, (T_ep,)) % 3).astype(np.float32).tolist()
    gamma, eps = 0.99, np.finfo(np.float32).eps.item()

    def finish():   # main_mp.py:62-77, verbatim in torch ops
        R, returns = 0.0, []
        for r in rewards[::-1]:
            R = r + gamma * R
            returns.insert(0, R)
        returns = torch.tensor(returns, device=dev)
        returns = (returns - returns.mean()) / (returns.std() + eps)
        return torch.cat([-lp * Rt for lp, Rt in zip(policy.saved_log_probs, returns)]).sum()

    def episode(n):
        agent.reset()
        agent.zero_grad(set_to_none=True)
        policy.saved_log_probs = []
        for t in range(n):
            policy(obs[t])
        return finish()

    def measure_one():
        torch.cuda.synchronize()
        base = torch.cuda.memory_allocated(dev)
        torch.cuda.reset_peak_memory_stats(dev)
        t0 = time.perf_counter()
        loss = episode(T_ep)
        t1 = time.perf_counter()
        held = torch.cuda.memory_allocated(dev) - base
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        loss.backward()
        e1.record()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        peak = torch.cuda.max_memory_allocated(dev) - base
        return {"ms_per_step_host": round((t1 - t0) / T_ep * 1e3, 3),
                "backward_ms_device": round(e0.elapsed_time(e1), 3), "backward_ms_host": round((t2 - t1) * 1e3, 3),
                "episode_frames_per_s": round(T_ep / (t2 - t0), 1),
                "graph_bytes_per_step": int(held // T_ep), "peak_bytes_per_step": int(peak // T_ep)}

    def measure(reps=5):
        # The host-bound leg moves with the box's host speed and scheduling noise: time
        # `reps` whole episodes and report the median one, with every episode's rate listed.
        episode(T_ep).backward()                 # warm-up (code objects; the segment workspace's allocator block)
        runs = sorted((measure_one() for _ in range(reps)), key=lambda r: r["episode_frames_per_s"])
        return {**runs[reps // 2], "episodes_timed": reps,
                "episode_frames_per_s_all": [r["episode_frames_per_s"] for r in runs]}

    agent.fuse_episode_backward = True
    out = {"pattern": "main_mp.py: T_ep x Policy.forward(obs) (B=1, 210x160, default basis, .item() per step) "
                      "-> finish_episode loss -> one loss.backward()",
           "steps": T_ep, **measure(),
           "path": "fused episode backward (episode.py): per-step forwards record into one episode; the backward "
                   "re-runs it as 64-step unrolls from checkpointed states, one hand-written BPTT call each",
           "note": "graph_bytes_per_step x main_mp.py:151's max_steps (10,000) is the device memory one "
                   "full-length episode's autograd graph would hold"}
    if per_step:
        agent.fuse_episode_backward = False
        out["per_step_path"] = {**measure(), "path": "one T=1 autograd node (own workspace) per step, T_ep backward calls"}
        agent.fuse_episode_backward = True
    if cpu:
        from oracle import ref_cpu
        cores, _ = _cpu_threads()
        torch.set_num_threads(cores)
        P = ref_cpu.tensor_params(detinit.deterministic_params(0, 18))
        X = torch.from_numpy(obs.astype(np.float32)).unsqueeze(1)    # (T_ep, 1, H, W, 3)
        c0 = time.perf_counter()
        lg, _, _ = ref_cpu.unroll(P, X, nq=4)                          # the reference op sequence, step by step
        R, returns = 0.0, []
        for r in rewards[::-1]:
            R = r + gamma * R
            returns.insert(0, R)
        returns = torch.tensor(returns)
        returns = (returns - returns.mean()) / (returns.std() + eps)
        acts = torch.from_numpy(detinit.frames_u8(4323, (T_ep,)).astype(np.int64) % 18)
        logp = torch.log_softmax(lg[:, 0], dim=1).gather(1, acts[:, None])[:, 0]
        (-(logp * returns)).sum().backward()
        c1 = time.perf_counter()
        out["cpu_oracle"] = {"ms_per_step": round((c1 - c0) / T_ep * 1e3, 2), "episode_frames_per_s":
                             round(T_ep / (c1 - c0), 1), "cores": cores,
                             "sample": f"one {T_ep}-step episode, oracle/ref_cpu.py fp32 (forward step by step "
                                       "+ finish_episode loss + backward)"}
    return out


def pmc_traffic(config, world, variant):
    """HBM bytes per launch of the dispatched kernel from the committed PMC
    passes (tools/pmc_cfg_r04.sh -> tools/pmc_traffic.py ->
    profiles/rNN/pmc_traffic_<config>.json, newest round first).  rocprofv3
    counters cannot be read from inside the timed run, so the value comes from
    a profile of the same config -- attached only when that profile holds the
    kernel the library reports it dispatched (the ``[kernel: a+b]`` marker of
    the variant: every substring must be in the profiled kernel's name);
    otherwise null with the reason."""
    import glob
    import re
    if world != 1:
        return {"traffic": None, "traffic_note": "PMC passes are single-GPU"}
    m = re.search(r"\[kernel: ([^\]]+)\]", variant or "")
    if not m:
        return {"traffic": None, "traffic_note": "the dispatched variant names no kernel"}
    subs = m.group(1).split("+")
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", f"pmc_traffic_{config}.json")), reverse=True):
        d = json.load(open(f))
        hits = [(k, e) for k, e in d.get("kernels", {}).items()
                if all(s in k for s in subs) and "hbm_bytes_per_launch" in e]
        if hits:
            k, e = max(hits, key=lambda kv: kv[1]["hbm_bytes_per_launch"])
            return {"traffic": round(e["hbm_bytes_per_launch"]), "traffic_unit": "bytes/launch",
                    "traffic_source": os.path.relpath(f, ROOT) + " (2*FETCH_SIZE + WRITE_SIZE, rocprofv3 --pmc)",
                    "traffic_kernel": k[:160], "pmc_mfma_util": e.get("mfma_util"),
                    "pmc_lds_conflict_rate": e.get("lds_conflict_rate")}
    return {"traffic": None, "traffic_note": f"no committed PMC profile of {subs} for {config}"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-dropin", action="store_true", help="skip the drop-in Agent API measurement")
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--no-episode", action="store_true", help="skip the main_mp.py episode leg (C2 line only)")
    ap.add_argument("--frames", default="u8", choices=["u8", "fp32"],
                    help="frame dtype in HBM: u8 (the environment's observation, cast in-kernel) or fp32 "
                         "(cast on the host as main_mp.py:53 does)")
    ap.add_argument("--no-kernel-timing", action="store_true",
                    help="A/B check only: time the steps without the library's per-kernel HIP events")
    ap.add_argument("--timed-steps", type=int, default=1,
                    help="how many of the last timed steps carry the library's per-kernel HIP events "
                         "(1: the last step only, ~0.4 %% of the run's time; K: every timed step)")
    ap.add_argument("--backend", default=os.environ.get("AAA_BENCH_BACKEND", "nccl"), choices=["nccl", "gloo"],
                    help="process-group backend for N > 1 (nccl = RCCL, the measured path; gloo only for the "
                         "one-GPU rehearsal of the N > 1 branch in tests/test_gpu_bench_dp.py)")
    ap.add_argument("--same-device", action="store_true",
                    default=os.environ.get("AAA_BENCH_SAME_DEVICE") == "1",
                    help="every rank on cuda:0 (the one-GPU rehearsal; RCCL refuses two ranks on one device)")
    ap.add_argument("--batch", type=int, default=0,
                    help="rows per rank instead of the config's (rehearsal only: two ranks sharing one GPU must "
                         "keep their frame-resident grids within half the CUs each)")
    args = ap.parse_args()
    cfg = dict(CONFIGS[args.config])
    if args.batch:
        cfg["B"] = args.batch
        cfg["desc"] = cfg["desc"] + f" [--batch {args.batch} per rank: rehearsal override]"

    import numpy as np
    import torch
    import torch.distributed as dist
    import attention  # noqa: F401  (registers aaa_amd)
    from aaa_amd import _native as N, detinit
    from aaa_amd.learner import Learner
    from aaa_amd.parallel import init_from_env

    local = 0 if args.same_device else int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)            # before the process group: RCCL binds this rank to its GPU
    dev = torch.device("cuda", local)
    rank, world, _ = init_from_env(args.backend, device=dev)
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using {world}")
    B, T, H, W, nq, dtype = cfg["B"], cfg["T"], cfg["H"], cfg["W"], cfg["nq"], cfg["dtype"]
    A = 18
    learner = Learner(B, T, H, W, nq, A, dtype, dev, frames_u8=args.frames == "u8")
    frames = torch.from_numpy(detinit.frames_u8(1234 + rank, (T, B, H, W, 3))).to(dev)
    if args.frames == "fp32":
        frames = frames.float()
    dl = torch.from_numpy(detinit.normal(2 + 7 * rank, (T, B, A))).to(dev)   # N(0,1), SURVEY.md §8d
    dv = torch.from_numpy(detinit.normal(3 + 7 * rank, (T, B, A))).to(dev)
    log(f"rank {rank}/{world} {cfg['desc']} workspace {learner.runner.ws_bytes / 2**20:.0f} MiB")

    for i in range(args.warmup):
        learner.step(frames, dl, dv, overlap=not args.no_overlap)
    torch.cuda.synchronize()
    log(f"warm-up done ({args.warmup} steps)")

    # Per-kernel HIP events (recorded by the library on its launch stream) are
    # live in the LAST timed step only: an event pair around every launch of
    # every step costs ~7 % of the step time at C2 (4.85 vs 4.54 ms/step,
    # tools/ab_timing.sh), so the sample keeps that cost to 1/K of it.
    timed = 0 if args.no_kernel_timing else max(1, min(args.timed_steps, args.steps))
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        last = i == args.steps - 1
        if timed and i == args.steps - timed:
            N.timing_enable(True)
        learner.step(frames, dl, dv, overlap=not args.no_overlap, comm_timing=last and world > 1)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    allk = {k: N.timing_stats(k) for k in range(N.TIMER_N)}
    kt = {k: allk[k] for k in (N.TIMER_FWD_STEP, N.TIMER_BPTT_STEP, N.TIMER_CORE_WGRAD)}
    ka = {k: allk[k] for k in (N.TIMER_ATTN_FWD, N.TIMER_ATTN_BWD)}
    N.timing_enable(False)
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms = elapsed / args.steps * 1e3
    frames_total = B * T * world * args.steps
    value = frames_total / elapsed
    if args.no_kernel_timing:
        if rank == 0:
            print(json.dumps({"metric": METRIC, "value": round(value, 2), "unit": "frames/s", "n_gpus": world,
                              "steps": args.steps, "ms_per_step": round(ms, 3), "kernel_timing": False}), flush=True)
        return

    # roofline of the dominant kernel class (largest total device time): the
    # library accounts each launch's algorithmic FLOP and names the variant it
    # dispatched (aaa_timing_stats), so nothing here re-derives its dispatch
    names = {N.TIMER_FWD_STEP: "ConvLSTM forward step", N.TIMER_BPTT_STEP: "ConvLSTM BPTT step",
             N.TIMER_CORE_WGRAD: "ConvLSTM weight-gradient GEMM"}
    dom = max(kt, key=lambda k: kt[k]["ms"])
    d = kt[dom]
    avg_ms = d["ms"] / max(d["launches"], 1)
    per_launch = d["work"] / max(d["launches"], 1)
    peak = SPLIT6_PEAK if split6_on(dtype) else PEAK_TFLOPS[dtype]
    achieved = per_launch / (avg_ms * 1e-3) / 1e12
    fpf = flop_per_frame(H, W, nq)
    kernels = {names[k]: {"avg_us": round(v["ms"] / max(v["launches"], 1) * 1e3, 2), "launches": v["launches"],
                          "flop_per_launch": v["work"] / max(v["launches"], 1),
                          "tflops": round(v["work"] / max(v["ms"] * 1e-3, 1e-12) / 1e12, 2),
                          "frac": round(v["work"] / max(v["ms"] * 1e-3, 1e-12) / 1e12 / peak, 4),
                          "variant": v["variant"], **pmc_traffic(args.config, world, v["variant"])}
               for k, v in kt.items() if v["launches"]}
    # the rest of the step, by timer class (library-recorded HIP events of the
    # last timed step): algorithmic FLOP where a GEMM dominates (tail classes
    # priced at the fp32 peak: their operands are fp32), time only for glue
    tail_peak = SPLIT6_PEAK if split6_on(dtype) else PEAK_TFLOPS["fp32"]
    other = {N.TIMER_PACK: ("weight packing", None), N.TIMER_VISION_FWD: ("vision encoder fwd (conv1+conv2)", peak),
             N.TIMER_TAIL_FWD: ("tail fwd (query pack, answer MLP, LSTMCell, heads)", tail_peak),
             N.TIMER_TAIL_BWD: ("tail bwd", tail_peak), N.TIMER_CORE_DX: ("batched dx (conv2-output grad)", peak),
             N.TIMER_VISION_BWD: ("vision bwd (conv2 wgrad+dgrad, conv1 wgrad)", peak),
             N.TIMER_MISC: ("state copies, memsets, bias column sums", None)}
    for k, (nm, pk) in other.items():
        v = allk[k]
        if not v["launches"]:
            continue
        e = {"ms": round(v["ms"], 4), "regions": v["launches"], "variant": v["variant"]}
        if pk and v["work"] > 0:
            e.update({"flop": v["work"], "tflops": round(v["work"] / max(v["ms"] * 1e-3, 1e-12) / 1e12, 2),
                      "frac": round(v["work"] / max(v["ms"] * 1e-3, 1e-12) / 1e12 / pk, 4), "peak_tflops": pk})
        if k == N.TIMER_CORE_DX:
            e.update(pmc_traffic(args.config, world, v["variant"]))
        kernels[nm] = e
    timed_ms = sum(allk[k]["ms"] for k in allk)
    coverage = {"timed_ms": round(timed_ms, 4), "ms_per_step": round(ms, 4), "frac": round(timed_ms / ms, 4),
                "note": "sum of every timer class's HIP-event time in the last timed step / the average step; the "
                        "remainder is launch gaps, host enqueue and the unattributed memsets"}

    out = {
        "metric": METRIC, "value": round(value, 2), "unit": "frames/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": dtype,
        "data": ("synthetic: seeded uint8 frames resident in HBM, cast to fp32 (raw 0..255) inside the first "
                 "kernel" if args.frames == "u8" else "synthetic: seeded uint8 frames cast to fp32 (raw 0..255) on "
                 "the host") + ", seeded uniform weights of the reference architecture, N(0,1) logits/values "
                 "cotangents (seeds 2, 3)",
        "config": {"workload": cfg["desc"], "global_batch": B * world, "seq_len": T, "frame": f"{H}x{W}",
                   "heads": nq, "parallelism": f"dp{world}",
                   **({"arithmetic": "fp32 operands split into three bf16 parts (8+8+8 mantissa bits), six products "
                                     "per fp32 product on the bf16 MFMA, fp32 accumulation (gemm.h SPLIT6); error vs "
                                     "the fp64 evaluation within 2x of the fp32 MFMA's "
                                     "(tests/test_gpu_parity.py::test_f32_split6_accuracy); roofline peak = bf16 "
                                     "dense / 6"} if split6_on(dtype) else {})},
        "roofline": {"bound": "mfma", "kernel": names[dom], "variant": d["variant"], "achieved": round(achieved, 2),
                     "peak": peak, "unit": "TFLOP/s", "frac": round(achieved / peak, 4),
                     **pmc_traffic(args.config, world, d["variant"]),
                     "flop_per_launch": per_launch, "avg_launch_us": round(avg_ms * 1e3, 2),
                     "timed_launches": d["launches"],
                     "timing": f"HIP events around each launch of the last {timed} timed step(s)",
                     **({"peak_fp32_mfma": PEAK_TFLOPS["fp32"],
                         "frac_vs_fp32_mfma": round(achieved / PEAK_TFLOPS["fp32"], 4),
                         "peak_note": "bound = the bf16 MFMA running six split products per fp32 product "
                                      "(bf16 dense 2500 / 6 = 416.7 TFLOP/s fp32-equivalent): the instruction "
                                      "mix the kernel executes; frac_vs_fp32_mfma prices the same work against "
                                      "the fp32 MFMA's 157.3 TFLOP/s dense peak"} if split6_on(dtype) else {})},
        "job_roofline": {"flop_per_frame": fpf, "achieved_tflops_per_gpu": round(value * fpf / world / 1e12, 2),
                         "frac": round(value * fpf / world / 1e12 / peak, 4),
                         **({"frac_vs_fp32_mfma": round(value * fpf / world / 1e12 / PEAK_TFLOPS["fp32"], 4)}
                            if split6_on(dtype) else {})},
        "kernels": kernels,
        "kernel_coverage": coverage,
        "hbm_kernels": attention_hbm(ka),
    }
    # The data-parallel overlap budget: Learner.step issues the
    # HEAD+CORE gradient all-reduce once the CORE phase is enqueued, and only the VISION
    # phase's kernels remain to hide it; the VISION bucket's all-reduce is exposed.
    vb = allk[N.TIMER_VISION_BWD]
    o_core, n_par = learner.bounds[1][0], learner.runner.n_params
    out["overlap_window_ms"] = round(vb["ms"], 4) if vb["launches"] else None
    out["allreduce_buckets_bytes"] = {"HEAD+CORE (+guard)": 4 * (n_par + 1 - o_core), "VISION": 4 * o_core}
    if world > 1:   # RCCL gradient all-reduce of the last timed step, per bucket
        out["comm"] = {**learner.comm_stats(), "backend": dist.get_backend(),
                       "note": "allreduce_ms: RCCL time per bucket on the comm stream; exposed_ms: comm still "
                               "running after the last backward phase finished (the part not overlapped)"}
    # fused Adam (excluded from the metric, which stops at
    # ready gradients): HBM-bound, 28 B per parameter (p, g, m, v read; p, m, v written)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n_opt = 50
    learner.optimizer_step()
    ev0.record()
    for i in range(n_opt):
        learner.optimizer_step()
    ev1.record()
    torch.cuda.synchronize()
    opt_us = ev0.elapsed_time(ev1) / n_opt * 1e3
    opt_bytes = 28 * learner.flat.numel()
    out["optimizer"] = {"kernel": "fused multi-tensor Adam (k_adam)", "avg_launch_us": round(opt_us, 2),
                        "params": learner.flat.numel(), "bytes_per_launch": opt_bytes,
                        "achieved_GBps": round(opt_bytes / (opt_us * 1e-6) / 1e9, 1), "peak_GBps": 8000.0,
                        "note": "working set (63.6 MB) is Infinity-Cache resident when stepped back to back"}
    if world == 1 and not args.no_dropin:
        out["dropin"] = dropin_api(cfg, dev, frames, dl, dv, args.steps, learner.flat)
    if world == 1 and args.config == "c2" and not args.no_episode:
        log("episode leg (main_mp.py call pattern)...")
        out["episode"] = episode_leg(dev, cpu=not args.no_cpu_baseline)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        log("timing the CPU baseline (oracle on host cores)...")
        out["cpu_baseline"] = cpu_baseline(cfg)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
