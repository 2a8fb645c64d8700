"""Actor-path latency: one environment step of the
reference's Policy.forward (main_mp.py:48-59) at B = 1.

Legs, each over ``--steps`` consecutive steps of one episode (the ConvLSTM
state carries, as in main_mp.py:100), on seeded synthetic uint8 frames:
  policy_item  aaa_amd.policy.Policy.forward: upload uint8 frame, HIP agent
               step, device draw, .item() host sync per step (the reference's
               contract: an int action for env.step)
  policy_async Policy.act: the same without the per-step host sync (one sync at the end)
  graph_item   GraphActor.step: the step captured once as a HIP graph, replayed per
               step, .item() per step (inference / actor-learner split); _chain = the
               actor chain (aaa_actor_step, six small-B launches), _forward = the
               learner's T=1 forward + aaa_sample_actions
  graph_async  GraphActor.step without the per-step sync
  device       graph replays back to back (device time per step, no host copy)
  cpu_ref      the oracle's restatement of the same step (reference op sequence,
               torch CPU fp32, host threads as stated) + softmax/Categorical draw
Prints one JSON line per frame size.  Frames: 210x160 (Seaquest's raw
observation; grid 27x20 = the reference's default SpatialBasis) and 84x84.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import attention  # noqa: E402
from aaa_amd import detinit  # noqa: E402
from aaa_amd.policy import GraphActor, Policy  # noqa: E402


def gpu_legs(H, W, steps, warmup, dev):
    params = detinit.deterministic_params(0, 18, 4)
    agent = attention.Agent(18, grid="auto")
    detinit.load_into(agent, params)
    agent.to(dev)
    pol = Policy(agent, seed=1)
    frames = detinit.frames_u8(77, (steps + warmup, H, W, 3))
    out = {}
    with torch.no_grad():
        for leg in ("policy_item", "policy_async"):
            agent.reset()
            for t in range(warmup):
                pol(frames[t])
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if leg == "policy_item":
                for t in range(steps):
                    pol(frames[warmup + t])
            else:
                for t in range(steps):
                    pol.act(frames[warmup + t])
                torch.cuda.synchronize()
            out[leg] = (time.perf_counter() - t0) / steps * 1e6
            pol.saved_log_probs.clear()
    for chain in (False, True):
        ga = GraphActor(agent, H, W, B=1, seed=1, chain=chain)
        tag = "chain" if chain else "forward"
        for leg in ("graph_item", "graph_async"):
            ga.reset()
            for t in range(warmup):
                int(ga.step(frames[t]).item())
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if leg == "graph_item":
                for t in range(steps):
                    int(ga.step(frames[warmup + t]).item())
            else:
                for t in range(steps):
                    ga.step(frames[warmup + t])
                torch.cuda.synchronize()
            out[f"{leg}_{tag}"] = (time.perf_counter() - t0) / steps * 1e6
        # device time per step: graph replays back to back on a device-resident frame
        dframe = torch.from_numpy(frames[0]).to(dev)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ga.step(dframe)
        ev0.record()
        for t in range(steps):
            ga.graph.replay()
        ev1.record()
        torch.cuda.synchronize()
        out[f"device_{tag}"] = ev0.elapsed_time(ev1) / steps * 1e3
    return out


def cpu_leg(H, W, steps, threads):
    from oracle import ref_cpu
    torch.set_num_threads(threads)
    P = ref_cpu.tensor_params(detinit.deterministic_params(0, 18, 4), requires_grad=False)
    frames = detinit.frames_u8(77, (steps + 1, H, W, 3))
    S = ref_cpu.spatial_basis(*ref_cpu.grid_of(H, W))
    state = None
    with torch.no_grad():
        # one untimed step, then the timed ones (state carried); frames as main_mp.py:53
        x = torch.from_numpy(frames[0]).float().unsqueeze(0).unsqueeze(0)
        *_, state = ref_cpu.unroll(P, x, S=S, state=state, return_state=True)
        t0 = time.perf_counter()
        for t in range(1, steps + 1):
            x = torch.from_numpy(frames[t]).float().unsqueeze(0).unsqueeze(0)
            lg, _, _, state = ref_cpu.unroll(P, x, S=S, state=state, return_state=True)
            probs = torch.softmax(lg[0], dim=-1)                              # main_mp.py:55-58
            dist = torch.distributions.Categorical(probs)
            a = dist.sample()
            dist.log_prob(a)
            int(a.item())
        return (time.perf_counter() - t0) / steps * 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--cpu-steps", type=int, default=20)
    ap.add_argument("--sizes", default="210x160,84x84")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    threads = min(16, len(os.sched_getaffinity(0)))
    for sz in args.sizes.split(","):
        H, W = (int(v) for v in sz.split("x"))
        g = gpu_legs(H, W, args.steps, args.warmup, dev)
        c = cpu_leg(H, W, args.cpu_steps, threads)
        rec = {"metric": "actor step latency (B=1, Policy.forward)", "unit": "us/step", "frame": sz,
               "steps": args.steps, "cpu_ref_us": round(c, 1), "cpu_threads": threads}
        rec.update({f"{k}_us": round(v, 1) for k, v in g.items()})
        rec["chain_graph_speedup_vs_cpu"] = round(c / g["graph_item_chain"], 2)
        rec["chain_vs_forward_device"] = round(g["device_forward"] / g["device_chain"], 2)
        print(json.dumps(rec), flush=True)

if __name__ == "__main__":
    main()
