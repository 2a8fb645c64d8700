"""Host-side profile of the reference's per-step call pattern (bench.episode_leg's
forward half): cProfile over 64 ``Policy.forward`` steps at 210x160, after a
warm-up episode.  Prints the functions by own time.
    python tools/episode_host_profile.py > gpurun_out/episode_host_profile.txt"""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

import attention  # noqa: E402
from aaa_amd import detinit  # noqa: E402
from aaa_amd.policy import Policy  # noqa: E402

if __name__ == "__main__":
    dev = torch.device("cuda:0")
    T_ep = 64
    agent = attention.Agent(18).to(dev)
    detinit.load_into(agent, detinit.deterministic_params(0, 18))
    agent.to(dev)
    policy = Policy(agent, seed=0)
    obs = detinit.frames_u8(4321, (T_ep, 210, 160, 3))

    def episode():
        agent.reset()
        agent.zero_grad(set_to_none=True)
        policy.saved_log_probs = []
        for t in range(T_ep):
            policy(obs[t])

    def episode_async():   # Policy.act: the same steps without the per-step .item() host sync
        agent.reset()
        agent.zero_grad(set_to_none=True)
        policy.saved_log_probs = []
        for t in range(T_ep):
            policy.act(obs[t])

    episode()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    episode()
    torch.cuda.synchronize()
    print(f"ms per step (no profiler): {(time.perf_counter() - t0) / T_ep * 1e3:.3f}")
    t0 = time.perf_counter()
    episode_async()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"ms per step without the .item() sync: host enqueue {(t1 - t0) / T_ep * 1e3:.3f}, "
          f"to device done {(t2 - t0) / T_ep * 1e3:.3f}")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    episode_async()
    e1.record()
    torch.cuda.synchronize()
    print(f"device ms per step (events around the async episode): {e0.elapsed_time(e1) / T_ep:.3f}")
    import gc
    for label in ("gc on", "gc off", "gc on"):
        if label == "gc off":
            gc.disable()
        ts = []
        for _ in range(5):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            episode()
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) / T_ep * 1e3)
        gc.enable()
        ts.sort()
        print(f"{label}: ms per step over 5 episodes: median {ts[2]:.3f} min {ts[0]:.3f} max {ts[-1]:.3f}")
    # one step at a time from an idle device: host time of Policy.act (returns after its launches)
    # and the device time left after it returns
    agent.reset()
    policy.saved_log_probs = []
    hs, ds = [], []
    for t in range(T_ep):
        torch.cuda.synchronize()
        a0 = time.perf_counter()
        act, _ = policy.act(obs[t])
        a1 = time.perf_counter()
        int(act.item())
        a2 = time.perf_counter()
        hs.append(a1 - a0)
        ds.append(a2 - a1)
    hs.sort(), ds.sort()
    print(f"isolated step: Policy.act host median {hs[T_ep // 2] * 1e3:.3f} ms, then .item() wait median "
          f"{ds[T_ep // 2] * 1e3:.3f} ms")
    if "--backward" in sys.argv:   # the bench's whole episode: forward steps + finish_episode loss + backward
        import numpy as np
        rewards = (detinit.frames_u8(4322, (T_ep,)) % 3).astype(np.float32).tolist()
        for _ in range(3):
            episode()
            R, returns = 0.0, []
            for r in rewards[::-1]:
                R = r + 0.99 * R
                returns.insert(0, R)
            returns = torch.tensor(returns, device=dev)
            returns = (returns - returns.mean()) / (returns.std() + 1e-7)
            loss = torch.cat([-lp * Rt for lp, Rt in zip(policy.saved_log_probs, returns)]).sum()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            e0.record()
            loss.backward()
            e1.record()
            torch.cuda.synchronize()
            print(f"backward: host {(time.perf_counter() - t0) * 1e3:.3f} ms, device {e0.elapsed_time(e1):.3f} ms")
        if "--phases" in sys.argv:   # wall-clock phases of the backward (the engine runs it on its own thread)
            from aaa_amd import episode as E
            marks = {}
            st0, ba0 = E.Episode.stash, E.Episode.backward_all

            def stash(self, *a, **k):
                marks.setdefault("first_stash", time.perf_counter())
                marks["last_stash"] = time.perf_counter()
                return st0(self, *a, **k)

            def backward_all(self, *a, **k):
                marks["bwd_all_start"] = time.perf_counter()
                out = ba0(self, *a, **k)
                marks["bwd_all_end"] = time.perf_counter()
                torch.cuda.synchronize()
                marks["bwd_all_synced"] = time.perf_counter()
                return out
            E.Episode.stash, E.Episode.backward_all = stash, backward_all
            for _ in range(3):
                episode()
                loss = torch.cat([-lp * Rt for lp, Rt in zip(policy.saved_log_probs, returns)]).sum()
                torch.cuda.synchronize()
                marks.clear()
                t0 = time.perf_counter()
                loss.backward()
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                print("backward phases (ms from loss.backward()):",
                      {k: round((v - t0) * 1e3, 3) for k, v in sorted(marks.items(), key=lambda kv: kv[1])},
                      "end", round((t1 - t0) * 1e3, 3))
            E.Episode.stash, E.Episode.backward_all = st0, ba0
        if "--cprofile" in sys.argv:
            episode()
            loss = torch.cat([-lp * Rt for lp, Rt in zip(policy.saved_log_probs, returns)]).sum()
            torch.cuda.synchronize()
            pr = cProfile.Profile()
            pr.enable()
            loss.backward()
            torch.cuda.synchronize()
            pr.disable()
            pstats.Stats(pr).sort_stats("tottime").print_stats(25)
            pstats.Stats(pr).sort_stats("cumulative").print_stats(25)
        sys.exit(0)
    pr = cProfile.Profile()
    pr.enable()
    episode()
    torch.cuda.synchronize()
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(30)
