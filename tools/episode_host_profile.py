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

    episode()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    episode()
    torch.cuda.synchronize()
    print(f"ms per step (no profiler): {(time.perf_counter() - t0) / T_ep * 1e3:.3f}")
    pr = cProfile.Profile()
    pr.enable()
    episode()
    torch.cuda.synchronize()
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(30)
