"""Host-side op census of the fused episode backward (bench.episode_leg's
pattern): torch.profiler over one episode's ``loss.backward()``, the ops and
their counts, so the per-step autograd nodes' launches can be attributed.
    python tools/episode_ops.py > gpurun_out/episode_ops.txt"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402
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
    agent.fuse_episode_backward = True
    policy = Policy(agent, seed=0)
    obs = detinit.frames_u8(4321, (T_ep, 210, 160, 3))
    rewards = (detinit.frames_u8(4322, (T_ep,)) % 3).astype(np.float32).tolist()
    eps = np.finfo(np.float32).eps.item()

    def episode():
        agent.reset()
        agent.zero_grad(set_to_none=True)
        policy.saved_log_probs = []
        for t in range(T_ep):
            policy(obs[t])
        R, returns = 0.0, []
        for r in rewards[::-1]:
            R = r + 0.99 * R
            returns.insert(0, R)
        returns = torch.tensor(returns, device=dev)
        returns = (returns - returns.mean()) / (returns.std() + eps)
        return torch.cat([-lp * Rt for lp, Rt in zip(policy.saved_log_probs, returns)]).sum()

    episode().backward()
    torch.cuda.synchronize()
    loss = episode()
    torch.cuda.synchronize()
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU]) as prof:
        loss.backward()
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=40))
