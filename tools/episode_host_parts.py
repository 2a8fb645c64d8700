"""Host cost of the pieces of one recorded episode step (Policy.act on the
actor chain), each timed alone in a loop on the GPU box -- where the ~150 us
of Python per step goes.
    python tools/episode_host_parts.py > gpurun_out/episode_host_parts.txt"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

import attention  # noqa: E402
from aaa_amd import detinit  # noqa: E402
from aaa_amd import _native as N  # noqa: E402
from aaa_amd.policy import Policy  # noqa: E402


def tm(name, f, n=200):
    for _ in range(10):
        f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        f()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    print(f"{name:48s} {(t1 - t0) / n * 1e6:8.2f} us/call (host)")


if __name__ == "__main__":
    dev = torch.device("cuda:0")
    agent = attention.Agent(18).to(dev)
    detinit.load_into(agent, detinit.deterministic_params(0, 18))
    agent.to(dev)
    policy = Policy(agent, seed=0)
    obs = detinit.frames_u8(4321, (64, 210, 160, 3))
    for t in range(64):
        policy(obs[t])
    ep = agent._episode
    X = policy._upload(obs[0])
    params = agent._param_list()
    runner = ep.runner
    tm("Policy._upload", lambda: policy._upload(obs[0]))
    tm("Agent._episode_params", lambda: agent._episode_params(X))
    tm("Agent._param_list", lambda: agent._param_list())
    tm("Agent._runner", lambda: agent._runner(1, 1, 210, 160, X.device, False, True))
    tm("Agent._basis_for", lambda: agent._basis_for(runner.h, runner.w, 210, 160, X.device))
    tm("Agent._packed_params", lambda: agent._packed_params(runner, params, agent))
    tm("torch.empty x6 (cuda)", lambda: [torch.empty(1, 1, 18, device=dev) for _ in range(6)])
    tm("N.stream_ptr", lambda: N.stream_ptr(dev))
    ar, ws = ep.actor, ep.ws
    shp = runner.state_shape()
    h, c = torch.zeros(shp, device=dev), torch.zeros(shp, device=dev)
    ho, co = torch.zeros(shp, device=dev), torch.zeros(shp, device=dev)
    lg, vl = torch.empty(1, 18, device=dev), torch.empty(1, 18, device=dev)
    at = torch.empty(1, runner.h, runner.w, 4, device=dev)
    acts, lp, jac = torch.empty(1, dtype=torch.int32, device=dev), torch.empty(1, device=dev), torch.empty(1, 18, device=dev)
    sampler = policy._sampler
    fr = X

    def step():
        ar.step(ep.flat, ep.packed, ep.basis, fr, ws, h, c, lg, vl, at, seed=sampler.seed, counter=sampler.counter,
                actions=acts, logp=lp, dlogp=jac, h_out=ho, c_out=co)
    tm("ActorRunner.step (checks + io + C call)", step)
    io = N.ActorIO()
    for k, v in dict(params=ep.flat, packed=ep.packed, basis=ep.basis, frames=fr, h=h, c=c, logits=lg, values=vl,
                     attn=at, workspace=ws, counter=sampler.counter, actions=acts, logp=lp, dlogp_dlogits=jac,
                     h_out=ho, c_out=co).items():
        setattr(io, k, v.data_ptr())
    import ctypes
    cref, ioref = ctypes.byref(ar.cfg), ctypes.byref(io)
    lib = N.load()
    st = N.stream_ptr(dev)
    tm("aaa_actor_step C call alone", lambda: lib.aaa_actor_step(cref, ioref, st))
    tm("Policy.act (whole step)", lambda: policy.act(obs[1]))
    torch.cuda.synchronize()
