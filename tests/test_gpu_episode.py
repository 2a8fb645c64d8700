"""Fused episode backward (episode.py) for the reference's call pattern:
per-step ``agent(state)`` calls (main_mp.py:49-59, :111) then one
``loss.backward()`` through all of them (main_mp.py:76-77).

The episode path must give the gradients of the per-step path it replaces
(``Agent.fuse_episode_backward = False``: one T=1 autograd node per call,
chained through the ConvLSTM state -- pinned to the oracle by
test_gpu_parity.py / test_gpu_actor.py) and of the CPU oracle, across segment
boundaries, with prev_reward / prev_action, when a later call continues from
the episode's state, across a parameter change mid-episode, and it must keep
a small, bounded amount of memory per step.
"""
import numpy as np
import pytest
import torch

from helpers import assert_close, detinit, rel_err
from oracle import ref_cpu

import attention
from aaa_amd import episode as E

pytestmark = pytest.mark.gpu

A = 18


def _agent(cuda, fuse, H=84, dtype="fp32"):
    grid = (11, 11) if H == 84 else None
    ag = attention.Agent(A, grid=grid, conv_dtype=dtype)
    detinit.load_into(ag, detinit.deterministic_params(0, A))
    ag.to(cuda)
    ag.fuse_episode_backward = fuse
    return ag


def _frames(T, B, H=84, W=84, seed=1234):
    return torch.from_numpy(detinit.frames_u8(seed, (T, B, H, W, 3)))


def _grads(agent):
    return {n: (p.grad.detach().cpu().clone() if p.grad is not None else torch.zeros_like(p).cpu())
            for n, p in agent.named_parameters()}


def _episode(agent, X, Gl, Gv, dev, pr=None, pa=None, u8=True):
    agent.reset()
    agent.zero_grad(set_to_none=True)
    loss, outs = 0, []
    for t in range(X.shape[0]):
        x = X[t].to(dev) if u8 else X[t].float().to(dev)
        kw = {}
        if pr is not None:
            kw = dict(prev_reward=pr[t].to(dev), prev_action=pa[t].to(dev))
        lg, vl = agent(x, **kw)
        outs.append(lg.detach().cpu())
        loss = loss + (lg * Gl[t].to(dev)).sum() + (vl * Gv[t].to(dev)).sum()
    loss.backward()
    torch.cuda.synchronize()
    return torch.stack(outs), _grads(agent)


def _cmp(a, b, tol, what):
    for n in b:
        if float(b[n].norm()) == 0.0:
            assert float(a[n].abs().max()) == 0.0, f"{what} {n}"
        else:
            assert rel_err(a[n].numpy(), b[n].numpy()) <= tol, f"{what} {n}: {rel_err(a[n].numpy(), b[n].numpy()):.3e}"


@pytest.mark.parametrize("T,B,seg,u8,extras", [(9, 2, 4, True, False), (7, 3, 64, False, True), (70, 1, 64, True, True)])
def test_episode_matches_per_step_path(cuda, monkeypatch, T, B, seg, u8, extras):
    """Segments of 4 (3 segments, ragged last), one segment, and 70 steps over
    the default 64-step segment; uint8 and fp32 frames; prev_reward/action."""
    monkeypatch.setattr(E, "EPISODE_SEGMENT", seg)
    X = _frames(T, B)
    Gl = torch.from_numpy(detinit.normal(2, (T, B, A)))
    Gv = torch.from_numpy(detinit.normal(3, (T, B, A)))
    pr = pa = None
    if extras:
        pr = torch.from_numpy(detinit.normal(5, (T, B)))
        pa = torch.from_numpy((detinit.frames_u8(6, (T, B)) % A).astype(np.float32))
    ag = _agent(cuda, True)
    lf, gf = _episode(ag, X, Gl, Gv, cuda, pr, pa, u8)
    assert isinstance(ag._episode, E.Episode) and len(ag._episode.steps) == T
    ref = _agent(cuda, False)
    lr_, gr = _episode(ref, X, Gl, Gv, cuda, pr, pa, u8)
    assert ref._episode is None
    assert torch.equal(lf, lr_)            # the forward is the per-step forward either way
    _cmp(gf, gr, 1e-5, "fused vs per-step")


def test_episode_matches_oracle(cuda, monkeypatch):
    monkeypatch.setattr(E, "EPISODE_SEGMENT", 3)
    T, B = 7, 2
    X = _frames(T, B)
    Gl = torch.from_numpy(detinit.normal(2, (T, B, A)))
    Gv = torch.from_numpy(detinit.normal(3, (T, B, A)))
    lf, gf = _episode(_agent(cuda, True), X, Gl, Gv, cuda)
    P = ref_cpu.tensor_params(detinit.deterministic_params(0, A))
    rl, rv, _ = ref_cpu.unroll(P, X.float())
    ((rl * Gl).sum() + (rv * Gv).sum()).backward()
    assert_close(lf.numpy(), rl.detach().numpy(), 1e-4, "logits")
    _cmp(gf, {n: (p.grad if p.grad is not None else torch.zeros_like(p)) for n, p in P.items()}, 1e-4,
         "fused vs oracle")


def test_episode_then_unroll_from_its_state(cuda, monkeypatch):
    """A later Agent.unroll continuing from the episode's state sends a state
    cotangent into the episode's last step (the BPTT's dhT / dcT)."""
    monkeypatch.setattr(E, "EPISODE_SEGMENT", 4)
    T1, T2, B = 6, 3, 2
    X = _frames(T1 + T2, B)
    G = torch.from_numpy(detinit.normal(2, (T1 + T2, B, A)))

    def run(fuse):
        ag = _agent(cuda, fuse)
        ag.reset()
        ag.zero_grad(set_to_none=True)
        loss = 0
        for t in range(T1):
            lg, _ = ag(X[t].to(cuda))
            loss = loss + (lg * G[t].to(cuda)).sum()
        lg2, _, _ = ag.unroll(X[T1:].to(cuda))
        loss = loss + (lg2 * G[T1:].to(cuda)).sum()
        loss.backward()
        torch.cuda.synchronize()
        return _grads(ag)
    _cmp(run(True), run(False), 1e-5, "episode + unroll")


def test_parameter_change_starts_new_episode(cuda, monkeypatch):
    """An optimizer step between two per-step calls (no backward yet) closes the
    episode: the next steps use the new weights and the gradient still flows
    back through the old steps (their state feeds the new episode)."""
    monkeypatch.setattr(E, "EPISODE_SEGMENT", 4)
    T, B = 6, 1
    X = _frames(T, B)
    G = torch.from_numpy(detinit.normal(2, (T, B, A)))

    def run(fuse):
        ag = _agent(cuda, fuse)
        ag.reset()
        ag.zero_grad(set_to_none=True)
        loss = 0
        eps = set()
        for t in range(T):
            if t == 3:
                with torch.no_grad():
                    ag.policy_head[0].bias.add_(0.01)
            lg, _ = ag(X[t].to(cuda))
            eps.add(id(ag._episode))
            loss = loss + (lg * G[t].to(cuda)).sum()
        loss.backward()
        torch.cuda.synchronize()
        return _grads(ag), len(eps)
    gf, n_eps = run(True)
    gr, _ = run(False)
    assert n_eps == 2
    _cmp(gf, gr, 1e-5, "parameter change")


def test_episode_memory_per_step(cuda):
    """The graph of a 210x160 episode keeps well under 1 MB per step (frames +
    a state checkpoint every 64 steps), not a T=1 workspace per step."""
    ag = attention.Agent(A).to(cuda)
    detinit.load_into(ag, detinit.deterministic_params(0, A))
    ag.to(cuda)
    T = 40
    obs = torch.from_numpy(detinit.frames_u8(7, (T, 1, 210, 160, 3))).to(cuda)
    ag.reset()
    lg, _ = ag(obs[0])          # warm-up: runner, workspace, packed weights
    torch.cuda.synchronize()
    base = torch.cuda.memory_allocated(cuda)
    loss = lg.sum()
    for t in range(1, T):
        lg, _ = ag(obs[t])
        loss = loss + lg.sum()
    torch.cuda.synchronize()
    per_step = (torch.cuda.memory_allocated(cuda) - base) / (T - 1)
    assert per_step < 1 << 20, per_step
    loss.backward()


def test_inplace_modified_frames_raise(cuda):
    ag = _agent(cuda, True)
    X = _frames(3, 1).to(cuda)
    ag.reset()
    loss = 0
    for t in range(3):
        lg, _ = ag(X[t])
        loss = loss + lg.sum()
    X[1].add_(1)          # the frames of step 1 change under the recorded episode
    with pytest.raises(RuntimeError, match="modified in place"):
        loss.backward()
