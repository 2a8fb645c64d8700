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


@pytest.mark.parametrize("T,B,seg,u8,extras,store", [(9, 2, 4, True, False, "1"), (7, 3, 64, False, True, "1"),
                                                    (70, 1, 64, True, True, "1"), (9, 2, 4, True, False, "0"),
                                                    (37, 1, 64, True, False, "1")])
def test_episode_matches_per_step_path(cuda, monkeypatch, T, B, seg, u8, extras, store):
    """Segments of 4 (3 segments, ragged last), one segment, and 70 steps over
    the default 64-step segment; uint8 and fp32 frames; prev_reward/action;
    the kept ConvLSTM products (16-step blocks, a ragged last block at 37) or
    the recomputed recurrence (AAA_EPISODE_STORE=0)."""
    monkeypatch.setattr(E, "EPISODE_SEGMENT", seg)
    monkeypatch.setenv("AAA_EPISODE_STORE", store)
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


@pytest.mark.parametrize("store", ["1", "0"])
def test_episode_memory_per_step(cuda, monkeypatch, store):
    """The graph of a 210x160 episode keeps a bounded amount per step, not a
    T=1 workspace (12.6 MB): frames + a state checkpoint every 64 steps (< 1 MB
    with AAA_EPISODE_STORE=0), plus the ConvLSTM products the backward imports
    instead of re-running the recurrence (1.66 MB, in 16-step blocks: < 3 MB)."""
    monkeypatch.setenv("AAA_EPISODE_STORE", store)
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
    assert per_step < (3 << 20 if store == "1" else 1 << 20), per_step
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


@pytest.mark.parametrize("u8", [True, False])
def test_core_import_replaces_the_recurrence(cuda, u8):
    """aaa_core_export of a full forward's ConvLSTM products, imported in two
    pieces into a fresh workspace, then aaa_forward_phases without CORE: the
    same logits bit for bit and the same gradients (up to the wgrad atomics'
    summation order) as the full forward + backward."""
    from aaa_amd import _native as N
    T, B = 5, 2
    ag = _agent(cuda, False)
    r = ag._runner(B, T, 84, 84, cuda, False, u8)
    S = ag._basis_for(r.h, r.w, 84, 84, cuda)
    flat, packed = ag._packed_params(r, list(ag.parameters()))
    X = _frames(T, B).to(cuda)
    X = X if u8 else X.float()
    dl = torch.from_numpy(detinit.normal(2, (T, B, A))).to(cuda)
    dv = torch.from_numpy(detinit.normal(3, (T, B, A))).to(cuda)
    ws1 = r.new_workspace()
    l1, v1, _, _, _ = r.forward(flat, packed, S, X, ws1, want_attn=False)
    core = [torch.empty(s, device=cuda) for s in r.core_shapes(T)]
    r.core_export(ws1, 0, T, *core)
    g1, _, _ = r.backward(flat, packed, S, X, ws1, dl, dv)
    ws2 = r.new_workspace()
    for t0, n in ((0, 2), (2, 3)):
        r.core_import(ws2, t0, n, *(x[t0:t0 + n] for x in core))
    l2, v2, _, _, _ = r.forward(flat, packed, S, X, ws2, want_attn=False, phases=N.FWD_VISION | N.FWD_TAIL)
    g2, _, _ = r.backward(flat, packed, S, X, ws2, dl, dv)
    torch.cuda.synchronize()
    assert torch.equal(l1, l2) and torch.equal(v1, v2)
    assert rel_err(g2.cpu().numpy(), g1.cpu().numpy()) < 1e-6
    with pytest.raises(ValueError, match="contiguous fp32"):
        r.core_import(ws2, 0, 2, core[0][:1], core[1][:2], core[2][:2])


def test_core_transfer_refuses_bf16_and_bad_ranges(cuda):
    ag = _agent(cuda, False, dtype="bf16")
    r = ag._runner(2, 3, 84, 84, cuda, False, True)
    ws = r.new_workspace()
    core = [torch.empty(s, device=cuda) for s in r.core_shapes(3)]
    with pytest.raises(RuntimeError, match="fp32 configs only"):
        r.core_export(ws, 0, 3, *core)
    agf = _agent(cuda, False)
    rf = agf._runner(2, 3, 84, 84, cuda, False, True)
    core = [torch.empty(s, device=cuda) for s in rf.core_shapes(2)]
    with pytest.raises(RuntimeError, match="steps"):
        rf.core_export(rf.new_workspace(), 2, 2, *core)


def test_bf16_episode_recomputes_and_matches_per_step_path(cuda, monkeypatch):
    """bf16 agents keep no ConvLSTM products (the store is fp32-only): the
    fused backward re-runs the recurrence and must still give the per-step
    path's gradients (same bf16 kernels and rounding points)."""
    monkeypatch.setattr(E, "EPISODE_SEGMENT", 4)
    T, B = 6, 2
    X = _frames(T, B)
    Gl = torch.from_numpy(detinit.normal(2, (T, B, A)))
    Gv = torch.from_numpy(detinit.normal(3, (T, B, A)))
    ag = _agent(cuda, True, dtype="bf16")
    lf, gf = _episode(ag, X, Gl, Gv, cuda)
    assert ag._episode.store is None
    lr_, gr = _episode(_agent(cuda, False, dtype="bf16"), X, Gl, Gv, cuda)
    assert torch.equal(lf, lr_)
    _cmp(gf, gr, 2e-2, "bf16 fused vs per-step")
