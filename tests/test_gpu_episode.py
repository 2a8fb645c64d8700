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


@pytest.mark.parametrize("T,B,seg,u8,extras,store,actor", [(9, 2, 4, True, False, "1", "0"),
                                                          (7, 3, 64, False, True, "1", "0"),
                                                          (70, 1, 64, True, True, "1", "0"),
                                                          (9, 2, 4, True, False, "0", "0"),
                                                          (37, 1, 64, True, False, "1", "0"),
                                                          (9, 2, 4, True, False, "1", "1"),
                                                          (7, 3, 64, False, True, "1", "1"),
                                                          (70, 1, 64, True, True, "1", "1")])
def test_episode_matches_per_step_path(cuda, monkeypatch, T, B, seg, u8, extras, store, actor):
    """Segments of 4 (3 segments, ragged last), one segment, and 70 steps over
    the default 64-step segment; uint8 and fp32 frames; prev_reward/action;
    the kept ConvLSTM products (16-step blocks, a ragged last block at 37) or
    the recomputed recurrence (AAA_EPISODE_STORE=0).  Recorded on the learner's
    T=1 forward (AAA_EPISODE_ACTOR=0: the per-step path's own kernels, so the
    logits are bit-identical and the gradients agree to 1e-5) or on the actor
    chain (its own fp32 kernels: logits within 1e-5, gradients within the fp32
    criterion 1e-4)."""
    monkeypatch.setattr(E, "EPISODE_SEGMENT", seg)
    monkeypatch.setenv("AAA_EPISODE_STORE", store)
    monkeypatch.setenv("AAA_EPISODE_ACTOR", actor)
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
    assert (ag._episode.actor is not None) == (actor == "1" and store == "1")
    ref = _agent(cuda, False)
    lr_, gr = _episode(ref, X, Gl, Gv, cuda, pr, pa, u8)
    assert ref._episode is None
    if actor == "0":
        assert torch.equal(lf, lr_)            # the forward is the per-step forward
        _cmp(gf, gr, 1e-5, "fused vs per-step")
    else:
        assert_close(lf.numpy(), lr_.numpy(), 1e-5, "actor-chain logits vs per-step")
        _cmp(gf, gr, 1e-4, "fused (actor chain) vs per-step")


@pytest.mark.parametrize("actor", ["1", "0"])
def test_episode_matches_oracle(cuda, monkeypatch, actor):
    monkeypatch.setattr(E, "EPISODE_SEGMENT", 3)
    monkeypatch.setenv("AAA_EPISODE_ACTOR", actor)
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


def test_long_actor_chain_episode_matches_oracle(cuda, monkeypatch):
    """an episode recorded on the actor chain (its own fp32 kernels'
    gates, c and h imported into the backward) while the backward recomputes the
    vision encoder and the tail with the learner's kernels -- two summation
    orders mixed in one BPTT.  Over 400 steps (7 segments of 64, the ConvLSTM
    state carried through all of them) the mix must still meet the fp32
    criterion against the CPU oracle: logits and every gradient at 1e-4."""
    monkeypatch.setenv("AAA_EPISODE_STORE", "1")
    monkeypatch.setenv("AAA_EPISODE_ACTOR", "1")
    T, B = 400, 1
    X = _frames(T, B, seed=4321)
    Gl = torch.from_numpy(detinit.normal(12, (T, B, A)))
    Gv = torch.from_numpy(detinit.normal(13, (T, B, A)))
    ag = _agent(cuda, True)
    lf, gf = _episode(ag, X, Gl, Gv, cuda)
    assert ag._episode.actor is not None and len(ag._episode.steps) == T
    torch.set_num_threads(16)
    P = ref_cpu.tensor_params(detinit.deterministic_params(0, A))
    rl, rv, _ = ref_cpu.unroll(P, X.float())
    ((rl * Gl).sum() + (rv * Gv).sum()).backward()
    assert_close(lf.numpy(), rl.detach().numpy(), 1e-4, "400-step actor-chain logits")
    _cmp(gf, {n: (p.grad if p.grad is not None else torch.zeros_like(p)) for n, p in P.items()}, 1e-4,
         "400-step actor-chain episode vs oracle")


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
    _cmp(gf, gr, 1e-4, "parameter change")   # recorded on the actor chain: the fp32 criterion


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
    with pytest.raises(ValueError, match="contiguous"):
        r.core_import(ws2, 0, 2, core[0][:1], core[1][:2], core[2][:2])


def test_core_transfer_bf16_types_and_bad_ranges(cuda):
    """bf16 runners move their own element types (fp16 gates, bf16 h: the
    workspace's storage, aaa_core_elem_bytes); fp32 buffers are refused, as are
    steps outside [0, T)."""
    from aaa_amd import _native as N
    T, B = 5, 2
    ag = _agent(cuda, False, dtype="bf16")
    r = ag._runner(B, T, 84, 84, cuda, False, True)
    assert r.core_dtypes() == (torch.float16, torch.float32, torch.bfloat16)
    ws = r.new_workspace()
    with pytest.raises(ValueError, match="contiguous"):
        r.core_export(ws, 0, 3, *[torch.empty(s, device=cuda) for s in r.core_shapes(3)])
    # round trip: export a forward's products, import them into a fresh workspace, VISION | TAIL only
    S = ag._basis_for(r.h, r.w, 84, 84, cuda)
    flat, packed = ag._packed_params(r, list(ag.parameters()))
    X = _frames(T, B).to(cuda)
    dl = torch.from_numpy(detinit.normal(2, (T, B, A))).to(cuda)
    l1, v1, _, _, _ = r.forward(flat, packed, S, X, ws, want_attn=False)
    core = [torch.empty(s, dtype=dt, device=cuda) for s, dt in zip(r.core_shapes(T), r.core_dtypes())]
    r.core_export(ws, 0, T, *core)
    g1, _, _ = r.backward(flat, packed, S, X, ws, dl)
    ws2 = r.new_workspace()
    r.core_import(ws2, 0, T, *core)
    l2, v2, _, _, _ = r.forward(flat, packed, S, X, ws2, want_attn=False, phases=N.FWD_VISION | N.FWD_TAIL)
    g2, _, _ = r.backward(flat, packed, S, X, ws2, dl)
    torch.cuda.synchronize()
    assert torch.equal(l1, l2) and torch.equal(v1, v2)
    assert rel_err(g2.cpu().numpy(), g1.cpu().numpy()) < 1e-5
    agf = _agent(cuda, False)
    rf = agf._runner(2, 3, 84, 84, cuda, False, True)
    core = [torch.empty(s, device=cuda) for s in rf.core_shapes(2)]
    with pytest.raises(RuntimeError, match="steps"):
        rf.core_export(rf.new_workspace(), 2, 2, *core)


@pytest.mark.parametrize("store", ["1", "0"])
def test_bf16_episode_matches_per_step_path(cuda, monkeypatch, store):
    """bf16 agents keep their ConvLSTM products too (fp16 gates, fp32 c, bf16
    h), so the fused backward imports them instead of re-running the
    recurrence (AAA_EPISODE_STORE=0: the re-run); either way the per-step
    path's gradients (same bf16 kernels and rounding points)."""
    monkeypatch.setattr(E, "EPISODE_SEGMENT", 4)
    monkeypatch.setenv("AAA_EPISODE_STORE", store)
    T, B = 6, 2
    X = _frames(T, B)
    Gl = torch.from_numpy(detinit.normal(2, (T, B, A)))
    Gv = torch.from_numpy(detinit.normal(3, (T, B, A)))
    ag = _agent(cuda, True, dtype="bf16")
    lf, gf = _episode(ag, X, Gl, Gv, cuda)
    assert (ag._episode.store is None) == (store == "0") and ag._episode.actor is None
    if store == "1":
        assert len(ag._episode.store) == 2     # two 4-step blocks (STORE_BLOCK capped by the segment)
    lr_, gr = _episode(_agent(cuda, False, dtype="bf16"), X, Gl, Gv, cuda)
    assert torch.equal(lf, lr_)
    _cmp(gf, gr, 2e-3, "bf16 fused vs per-step")


@pytest.mark.parametrize("actor,store", [("1", "1"), ("0", "1"), ("0", "0")])
def test_state_cotangent_at_intermediate_steps(cuda, monkeypatch, actor, store):
    """The reference keeps a live (h, c) in ``prev_hidden`` after every step
    (attention.py:125), so a loss may use any step's state: here the logits of
    every step plus the ConvLSTM state after steps 2, 5 (a segment boundary),
    8 and the last -- h and c with different weights.  The fused episode cuts
    its segments after each such step and adds the cotangent to the carry; it
    must match the per-step path (one autograd node per call)."""
    monkeypatch.setattr(E, "EPISODE_SEGMENT", 6)
    monkeypatch.setenv("AAA_EPISODE_ACTOR", actor)
    monkeypatch.setenv("AAA_EPISODE_STORE", store)
    T, B = 11, 2
    X = _frames(T, B)
    G = torch.from_numpy(detinit.normal(2, (T, B, A)))
    taps = {2: 0.7, 5: -0.4, 8: 1.3, T - 1: 0.5}

    def run(fuse):
        ag = _agent(cuda, fuse)
        ag.reset()
        ag.zero_grad(set_to_none=True)
        loss = 0
        for t in range(T):
            lg, _ = ag(X[t].to(cuda))
            loss = loss + (lg * G[t].to(cuda)).sum()
            if t in taps:
                h, c = ag.vision.vision_lstm.prev_hidden
                wh = torch.from_numpy(detinit.normal(10 + t, tuple(h.shape))).to(cuda)
                loss = loss + taps[t] * (h * wh).sum() + 0.3 * (c * c).sum()
        loss.backward()
        torch.cuda.synchronize()
        return _grads(ag)
    _cmp(run(True), run(False), 1e-5 if actor == "0" else 1e-4, "state cotangents mid-episode")


def test_policy_mixed_act_and_forward(cuda, monkeypatch):
    """One episode whose steps come from Policy.act (the draw fused into the step
    node) and from plain agent(x) calls: the log-prob cotangents fold in where a
    draw was recorded and nowhere else (no missing-Jacobian error)."""
    from aaa_amd.policy import Policy
    monkeypatch.setattr(E, "EPISODE_SEGMENT", 4)
    T = 9
    X = _frames(T, 1)
    G = torch.from_numpy(detinit.normal(2, (T, 1, A)))

    def run(fuse):
        ag = _agent(cuda, fuse)
        pol = Policy(ag, seed=3)
        ag.reset()
        ag.zero_grad(set_to_none=True)
        loss = 0
        for t in range(T):
            if t % 3 == 1:
                lg, _ = ag(X[t].to(cuda))
                loss = loss + (lg * G[t].to(cuda)).sum()
            else:
                _, logp = pol.act(X[t, 0].to(cuda))
                loss = loss - (t + 1) * 0.1 * logp.sum()
        loss.backward()
        torch.cuda.synchronize()
        return _grads(ag)
    _cmp(run(True), run(False), 1e-4, "mixed act/forward episode")


def test_episode_store_budget(cuda, monkeypatch):
    """AAA_EPISODE_STORE_MB caps the kept ConvLSTM products: past
    the budget the steps are recomputed from checkpoints, with the same result."""
    monkeypatch.setattr(E, "EPISODE_SEGMENT", 8)
    monkeypatch.setenv("AAA_EPISODE_STORE_MB", "1")   # one 16-step block at B = 2, 84x84: 2 x 16 x 242 x 768 x 4 B = 23.8 MB > 1 MB
    T, B = 20, 2
    X = _frames(T, B)
    Gl = torch.from_numpy(detinit.normal(2, (T, B, A)))
    Gv = torch.from_numpy(detinit.normal(3, (T, B, A)))
    ag = _agent(cuda, True)
    _, gf = _episode(ag, X, Gl, Gv, cuda)
    assert ag._episode.store == {} and ag._episode.store_bytes == 0
    _, gr = _episode(_agent(cuda, False), X, Gl, Gv, cuda)
    _cmp(gf, gr, 1e-4, "store past its budget")
