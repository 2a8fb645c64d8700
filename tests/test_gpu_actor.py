"""Actor path: the device sampler (aaa_sample_actions)
against the oracle's restatement, and the drop-in Policy (main_mp.py:40-59)
through a whole episode + finish_episode (main_mp.py:62-77) against the oracle
unroll with the same actions.
"""
import numpy as np
import pytest
import torch

from helpers import assert_close, detinit
from oracle import ref_cpu

import attention
from aaa_amd.policy import ActionSampler, Policy, sample_actions

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("B,A,scale", [(4096, 18, 1.0), (1000, 18, 8.0), (257, 5, 0.2), (64, 130, 2.0)])
def test_sampler_matches_oracle(cuda, B, A, scale):
    g = torch.Generator().manual_seed(B + A)
    logits = torch.randn(B, A, generator=g) * scale
    counter = torch.tensor([41], dtype=torch.int64, device=cuda)
    a, lp = sample_actions(logits.to(cuda), seed=1234, counter=counter)
    torch.cuda.synchronize()
    ra, rlp, margin = ref_cpu.sample_actions(logits.numpy(), 1234, 41)
    a = a.cpu().numpy()
    sure = margin > 1e-5          # draws within fp32 rounding of a CDF boundary may differ
    assert sure.mean() > 0.99
    assert np.array_equal(a[sure], ra[sure]), int((a[sure] != ra[sure]).sum())
    ref = torch.distributions.Categorical(torch.softmax(logits, -1)).log_prob(torch.from_numpy(a).long())
    assert np.abs(lp.cpu().numpy() - ref.numpy()).max() <= 2e-6 * max(1.0, float(ref.abs().max()))
    assert int(counter.item()) == 42


def test_sampler_counter_advances_and_seeds_differ(cuda):
    logits = torch.zeros(512, 18, device=cuda)
    s = ActionSampler(7, cuda)
    a0, _ = s(logits)
    a1, _ = s(logits)
    b0, _ = ActionSampler(8, cuda)(logits)
    torch.cuda.synchronize()
    assert int(s.counter.item()) == 2
    assert (a0 != a1).float().mean() > 0.8 and (a0 != b0).float().mean() > 0.8
    ra0, _, _ = ref_cpu.sample_actions(np.zeros((512, 18), np.float32), 7, 0)
    ra1, _, _ = ref_cpu.sample_actions(np.zeros((512, 18), np.float32), 7, 1)
    assert np.array_equal(a0.cpu().numpy(), ra0) and np.array_equal(a1.cpu().numpy(), ra1)


def test_sampler_distribution(cuda):
    logits = torch.tensor([[2.0, 0.0, -1.0, 1.0, 0.5, -3.0]])
    p = torch.softmax(logits, -1)[0].numpy()
    n = 200000
    a, _ = sample_actions(logits.repeat(n, 1).to(cuda), seed=3)
    freq = np.bincount(a.cpu().numpy(), minlength=6) / n
    chi2 = float((((freq - p) ** 2) / p).sum() * n)
    assert chi2 < 25.0, (chi2, freq, p)


def test_sampler_log_prob_gradient(cuda):
    g = torch.Generator().manual_seed(5)
    logits = torch.randn(32, 18, generator=g) * 2
    logits[0, 3] = 60.0                       # saturated row: clamp at 1 - eps passes no gradient
    w = torch.randn(32, generator=g)
    dl = logits.to(cuda).requires_grad_(True)
    a, lp = sample_actions(dl, seed=11)
    (lp * w.to(cuda)).sum().backward()
    rl = logits.clone().requires_grad_(True)
    ref = torch.distributions.Categorical(torch.softmax(rl, -1)).log_prob(a.cpu().long())
    (ref * w).sum().backward()
    assert torch.allclose(dl.grad.cpu(), rl.grad, rtol=1e-5, atol=1e-6)
    assert float(dl.grad[0].abs().max()) == 0.0


def _finish_episode_loss(saved_log_probs, rewards, gamma=0.99):
    """finish_episode's loss (main_mp.py:62-76) on the saved log-prob tensors."""
    eps = np.finfo(np.float32).eps.item()
    R, returns = 0, []
    for r in rewards[::-1]:
        R = r + gamma * R
        returns.insert(0, R)
    returns = torch.tensor(returns, device=saved_log_probs[0].device)
    returns = (returns - returns.mean()) / (returns.std() + eps)
    return torch.cat([-lp * Rt for lp, Rt in zip(saved_log_probs, returns)]).sum()


@pytest.mark.parametrize("T", [1 + 5, 12])
def test_policy_episode_matches_oracle(cuda, T):
    """Policy.forward per step (uint8 frames, device draw, .item()) -> finish_episode
    -> loss.backward through T chained per-step agent calls, vs the oracle unroll
    of the same frames and actions."""
    params = detinit.deterministic_params(0, 18, 4)
    agent = attention.Agent(18, grid=(11, 11))
    detinit.load_into(agent, params)
    agent.to(cuda)
    policy = Policy(agent, seed=17)
    frames = detinit.frames_u8(1234 + T, (T, 84, 84, 3))
    rewards = [float(r) for r in (np.arange(T) % 3 == 1) * 5.0]
    agent.reset()
    actions = [policy(frames[t]) for t in range(T)]
    policy.rewards = rewards
    loss = _finish_episode_loss(policy.saved_log_probs, policy.rewards)
    loss.backward()
    torch.cuda.synchronize()

    P = ref_cpu.tensor_params(params)
    X = torch.from_numpy(frames.astype(np.float32)).unsqueeze(1)
    rl, _, _ = ref_cpu.unroll(P, X)
    ref_loss = ref_cpu.reinforce_loss(rl, actions, rewards)
    ref_loss.backward()
    # the policy drew from its own logits: check those draws are the oracle's for the oracle logits
    for t in range(T):
        ra, _, margin = ref_cpu.sample_actions(rl[t].detach().numpy(), 17, t)
        if margin[0] > 1e-4:
            assert actions[t] == int(ra[0]), t
    assert abs(float(loss) - float(ref_loss)) <= 1e-4 * max(1.0, abs(float(ref_loss)))
    for n, p in agent.named_parameters():
        gr = P[n].grad if P[n].grad is not None else torch.zeros_like(P[n])
        g = p.grad if p.grad is not None else torch.zeros_like(p)
        if float(gr.norm()) > 0:
            assert_close(g.cpu().numpy(), gr.numpy(), 1e-4, n)
        else:
            assert float(g.abs().max()) == 0.0, n


@pytest.mark.parametrize("optim", ["torch", "aaa"])
def test_packed_weights_follow_parameter_updates(cuda, optim):
    """The per-runner packed-weight cache re-packs after an in-place update --
    also after the fused aaa_amd.optim.Adam, which writes the parameters through
    raw pointers and bumps their version counters itself."""
    params = detinit.deterministic_params(0, 18, 4)
    agent = attention.Agent(18, grid=(11, 11))
    detinit.load_into(agent, params)
    agent.to(cuda)
    x = torch.from_numpy(detinit.frames_u8(5, (1, 84, 84, 3)).astype(np.float32)).to(cuda)
    agent.reset()
    l0, _ = agent(x)
    agent.reset()
    l1, _ = agent(x)
    assert torch.equal(l0, l1)
    from aaa_amd.optim import Adam as FusedAdam
    opt = (torch.optim.Adam if optim == "torch" else FusedAdam)(agent.parameters(), lr=1e-2)
    (l1.sum()).backward()
    opt.step()
    agent.reset()
    l2, _ = agent(x)
    P = ref_cpu.tensor_params({n: p.detach().cpu().numpy() for n, p in agent.named_parameters()})
    rl, _, _ = ref_cpu.unroll(P, x.cpu().unsqueeze(0))
    assert not torch.equal(l1, l2)
    assert_close(l2.detach().cpu().numpy(), rl[0].detach().numpy(), 1e-4, "logits after update")


@pytest.mark.parametrize("chain", [True, False])
def test_graph_actor_matches_eager_steps(cuda, chain):
    """The captured one-step graph -- on the actor chain (aaa_actor_step) or the
    learner's T=1 forward -- reproduces the oracle's per-step agent (same
    logits, carried ConvLSTM state, the same draws for the same counter), and
    picks up a parameter update."""
    from aaa_amd.policy import GraphActor
    params = detinit.deterministic_params(0, 18, 4)
    agent = attention.Agent(18, grid=(11, 11))
    detinit.load_into(agent, params)
    agent.to(cuda)
    T = 5
    frames = detinit.frames_u8(31, (T, 84, 84, 3))
    ga = GraphActor(agent, 84, 84, B=1, seed=9, chain=chain)
    assert ga.chain == chain
    ga.reset()
    got_a, got_l = [], []
    for t in range(T):
        a = ga.step(frames[t])
        got_a.append(int(a.item()))
        got_l.append(ga.logits.clone())
    P = ref_cpu.tensor_params(params, requires_grad=False)
    rl, _, ra = ref_cpu.unroll(P, torch.from_numpy(frames.astype(np.float32)).unsqueeze(1))
    for t in range(T):
        assert_close(got_l[t].cpu().numpy(), rl[t].numpy(), 1e-4, f"logits t={t}")
        oa, _, margin = ref_cpu.sample_actions(rl[t].numpy(), 9, t)
        if margin[0] > 1e-4:
            assert got_a[t] == int(oa[0]), t
    assert_close(ga.attention.cpu().numpy(), ra[T - 1].numpy(), 1e-4, "attention")
    # reset restarts the episode; an in-place update is re-packed
    with torch.no_grad():
        agent.policy_head[0].bias.add_(1.0)
    ga.reset()
    ga.step(frames[0])
    assert_close(ga.logits.cpu().numpy(), rl[0].numpy() + 1.0, 1e-4, "logits after bias update")


@pytest.mark.parametrize("H,W,B,nq,u8", [(84, 84, 1, 4, True), (84, 84, 3, 8, False), (210, 160, 2, 4, True),
                                         (84, 84, 16, 4, True)])
def test_actor_chain_matches_learner_forward(cuda, H, W, B, nq, u8):
    """aaa_actor_step (six small-B launches) against aaa_forward with T=1 on the
    same carried state, prev_reward/prev_action, frames and packed weights:
    logits, values, attention, h_t, c_t at 1e-4 (only the fp32 summation order
    differs), over three chained steps; and its fused draw is bit-identical to
    aaa_sample_actions on its own logits with the same seed and counter."""
    from aaa_amd.runtime import ActorRunner, UnrollRunner
    A = 18
    params = detinit.deterministic_params(3, A, nq)
    ar = ActorRunner(B, H, W, nq, A, cuda, frames_u8=u8)
    ur = UnrollRunner(B, 1, H, W, nq, A, "fp32", cuda, frames_u8=u8)
    agent = attention.Agent(A, num_queries=nq, grid=(ar.h, ar.w))
    detinit.load_into(agent, params)
    flat = torch.cat([p.detach().reshape(-1) for p in agent.parameters()]).to(cuda)
    assert flat.numel() == ar.n_params
    packed = ar.new_packed()
    ar.pack(flat, packed)
    S = agent.spatial.S.to(cuda).contiguous()
    g = torch.Generator().manual_seed(H + B + nq)
    h = (torch.rand(ar.state_shape(), generator=g) * 2 - 1).to(cuda) * 0.5
    c = (torch.rand(ar.state_shape(), generator=g) * 2 - 1).to(cuda)
    ws, uws = ar.new_workspace(), ur.new_workspace()
    counter = torch.tensor([5], dtype=torch.int64, device=cuda)
    for step in range(3):
        fr = torch.from_numpy(detinit.frames_u8(40 + step, (B, H, W, 3))).to(cuda)
        if not u8:
            fr = fr.float() * 0.5
        pr = torch.rand(B, generator=g).to(cuda)
        pa = torch.randint(0, A, (B,), generator=g).float().to(cuda)
        rl, rv, ra, rh, rc = ur.forward(flat, packed, S, fr.unsqueeze(0), uws, prev_reward=pr, prev_action=pa,
                                        h0=h, c0=c, want_attn=True, want_state=True)
        logits = torch.empty(B, A, device=cuda)
        values = torch.empty(B, A, device=cuda)
        attn = torch.empty(B, ar.h, ar.w, nq, device=cuda)
        acts = torch.empty(B, dtype=torch.int32, device=cuda)
        logp = torch.empty(B, device=cuda)
        jac = torch.empty(B, A, device=cuda)
        c_before = counter.clone()
        ar.step(flat, packed, S, fr, ws, h, c, logits, values, attn=attn, prev_reward=pr, prev_action=pa,
                seed=77, counter=counter, actions=acts, logp=logp, dlogp=jac)
        torch.cuda.synchronize()
        assert_close(logits.cpu().numpy(), rl[0].cpu().numpy(), 1e-4, f"logits step {step}")
        assert_close(values.cpu().numpy(), rv[0].cpu().numpy(), 1e-4, f"values step {step}")
        assert_close(attn.cpu().numpy(), ra[0].cpu().numpy(), 1e-4, f"attention step {step}")
        assert_close(h.cpu().numpy(), rh.cpu().numpy(), 1e-4, f"h step {step}")
        assert_close(c.cpu().numpy(), rc.cpu().numpy(), 1e-4, f"c step {step}")
        assert int(counter.item()) == int(c_before.item()) + 1
        sa, slp = sample_actions(logits, seed=77, counter=c_before)
        assert torch.equal(sa, acts) and torch.equal(slp, logp)
        pj = torch.softmax(logits, -1)
        ref_jac = torch.nn.functional.one_hot(acts.long(), A).float() - pj
        assert float((jac - ref_jac).abs().max()) <= 1e-6
        # continue from the learner's state so both paths see the same inputs next step
        h.copy_(rh)
        c.copy_(rc)


def test_actor_chain_refuses_unsupported(cuda):
    """bf16, stateful-core, T > 1 and B > 16 configurations are refused with AAA_E_ARG
    (they run on aaa_forward), never silently computed."""
    import ctypes
    from aaa_amd import _native as N
    lib = N.load()
    for cfg in (N.Cfg(1, 1, 84, 84, 4, 18, N.BF16, 0), N.Cfg(1, 1, 84, 84, 4, 18, N.F32, N.FLAG_STATEFUL_CORE),
                N.Cfg(1, 2, 84, 84, 4, 18, N.F32, 0), N.Cfg(17, 1, 84, 84, 4, 18, N.F32, 0)):
        assert lib.aaa_actor_workspace_bytes(ctypes.byref(cfg)) == 0
        io = N.ActorIO()
        assert lib.aaa_actor_step(ctypes.byref(cfg), ctypes.byref(io), None) == -1
