"""Device REINFORCE loss (csrc/loss.hip, aaa_reinforce) against the oracle's
restatement of finish_episode (main_mp.py:62-77), which is pinned to the
reference by golden fixture G5 (recorded actions / rewards of a T=12 episode).
"""
import numpy as np
import pytest
import torch

from helpers import assert_close, check_fp, detinit
from oracle import ref_cpu

import attention
from aaa_amd.reinforce import reinforce_loss

pytestmark = pytest.mark.gpu


def _oracle(logits_cpu, actions, rewards, gamma=0.99):
    l = logits_cpu.clone().requires_grad_(True)
    loss = ref_cpu.reinforce_loss(l, actions, rewards, gamma)
    loss.backward()
    return float(loss), l.grad


@pytest.mark.parametrize("T,A,seed", [(12, 18, 0), (1000, 18, 1), (3, 5, 2), (517, 18, 3)])
def test_reinforce_matches_oracle(cuda, T, A, seed):
    g = torch.Generator().manual_seed(seed)
    logits = torch.randn(T, 1, A, generator=g) * 3
    actions = torch.randint(0, A, (T,), generator=g).tolist()
    rewards = (torch.rand(T, generator=g) < 0.2).double().mul(10).tolist()
    rl, rg = _oracle(logits, actions, rewards)
    dl = logits.to(cuda).requires_grad_(True)
    loss = reinforce_loss(dl, actions, rewards)
    loss.backward()
    torch.cuda.synchronize()
    assert abs(float(loss) - rl) <= 1e-4 * max(1.0, abs(rl))   # the reference sums T float32 terms in float32
    err = float((dl.grad.cpu() - rg).abs().max())
    assert err <= 1e-5 * max(float(rg.abs().max()), 1e-30), err


def test_reinforce_batched_episodes_are_independent(cuda):
    g = torch.Generator().manual_seed(9)
    T, B, A = 40, 6, 18
    logits = torch.randn(T, B, A, generator=g)
    actions = torch.randint(0, A, (T, B), generator=g)
    rewards = torch.randn(T, B, generator=g)
    dl = logits.to(cuda).requires_grad_(True)
    loss = reinforce_loss(dl, actions, rewards, gamma=0.95)
    loss.backward()
    tot = 0.0
    for b in range(B):
        rl, rg = _oracle(logits[:, b:b + 1], actions[:, b].tolist(), rewards[:, b].tolist(), gamma=0.95)
        tot += rl
        err = float((dl.grad[:, b:b + 1].cpu() - rg).abs().max())
        assert err <= 1e-5 * max(float(rg.abs().max()), 1e-30), (b, err)
    assert abs(float(loss) - tot) <= 1e-4 * max(1.0, abs(tot))


def test_reinforce_saturated_policy_clamp(cuda):
    """A probability clamped to [eps, 1-eps] (torch's probs_to_logits) passes no gradient."""
    T, A = 4, 6
    logits = torch.zeros(T, 1, A)
    logits[0, 0, 2] = 60.0            # p ~ 1 -> clamped at 1 - eps
    logits[1, 0, 3] = -60.0           # chosen action with p ~ 0 -> clamped at eps
    actions = [2, 3, 1, 0]
    rewards = [1.0, 0.0, 2.0, 1.0]
    rl, rg = _oracle(logits, actions, rewards)
    dl = logits.to(cuda).requires_grad_(True)
    loss = reinforce_loss(dl, actions, rewards)
    loss.backward()
    assert abs(float(loss) - rl) <= 1e-4 * max(1.0, abs(rl))   # the reference sums T float32 terms in float32
    assert torch.allclose(dl.grad.cpu(), rg, rtol=1e-5, atol=1e-7)
    assert float(dl.grad[0].abs().max()) == 0.0 and float(dl.grad[1].abs().max()) == 0.0


def test_reinforce_episode_through_agent_matches_g5(cuda, golden):
    """G5 end to end: unroll the recorded episode on the HIP path, device REINFORCE
    loss, hand-written backward -> parameter gradients vs the reference's."""
    g = golden("G5")
    T = int(g["T"])
    ag = attention.Agent(18, grid=(11, 11))
    detinit.load_into(ag, detinit.deterministic_params(0, 18, 4))
    ag.to(cuda)
    X = torch.from_numpy(detinit.frames_u8(1234, (T, 84, 84, 3)).astype(np.float32)).unsqueeze(1).to(cuda)
    ag.reset()
    lg, _, _ = ag.unroll(X)
    assert_close(lg.detach().cpu().numpy(), g["logits"], 1e-4, "logits")
    loss = reinforce_loss(lg, g["actions"], g["rewards"])
    loss.backward()
    torch.cuda.synchronize()
    for n, p in ag.named_parameters():
        v = (p.grad if p.grad is not None else torch.zeros_like(p)).detach().cpu().numpy()
        assert check_fp(g, "g_", n, v, 1e-4) <= 1e-4, n
