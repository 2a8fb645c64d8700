"""CPU checks of the oracle's actor-sampling restatement (oracle/ref_cpu.py
sample_uniform / sample_actions), which the GPU sampler is compared against.

log_prob is pinned to torch.distributions.Categorical -- the object the
reference builds at main_mp.py:55-58 -- and the draw to its distribution.
"""
import numpy as np
import torch

from oracle import ref_cpu


def test_uniform_is_deterministic_and_in_range():
    u = [ref_cpu.sample_uniform(123, c, r) for c in range(4) for r in range(256)]
    assert u == [ref_cpu.sample_uniform(123, c, r) for c in range(4) for r in range(256)]
    u = np.array(u)
    assert u.min() >= 0.0 and u.max() < 1.0
    assert abs(u.mean() - 0.5) < 0.03 and abs(u.var() - 1 / 12) < 0.01
    assert len(set(u.tolist())) > 0.99 * u.size          # counters and rows give distinct draws
    assert np.all(u * 16777216.0 == np.floor(u * 16777216.0))   # 24-bit grid: exact in fp32


def test_log_prob_matches_categorical():
    g = torch.Generator().manual_seed(0)
    for scale in (0.1, 3.0, 30.0):
        logits = torch.randn(64, 18, generator=g) * scale
        acts, logp, _ = ref_cpu.sample_actions(logits.numpy(), 5, 1)
        ref = torch.distributions.Categorical(torch.softmax(logits, -1)).log_prob(torch.from_numpy(acts))
        assert np.abs(ref.numpy() - logp).max() <= 2e-6 * max(1.0, float(ref.abs().max()))


def test_draws_follow_softmax():
    logits = np.array([[2.0, 0.0, -1.0, 1.0, 0.5, -3.0]], np.float32)
    p = np.exp(logits[0] - logits[0].max())
    p /= p.sum()
    n = 20000
    acts, _, _ = ref_cpu.sample_actions(np.repeat(logits, n, 0), 99, 0)
    freq = np.bincount(acts, minlength=6) / n
    chi2 = float((((freq - p) ** 2) / p).sum() * n)
    assert chi2 < 25.0, (chi2, freq, p)                    # 5 dof: p(chi2 > 25) ~ 1e-4
