"""Fused Adam (csrc/optim.hip, aaa_adam_step) against torch.optim.Adam on the
CPU -- the optimizer the reference builds at main_mp.py:92 and steps at
main_mp.py:78.  Parameters are compared after several steps at 1e-6 relative
(the kernel evaluates torch's op sequence in fp32; differences are ulps)."""
import numpy as np
import pytest
import torch

import attention  # noqa: F401  (registers aaa_amd)
from aaa_amd import detinit
from aaa_amd.optim import Adam, adam_flat_

pytestmark = pytest.mark.gpu


def _shapes():
    # the 34 reference tensors plus odd sizes (vector tail, scalar path)
    return [tuple(v.shape) for v in detinit.deterministic_params(0, 18, 4).values()] + [(1,), (3,), (1025,), (7, 9)]


def _run(dev, steps=4, **kw):
    g = torch.Generator().manual_seed(5)
    cpu = [torch.randn(s, generator=g) for s in _shapes()]
    grads = [[torch.randn(s, generator=g) * (10.0 ** (i % 3 - 1)) for s in _shapes()] for i in range(steps)]
    for gs in grads:      # exactly-zero gradients (Q1's weight_hh / query.0.weight) stay exactly put
        gs[27].zero_()
    ref = [p.clone().requires_grad_(True) for p in cpu]
    dut = [torch.nn.Parameter(p.clone().to(dev)) for p in cpu]
    o_ref = torch.optim.Adam(ref, foreach=False, **kw)
    o_dut = Adam(dut, **kw)
    for gs in grads:
        for p, q, gg in zip(ref, dut, gs):
            p.grad = gg.clone()
            q.grad = gg.clone().to(dev)
        o_ref.step()
        o_dut.step()
    torch.cuda.synchronize()
    return ref, dut, o_ref, o_dut


@pytest.mark.parametrize("kw", [dict(lr=1e-3), dict(lr=3e-3, weight_decay=0.01), dict(lr=1e-3, amsgrad=True),
                                dict(lr=1e-3, betas=(0.8, 0.99), eps=1e-6, maximize=True)])
def test_adam_matches_torch(cuda, kw):
    ref, dut, o_ref, o_dut = _run(cuda, **kw)
    for i, (p, q) in enumerate(zip(ref, dut)):
        a, b = q.detach().cpu().double(), p.detach().double()
        err = float((a - b).abs().max() / max(float(b.abs().max()), 1e-30))
        assert err < 1e-6, (i, err)
    # state compatible with torch.optim.Adam: same keys, same moments
    sd_r, sd_d = o_ref.state_dict(), o_dut.state_dict()
    for k in sd_r["state"]:
        assert set(sd_r["state"][k]) == set(sd_d["state"][k])
        assert float(sd_r["state"][k]["step"]) == float(sd_d["state"][k]["step"])
        for name in ("exp_avg", "exp_avg_sq"):
            x, y = sd_d["state"][k][name].cpu().double(), sd_r["state"][k][name].double()
            assert float((x - y).abs().max()) <= 1e-6 * max(float(y.abs().max()), 1e-30)
    if not kw.get("weight_decay"):   # zero grad and no decay -> the parameter does not move
        assert torch.equal(dut[27].detach().cpu(), ref[27].detach())


def test_adam_on_agent_after_backward(cuda):
    """The reference loop: backward through the drop-in Agent, then optimizer.step()."""
    ag = attention.Agent(18, grid=(11, 11))
    detinit.load_into(ag, detinit.deterministic_params(0, 18, 4))
    ag.to(cuda)
    opt = Adam(ag.parameters(), lr=1e-3)
    X = torch.from_numpy(detinit.frames_u8(1234, (3, 2, 84, 84, 3)).astype(np.float32)).to(cuda)
    ag.reset()
    lg, vl, _ = ag.unroll(X)
    (lg.sum() + vl.sum()).backward()
    before = {n: p.detach().clone() for n, p in ag.named_parameters()}
    grads = {n: p.grad.detach().cpu() for n, p in ag.named_parameters()}
    opt.step()
    torch.cuda.synchronize()
    ref_params = [before[n].cpu().clone().requires_grad_(True) for n in before]
    o = torch.optim.Adam(ref_params, lr=1e-3, foreach=False)
    for p, n in zip(ref_params, before):
        p.grad = grads[n]
    o.step()
    for (n, p), r in zip(ag.named_parameters(), ref_params):
        err = float((p.detach().cpu() - r.detach()).abs().max())
        assert err <= 1e-6 * max(float(r.detach().abs().max()), 1e-30) + 1e-9, (n, err)
    assert torch.equal(ag.policy_core.weight_hh.detach(), before["policy_core.weight_hh"])
    # the next forward runs on the updated weights (the fused step bumps the
    # parameters' version counters, so the packed-weight cache re-packs)
    fresh = attention.Agent(18, grid=(11, 11))
    fresh.load_state_dict(ag.state_dict())
    fresh.to(cuda)
    ag.reset()
    fresh.reset()
    with torch.no_grad():
        l_next, _, _ = ag.unroll(X)
        l_fresh, _, _ = fresh.unroll(X)
    assert torch.equal(l_next, l_fresh)
    assert not torch.equal(l_next, lg.detach())


def test_adam_flat_matches_torch(cuda):
    g = torch.Generator().manual_seed(7)
    p = torch.randn(2_270_276, generator=g)
    ref = p.clone().requires_grad_(True)
    o = torch.optim.Adam([ref], lr=1e-3, foreach=False)
    dp, dm, dv = p.to(cuda), torch.zeros_like(p, device=cuda), torch.zeros_like(p, device=cuda)
    for step in range(1, 4):
        gr = torch.randn(p.shape, generator=g)
        ref.grad = gr
        o.step()
        adam_flat_(dp, gr.to(cuda), dm, dv, step, lr=1e-3)
    torch.cuda.synchronize()
    err = float((dp.cpu() - ref.detach()).abs().max())
    assert err <= 1e-6 * float(ref.detach().abs().max())
