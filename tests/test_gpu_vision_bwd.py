"""The frame-resident bf16 vision backward (csrc/vision_bwd.h, round 6): conv2's
weight gradient, conv2's dgrad and conv1's weight gradient of every frame in
one persistent launch (dY1 kept in LDS, the RGBx image rebuilt from the
uint8 observation) against the three layered launches it replaces
(AAA_VIS_BWD_FRAMES=0) -- same bf16 operands, fp32 sums in another order --
and against the bf16-emulated CPU oracle.  The kernel takes uint8
observations only (the environment's dtype); fp32 frames keep the layered
launches.  Reference: attention.py:153-170 (VisionNetwork.vision_cnn) and its
autograd backward through main_mp.py:77."""
import pytest
import torch

from helpers import assert_close, oracle_masks, rel_err
from test_gpu_parity import _agent, _cot, _frames, _grads, _oracle, _run_unroll

import attention

pytestmark = pytest.mark.gpu
N = attention._pkg._native
CONV = ["vision.vision_cnn.0.weight", "vision.vision_cnn.0.bias", "vision.vision_cnn.1.weight",
        "vision.vision_cnn.1.bias"]


def _run_u8(agent, T, B, dev, A=18):
    """tests/test_gpu_parity._run_unroll on the uint8 observations themselves."""
    X = _frames(T, B).to(torch.uint8).to(dev)
    agent.reset()
    lg, vl, at = agent.unroll(X)
    Gl, Gv = _cot(T, B, A)
    ((lg * Gl.to(dev)).sum() + (vl * Gv.to(dev)).sum()).backward()
    torch.cuda.synchronize()
    return lg.detach().cpu(), vl.detach().cpu(), at.detach().cpu(), _grads(agent)


def _grads_with(monkeypatch, cuda, T, B, on, u8=True):
    monkeypatch.setenv("AAA_VIS_BWD_FRAMES", "1" if on else "0")
    monkeypatch.setenv("AAA_VBWD_MINF", "0")   # (the default: no frames-per-CU floor)
    N.timing_enable(True)
    try:
        ag = _agent(cuda, conv_dtype="bf16")
        out = _run_u8(ag, T, B, cuda) if u8 else _run_unroll(ag, T, B, cuda, scale=1.0 / 255.0)
        var = N.timing_stats(N.TIMER_VISION_BWD)["variant"]
    finally:
        N.timing_enable(False)
    return out, var


@pytest.mark.parametrize("T,B", [(3, 3), (2, 40), (20, 16)])
def test_frame_resident_vision_bwd_matches_layered(cuda, monkeypatch, T, B):
    """Every gradient of the fused path against the layered path: the conv
    weight / bias grads within fp32 summation-order noise, the rest identical
    up to that noise (the vision grads feed nothing else)."""
    fused, var = _grads_with(monkeypatch, cuda, T, B, True)
    assert "k_vision_bwd_frames" in var, var
    ref, var0 = _grads_with(monkeypatch, cuda, T, B, False)
    assert "k_vision_bwd_frames" not in var0, var0
    for a, b in zip(fused[:3], ref[:3]):
        assert torch.equal(a, b)   # the forward is untouched
    names = [n for n in CONV if n in fused[3]]
    assert len(names) == 4, sorted(fused[3])
    for n in fused[3]:
        g, r = fused[3][n], ref[3][n]
        if float(r.norm()) == 0.0:
            assert float(g.abs().max()) == 0.0, n
            continue
        tol = 1e-4 if n in CONV else 1e-6
        assert rel_err(g.numpy(), r.numpy()) <= tol, (n, rel_err(g.numpy(), r.numpy()))


def test_fp32_frames_keep_layered_vision_bwd(cuda, monkeypatch):
    """fp32 observations never reach the fused kernel (uint8 only)."""
    _, var = _grads_with(monkeypatch, cuda, 2, 3, True, u8=False)
    assert "k_vision_bwd_frames" not in var, var


def test_frame_resident_vision_bwd_vs_oracle(cuda, monkeypatch):
    """The conv grads of the fused path (uint8 frames) against the bf16-emulated
    oracle on the same pixel values (2e-2), the oracle run through the HIP
    path's own ReLU masks as in every bf16 check."""
    T, B = 4, 5
    monkeypatch.setenv("AAA_VIS_BWD_FRAMES", "1")
    monkeypatch.setenv("AAA_VBWD_MINF", "0")
    ag = _agent(cuda, conv_dtype="bf16")
    ag.relu_trace = []
    out = _run_u8(ag, T, B, cuda)
    ref = _oracle(T, B, conv_mode="bf16", kink_limit=0, masks=oracle_masks(ag.relu_trace, B))
    for n in CONV:
        assert_close(out[3][n].numpy(), ref[3][n].float().numpy(), 2e-2, f"fused vision bwd {n}")
