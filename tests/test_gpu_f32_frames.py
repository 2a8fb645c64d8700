"""The fp32 frame-group ConvLSTM recurrence (csrc/recur_f32.h: G = 8 or 4
workgroups own a frame for all T steps and exchange h_t through L2; with G = 8
also the frame-group BPTT, csrc/recur_bwd_f32.h, which exchanges dZ) against
the CPU oracle at the fp32 tolerance (1e-4) and against the
per-step launches it replaces (AAA_F32_FRAMES=0).

Reference: attention.py:110-126 (ConvLSTMCell.forward, x- and h-gate convs,
cell update) over T steps from reset(), and its autograd backward.
"""
import numpy as np
import pytest
import torch

from helpers import assert_close, rel_err
from test_gpu_parity import RTOL, _agent, _compare, _frames, _cot, _grads, _oracle, _run_unroll

import attention

pytestmark = pytest.mark.gpu
N = attention._pkg._native


@pytest.mark.parametrize("G", ["8", "4"])
@pytest.mark.parametrize("T,B", [(1, 1), (3, 5), (5, 4), (20, 3), (2, 9)])
def test_f32_frames_vs_oracle(cuda, monkeypatch, T, B, G):
    """Single step, ragged B (padding workgroups of the last XCD column),
    a full T=20 unroll, B not a multiple of 8."""
    monkeypatch.setenv("AAA_F32_FRAMES", G)
    N.timing_enable(True)
    try:
        out = _run_unroll(_agent(cuda), T, B, cuda)
        var = N.timing_stats(N.TIMER_FWD_STEP)["variant"]
        bvar = N.timing_stats(N.TIMER_BPTT_STEP)["variant"]
    finally:
        N.timing_enable(False)
    assert f"{G} WG per frame" in var, var
    if T > 1:
        assert ("frame-group BPTT" in bvar) == (G == "8"), bvar
    _compare(out, _oracle(T, B), RTOL, f"f32 frames G={G} T={T} B={B}: ")
    assert N.pair_status(clear=True) == 0
    monkeypatch.setenv("AAA_F32_FRAMES", "0")
    step = _run_unroll(_agent(cuda), T, B, cuda)
    for a, b, n in zip(out[:3], step[:3], ("logits", "values", "attn")):
        assert_close(a.numpy(), b.numpy(), 1e-5, f"f32 frames vs per-step {n}")
    # the frame-group BPTT (G = 8 only; G = 4 keeps the per-step BPTT) against the per-step launches
    for n in out[3]:
        if float(step[3][n].norm()) > 0:
            assert rel_err(out[3][n].numpy(), step[3][n].numpy()) <= 1e-5, f"f32 frames vs per-step grad {n}"


def test_f32_frames_small_grid_vs_oracle(cuda, monkeypatch):
    """P = 64 (64x64 frames: an 8x8 grid) on the pre-split frame-group kernels.
    The forward's epilogue staging aliases the front of its x image; the images'
    off-grid zero pixels must lie beyond it (round 6: the two slot-matched zero
    pixels at the image end; the single zero pixel at P of round 5 sat inside
    the staging for P < 88)."""
    monkeypatch.setenv("AAA_F32_FRAMES", "8")
    T, B = 4, 3
    N.timing_enable(True)
    try:
        out = _run_unroll(_agent(cuda, grid=(8, 8)), T, B, cuda, H=64, W=64)
        var = N.timing_stats(N.TIMER_FWD_STEP)["variant"]
        bvar = N.timing_stats(N.TIMER_BPTT_STEP)["variant"]
    finally:
        N.timing_enable(False)
    assert "8 WG per frame" in var and "frame-group BPTT" in bvar, (var, bvar)
    _compare(out, _oracle(T, B, H=64, W=64), RTOL, "f32 frames 8x8 grid: ")
    assert N.pair_status(clear=True) == 0


@pytest.mark.parametrize("G", ["8", "4"])
def test_f32_frames_carried_state(cuda, monkeypatch, G):
    """T per-step agent(X_t) calls (main_mp.py:54) -- every call after the first
    starts from a carried, non-zero h (the kernel's h-part at t = 0) -- then one
    backward through all of them (main_mp.py:77)."""
    monkeypatch.setenv("AAA_F32_FRAMES", G)
    T, B = 4, 3
    agent = _agent(cuda)
    X = _frames(T, B).to(cuda)
    Gl, Gv = _cot(T, B)
    agent.reset()
    loss = 0
    lgs = []
    for t in range(T):
        lg, vl = agent(X[t])
        lgs.append(lg.detach().cpu())
        loss = loss + (lg * Gl[t].to(cuda)).sum() + (vl * Gv[t].to(cuda)).sum()
    loss.backward()
    ref = _oracle(T, B)
    assert_close(torch.stack(lgs).numpy(), ref[0].numpy(), RTOL, "carried logits")
    g = _grads(agent)
    for n in ref[3]:
        if float(ref[3][n].norm()) > 0:
            assert_close(g[n].numpy(), ref[3][n].numpy(), RTOL, "carried grad " + n)
