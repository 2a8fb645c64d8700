"""Band-mode frame-resident bf16 ConvLSTM forward (csrc/recur.h BAND) and BPTT
(csrc/recur_bwd.h BAND): 168x168 frames (21x21 grid, config 5) split into four
row bands, one workgroup each, exchanging their boundary rows of h_t (forward)
or dZ_t (BPTT) through L2 every step.

Against the bf16-emulated oracle (2e-2) and against the
per-step launches it replaces (AAA_FRAMES_BAND=0: same bf16 operands and fp32
accumulation, only the summation order and gate approximations differ).
Reference: attention.py:110-126 (ConvLSTMCell.forward) over the unroll.
"""
import pytest
import torch

from helpers import assert_close, oracle_masks, rel_err
from test_gpu_parity import _agent, _compare, _cot, _frames, _grads, _oracle, _run_unroll

import attention

pytestmark = pytest.mark.gpu
N = attention._pkg._native


def _run(cuda, monkeypatch, band, T, B, nq=8, trace=None):
    monkeypatch.setenv("AAA_FRAMES_BAND", band)
    N.timing_enable(True)
    try:
        ag = _agent(cuda, nq=nq, grid=(21, 21), conv_dtype="bf16")
        ag.relu_trace = trace
        out = _run_unroll(ag, T, B, cuda, H=168, W=168)
        var = N.timing_stats(N.TIMER_FWD_STEP)["variant"]
        sb = N.timing_stats(N.TIMER_BPTT_STEP)
    finally:
        N.timing_enable(False)
    assert ("band-mode" in var) == (band == "1"), var
    if band == "1":   # one band-mode BPTT launch for the whole chain
        assert sb["launches"] == 1 and "band-mode" in sb["variant"], sb
    else:             # per-step launches (none at T = 1: no dh of an earlier step)
        assert "band-mode" not in sb["variant"], sb
    return out


@pytest.mark.parametrize("T,B,nq", [(1, 1, 8), (3, 5, 8), (4, 9, 4), (50, 2, 8)])
def test_band_forward_vs_per_step(cuda, monkeypatch, T, B, nq):
    """Single step, ragged B (padding workgroups of the last XCD column), B > 8,
    nq 4 and 8, a full T=50 unroll (config 5's length)."""
    band = _run(cuda, monkeypatch, "1", T, B, nq)
    assert N.pair_status(clear=True) == 0
    step = _run(cuda, monkeypatch, "0", T, B, nq)
    for a, b, n in zip(band[:3], step[:3], ("logits", "values", "attn")):
        assert_close(a.numpy(), b.numpy(), 2e-3, f"band vs per-step {n}")
    for n in band[3]:
        if float(step[3][n].norm()) > 0:
            assert rel_err(band[3][n].numpy(), step[3][n].numpy()) <= 5e-3, f"band vs per-step grad {n}"


def test_band_forward_vs_emulated_oracle(cuda, monkeypatch):
    T, B = 3, 5
    trace = []
    out = _run(cuda, monkeypatch, "1", T, B, trace=trace)
    _compare(out, _oracle(T, B, nq=8, conv_mode="bf16", H=168, W=168, masks=oracle_masks(trace, B)), 2e-2,
             "band T=3 B=5: ")


def test_band_carried_state(cuda, monkeypatch):
    """T per-step agent(X_t) calls (main_mp.py:54): every call after the first
    starts the band kernel from a carried h (its halo rows included), then one
    backward through all of them (main_mp.py:77)."""
    T, B = 12, 3

    def run(band):
        monkeypatch.setenv("AAA_FRAMES_BAND", band)
        agent = _agent(cuda, nq=8, grid=(21, 21), conv_dtype="bf16")
        X = _frames(T, B, 168, 168).to(cuda)
        Gl, Gv = _cot(T, B)
        agent.reset()
        loss, lgs = 0, []
        for t in range(T):
            lg, vl = agent(X[t])
            lgs.append(lg.detach().cpu())
            loss = loss + (lg * Gl[t].to(cuda)).sum() + (vl * Gv[t].to(cuda)).sum()
        loss.backward()
        torch.cuda.synchronize()
        return torch.stack(lgs), _grads(agent)

    lb, gb = run("1")
    assert N.pair_status(clear=True) == 0
    ls, gs = run("0")
    assert_close(lb.numpy(), ls.numpy(), 2e-3, "carried band logits")
    for n in gs:
        if float(gs[n].norm()) > 0:
            assert rel_err(gb[n].numpy(), gs[n].numpy()) <= 5e-3, f"carried band grad {n}"
