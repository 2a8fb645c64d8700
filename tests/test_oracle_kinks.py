"""The kink envelope of the bf16 gradient comparisons (helpers.kink_envelope),
justified on the oracle alone (CPU).

The reference's gradient is discontinuous at the answer MLP's ReLU
(attention.py:277-282): where a pre-activation of answer_processor.0 sits
within a few 1e-6 of zero, any evaluation whose forward differs by rounding
may put that unit on the other side, which switches the frame's cotangent
path through it.  On the bf16 path the readout reads h_t rounded to bf16, so
rounding flips of single h elements move those pre-activations by ~1e-6.

Pinned here: at T=20, B=3 (test_gpu_parity's frame-resident case) perturbing
h_t by 1e-6 (relative) before its bf16 rounding flips exactly one near-zero
unit, which moves the ConvLSTM weight gradients by ~2% norm-relative --
beyond the 2e-2 criterion -- while the perturbed gradients stay inside the
oracle's own kink envelope; without the bf16 rounding the same perturbation
moves them by ~1e-6.
"""
import numpy as np
import torch

from helpers import assert_close, detinit, kink_envelope, rel_err
from oracle import ref_cpu

T, B, A = 20, 3, 18


def _run(pert, h_store="bf16", probe=None):
    P = ref_cpu.tensor_params(detinit.deterministic_params(0, A, 4))
    X = torch.from_numpy(detinit.frames_u8(1234, (T, B, 84, 84, 3)).astype(np.float32))
    Gl = torch.from_numpy(detinit.cotangent(2, (T, B, A)))
    Gv = torch.from_numpy(detinit.cotangent(3, (T, B, A)))
    gen = torch.Generator().manual_seed(7)
    rb = ref_cpu._RoundBf16

    class Perturbed(torch.autograd.Function):
        @staticmethod
        def forward(ctx, h):
            hp = h * (1 + pert * torch.randn(h.shape, generator=gen))
            return ref_cpu._bf(hp) if h_store == "bf16" else hp

        @staticmethod
        def backward(ctx, g):
            return g

    ref_cpu._RoundBf16 = Perturbed
    try:
        lg, vl, _ = ref_cpu.unroll(P, X, conv_mode="bf16", h_store="bf16", kinks=probe)
    finally:
        ref_cpu._RoundBf16 = rb
    loss = (lg * Gl).sum() + (vl * Gv).sum()
    return P, loss, lg.detach()


def test_one_near_zero_relu_unit_moves_the_gradient_and_the_envelope_covers_it():
    torch.set_num_threads(min(8, torch.get_num_threads()))
    probe = ref_cpu.KinkProbe()
    P, loss, lg = _run(0.0, probe=probe)
    g, env, units = kink_envelope(loss, P, probe)
    assert units, "no answer-MLP pre-activation within KINK_EPS of zero at this input"
    assert units[0][2] < 2e-6, units[0]          # the unit the perturbation flips (step 7: -1.4e-6)
    Pp, lossp, lgp = _run(1e-6)
    lossp.backward()
    assert rel_err(lgp.numpy(), lg.numpy()) < 1e-5           # the forward barely moves
    n = "vision.vision_lstm.Wxc.weight"
    moved = rel_err(Pp[n].grad.numpy(), g[n].numpy())
    assert moved > 5e-3, moved                                # ... the gradient jumps (measured 1.8e-2)
    for k in g:
        if float(g[k].norm()) > 0:
            assert_close(Pp[k].grad.numpy(), g[k].numpy(), 2e-2, "perturbed oracle " + k, envelope=env[k].numpy())


def test_without_rounding_the_same_perturbation_is_smooth():
    P, loss, _ = _run(0.0, h_store="fp32")
    loss.backward()
    Pp, lossp, _ = _run(1e-6, h_store="fp32")
    lossp.backward()
    n = "vision.vision_lstm.Wxc.weight"
    assert rel_err(Pp[n].grad.numpy(), P[n].grad.numpy()) < 1e-4
