"""The paired frame-resident ConvLSTM kernels (two cooperating workgroups per
frame: recur.h G = 2, recur_bwd.h k_convlstm_bwd_pairs) report a partner wait
that times out instead of returning results computed from a stale half.

Reference: the recurrence they run is attention.py:117-125 (ConvLSTMCell
forward) and its autograd backward (main_mp.py:77).  These tests only pin the
health channel -- the numerics of the same launches are covered by
test_gpu_parity.py::test_c3_c4_full_size_bf16_vs_emulated_oracle[128].
"""
import numpy as np
import pytest
import torch

from helpers import detinit
import attention

N = attention._pkg._native
R = attention._pkg.runtime

pytestmark = pytest.mark.gpu

T, B = 20, 128   # config 4's per-GPU shape: B below the CU count -> the paired kernels


def _run(cuda, runner, flat, packed, basis, frames, ws, dl):
    runner.forward(flat, packed, basis, frames, ws, want_attn=False)
    runner.backward(flat, packed, basis, frames, ws, dl)


def _setup(cuda):
    runner = R.UnrollRunner(B, T, 84, 84, dtype="bf16", device=cuda, frames_u8=True)
    params = detinit.deterministic_params(0, 18)
    flat = torch.cat([torch.from_numpy(np.asarray(v, np.float32)).reshape(-1) for v in params.values()]).to(cuda)
    packed, ws = runner.new_packed(), runner.new_workspace()
    runner.pack(flat, packed)
    basis = attention.SpatialBasis(11, 11).S.to(cuda).contiguous()
    frames = torch.from_numpy(detinit.frames_u8(1234, (T, B, 84, 84, 3))).to(cuda)
    dl = torch.from_numpy(detinit.cotangent(2, (T, B, 18))).to(cuda)
    return runner, flat, packed, basis, frames, ws, dl


def test_paired_kernels_run_and_report_clean(cuda):
    """At C4's per-GPU shape the forward and the BPTT dispatch the paired
    kernels (the variant the library reports), and no partner wait times out."""
    args = _setup(cuda)
    N.pair_status(clear=True)
    N.timing_enable(True)
    try:
        _run(cuda, *args)
        fwd = N.timing_stats(N.TIMER_FWD_STEP)
        bwd = N.timing_stats(N.TIMER_BPTT_STEP)
    finally:
        N.timing_enable(False)
    assert "2 WG per frame" in fwd["variant"], fwd
    assert "2 WG per frame" in bwd["variant"], bwd
    assert N.pair_status(clear=True) == 0


def test_stranded_pair_is_reported(cuda):
    """With half the CUs held by a filler kernel past the partner-wait budget,
    some wait expires: the report word counts it, and the next API
    call fails with AAA_E_STRANDED (once) instead of silently continuing."""
    from test_gpu_coresidency import strand_next_launch
    args = _setup(cuda)
    N.pair_status(clear=True)
    with strand_next_launch(cuda):
        runner, flat, packed, basis, frames, ws, dl = args
        runner.forward(flat, packed, basis, frames, ws, want_attn=False)
    n = N.pair_status(clear=False)
    assert n > 0, "no partner wait expired beside the filler"
    with pytest.raises(RuntimeError, match=r"status -5"):
        runner.forward(flat, packed, basis, frames, ws, want_attn=False)
    assert N.pair_status(clear=True) == 0   # consumed by the failing call
    _run(cuda, *args)                       # default budget: clean again
    assert N.pair_status(clear=True) == 0
