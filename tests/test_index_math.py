"""Index arithmetic and size limits of the kernels (host-side, no GPU).

Every pixel / tap / tile index in the GEMM loaders and epilogues is divided by
a runtime constant through one multiply-shift divider (csrc/common.h FastDiv).
Round 1's divider was exact only while n*d < 2^32, which conv1's 5.38 M pixel
rows at 168x168 (config 5, d = 1681) broke.  Here the divider is checked
against the exact quotient over its WHOLE domain (every n < 2^31) for every
divisor the geometry of configs C1-C5 -- per GPU and as global batches --
produces, and the runtime must refuse shapes whose operands leave the 32-bit
buffer-descriptor range instead of wrapping.
"""
import ctypes
import random

import pytest

import attention  # noqa: F401
from aaa_amd import _native as N

FULL = 1 << 31

# (name, B, T, H, W, nq): BASELINE.json configs; C4/C5 per GPU under DP and as
# the global batch; G6 is the reference's own 210x160 default-basis frame
CONFIGS = [
    ("C1", 1, 20, 84, 84, 4), ("C2", 32, 20, 84, 84, 4), ("C3", 256, 20, 84, 84, 4),
    ("C4/gpu", 128, 20, 84, 84, 4), ("C5/gpu", 64, 50, 168, 168, 8),
    ("C4/global", 1024, 20, 84, 84, 4), ("C5/global", 512, 50, 168, 168, 8), ("G6", 1, 2, 210, 160, 4),
]


def _geometry(H, W):
    def out(n, k, s, p):
        return (n + 2 * p - k) // s + 1
    H1, W1 = out(H, 8, 4, 1), out(W, 8, 4, 1)
    h, w = out(H1, 4, 2, 2), out(W1, 4, 2, 2)
    return H1, W1, h, w


def _divisors(H, W):
    """The divisors runtime.hip builds for one frame size: ConvGeo's Cin / KW /
    Wout / Hout*Wout of every conv (conv1 on the bordered RGBx image, conv2,
    the ConvLSTM x / h / [x|h] convs, their dgrad and wgrad gathers, conv2's
    four dgrad parity classes) and the parity-class epilogue's Ha*Wa / Wa."""
    H1, W1, h, w = _geometry(H, W)
    ds = {4, 32, 64, 128, 192, 512,              # Cin
          8, 4, 3, 2,                            # KW
          W1, w, H1 * W1, h * w}                 # Wout, Hout*Wout
    for py in (0, 1):
        for px in (0, 1):
            Ha, Wa = (H1 - py + 1) // 2, (W1 - px + 1) // 2
            ds |= {Wa, Ha * Wa}
    return sorted(ds)


def test_divider_exact_over_its_whole_domain_for_every_config_divisor():
    ds = set()
    for _, B, T, H, W, _ in CONFIGS:
        ds |= set(_divisors(H, W))
    bad = {d: N.fastdiv_check(d, 0, FULL) for d in sorted(ds)}
    assert not any(bad.values()), {d: n for d, n in bad.items() if n}


def test_round1_divider_would_have_failed_at_c5():
    """The failure mode this replaces: with m = ceil(2^32 / 1681), q = n*m >> 32
    is one too large first at conv1 row 3,728,457 of config 5 (frame 2217,
    pixel 1680) -- inside the 5,379,200 rows C5 has per GPU."""
    d, rows = 1681, 64 * 50 * 41 * 41
    m = ((1 << 32) + d - 1) // d
    first = next(n for n in range(3_700_000, rows) if (n * m) >> 32 != n // d)
    assert first == 3_728_457 < rows
    assert N.fastdiv_check(d, 0, rows) == 0


def test_divider_random_divisors_and_edges():
    rng = random.Random(7)
    for d in [1, 2, 3, 5, 7, (1 << 31) - 1, (1 << 30) + 1, 65535, 65537] + [rng.randrange(1, 1 << 31) for _ in range(40)]:
        assert N.fastdiv_check(d, 0, 1 << 16) == 0, d
        assert N.fastdiv_check(d, FULL - (1 << 16), FULL) == 0, d
        lo = rng.randrange(0, FULL - (1 << 16))
        assert N.fastdiv_check(d, lo, lo + (1 << 16)) == 0, d


def test_divider_rejects_bad_arguments():
    bad = ctypes.c_ulonglong()
    lib = N.load()
    assert lib.aaa_fastdiv_check(0, 0, 10, ctypes.byref(bad)) == -1
    assert lib.aaa_fastdiv_check(3, 0, FULL + 1, ctypes.byref(bad)) == -1


def _cfg(B, T, H, W, nq, dtype):
    return N.Cfg(B, T, H, W, nq, 18, N.BF16 if dtype == "bf16" else N.F32, 0)


@pytest.mark.parametrize("name,B,T,H,W,nq", CONFIGS)
@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_size_limits(name, B, T, H, W, nq, dtype):
    """The whole-batch conv GEMMs run in frame chunks whose descriptor-addressed
    operands stay below 2 GiB, so a batch is limited only by one step's
    operands fitting one descriptor and by the int element range of the
    activations; beyond that the shape is refused (AAA_E_ARG), never wrapped."""
    lib = N.load()
    H1, W1, h, w = _geometry(H, W)
    F, e = B * T, (2 if dtype == "bf16" else 4)
    per_frame = max(h * w * 512 * e, (H + 2) * (W + 2) * 4 * e, H1 * W1 * 32 * e, H * W * 3 * 4)
    elems = max(F * h * w * 512, F * H * W * 3)
    ws = lib.aaa_workspace_bytes(ctypes.byref(_cfg(B, T, H, W, nq, dtype)))
    if B * per_frame < FULL and elems < FULL:
        assert ws > 0, lib.aaa_last_error()
        assert F * H1 * W1 < FULL      # every row index of the kernels is an exact int
    else:
        assert ws == 0
        assert b"2 GiB" in lib.aaa_last_error() or b"int index" in lib.aaa_last_error()
        assert name == "C5/global", name     # only C5's undistributed 25,600-frame batch is refused


def test_per_gpu_shapes_of_the_baseline_configs_fit():
    for name, B, T, H, W, nq in CONFIGS:
        if name == "C5/global":
            continue
        for dt in ("fp32", "bf16"):
            assert N.load().aaa_workspace_bytes(ctypes.byref(_cfg(B, T, H, W, nq, dt))) > 0, (name, dt)


def test_conv_entry_refuses_descriptor_overflow():
    lib = N.load()
    d = N.ConvDesc(40000, 168, 168, 32, 168, 168, 32, 3, 3, 1, 1, N.F32)   # 144 GB input
    assert lib.aaa_conv2d_nhwc(ctypes.byref(d), 16, 16, None, 16, None) == -1
    assert b"2 GiB" in lib.aaa_last_error()


def test_component_layouts():
    lib = N.load()
    c = N.CellDesc(4, 11, 11, N.F32)
    assert lib.aaa_convlstm_packed_bytes(ctypes.byref(c)) >= 512 * 1728 * 4
    assert lib.aaa_convlstm_workspace_bytes(ctypes.byref(c)) >= 4 * 121 * 512 * 4
    assert lib.aaa_convlstm_workspace_bytes(ctypes.byref(N.CellDesc(0, 11, 11, N.F32))) == 0
    assert lib.aaa_convlstm_workspace_bytes(ctypes.byref(N.CellDesc(1 << 16, 64, 64, N.F32))) == 0   # > 2 GiB
    v = N.CnnDesc(8, 84, 84, N.BF16)
    assert 0 < lib.aaa_vision_cnn_packed_bytes(ctypes.byref(v)) < lib.aaa_packed_bytes(
        ctypes.byref(_cfg(8, 1, 84, 84, 4, "bf16")))
    assert lib.aaa_vision_cnn_workspace_bytes(ctypes.byref(v)) > 8 * 86 * 86 * 4 * 2
    assert lib.aaa_attn_fwd(1, 11, 11, 5, 16, 16, 16, 0, None, None, 16, 16, None) == -1
    assert b"nq" in lib.aaa_last_error()
