"""Single-kernel numerics: the gfx950 implicit-GEMM conv (fwd / dgrad / wgrad)
and linear kernels against plain PyTorch on the CPU (fp64 accumulation of the
same fp32 -- or bf16-rounded -- operands)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from helpers import assert_close

import attention  # noqa: F401
from aaa_amd import _native as N

pytestmark = pytest.mark.gpu

CONVS = {
    # name: (N, Hin, Win, Cin, Cout, K, stride, pad)  -- the three convs of the path
    "conv1": (3, 84, 84, 3, 32, 8, 4, 1),
    "conv2": (3, 20, 20, 32, 64, 4, 2, 2),
    "convlstm": (2, 11, 11, 192, 512, 3, 1, 1),
    "odd": (2, 13, 9, 8, 12, 3, 2, 1),
    "conv1_rgbx": (2, 84, 84, 4, 32, 8, 4, 1),   # conv1 on RGBx frames (multi-tap K tiles)
}


def _desc(name, dtype):
    n, H, W, ci, co, k, s, p = CONVS[name]
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    return N.ConvDesc(n, H, W, ci, Ho, Wo, co, k, k, s, p, dtype), (n, H, W, ci, co, k, s, p, Ho, Wo)


def _rnd(shape, seed, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.rand(shape, generator=g) * 2 - 1) * scale


def _r(t, dtype):
    return t.to(torch.bfloat16).float() if dtype == N.BF16 else t


def _tol(dtype):
    return 2e-5 if dtype == N.F32 else 2e-5  # bf16 compares against bf16-rounded operands


@pytest.mark.parametrize("dtype", [N.F32, N.BF16])
@pytest.mark.parametrize("name", list(CONVS))
def test_conv_fwd(cuda, name, dtype):
    d, (n, H, W, ci, co, k, s, p, Ho, Wo) = _desc(name, dtype)
    x = _rnd((n, ci, H, W), 1, 255.0 if ci == 3 else 1.0)
    w = _rnd((co, ci, k, k), 2, 0.1)
    b = _rnd((co,), 3)
    ref = F.conv2d(_r(x, dtype).double(), _r(w, dtype).double(), b.double(), stride=s, padding=p)
    xd = x.permute(0, 2, 3, 1).contiguous().to(cuda)
    wd = w.permute(0, 2, 3, 1).contiguous().to(cuda)
    bd = b.to(cuda)
    y = torch.empty(n, Ho, Wo, co, device=cuda)
    N.check(N.load().aaa_conv2d_nhwc(d, xd.data_ptr(), wd.data_ptr(), bd.data_ptr(), y.data_ptr(),
                                     N.stream_ptr()))
    assert_close(y.permute(0, 3, 1, 2).cpu().numpy(), ref.numpy(), _tol(dtype), f"{name} fwd")


@pytest.mark.parametrize("dtype", [N.F32, N.BF16])
@pytest.mark.parametrize("name", list(CONVS))
def test_conv_dgrad(cuda, name, dtype):
    d, (n, H, W, ci, co, k, s, p, Ho, Wo) = _desc(name, dtype)
    if co % 4:
        pytest.skip("dgrad needs Cout % 4 == 0")
    w = _rnd((co, ci, k, k), 2, 0.1)
    dy = _rnd((n, co, Ho, Wo), 4)
    ref = torch.nn.grad.conv2d_input((n, ci, H, W), _r(w, dtype).double(), _r(dy, dtype).double(),
                                     stride=s, padding=p)
    dyd = dy.permute(0, 2, 3, 1).contiguous().to(cuda)
    wT = w.permute(1, 2, 3, 0).contiguous().to(cuda)
    dx = torch.empty(n, H, W, ci, device=cuda)
    N.check(N.load().aaa_conv2d_nhwc_dgrad(d, dyd.data_ptr(), wT.data_ptr(), dx.data_ptr(), N.stream_ptr()))
    assert_close(dx.permute(0, 3, 1, 2).cpu().numpy(), ref.numpy(), _tol(dtype), f"{name} dgrad")


@pytest.mark.parametrize("dtype", [N.F32, N.BF16])
@pytest.mark.parametrize("name", list(CONVS))
def test_conv_wgrad(cuda, name, dtype):
    d, (n, H, W, ci, co, k, s, p, Ho, Wo) = _desc(name, dtype)
    x = _rnd((n, ci, H, W), 1, 255.0 if ci == 3 else 1.0)
    dy = _rnd((n, co, Ho, Wo), 4)
    ref = torch.nn.grad.conv2d_weight(_r(x, dtype).double(), (co, ci, k, k), _r(dy, dtype).double(),
                                      stride=s, padding=p)
    xd = x.permute(0, 2, 3, 1).contiguous().to(cuda)
    dyd = dy.permute(0, 2, 3, 1).contiguous().to(cuda)
    dw = torch.empty(co, k, k, ci, device=cuda)
    N.check(N.load().aaa_conv2d_nhwc_wgrad(d, xd.data_ptr(), dyd.data_ptr(), dw.data_ptr(), N.stream_ptr()))
    assert_close(dw.permute(0, 3, 1, 2).cpu().numpy(), ref.numpy(), _tol(dtype), f"{name} wgrad")


@pytest.mark.parametrize("M,Nn,K", [(640, 512, 1032), (37, 36, 256), (5, 1024, 256)])
def test_linear(cuda, M, Nn, K):
    x = _rnd((M, K), 5)
    w = _rnd((Nn, K), 6, 0.05)
    b = _rnd((Nn,), 7)
    ref = F.linear(x.double(), w.double(), b.double())
    y = torch.empty(M, Nn, device=cuda)
    xd, wd, bd = x.to(cuda), w.to(cuda), b.to(cuda)   # keep alive until the kernel has run
    N.check(N.load().aaa_linear(M, Nn, K, xd.data_ptr(), wd.data_ptr(), bd.data_ptr(), y.data_ptr(),
                                N.stream_ptr()))
    torch.cuda.synchronize()
    assert_close(y.cpu().numpy(), ref.numpy(), 2e-5, "linear")
