"""Diagnostic: the fp32 frame-group BPTT (AAA_F32_FRAMES_BWD=1) against the
per-step BPTT (=0) on the same frame-group forward: per-tensor gradient and
dh0/dc0 relative errors for a few (T, B)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import attention  # noqa: E402,F401
from aaa_amd import _native as N, detinit  # noqa: E402
from aaa_amd.runtime import UnrollRunner  # noqa: E402


def run(T, B, bwd):
    os.environ["AAA_F32_FRAMES"] = "8"
    os.environ["AAA_F32_FRAMES_BWD"] = bwd
    dev = torch.device("cuda:0")
    r = UnrollRunner(B, T, 84, 84, 4, 18, "fp32", dev)
    params = detinit.deterministic_params(0, 18)
    flat = torch.from_numpy(np.concatenate([v.reshape(-1) for v in params.values()])).to(dev)
    pk, ws = r.new_packed(), r.new_workspace()
    r.pack(flat, pk)
    basis = attention.SpatialBasis(11, 11).S.to(dev).contiguous()
    X = torch.from_numpy(detinit.frames_u8(1234, (T, B, 84, 84, 3)).astype(np.float32)).to(dev)
    dl = torch.from_numpy(detinit.normal(2, (T, B, 18))).to(dev)
    dv = torch.from_numpy(detinit.normal(3, (T, B, 18))).to(dev)
    r.forward(flat, pk, basis, X, ws, want_attn=False)
    g, dh0, dc0 = r.backward(flat, pk, basis, X, ws, dl, dv, want_state_grads=True)
    torch.cuda.synchronize()
    return g.cpu(), dh0.cpu(), dc0.cpu(), r


for T, B in [(2, 1), (2, 8), (3, 5), (3, 8), (5, 32)]:
    a, ah, ac, r = run(T, B, "1")
    b, bh, bc, _ = run(T, B, "0")
    names = [n for n, _ in detinit.param_shapes(18)]
    errs = []
    for n, o, s in zip(names, r.offsets, r.sizes):
        x, y = a[o:o + s], b[o:o + s]
        if float(y.norm()) > 0:
            errs.append((float((x - y).norm() / y.norm()), n))
    errs.sort(reverse=True)
    print(f"T={T} B={B}: dh0 {float((ah - bh).norm() / bh.norm()):.2e} dc0 {float((ac - bc).norm() / bc.norm()):.2e} "
          f"worst grads {[(f'{e:.1e}', n.split('.')[-2] + '.' + n.split('.')[-1]) for e, n in errs[:6]]}", flush=True)
    print("   pair_status", N.pair_status(clear=True))
