"""Diagnostic: the fused vision backward vs the layered launches, per conv tensor, uint8 and fp32 frames."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np, torch
import attention
from aaa_amd import detinit
from helpers import rel_err
A = 18
def run(on, u8, T=3, B=3):
    os.environ["AAA_VIS_BWD_FRAMES"] = "1" if on else "0"
    ag = attention.Agent(A, grid=(11, 11), conv_dtype="bf16")
    detinit.load_into(ag, detinit.deterministic_params(0, A)); ag.to("cuda")
    X = torch.from_numpy(detinit.frames_u8(1234, (T, B, 84, 84, 3)))
    X = (X if u8 else X.float()).cuda()
    ag.reset(); lg, vl, at = ag.unroll(X)
    Gl = torch.from_numpy(detinit.cotangent(2, (T, B, A))).cuda(); Gv = torch.from_numpy(detinit.cotangent(3, (T, B, A))).cuda()
    ((lg * Gl).sum() + (vl * Gv).sum()).backward(); torch.cuda.synchronize()
    return {n: p.grad.detach().cpu().clone() for n, p in ag.named_parameters() if "vision_cnn" in n}
for u8 in (True, False):
    a, b = run(True, u8), run(False, u8)
    for n in a:
        print("u8" if u8 else "f32", n, "rel", rel_err(a[n].numpy(), b[n].numpy()))
    w, r = a["vision.vision_cnn.0.weight"], b["vision.vision_cnn.0.weight"]   # (32, 3, 8, 8)
    d = (w - r).abs().amax(dim=(0, 1))
    print("conv1 max |diff| per (kh, kw):\n", (d / r.abs().max()).numpy().round(3))
