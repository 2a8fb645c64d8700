"""Diagnostic: per-tensor errors of the GPU path and the fp32 oracle vs an fp64 oracle."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np, torch
from helpers import detinit, rel_err
from oracle import ref_cpu
import attention

T, B = int(sys.argv[1]), int(sys.argv[2])
dt = sys.argv[3] if len(sys.argv) > 3 else "fp32"
torch.set_num_threads(16)
dev = torch.device("cuda:0")
prm = detinit.deterministic_params(0, 18)
X = torch.from_numpy(detinit.frames_u8(1234, (T, B, 84, 84, 3)).astype(np.float32))
Gl = torch.from_numpy(detinit.cotangent(2, (T, B, 18))); Gv = torch.from_numpy(detinit.cotangent(3, (T, B, 18)))
ag = attention.Agent(18, grid=(11, 11), conv_dtype=dt); detinit.load_into(ag, prm); ag.to(dev)
ag.reset(); lg, vl, at = ag.unroll(X.to(dev)); ((lg*Gl.to(dev)).sum() + (vl*Gv.to(dev)).sum()).backward()
G = {n: p.grad.detach().cpu().double() for n, p in ag.named_parameters()}
def orc(dtype, mode="fp32"):
    P = ref_cpu.tensor_params(prm, dtype=dtype)
    t0 = time.time()
    l, v, a = ref_cpu.unroll(P, X.to(dtype), conv_mode=mode)
    ((l*Gl.to(dtype)).sum() + (v*Gv.to(dtype)).sum()).backward()
    print(f"oracle {dtype} {mode}: {time.time()-t0:.1f}s")
    return l.detach().double(), {n: (p.grad if p.grad is not None else torch.zeros_like(p)).double() for n, p in P.items()}
l32, g32 = orc(torch.float32, "bf16" if dt == "bf16" else "fp32")
l64, g64 = orc(torch.float64) if dt == "fp32" else (l32, g32)
print(f"logits: gpu-vs-64 {rel_err(lg.detach().cpu().numpy(), l64.numpy()):.2e}  o32-vs-64 {rel_err(l32.numpy(), l64.numpy()):.2e}")
for n in g64:
    if float(g64[n].norm()) == 0: continue
    print(f"{n:40s} gpu-vs-64 {rel_err(G[n].numpy(), g64[n].numpy()):.2e}  o32-vs-64 {rel_err(g32[n].numpy(), g64[n].numpy()):.2e}  gpu-vs-o32 {rel_err(G[n].numpy(), g32[n].numpy()):.2e}")
