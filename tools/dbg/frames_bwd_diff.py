"""Debug: per-parameter gradient difference of the frame-resident BPTT vs the per-step path (bf16)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import torch
import test_gpu_parity as tp
from helpers import rel_err
dev = torch.device("cuda")
for T, B in ((1, 1), (3, 2)):
    res = {}
    for fb in ("0", "1"):
        os.environ["AAA_FRAMES_FWD"] = "1"
        os.environ["AAA_FRAMES_BWD"] = fb
        res[fb] = tp._run_unroll(tp._agent(dev, conv_dtype="bf16"), T, B, dev)
    for n in res["0"][3]:
        a, b = res["1"][3][n], res["0"][3][n]
        if float(b.norm()) > 0:
            print(T, B, n, f"{rel_err(a.numpy(), b.numpy()):.3e}", flush=True)
