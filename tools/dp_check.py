"""Data-parallel learner self-check on ONE GPU (tests/test_gpu_dp.py launches it).

Launched by torch.distributed.run with N ranks that all use cuda:0 and the
gloo backend (RCCL refuses two ranks on one device; the driver's N-GPU runs
use RCCL with one rank per GPU).  Each rank runs aaa_amd.learner.Learner.step
on its B/N rows -- the three backward phases with each gradient bucket
all-reduced while the next phase runs -- and rank 0 checks the summed
gradient against a single-process backward of the full batch (SUM, SURVEY.md
§8e).  Prints one JSON line on rank 0; exit status 1 on a mismatch.
"""
import json
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import attention  # noqa: E402,F401
from aaa_amd import detinit  # noqa: E402
from aaa_amd.learner import Learner  # noqa: E402
from aaa_amd.runtime import UnrollRunner  # noqa: E402


def main():
    dist.init_process_group(os.environ.get("AAA_DP_BACKEND", "gloo"))
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    T, Bt, A = 3, 2 * world, 18
    dtype = os.environ.get("AAA_DP_DTYPE", "fp32")
    X = torch.from_numpy(detinit.frames_u8(1234, (T, Bt, 84, 84, 3)).astype(np.float32))
    Gl = torch.from_numpy(detinit.cotangent(2, (T, Bt, A)))
    Gv = torch.from_numpy(detinit.cotangent(3, (T, Bt, A)))
    b = Bt // world
    rows = slice(rank * b, (rank + 1) * b)
    worst = {}
    for overlap in (True, False):
        lr = Learner(b, T, 84, 84, 4, A, dtype, dev)
        lr.step(X[:, rows].contiguous().to(dev), Gl[:, rows].contiguous().to(dev), Gv[:, rows].contiguous().to(dev),
                overlap=overlap, comm_timing=True)
        torch.cuda.synchronize()
        cs = lr.comm_stats()
        assert len(cs["buckets"]) == 3 and all(x["allreduce_ms"] >= 0 for x in cs["buckets"]), cs
        if rank == 0:   # single-process reference over the whole batch, same weights
            r = UnrollRunner(Bt, T, 84, 84, 4, A, dtype, dev)
            pk, ws = r.new_packed(), r.new_workspace()
            r.pack(lr.flat, pk)
            r.forward(lr.flat, pk, lr.basis, X.to(dev), ws, want_attn=False)
            g, _, _ = r.backward(lr.flat, pk, lr.basis, X.to(dev), ws, Gl.to(dev), Gv.to(dev))
            torch.cuda.synchronize()
            err = float((lr.grads - g).norm() / g.norm())
            worst[f"overlap={overlap}"] = err
        dist.barrier()
    if rank == 0:
        ok = all(v <= 1e-5 for v in worst.values())
        print(json.dumps({"world": world, "backend": dist.get_backend(), "dtype": dtype, "rel_err": worst, "ok": ok}),
              flush=True)
    dist.barrier()
    dist.destroy_process_group()
    if rank == 0 and not ok:
        sys.exit(1)


if __name__ == "__main__":
    main()
