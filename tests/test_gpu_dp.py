"""The data-parallel learner on the GPU: tools/dp_check.py under
torch.distributed.run, 2 and 3 ranks on cuda:0 over gloo (one device on this
box; the N-GPU driver runs use RCCL, one rank per GPU).  The summed bucketed
gradient must equal the single-process full-batch gradient and the CPU
oracle's full-batch gradient, and no backward phase may write a bucket whose
all-reduce an earlier phase already issued."""
import json
import os
import socket
import subprocess
import sys

import pytest

from helpers import ROOT

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


# (world, dtype, rows per rank): fp32 per-step kernels; bf16 at B = 32 per rank
# runs the paired frame-resident kernels, at B = 160 the one-workgroup ones
# (256-CU part); each against the full-batch oracle (1e-4 / 2e-2)
@pytest.mark.parametrize("world,dtype,b", [(2, "fp32", 2), (3, "fp32", 2), (2, "bf16", 32), (2, "bf16", 160)])
def test_dp_learner_sums_to_full_batch(world, dtype, b):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", os.path.join(ROOT, "tools", "dp_check.py")]
    env = dict(os.environ, AAA_DP_BACKEND="gloo", OMP_NUM_THREADS="2", AAA_DP_DTYPE=dtype, AAA_DP_B=str(b),
               AAA_DP_T="3", AAA_DP_ORACLE_THREADS="16")
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert p.returncode == 0 and lines, p.stdout[-2000:] + p.stderr[-4000:]
    res = json.loads(lines[-1])
    assert res["ok"] and res["world"] == world, res
    if dtype == "bf16":   # the per-rank kernels are the frame-resident ones this case is meant to cover
        want = "2 WG per frame" if b < 160 else "1 WG per frame"
        assert all(want in v for v in res["variants_per_rank"].values()), res
