"""The data-parallel learner on the GPU: tools/dp_check.py under
torch.distributed.run, 2 and 3 ranks on cuda:0 over gloo (one device on this
box; the N-GPU driver runs use RCCL, one rank per GPU).  The summed bucketed
gradient must equal the single-process full-batch gradient."""
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


@pytest.mark.parametrize("world", [2, 3])
def test_dp_learner_sums_to_full_batch(world):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", os.path.join(ROOT, "tools", "dp_check.py")]
    env = dict(os.environ, AAA_DP_BACKEND="gloo", OMP_NUM_THREADS="2")
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert p.returncode == 0 and lines, p.stdout[-2000:] + p.stderr[-4000:]
    res = json.loads(lines[-1])
    assert res["ok"] and res["world"] == world, res
