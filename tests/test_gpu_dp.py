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


# (world, dtype, rows per rank, frame side, heads): fp32 per-step kernels (B = 2) and the fp32
# frame-group kernels (B = 16: 8 workgroups per frame); bf16 at B = 32 per rank the paired
# frame-resident kernels, at B = 160 the one-workgroup ones (256-CU part), at 168x168 and B = 16
# the band-mode kernels (4 row bands per frame); each against the full-batch oracle (1e-4 / 2e-2).
# The ranks share ONE GPU here, so a per-rank grid of frame-resident workgroups that need each
# other (frame-group, paired, band) is kept to half the CUs (B = 16 -> 128 workgroups): two ranks'
# grids that together exceed the chip could each hold CUs the other's partners need.  The N-GPU
# driver runs (one rank per GPU) use the full per-GPU shapes.
CASES = [(2, "fp32", 2, 84, 4, None), (3, "fp32", 2, 84, 4, None), (2, "fp32", 16, 84, 4, "frame-group"),
         (2, "bf16", 32, 84, 4, "2 WG per frame"), (2, "bf16", 160, 84, 4, "1 WG per frame"),
         (2, "bf16", 16, 168, 8, "band-mode")]


@pytest.mark.parametrize("world,dtype,b,H,nq,want", CASES)
def test_dp_learner_sums_to_full_batch(world, dtype, b, H, nq, want):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", os.path.join(ROOT, "tools", "dp_check.py")]
    env = dict(os.environ, AAA_DP_BACKEND="gloo", OMP_NUM_THREADS="2", AAA_DP_DTYPE=dtype, AAA_DP_B=str(b),
               AAA_DP_T="3", AAA_DP_H=str(H), AAA_DP_NQ=str(nq), AAA_DP_ORACLE_THREADS="16")
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert p.returncode == 0 and lines, p.stdout[-2000:] + p.stderr[-4000:]
    res = json.loads(lines[-1])
    assert res["ok"] and res["world"] == world, res
    if want:   # the per-rank kernels are the multi-workgroup ones this case is meant to cover
        assert all(want in v for v in res["variants_per_rank"].values()), res


def test_dp_stranded_step_skipped_on_every_rank():
    """a rank whose frame-resident launch strands must not raise
    between its collectives (its peers would hang in an unmatched all-reduce);
    the guard slot skips the update -- and the device-side Adam step count --
    on every rank, check_health() raises afterwards, and the next clean step
    updates every rank identically (tools/dp_check.py AAA_DP_STRAND=1)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", os.path.join(ROOT, "tools", "dp_check.py")]
    env = dict(os.environ, AAA_DP_BACKEND="gloo", OMP_NUM_THREADS="2", AAA_DP_STRAND="1", AAA_DP_B="32")
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert p.returncode == 0 and lines, p.stdout[-2000:] + p.stderr[-4000:]
    res = json.loads(lines[-1])
    assert res["ok"] and res["raised_mid_step"] is None, res
    if not res.get("stranded", True):
        pytest.skip("the filler stranded no rank's launch on this box (premise unmet; both steps ordinary and "
                    "identical on every rank)")
