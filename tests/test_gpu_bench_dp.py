"""bench.py's N > 1 branch, rehearsed on one GPU (VERDICT r05 "make the
multi-GPU path ready for its first run").

The driver's scaling runs launch ``bench.py --gpus N`` under torch.distributed.run
with one rank per GPU over RCCL; that branch (the barrier around the timed
region, the MAX all-reduce of the elapsed time, the per-bucket ``comm`` block
of Learner.comm_stats) otherwise first executes there.  Here two ranks run it
on cuda:0 over gloo (RCCL refuses two ranks on one device) at a per-rank batch
that keeps both ranks' frame-resident grids within the chip together, and
rank 0's JSON line must be the N = 2 line: n_gpus 2, dp2, the whole-job value
over both ranks' frames, and a comm block with both buckets timed.  The
gradient sums themselves are checked against the full-batch oracle by
tests/test_gpu_dp.py (the same Learner)."""
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


# (config, rows per rank, the recurrence variant those rows select): fp32 frame-group kernels
# (B = 16: 128 workgroups per rank) and the bf16 paired frame-resident kernels (B = 32: 64)
CASES = [("c2", 16, "frame-group"), ("c4", 32, "2 WG per frame")]


@pytest.mark.parametrize("config,b,variant", CASES)
def test_bench_two_ranks_line(config, b, variant):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "3", "--warmup", "2", "--config", config, "--batch", str(b),
           "--backend", "gloo", "--same-device"]
    env = dict(os.environ, OMP_NUM_THREADS="2")
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert p.returncode == 0 and len(lines) == 1, p.stdout[-2000:] + p.stderr[-4000:]   # rank 0 prints ONE line
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2" and d["config"]["global_batch"] == 2 * b, d
    assert d["steps"] == 3 and d["scaling"] == "weak" and d["higher_is_better"] is True
    # value = both ranks' frames over the max-over-ranks time of the timed steps
    T = d["config"]["seq_len"]
    assert abs(d["value"] - 2 * b * T * 3 / (d["ms_per_step"] * 3e-3)) <= 1e-3 * d["value"] + 1.0, d["value"]
    comm = d["comm"]
    assert comm["backend"] == "gloo"
    names = [x["bucket"] for x in comm["buckets"]]
    assert names == ["HEAD+CORE (+guard)", "VISION"], names
    assert all(x["allreduce_ms"] >= 0 and x["bytes"] > 0 for x in comm["buckets"]), comm
    assert sum(x["bytes"] for x in comm["buckets"]) == sum(d["allreduce_buckets_bytes"].values()), comm
    assert comm["exposed_ms"] >= 0
    assert variant in d["roofline"]["variant"] or any(variant in k.get("variant", "") for k in d["kernels"].values()), d
