"""share_memory(), parameters() and .to() keep working in
main_mp.py's own process structure (main_mp.py:91-92,178-184): a CPU agent
shared by the parent, two spawned workers that each move it to the GPU, run a
3-step Policy.forward episode, back-propagate the reference's REINFORCE loss
and step torch.optim.Adam; each worker's gradients against the CPU oracle at
1e-4 (tools/share_check.py)."""
import json
import os
import subprocess
import sys

import pytest

from helpers import ROOT

pytestmark = pytest.mark.gpu


def test_share_memory_spawned_workers_train_on_gpu():
    cmd = [sys.executable, os.path.join(ROOT, "tools", "share_check.py")]
    env = dict(os.environ, OMP_NUM_THREADS="4", AAA_SHARE_PROCS="2")
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert lines, p.stdout[-2000:] + p.stderr[-4000:]
    res = json.loads(lines[-1])
    assert p.returncode == 0 and res["ok"], json.dumps(res)[:4000]
    assert res["shared_in_parent"] and res["parent_shared_params_untouched"] and res["state_dict_keys"] == 34
    for w in res["workers"]:
        assert w["shared_in_worker"] and w["params_on_gpu"] and w["params_moved_by_adam"] > 0, w
        assert w["grad_worst_rel_vs_oracle"] <= 1e-4 and w["zero_grads_exact"], w
