"""The bench's episode leg alone (bench.episode_leg, no CPU oracle), for a
rocprofv3 kernel trace of the fused episode backward and for tile A/B runs:
    rocprofv3 --kernel-trace --stats -d DIR -o run -- python tools/episode_trace.py
    AAA_FUSED_TILE=4 python tools/episode_trace.py --fused-only --reps 3"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--fused-only", action="store_true", help="skip the per-step autograd path")
    ap.add_argument("--reps", type=int, default=1)
    a = ap.parse_args()
    keys = ("backward_ms_device", "ms_per_step_host", "episode_frames_per_s", "graph_bytes_per_step")
    env = {k: v for k, v in os.environ.items() if k.startswith("AAA_")}
    for _ in range(a.reps):
        out = bench.episode_leg(torch.device("cuda:0"), cpu=False, per_step=not a.fused_only)
        row = {"env": env, **{k: out[k] for k in keys}}
        if "per_step_path" in out:
            row["per_step_backward_ms_device"] = out["per_step_path"]["backward_ms_device"]
        print(json.dumps(row), flush=True)
