"""Data-parallel gradient exchange for the learner.

Each rank runs the full T-step unroll on its own B rows; the only collective
is a SUM all-reduce of the flat fp32 gradient buffer (SUM, not mean, so the
result equals the single-device gradient of the concatenated batch).  The
buffer is cut into three contiguous buckets that become final in backward
phase order, so each bucket's all-reduce is issued as soon as its phase has
been enqueued and overlaps the remaining phases:

  bucket HEAD   = state_dict tensors 16..33 (query MLP, answer MLP, LSTMCell, heads)
  bucket CORE   = tensors 4..15  (ConvLSTM)
  bucket VISION = tensors 0..3   (conv1, conv2)

The reference has no DP at all (Hogwild on CPU, main_mp.py:182-184); this
replaces it with synchronous, deterministic-order RCCL collectives.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import torch
import torch.distributed as dist

HEAD_FIRST, CORE_FIRST, N_TENSORS = 16, 4, 34


def bucket_bounds(offsets: Sequence[int], total: int) -> List[Tuple[int, int]]:
    """[(lo, hi)] element ranges of the HEAD, CORE, VISION buckets (phase order)."""
    assert len(offsets) == N_TENSORS
    return [(offsets[HEAD_FIRST], total), (offsets[CORE_FIRST], offsets[HEAD_FIRST]), (0, offsets[CORE_FIRST])]


def allreduce_buckets(grads: torch.Tensor, bounds, group=None, async_op: bool = True):
    """Issue one SUM all-reduce per bucket; returns the work handles."""
    works = []
    for lo, hi in bounds:
        works.append(dist.all_reduce(grads[lo:hi], op=dist.ReduceOp.SUM, group=group, async_op=async_op))
    return works


def init_from_env(backend: str = "nccl", device=None):
    """torch.distributed init from torchrun's env (RANK/WORLD_SIZE/MASTER_*).
    Call torch.cuda.set_device(LOCAL_RANK) first and pass that ``device``: RCCL
    then binds the communicator to this rank's GPU eagerly."""
    import os
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1:
        return 0, 1, int(os.environ.get("LOCAL_RANK", "0"))
    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        kw = {"device_id": device} if device is not None and backend == "nccl" else {}
        dist.init_process_group(backend=backend, **kw)
    return dist.get_rank(), dist.get_world_size(), int(os.environ.get("LOCAL_RANK", "0"))
