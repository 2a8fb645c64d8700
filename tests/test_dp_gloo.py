"""Data-parallel gradient exchange on CPU (gloo, world_size 2).

Each rank computes the oracle gradients of its half of the batch and the
ranks exchange them with aaa_amd.parallel.allreduce_buckets -- the exact
bucketed SUM all-reduce the GPU learner issues after each backward phase.
The result must equal the single-process gradient of the full batch
(SUM, not mean).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from helpers import detinit

import attention  # noqa: F401
from aaa_amd import parallel

T, B = 2, 4


def _flat_grads(P):
    return torch.cat([(p.grad if p.grad is not None else torch.zeros_like(p)).reshape(-1) for p in P.values()])


def _oracle_grads(rows):
    from oracle import ref_cpu
    P = ref_cpu.tensor_params(detinit.deterministic_params(0, 18))
    X = torch.from_numpy(detinit.frames_u8(1234, (T, B, 84, 84, 3)).astype(np.float32))[:, rows]
    Gl = torch.from_numpy(detinit.cotangent(2, (T, B, 18)))[:, rows]
    Gv = torch.from_numpy(detinit.cotangent(3, (T, B, 18)))[:, rows]
    lg, vl, _ = ref_cpu.unroll(P, X)
    ((lg * Gl).sum() + (vl * Gv).sum()).backward()
    return _flat_grads(P)


def _offsets():
    sizes = [int(np.prod(s)) for _, s in detinit.param_shapes(18, 4)]
    return list(np.cumsum([0] + sizes[:-1])), sum(sizes)


def _worker(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    half = B // world
    g = _oracle_grads(slice(rank * half, (rank + 1) * half)).contiguous()
    offs, total = _offsets()
    works = []
    for bnd in parallel.bucket_bounds(offs, total):   # phase order, async like the learner
        works += parallel.allreduce_buckets(g, [bnd], async_op=True)
    for w in works:
        w.wait()
    if rank == 0:
        torch.save(g, out_path)
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_bucket_bounds_partition_the_flat_buffer():
    offs, total = _offsets()
    b = parallel.bucket_bounds(offs, total)
    assert b[0][1] == total and b[-1][0] == 0
    assert b[0][0] == b[1][1] and b[1][0] == b[2][1]
    # HEAD bucket = tensors 16..33, CORE = 4..15, VISION = 0..3 (backward phase ownership)
    assert b[0][0] == offs[16] and b[1][0] == offs[4]


def test_init_from_env_single_process(monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert parallel.init_from_env("gloo")[:2] == (0, 1)


@pytest.mark.timeout(300)
def test_two_rank_sum_equals_full_batch(tmp_path):
    out = str(tmp_path / "g.pt")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    got = torch.load(out, weights_only=True)
    ref = _oracle_grads(slice(0, B))
    err = float((got - ref).norm() / ref.norm())
    assert err < 1e-5, err
