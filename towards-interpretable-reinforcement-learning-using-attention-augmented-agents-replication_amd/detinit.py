"""Framework-independent deterministic weights and synthetic inputs.

Everything here is exact IEEE fp32 arithmetic on splitmix64 streams, so the
same seed gives bit-identical tensors in the fixture generator (this container,
which imports the reference), in the tests on the GPU box and in bench.py.
That is what lets the golden fixtures under tests/golden/ store only seeds and
fingerprints instead of the 9 MB of weights.

Shapes follow the reference state_dict (attention.py:257-291, listed in
SURVEY.md §8b); ``num_queries`` generalises the query MLP / answer width the
way SURVEY.md Q5 describes (identical to the reference at nq=4).
"""
from __future__ import annotations

import math
from collections import OrderedDict

import numpy as np

_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def splitmix64(seed: int, n: int) -> np.ndarray:
    """n successive outputs of splitmix64 started at ``seed`` (uint64 array)."""
    idx = np.arange(1, n + 1, dtype=np.uint64)
    base = np.full(n, seed & 0xFFFFFFFFFFFFFFFF, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = base + idx * _GOLDEN
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        z = z ^ (z >> np.uint64(31))
    return z


def uniform01(seed: int, n: int) -> np.ndarray:
    """fp32 uniform [0,1) with 24 random bits (exact)."""
    z = splitmix64(seed, n)
    return (z >> np.uint64(40)).astype(np.float32) * np.float32(2.0 ** -24)


def uniform_pm(seed: int, n: int, bound: float) -> np.ndarray:
    """fp32 uniform [-bound, bound): (2u-1) is exact, one rounding for *bound."""
    u = uniform01(seed, n)
    return (u * np.float32(2.0) - np.float32(1.0)) * np.float32(bound)


def param_shapes(num_actions: int = 18, num_queries: int = 4, hidden: int = 256):
    """Ordered (name, shape) list == reference state_dict order (34 tensors)."""
    nq = num_queries
    qd = 72 * nq
    ans_in = (120 + 64) * nq + (8 + 64) * nq + 2
    s = [
        ("vision.vision_cnn.0.weight", (32, 3, 8, 8)),
        ("vision.vision_cnn.0.bias", (32,)),
        ("vision.vision_cnn.1.weight", (64, 32, 4, 4)),
        ("vision.vision_cnn.1.bias", (64,)),
    ]
    for g in "ifco":
        s.append((f"vision.vision_lstm.Wx{g}.weight", (128, 64, 3, 3)))
        s.append((f"vision.vision_lstm.Wx{g}.bias", (128,)))
        s.append((f"vision.vision_lstm.Wh{g}.weight", (128, 128, 3, 3)))
    s += [
        ("query.model.0.weight", (128, hidden)),
        ("query.model.0.bias", (128,)),
        ("query.model.2.weight", (qd, 128)),
        ("query.model.2.bias", (qd,)),
        ("query.model.4.weight", (qd, qd)),
        ("query.model.4.bias", (qd,)),
        ("answer_processor.0.weight", (512, ans_in)),
        ("answer_processor.0.bias", (512,)),
        ("answer_processor.2.weight", (hidden, 512)),
        ("answer_processor.2.bias", (hidden,)),
        ("policy_core.weight_ih", (4 * hidden, hidden)),
        ("policy_core.weight_hh", (4 * hidden, hidden)),
        ("policy_core.bias_ih", (4 * hidden,)),
        ("policy_core.bias_hh", (4 * hidden,)),
        ("policy_head.0.weight", (num_actions, hidden)),
        ("policy_head.0.bias", (num_actions,)),
        ("values_head.0.weight", (num_actions, hidden)),
        ("values_head.0.bias", (num_actions,)),
    ]
    return s


def _fan_in(name: str, shapes: dict) -> int:
    if name.startswith("policy_core."):
        return shapes["policy_core.weight_ih"][1]  # torch LSTMCell: 1/sqrt(hidden)
    wname = name[: -len("bias")] + "weight" if name.endswith("bias") else name
    shp = shapes[wname]
    return int(np.prod(shp[1:]))


def deterministic_params(seed: int = 0, num_actions: int = 18, num_queries: int = 4):
    """OrderedDict name -> fp32 numpy array, uniform(+-1/sqrt(fan_in))."""
    lst = param_shapes(num_actions, num_queries)
    shapes = dict(lst)
    out = OrderedDict()
    for i, (name, shp) in enumerate(lst):
        n = int(np.prod(shp))
        bound = 1.0 / math.sqrt(_fan_in(name, shapes))
        out[name] = uniform_pm((seed << 20) + 7919 * (i + 1), n, bound).reshape(shp)
    return out


def frames_u8(seed: int, shape) -> np.ndarray:
    """uint8 uniform [0,255] frames (splitmix64 seed 1234)."""
    n = int(np.prod(shape))
    return (splitmix64(seed, n) >> np.uint64(56)).astype(np.uint8).reshape(shape)


def normal(seed: int, shape) -> np.ndarray:
    """fp32 N(0, 1) by Box-Muller on two splitmix64 uniform streams (seed, seed
    + 2^32); computed in float64 and rounded once (bench cotangents, SURVEY.md
    §8d: G_l, G_v ~ N(0,1), seed 2)."""
    n = int(np.prod(shape))
    u1 = (splitmix64(seed, n) >> np.uint64(11)).astype(np.float64) * 2.0 ** -53
    u2 = (splitmix64(seed + (1 << 32), n) >> np.uint64(11)).astype(np.float64) * 2.0 ** -53
    r = np.sqrt(-2.0 * np.log1p(-u1))          # u1 in [0, 1): 1 - u1 in (0, 1]
    return (r * np.cos(2.0 * np.pi * u2)).astype(np.float32).reshape(shape)


def cotangent(seed: int, shape) -> np.ndarray:
    """fp32 uniform [-1,1) loss cotangents for logits / values."""
    n = int(np.prod(shape))
    return uniform_pm(seed, n, 1.0).reshape(shape)


def load_into(module, params: dict) -> None:
    """Copy a name->array dict into a torch module's state_dict (any device)."""
    import torch

    sd = module.state_dict()
    with torch.no_grad():
        for k, v in params.items():
            sd[k].copy_(torch.from_numpy(np.ascontiguousarray(v)))
