"""CPU-side checks of the C ABI: the library loads, exports every symbol
include/aaa.h declares, and its layout queries agree with the reference's
state_dict (no GPU compute is issued here)."""
import ctypes
import os
import re

import numpy as np
import pytest

from helpers import ROOT, detinit

import attention  # noqa: F401
from aaa_amd import _native as N

HEADER = os.path.join(ROOT, "include", "aaa.h")


def _declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(aaa_[a-z0-9_]+)\s*\(", src)))


def test_header_matches_binding_list():
    assert _declared() == sorted(N.EXPORTS)


def test_library_exports_every_declared_symbol():
    lib = N.load()
    for name in _declared():
        assert hasattr(lib, name), name


def test_abi_version():
    assert N.load().aaa_abi_version() == N.ABI_VERSION == 9


@pytest.mark.parametrize("H,W,hw", [(84, 84, (11, 11)), (168, 168, (21, 21)), (210, 160, (27, 20))])
def test_grid(H, W, hw):
    assert N.grid(H, W) == hw


@pytest.mark.parametrize("nq,total", [(4, 2270276), (8, 3080836)])
def test_param_layout_matches_state_dict(nq, total):
    cfg = N.Cfg(2, 3, 84, 84, nq, 18, N.F32, 0)
    n, offs, sizes = N.param_layout(cfg)
    assert n == total
    shapes = detinit.param_shapes(18, nq)
    assert sizes == [int(np.prod(s)) for _, s in shapes]
    assert offs == list(np.cumsum([0] + sizes[:-1]))


def test_layout_sizes_and_errors():
    lib = N.load()
    ok = N.Cfg(32, 20, 84, 84, 4, 18, N.F32, 0)
    ws = lib.aaa_workspace_bytes(ctypes.byref(ok))
    pk = lib.aaa_packed_bytes(ctypes.byref(ok))
    assert ws > 32 * 20 * 121 * 128 * 4 and pk > 512 * 1728 * 4
    bf = N.Cfg(32, 20, 84, 84, 4, 18, N.BF16, 0)
    assert lib.aaa_packed_bytes(ctypes.byref(bf)) < pk
    bad = N.Cfg(32, 20, 84, 84, 5, 18, N.F32, 0)
    assert lib.aaa_workspace_bytes(ctypes.byref(bad)) == 0
    assert b"nq" in lib.aaa_last_error()
    bad_rc = lib.aaa_forward(ctypes.byref(bad), None, None)
    assert bad_rc == -1


def test_agent_refuses_cpu_tensors():
    import torch
    agent = attention.Agent(18, grid=(11, 11))
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        agent(torch.zeros(1, 84, 84, 3))


def test_state_dict_keys_match_reference_order():
    agent = attention.Agent(18)
    keys = list(agent.state_dict().keys())
    assert keys == [n for n, _ in detinit.param_shapes(18, 4)]
    assert len(list(agent.buffers())) == 0


def test_adam_rejects_bad_args_without_gpu():
    lib = N.load()
    hp = N.AdamHP(1e-3, 0.9, 0.999, 1e-8, 0.0, 0, 0)
    assert lib.aaa_adam_step(ctypes.byref(hp), 0, 0, None, None, None, None, None, None, None) == -1   # step < 1
    assert b"step" in lib.aaa_last_error()
    bad = N.AdamHP(1e-3, 1.0, 0.999, 1e-8, 0.0, 0, 0)
    assert lib.aaa_adam_step(ctypes.byref(bad), 1, 0, None, None, None, None, None, None, None) == -1
    ams = N.AdamHP(1e-3, 0.9, 0.999, 1e-8, 0.0, 1, 0)
    one = (ctypes.c_void_p * 1)(16)
    n = (ctypes.c_size_t * 1)(4)
    assert lib.aaa_adam_step(ctypes.byref(ams), 1, 1, one, one, one, one, None, n, None) == -1     # amsgrad w/o vmax


def test_adam_optimizer_has_no_cpu_fallback():
    import torch
    from aaa_amd.optim import Adam
    p = torch.nn.Parameter(torch.zeros(4))
    p.grad = torch.ones(4)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        Adam([p]).step()


def test_reinforce_rejects_bad_args_without_gpu():
    lib = N.load()
    assert lib.aaa_reinforce(0, 1, 18, 16, 16, 16, 0.99, 16, 16, 16, None) == -1
    assert lib.aaa_reinforce(4, 1, 18, None, 16, 16, 0.99, 16, 16, 16, None) == -1
    assert lib.aaa_reinforce(4, 1, 18, 16, 16, 16, 1.5, 16, 16, 16, None) == -1
    assert b"gamma" in lib.aaa_last_error()


def test_reinforce_loss_has_no_cpu_fallback():
    import torch
    from aaa_amd.reinforce import reinforce_loss
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        reinforce_loss(torch.zeros(3, 1, 18), [0, 1, 2], [1.0, 0.0, 1.0])


def test_actor_layout_refuses_readout_overflow():
    """The actor chain's readout merges at most kActMaxChunks position chunks
    per frame (csrc/actor.h; P <= 2048): a larger grid is refused by the layout
    query (GraphActor then takes the learner's T=1 forward) instead of failing
    at launch."""
    lib = N.load()
    small = N.Cfg(1, 1, 210, 160, 8, 18, N.F32, N.FLAG_FRAMES_U8)
    big = N.Cfg(1, 1, 506, 506, 8, 18, N.F32, N.FLAG_FRAMES_U8)   # 64x64 grid: 4096 x 8 logits
    assert N.grid(506, 506) == (64, 64)
    assert lib.aaa_actor_workspace_bytes(ctypes.byref(small)) > 0
    assert lib.aaa_actor_workspace_bytes(ctypes.byref(big)) == 0


def test_timer_classes_match_header():
    """Every timer class the header enumerates has its binding constant (the
    bench reads all of them to attribute the whole step)."""
    src = open(HEADER).read()
    enum = dict((k, int(v)) for k, v in re.findall(r"AAA_TIMER_([A-Z_]+)\s*=\s*(\d+)", src))
    assert enum.pop("N") == N.TIMER_N == 12
    for name, val in enum.items():
        assert getattr(N, "TIMER_" + name) == val, name


def test_timing_stats_rejects_unknown_class():
    lib = N.load()
    s = N.TimerStats()
    assert lib.aaa_timing_stats(N.TIMER_N, ctypes.byref(s)) == -1
    assert lib.aaa_timing_stats(N.TIMER_MISC, ctypes.byref(s)) == 0 and s.launches == 0


def test_no_test_hooks_in_the_product_library():
    """The partner-wait budget has no override in libaaa.so:
    the stranded-launch tests strand a launch with a filler held past the
    default budget instead."""
    lib = N.load()
    assert not hasattr(lib, "aaa_debug_pair_spin")


def test_defer_stranded_flag_accepted():
    """AAA_FLAG_DEFER_STRANDED is a known cfg flag (layout queries need no GPU)."""
    lib = N.load()
    cfg = N.Cfg(2, 3, 84, 84, 4, 18, N.F32, N.FLAG_DEFER_STRANDED | N.FLAG_FRAMES_U8)
    assert lib.aaa_workspace_bytes(ctypes.byref(cfg)) > 0
    bad = N.Cfg(2, 3, 84, 84, 4, 18, N.F32, 8)
    assert lib.aaa_workspace_bytes(ctypes.byref(bad)) == 0


def test_adam_counted_rejects_null_counter():
    lib = N.load()
    hp = N.AdamHP(1e-3, 0.9, 0.999, 1e-8, 0.0, 0, 0)
    assert lib.aaa_adam_step_counted(ctypes.byref(hp), None, None, 0, None, None, None, None, None, None, None) == -1


def test_package_modules_import():
    """Every host module of the package imports on a CPU-only box (no GPU call)."""
    import importlib
    for m in ("learner", "policy", "optim", "parallel", "reinforce", "runtime", "attention"):
        importlib.import_module(f"aaa_amd.{m}")


def test_param_cache_follows_replaced_parameters():
    """Agent._param_list (the per-step parameter list the actor / episode paths
    use) is re-made when a Parameter object is replaced without a registration
    hook or a count change: a direct ``_parameters[k] = ...`` and ``.to()``
    under the overwrite-on-conversion future flag."""
    import torch
    import attention
    a = attention.Agent(num_actions=18)
    ps = a._param_list()
    assert ps == list(a.parameters()) and a._param_list() is ps
    w = a.policy_head[0].weight
    a.policy_head[0]._parameters["weight"] = torch.nn.Parameter(w.detach().clone())
    ps2 = a._param_list()
    assert ps2 is not ps and ps2 == list(a.parameters())
    assert any(p is a.policy_head[0].weight for p in ps2) and not any(p is w for p in ps2)
    prev = torch.__future__.get_overwrite_module_params_on_conversion()
    torch.__future__.set_overwrite_module_params_on_conversion(True)
    try:
        a.double()
        ps3 = a._param_list()
        assert ps3 == list(a.parameters()) and all(p.dtype == torch.float64 for p in ps3)
    finally:
        torch.__future__.set_overwrite_module_params_on_conversion(prev)
