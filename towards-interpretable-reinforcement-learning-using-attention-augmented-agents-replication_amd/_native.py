"""ctypes binding of libaaa.so (C ABI in include/aaa.h).

There is no fallback: if the library is missing or the device is not gfx950,
every entry point raises.  Build with ``python -c "import __graft_entry__ as g; g.build()"``
(or ``make -C <pkg>/csrc``).
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# AAA_LIB overrides the library path (A/B runs of two builds on one GPU box).
LIB_PATH = os.environ.get("AAA_LIB") or os.path.join(_HERE, "libaaa.so")

F32, BF16 = 0, 1
BWD_HEAD, BWD_CORE, BWD_VISION, BWD_ALL = 1, 2, 4, 7

# Every symbol include/aaa.h declares (checked by tests/test_native_abi.py).
EXPORTS = (
    "aaa_abi_version", "aaa_last_error", "aaa_grid", "aaa_param_layout", "aaa_packed_bytes",
    "aaa_workspace_bytes", "aaa_pack_weights", "aaa_forward", "aaa_backward", "aaa_conv2d_nhwc",
    "aaa_conv2d_nhwc_dgrad", "aaa_conv2d_nhwc_wgrad", "aaa_linear", "aaa_timing_enable", "aaa_timing_read",
    "aaa_adam_step", "aaa_reinforce", "aaa_sample_actions",
)
TIMER_FWD_STEP, TIMER_BPTT_STEP, TIMER_CORE_WGRAD, TIMER_ATTN_FWD, TIMER_ATTN_BWD = 0, 1, 2, 3, 4


class Cfg(ctypes.Structure):
    _fields_ = [("B", ctypes.c_int), ("T", ctypes.c_int), ("H", ctypes.c_int), ("W", ctypes.c_int),
                ("nq", ctypes.c_int), ("A", ctypes.c_int), ("dtype", ctypes.c_int), ("flags", ctypes.c_int)]


IO_FIELDS = ("params", "packed", "basis", "frames", "prev_reward", "prev_action", "h0", "c0",
             "logits", "values", "attn", "hT", "cT", "dlogits", "dvalues", "dhT", "dcT",
             "grads", "dh0", "dc0", "workspace",
             "core_h0", "core_c0", "core_hT", "core_cT", "dcore_hT", "dcore_cT", "dcore_h0", "dcore_c0")
FLAG_STATEFUL_CORE = 1


class IO(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in IO_FIELDS]


class AdamHP(ctypes.Structure):
    _fields_ = [("lr", ctypes.c_double), ("beta1", ctypes.c_double), ("beta2", ctypes.c_double),
                ("eps", ctypes.c_double), ("weight_decay", ctypes.c_double), ("amsgrad", ctypes.c_int),
                ("maximize", ctypes.c_int)]


class ConvDesc(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in
                ("N", "Hin", "Win", "Cin", "Hout", "Wout", "Cout", "KH", "KW", "stride", "pad", "dtype")]


_lib = None
_lock = threading.Lock()


def load(path: str = LIB_PATH):
    """Load libaaa.so (raises if absent).  Safe to call without a GPU."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.isfile(path):
            raise RuntimeError(f"aaa: native library {path} is missing; build it with "
                               f"`make -C {os.path.join(_HERE, 'csrc')}` -- there is no CPU fallback")
        lib = ctypes.CDLL(path)
        P, I, S = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
        CP = ctypes.POINTER(Cfg)
        sig = {
            "aaa_abi_version": (I, []),
            "aaa_last_error": (ctypes.c_char_p, []),
            "aaa_grid": (I, [I, I, ctypes.POINTER(I), ctypes.POINTER(I)]),
            "aaa_param_layout": (I, [CP, ctypes.POINTER(S), ctypes.POINTER(S), ctypes.POINTER(S)]),
            "aaa_packed_bytes": (S, [CP]),
            "aaa_workspace_bytes": (S, [CP]),
            "aaa_pack_weights": (I, [CP, P, P, P]),
            "aaa_forward": (I, [CP, ctypes.POINTER(IO), P]),
            "aaa_backward": (I, [CP, ctypes.POINTER(IO), I, P]),
            "aaa_conv2d_nhwc": (I, [ctypes.POINTER(ConvDesc), P, P, P, P, P]),
            "aaa_conv2d_nhwc_dgrad": (I, [ctypes.POINTER(ConvDesc), P, P, P, P]),
            "aaa_conv2d_nhwc_wgrad": (I, [ctypes.POINTER(ConvDesc), P, P, P, P]),
            "aaa_linear": (I, [I, I, I, P, P, P, P, P]),
            "aaa_timing_enable": (I, [I]),
            "aaa_timing_read": (I, [I, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_long)]),
            "aaa_adam_step": (I, [ctypes.POINTER(AdamHP), ctypes.c_long, I, P, P, P, P, P, P, P]),
            "aaa_reinforce": (I, [I, I, I, P, P, P, ctypes.c_double, P, P, P, P]),
            "aaa_sample_actions": (I, [I, I, P, ctypes.c_ulonglong, P, P, P, P, P]),
        }
        for name, (res, args) in sig.items():
            if not hasattr(lib, name):   # an older build (A/B runs); calling it raises AttributeError
                continue
            fn = getattr(lib, name)
            fn.restype, fn.argtypes = res, args
        _lib = lib
        return lib


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = load().aaa_last_error().decode(errors="replace")
        raise RuntimeError(f"aaa{(' ' + what) if what else ''}: {msg} (status {rc})")


def ptr(t) -> int | None:
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return t.data_ptr()


def stream_ptr(device=None) -> int:
    import torch
    return torch.cuda.current_stream(device).cuda_stream


def grid(H: int, W: int):
    h, w = ctypes.c_int(), ctypes.c_int()
    check(load().aaa_grid(H, W, ctypes.byref(h), ctypes.byref(w)), "grid")
    return h.value, w.value


def param_layout(cfg: Cfg):
    total = ctypes.c_size_t()
    offs = (ctypes.c_size_t * 34)()
    sizes = (ctypes.c_size_t * 34)()
    check(load().aaa_param_layout(ctypes.byref(cfg), ctypes.byref(total), offs, sizes), "param_layout")
    return total.value, list(offs), list(sizes)


def timing_enable(on: bool = True) -> None:
    check(load().aaa_timing_enable(1 if on else 0), "timing_enable")


def timing_read(kind: int):
    """(total_ms, launches) of kernel class ``kind`` since the last read."""
    ms, n = ctypes.c_double(), ctypes.c_long()
    check(load().aaa_timing_read(kind, ctypes.byref(ms), ctypes.byref(n)), "timing_read")
    return ms.value, n.value


def adam_step(hp: AdamHP, step: int, params, grads, exp_avg, exp_avg_sq, max_exp_avg_sq=None, stream=None) -> None:
    """One fused Adam launch over lists of same-length fp32 device tensors (aaa_adam_step)."""
    n = len(params)
    VP = ctypes.c_void_p * max(n, 1)
    def arr(ts):
        return VP(*[t.data_ptr() for t in ts]) if ts is not None else None
    numel = (ctypes.c_size_t * max(n, 1))(*[t.numel() for t in params])
    for group in (grads, exp_avg, exp_avg_sq) + ((max_exp_avg_sq,) if max_exp_avg_sq is not None else ()):
        assert len(group) == n
    mx = arr(max_exp_avg_sq)
    check(load().aaa_adam_step(ctypes.byref(hp), int(step), n, arr(params), arr(grads), arr(exp_avg),
                               arr(exp_avg_sq), mx, numel, stream if stream is not None else stream_ptr()),
          "adam_step")
