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
ABI_VERSION = 9   # include/aaa.h AAA_ABI_VERSION
E_STRANDED = -5   # AAA_E_STRANDED
BWD_HEAD, BWD_CORE, BWD_VISION, BWD_ALL = 1, 2, 4, 7
FWD_VISION, FWD_CORE, FWD_TAIL, FWD_ALL = 1, 2, 4, 7

# Every symbol include/aaa.h declares (checked by tests/test_native_abi.py).
EXPORTS = (
    "aaa_abi_version", "aaa_last_error", "aaa_grid", "aaa_param_layout", "aaa_packed_bytes",
    "aaa_workspace_bytes", "aaa_pack_weights", "aaa_forward", "aaa_backward", "aaa_conv2d_nhwc",
    "aaa_conv2d_nhwc_dgrad", "aaa_conv2d_nhwc_wgrad", "aaa_linear", "aaa_timing_enable", "aaa_timing_read", "aaa_timing_stats",
    "aaa_adam_step", "aaa_reinforce", "aaa_sample_actions", "aaa_fastdiv_check", "aaa_divisor_log",
    "aaa_convlstm_packed_bytes", "aaa_convlstm_workspace_bytes", "aaa_convlstm_pack", "aaa_convlstm_cell_fwd",
    "aaa_convlstm_cell_bwd", "aaa_vision_cnn_packed_bytes", "aaa_vision_cnn_workspace_bytes", "aaa_vision_cnn_pack",
    "aaa_vision_cnn_fwd", "aaa_vision_cnn_bwd", "aaa_attn_fwd", "aaa_attn_bwd",
    "aaa_actor_workspace_bytes", "aaa_actor_step", "aaa_pair_status", "aaa_pair_flag", "aaa_pair_flag_at",
    "aaa_adam_step_guarded", "aaa_adam_step_counted", "aaa_workspace_region",
    "aaa_core_elem_bytes", "aaa_forward_phases", "aaa_core_export", "aaa_core_import",
)
# include/aaa.h enum aaa_timer
TIMER_FWD_STEP, TIMER_BPTT_STEP, TIMER_CORE_WGRAD, TIMER_ATTN_FWD, TIMER_ATTN_BWD = 0, 1, 2, 3, 4
TIMER_PACK, TIMER_VISION_FWD, TIMER_TAIL_FWD, TIMER_TAIL_BWD, TIMER_CORE_DX, TIMER_VISION_BWD, TIMER_MISC = range(5, 12)
TIMER_N = 12


class Cfg(ctypes.Structure):
    _fields_ = [("B", ctypes.c_int), ("T", ctypes.c_int), ("H", ctypes.c_int), ("W", ctypes.c_int),
                ("nq", ctypes.c_int), ("A", ctypes.c_int), ("dtype", ctypes.c_int), ("flags", ctypes.c_int)]


IO_FIELDS = ("params", "packed", "basis", "frames", "prev_reward", "prev_action", "h0", "c0",
             "logits", "values", "attn", "hT", "cT", "dlogits", "dvalues", "dhT", "dcT",
             "grads", "dh0", "dc0", "workspace",
             "core_h0", "core_c0", "core_hT", "core_cT", "dcore_hT", "dcore_cT", "dcore_h0", "dcore_c0")
FLAG_STATEFUL_CORE = 1
FLAG_FRAMES_U8 = 2
FLAG_DEFER_STRANDED = 4
# include/aaa.h enum aaa_ws_region
WS_ANSWER_HIDDEN, WS_QUERY_HIDDEN0, WS_QUERY_HIDDEN1 = 0, 1, 2


class TimerStats(ctypes.Structure):
    _fields_ = [("total_ms", ctypes.c_double), ("launches", ctypes.c_long), ("work", ctypes.c_double),
                ("variant", ctypes.c_char * 192)]


class IO(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in IO_FIELDS]


ACTOR_IO_FIELDS = ("params", "packed", "basis", "frames", "prev_reward", "prev_action", "h", "c",
                   "logits", "values", "attn", "workspace")


class ActorIO(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in ACTOR_IO_FIELDS] + [
        ("seed", ctypes.c_ulonglong), ("counter", ctypes.c_void_p), ("actions", ctypes.c_void_p),
        ("logp", ctypes.c_void_p), ("dlogp_dlogits", ctypes.c_void_p), ("gates", ctypes.c_void_p),
        ("h_out", ctypes.c_void_p), ("c_out", ctypes.c_void_p)]


class AdamHP(ctypes.Structure):
    _fields_ = [("lr", ctypes.c_double), ("beta1", ctypes.c_double), ("beta2", ctypes.c_double),
                ("eps", ctypes.c_double), ("weight_decay", ctypes.c_double), ("amsgrad", ctypes.c_int),
                ("maximize", ctypes.c_int)]


class CellDesc(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in ("B", "h", "w", "dtype")]


class CnnDesc(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in ("N", "H", "W", "dtype")]


class ConvDesc(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in
                ("N", "Hin", "Win", "Cin", "Hout", "Wout", "Cout", "KH", "KW", "stride", "pad", "dtype")]


_lib = None
_lock = threading.Lock()


def ablation_build() -> bool:
    """Whether the loaded library is the A/B build (make ablation; AAA_LIB=.../libaaa_ablation.so):
    the measured-slower variants and the A/B environment knobs exist only there."""
    return hasattr(load(), "aaa_ablation_build")


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
            "aaa_forward_phases": (I, [CP, ctypes.POINTER(IO), I, P]),
            "aaa_core_export": (I, [CP, P, I, I, P, P, P, P]),
            "aaa_core_import": (I, [CP, P, I, I, P, P, P, P]),
            "aaa_conv2d_nhwc": (I, [ctypes.POINTER(ConvDesc), P, P, P, P, P]),
            "aaa_conv2d_nhwc_dgrad": (I, [ctypes.POINTER(ConvDesc), P, P, P, P]),
            "aaa_conv2d_nhwc_wgrad": (I, [ctypes.POINTER(ConvDesc), P, P, P, P]),
            "aaa_linear": (I, [I, I, I, P, P, P, P, P]),
            "aaa_timing_enable": (I, [I]),
            "aaa_timing_read": (I, [I, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_long)]),
            "aaa_timing_stats": (I, [I, ctypes.POINTER(TimerStats)]),
            "aaa_adam_step": (I, [ctypes.POINTER(AdamHP), ctypes.c_long, I, P, P, P, P, P, P, P]),
            "aaa_adam_step_guarded": (I, [ctypes.POINTER(AdamHP), ctypes.c_long, P, I, P, P, P, P, P, P, P]),
            "aaa_pair_flag": (I, [P, P]),
            "aaa_pair_flag_at": (I, [P, P, P]),
            "aaa_adam_step_counted": (I, [ctypes.POINTER(AdamHP), P, P, I, P, P, P, P, P, P, P]),
            "aaa_core_elem_bytes": (I, [ctypes.POINTER(Cfg), ctypes.POINTER(I), ctypes.POINTER(I)]),
            "aaa_workspace_region": (I, [ctypes.POINTER(Cfg), I, ctypes.POINTER(ctypes.c_size_t),
                                         ctypes.POINTER(ctypes.c_size_t)]),
            "aaa_reinforce": (I, [I, I, I, P, P, P, ctypes.c_double, P, P, P, P]),
            "aaa_sample_actions": (I, [I, I, P, ctypes.c_ulonglong, P, P, P, P, P]),
            "aaa_convlstm_packed_bytes": (S, [ctypes.POINTER(CellDesc)]),
            "aaa_convlstm_workspace_bytes": (S, [ctypes.POINTER(CellDesc)]),
            "aaa_convlstm_pack": (I, [ctypes.POINTER(CellDesc), P, P, P]),
            "aaa_convlstm_cell_fwd": (I, [ctypes.POINTER(CellDesc), P, P, P, P, P, P, P, P]),
            "aaa_convlstm_cell_bwd": (I, [ctypes.POINTER(CellDesc), P, P, P, P, P, P, P, P, P]),
            "aaa_vision_cnn_packed_bytes": (S, [ctypes.POINTER(CnnDesc)]),
            "aaa_vision_cnn_workspace_bytes": (S, [ctypes.POINTER(CnnDesc)]),
            "aaa_vision_cnn_pack": (I, [ctypes.POINTER(CnnDesc), P, P, P]),
            "aaa_vision_cnn_fwd": (I, [ctypes.POINTER(CnnDesc), P, P, P, P, P, P, P]),
            "aaa_vision_cnn_bwd": (I, [ctypes.POINTER(CnnDesc), P, P, P, P, P, P]),
            "aaa_attn_fwd": (I, [I, I, I, I, P, P, P, I, P, P, P, P, P]),
            "aaa_attn_bwd": (I, [I, I, I, I, P, P, P, I, P, P, P, P, P]),
            "aaa_fastdiv_check": (I, [ctypes.c_uint, ctypes.c_uint, ctypes.c_uint, ctypes.POINTER(ctypes.c_ulonglong)]),
            "aaa_divisor_log": (I, [I, ctypes.POINTER(ctypes.c_uint), I]),
            "aaa_actor_workspace_bytes": (S, [CP]),
            "aaa_actor_step": (I, [CP, ctypes.POINTER(ActorIO), P]),
            "aaa_pair_status": (I, [P, I]),
        }
        ab_override = "AAA_LIB" in os.environ
        missing = [name for name in sig if not hasattr(lib, name)]
        if missing and not ab_override:
            raise RuntimeError(f"aaa: {path} does not export {missing}; it is older than these bindings -- "
                               f"rebuild it (make -C {os.path.join(_HERE, 'csrc')})")
        for name, (res, args) in sig.items():
            if name in missing:   # only with an explicit AAA_LIB (A/B runs of an older build)
                continue
            fn = getattr(lib, name)
            fn.restype, fn.argtypes = res, args
        abi = lib.aaa_abi_version()
        if abi != ABI_VERSION and not ab_override:
            raise RuntimeError(f"aaa: {path} has ABI version {abi}, these bindings expect {ABI_VERSION}; "
                               f"rebuild it (make -C {os.path.join(_HERE, 'csrc')})")
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


def fastdiv_check(d: int, lo: int = 0, hi: int = 1 << 31) -> int:
    """Mismatches of the kernels' divider for d over every dividend in [lo, hi) (host)."""
    bad = ctypes.c_ulonglong()
    check(load().aaa_fastdiv_check(d, lo, hi, ctypes.byref(bad)), "fastdiv_check")
    return bad.value


def divisor_log(enable: int = -1):
    """Divisors the runtime built since recording started (enable: 1 start, 0 stop+clear, -1 read)."""
    n = load().aaa_divisor_log(-1, None, 0)
    buf = (ctypes.c_uint * max(n, 1))()
    n = load().aaa_divisor_log(enable, buf, n)
    return sorted(set(buf[:n]))


def timing_enable(on: bool = True) -> None:
    check(load().aaa_timing_enable(1 if on else 0), "timing_enable")


def timing_read(kind: int):
    """(total_ms, launches) of kernel class ``kind`` since the last read."""
    ms, n = ctypes.c_double(), ctypes.c_long()
    check(load().aaa_timing_read(kind, ctypes.byref(ms), ctypes.byref(n)), "timing_read")
    return ms.value, n.value


def timing_stats(kind: int) -> dict:
    """Kernel class ``kind`` since the last read: device ms, launches, the
    launches' algorithmic work (FLOP for classes 0-2 and 6-10, bytes for 3-4) as the
    runtime accounts it, and the variant it dispatched."""
    s = TimerStats()
    check(load().aaa_timing_stats(kind, ctypes.byref(s)), "timing_stats")
    return {"ms": s.total_ms, "launches": s.launches, "work": s.work, "variant": s.variant.decode()}


def pair_status(clear: bool = True, stream=None) -> int:
    """Synchronise ``stream`` (default: torch's current) and return how many
    partner waits of the paired frame-resident kernels timed out since the
    last clear (0 = every paired launch ran on a co-resident pair)."""
    n = load().aaa_pair_status(stream if stream is not None else stream_ptr(), 1 if clear else 0)
    if n < 0:
        check(n, "pair_status")
    return n


def pair_flag(dst, stream=None, base=None) -> None:
    """Enqueue a kernel writing into the one-element fp32 device tensor ``dst``
    the partner timeouts reported since the previous pair_flag on this device
    (stream order, no host sync; independent of host-side consumption).  With
    ``base`` (a one-element int32 device tensor the caller owns) the count is
    taken against that snapshot instead of the library's per-device one, so
    other readers on the device cannot consume it (aaa_pair_flag_at)."""
    st = stream if stream is not None else stream_ptr(dst.device)
    if base is None:
        check(load().aaa_pair_flag(dst.data_ptr(), st), "pair_flag")
    else:
        import torch
        if base.dtype != torch.int32 or base.device != dst.device:
            raise ValueError("pair_flag: base must be an int32 tensor on dst's device")
        check(load().aaa_pair_flag_at(dst.data_ptr(), base.data_ptr(), st), "pair_flag_at")


def adam_step(hp: AdamHP, step: int, params, grads, exp_avg, exp_avg_sq, max_exp_avg_sq=None, stream=None,
              guard=None, step_dev=None) -> None:
    """One fused Adam launch over lists of same-length fp32 device tensors
    (aaa_adam_step; with ``guard``, a one-element fp32 device tensor,
    aaa_adam_step_guarded: no update when guard != 0; with ``step_dev``, a
    one-element int32 device tensor, aaa_adam_step_counted: ``step`` is
    ignored, the update is number step_dev + 1 and step_dev advances on the
    device only when the update was applied)."""
    n = len(params)
    VP = ctypes.c_void_p * max(n, 1)
    def arr(ts):
        return VP(*[t.data_ptr() for t in ts]) if ts is not None else None
    numel = (ctypes.c_size_t * max(n, 1))(*[t.numel() for t in params])
    for group in (grads, exp_avg, exp_avg_sq) + ((max_exp_avg_sq,) if max_exp_avg_sq is not None else ()):
        assert len(group) == n
    mx = arr(max_exp_avg_sq)
    st = stream if stream is not None else stream_ptr()
    if step_dev is not None:
        assert step_dev.numel() == 1 and step_dev.is_cuda and str(step_dev.dtype) == "torch.int32"
        check(load().aaa_adam_step_counted(ctypes.byref(hp), step_dev.data_ptr(),
                                           guard.data_ptr() if guard is not None else None, n, arr(params),
                                           arr(grads), arr(exp_avg), arr(exp_avg_sq), mx, numel, st),
              "adam_step_counted")
    elif guard is not None:
        check(load().aaa_adam_step_guarded(ctypes.byref(hp), int(step), guard.data_ptr(), n, arr(params), arr(grads),
                                           arr(exp_avg), arr(exp_avg_sq), mx, numel, st), "adam_step_guarded")
    else:
        check(load().aaa_adam_step(ctypes.byref(hp), int(step), n, arr(params), arr(grads), arr(exp_avg),
                                   arr(exp_avg_sq), mx, numel, st), "adam_step")
