"""Host runtime around the C ABI: buffers for one unroll configuration.

``UnrollRunner`` owns nothing but torch-allocated device memory (the caching
allocator is the allocator, per the C ABI's ownership rule) and issues the
library calls on torch's current HIP stream.
"""
from __future__ import annotations

import ctypes

import torch

from . import _native as N


class UnrollRunner:
    def __init__(self, B: int, T: int, H: int, W: int, nq: int = 4, A: int = 18,
                 dtype: str = "fp32", device=None, stateful_core: bool = False, frames_u8: bool = False,
                 defer_stranded: bool = False):
        if dtype not in ("fp32", "bf16"):
            raise ValueError(f"dtype must be 'fp32' or 'bf16', got {dtype!r}")
        self.lib = N.load()
        self.device = torch.device(device if device is not None else "cuda")
        if self.device.type != "cuda":
            raise RuntimeError("aaa: the HIP path needs a ROCm GPU tensor device (no CPU fallback)")
        self.stateful_core = bool(stateful_core)
        self.frames_u8 = bool(frames_u8)
        self.cfg = N.Cfg(B, T, H, W, nq, A, N.BF16 if dtype == "bf16" else N.F32,
                         (N.FLAG_STATEFUL_CORE if stateful_core else 0) | (N.FLAG_FRAMES_U8 if frames_u8 else 0)
                         | (N.FLAG_DEFER_STRANDED if defer_stranded else 0))
        self.B, self.T, self.H, self.W, self.nq, self.A, self.dtype = B, T, H, W, nq, A, dtype
        self.h, self.w = N.grid(H, W)
        self.P = self.h * self.w
        self.n_params, self.offsets, self.sizes = N.param_layout(self.cfg)
        self.ws_bytes = self.lib.aaa_workspace_bytes(ctypes.byref(self.cfg))
        self.pk_bytes = self.lib.aaa_packed_bytes(ctypes.byref(self.cfg))
        if not self.ws_bytes or not self.pk_bytes:
            N.check(-1, "layout")

    # -- buffers ----------------------------------------------------------
    def new_workspace(self):
        return torch.empty(self.ws_bytes, dtype=torch.uint8, device=self.device)

    def new_packed(self):
        return torch.empty(self.pk_bytes, dtype=torch.uint8, device=self.device)

    def state_shape(self):
        return (self.B, self.h, self.w, 128)

    def workspace_region(self, workspace, region: int):
        """A forward product inside ``workspace`` (aaa_workspace_region): an
        (T*B, n) fp32 view, e.g. N.WS_ANSWER_HIDDEN = relu(answer_processor.0)."""
        off, nb = ctypes.c_size_t(), ctypes.c_size_t()
        N.check(self.lib.aaa_workspace_region(ctypes.byref(self.cfg), int(region), ctypes.byref(off),
                                              ctypes.byref(nb)), "workspace_region")
        F = self.T * self.B
        return workspace[off.value:off.value + nb.value].view(torch.float32).view(F, nb.value // (4 * F))

    def relu_masks(self, workspace):
        """The on/off pattern of every ReLU the hand-written backward masks with,
        after a forward into ``workspace`` (host bool tensors, (T*B, n)):
        "answer" = answer_processor.0 (attention.py:277-282) and, in the stateful
        core, "q0" / "q1" = the query MLP's two (attention.py:184-198).  For
        checkers: the mask-matched oracle (oracle/ref_cpu.py KinkProbe.masks)."""
        out = {"answer": self.workspace_region(workspace, N.WS_ANSWER_HIDDEN) > 0}
        if self.stateful_core:
            out["q0"] = self.workspace_region(workspace, N.WS_QUERY_HIDDEN0) > 0
            out["q1"] = self.workspace_region(workspace, N.WS_QUERY_HIDDEN1) > 0
        return {k: v.cpu() for k, v in out.items()}

    # -- calls ------------------------------------------------------------
    def pack(self, flat_params, packed):
        assert flat_params.dtype == torch.float32 and flat_params.is_contiguous()
        assert flat_params.numel() == self.n_params, (flat_params.numel(), self.n_params)
        N.check(self.lib.aaa_pack_weights(ctypes.byref(self.cfg), N.ptr(flat_params), N.ptr(packed),
                                          N.stream_ptr(self.device)), "pack_weights")

    def _io(self, **kw):
        io = N.IO()
        for k, v in kw.items():
            setattr(io, k, None if v is None else (v if isinstance(v, int) else v.data_ptr()))
        return io

    def forward(self, flat_params, packed, basis, frames, workspace, prev_reward=None, prev_action=None,
                h0=None, c0=None, want_attn=True, want_state=False, core=None, phases=N.FWD_ALL):
        """Returns (logits, values, attn, hT, cT); a stateful-core runner also
        returns the core state (core_hT, core_cT) (B, 256), starting from
        ``core`` = (h0, c0) or zeros.  ``phases`` = FWD_VISION | FWD_TAIL skips
        the ConvLSTM recurrence (its products imported first: core_import)."""
        T, B, A = self.T, self.B, self.A
        dev = self.device
        self._check_frames(frames)
        logits = torch.empty(T, B, A, device=dev)
        values = torch.empty(T, B, A, device=dev)
        attn = torch.empty(T, B, self.h, self.w, self.nq, device=dev) if want_attn else None
        hT = torch.empty(self.state_shape(), device=dev) if want_state else None
        cT = torch.empty(self.state_shape(), device=dev) if want_state else None
        # keep converted inputs alive until the launches are enqueued
        keep = dict(prev_reward=_f32(prev_reward, (T, B)), prev_action=_f32(prev_action, (T, B)),
                    h0=_f32(h0, self.state_shape()), c0=_f32(c0, self.state_shape()))
        extra = {}
        if self.stateful_core:
            ch0, cc0 = core if core is not None else (None, None)
            extra = dict(core_h0=_f32(ch0, (B, 256)), core_c0=_f32(cc0, (B, 256)),
                         core_hT=torch.empty(B, 256, device=dev), core_cT=torch.empty(B, 256, device=dev))
        io = self._io(params=flat_params, packed=packed, basis=basis, frames=frames,
                      logits=logits, values=values, attn=attn, hT=hT, cT=cT, workspace=workspace, **keep, **extra)
        if phases == N.FWD_ALL:
            N.check(self.lib.aaa_forward(ctypes.byref(self.cfg), ctypes.byref(io), N.stream_ptr(dev)), "forward")
        else:
            N.check(self.lib.aaa_forward_phases(ctypes.byref(self.cfg), ctypes.byref(io), int(phases),
                                                N.stream_ptr(dev)), "forward_phases")
        if self.stateful_core:
            return logits, values, attn, hT, cT, extra["core_hT"], extra["core_cT"]
        return logits, values, attn, hT, cT

    def core_shapes(self, n):
        """Shapes of n steps' (gates, c, h) for core_export / core_import."""
        M = self.B * self.h * self.w
        return (n, M, 512), (n, M, 128), (n, M, 128)

    def core_dtypes(self):
        """Element types of (gates, c, h) in core_export / core_import: fp32 runners
        all fp32; bf16 runners the workspace's gate storage (fp16) and bf16 h.  None
        where the geometry's products cannot be transferred (the channel-quad-major
        slices of large-batch bf16 runs)."""
        if not hasattr(self, "_core_dt"):
            ge, he = ctypes.c_int(), ctypes.c_int()
            N.check(self.lib.aaa_core_elem_bytes(ctypes.byref(self.cfg), ctypes.byref(ge), ctypes.byref(he)),
                    "core_elem_bytes")
            self._core_dt = None if ge.value == 0 else (torch.float16 if ge.value == 2 else torch.float32,
                                                        torch.float32,
                                                        torch.bfloat16 if he.value == 2 else torch.float32)
        return self._core_dt

    def _core_dts(self):
        dts = self.core_dtypes()
        if dts is None:
            raise RuntimeError("aaa: this geometry keeps the recurrence's products in channel-quad-major slices; "
                               "core_export / core_import do not apply (core_dtypes() is None)")
        return dts

    def core_export(self, workspace, t0, n, gates, c, h):
        """Steps [t0, t0+n) of the recurrence's products -> gates, c, h (core_shapes, core_dtypes)."""
        for x, shp, dt in zip((gates, c, h), self.core_shapes(n), self._core_dts()):
            _check_out(x, shp, dt)
        N.check(self.lib.aaa_core_export(ctypes.byref(self.cfg), N.ptr(workspace), int(t0), int(n), N.ptr(gates),
                                         N.ptr(c), N.ptr(h), N.stream_ptr(self.device)), "core_export")

    def core_import(self, workspace, t0, n, gates, c, h):
        """The inverse of core_export, into a workspace for forward(phases=FWD_VISION | FWD_TAIL)."""
        for x, shp, dt in zip((gates, c, h), self.core_shapes(n), self._core_dts()):
            _check_out(x, shp, dt)
        N.check(self.lib.aaa_core_import(ctypes.byref(self.cfg), N.ptr(workspace), int(t0), int(n), N.ptr(gates),
                                         N.ptr(c), N.ptr(h), N.stream_ptr(self.device)), "core_import")

    def backward(self, flat_params, packed, basis, frames, workspace, dlogits, dvalues=None, dhT=None,
                 dcT=None, grads=None, want_state_grads=False, phases=N.BWD_ALL, dcore=None, want_core_grads=False):
        """Returns (grads, dh0, dc0); a stateful-core runner also returns the
        core-state grads (dcore_h0, dcore_c0) when ``want_core_grads``."""
        dev = self.device
        B = self.B
        if grads is None:
            grads = torch.empty(self.n_params, device=dev)
        dh0 = torch.empty(self.state_shape(), device=dev) if want_state_grads else None
        dc0 = torch.empty(self.state_shape(), device=dev) if want_state_grads else None
        keep = dict(dlogits=_f32(dlogits, (self.T, self.B, self.A)),
                    dvalues=_f32(dvalues, (self.T, self.B, self.A)),
                    dhT=_f32(dhT, self.state_shape()), dcT=_f32(dcT, self.state_shape()))
        extra = {}
        if self.stateful_core:
            dch, dcc = dcore if dcore is not None else (None, None)
            extra = dict(dcore_hT=_f32(dch, (B, 256)), dcore_cT=_f32(dcc, (B, 256)),
                         dcore_h0=torch.empty(B, 256, device=dev) if want_core_grads else None,
                         dcore_c0=torch.empty(B, 256, device=dev) if want_core_grads else None)
        io = self._io(params=flat_params, packed=packed, basis=basis, frames=frames, workspace=workspace,
                      grads=grads, dh0=dh0, dc0=dc0, **keep, **extra)
        N.check(self.lib.aaa_backward(ctypes.byref(self.cfg), ctypes.byref(io), phases, N.stream_ptr(dev)),
                "backward")
        if self.stateful_core:
            return grads, dh0, dc0, extra["dcore_h0"], extra["dcore_c0"]
        return grads, dh0, dc0

    def _check_frames(self, frames):
        exp = (self.T, self.B, self.H, self.W, 3)
        dt = torch.uint8 if self.frames_u8 else torch.float32
        if tuple(frames.shape) != exp or frames.dtype != dt or not frames.is_contiguous():
            raise ValueError(f"frames must be contiguous {dt} {exp}, got {tuple(frames.shape)} {frames.dtype}")
        if frames.device != self.device and frames.device.type != "cuda":
            raise RuntimeError("frames must be on the GPU")


def _check_out(t, shape, dtype=torch.float32):
    if (t is None or tuple(t.shape) != tuple(shape) or t.dtype != dtype or not t.is_contiguous()
            or t.device.type != "cuda"):
        raise ValueError(f"expected a contiguous {dtype} device tensor {tuple(shape)}, got "
                         f"{None if t is None else (tuple(t.shape), t.dtype, t.device)}")


def _f32(t, shape):
    if t is None:
        return None
    t = t.reshape(shape)
    if t.dtype != torch.float32:
        t = t.float()
    return t.contiguous()


class CellRunner:
    """ConvLSTMCell(64, 128, 3) steps of one (B, h, w) shape on the C ABI
    (aaa_convlstm_*; attention.py:110-126).  Tensors are NHWC: the reference's
    (B, C, a, b) permuted (0, 3, 2, 1)."""

    def __init__(self, B: int, h: int, w: int, dtype: str = "fp32", device=None):
        self.lib = N.load()
        self.device = torch.device(device if device is not None else "cuda")
        if self.device.type != "cuda":
            raise RuntimeError("aaa: the HIP path needs a ROCm GPU tensor device (no CPU fallback)")
        self.B, self.h, self.w, self.dtype = B, h, w, dtype
        self.desc = N.CellDesc(B, h, w, N.BF16 if dtype == "bf16" else N.F32)
        self.pk_bytes = self.lib.aaa_convlstm_packed_bytes(ctypes.byref(self.desc))
        self.ws_bytes = self.lib.aaa_convlstm_workspace_bytes(ctypes.byref(self.desc))
        if not self.pk_bytes or not self.ws_bytes:
            N.check(-1, "convlstm layout")

    def pack(self, cell_flat):
        packed = torch.empty(self.pk_bytes, dtype=torch.uint8, device=self.device)
        N.check(self.lib.aaa_convlstm_pack(ctypes.byref(self.desc), N.ptr(cell_flat), N.ptr(packed),
                                           N.stream_ptr(self.device)), "convlstm_pack")
        return packed

    def forward(self, packed, x, h0=None, c0=None):
        """x (B,h,w,64), h0/c0 (B,h,w,128) or None -> (h1, c1, workspace)."""
        shp = (self.B, self.h, self.w, 128)
        x = _f32(x, (self.B, self.h, self.w, 64))
        h0, c0 = _f32(h0, shp), _f32(c0, shp)
        ws = torch.empty(self.ws_bytes, dtype=torch.uint8, device=self.device)
        h1 = torch.empty(shp, device=self.device)
        c1 = torch.empty(shp, device=self.device)
        N.check(self.lib.aaa_convlstm_cell_fwd(ctypes.byref(self.desc), N.ptr(packed), N.ptr(x), N.ptr(h0), N.ptr(c0),
                                               N.ptr(h1), N.ptr(c1), N.ptr(ws), N.stream_ptr(self.device)),
                "convlstm_cell_fwd")
        return h1, c1, ws

    def backward(self, packed, ws, dh1=None, dc1=None, want_dx=True, want_dh0=True, want_dc0=True,
                 want_grads=True):
        shp = (self.B, self.h, self.w, 128)
        dh1, dc1 = _f32(dh1, shp), _f32(dc1, shp)
        dev = self.device
        dx = torch.empty(self.B, self.h, self.w, 64, device=dev) if want_dx else None
        dh0 = torch.empty(shp, device=dev) if want_dh0 else None
        dc0 = torch.empty(shp, device=dev) if want_dc0 else None
        grads = torch.empty(4 * (128 * 64 * 9 + 128 + 128 * 128 * 9), device=dev) if want_grads else None
        N.check(self.lib.aaa_convlstm_cell_bwd(ctypes.byref(self.desc), N.ptr(packed), N.ptr(dh1), N.ptr(dc1),
                                               N.ptr(dx), N.ptr(dh0), N.ptr(dc0), N.ptr(grads), N.ptr(ws),
                                               N.stream_ptr(dev)), "convlstm_cell_bwd")
        return dx, dh0, dc0, grads


class CnnRunner:
    """VisionNetwork.vision_cnn over N frames (aaa_vision_cnn_*; attention.py:155-170
    on X.transpose(1,3)): frames (N,H,W,3) -> (N,h,w,64) NHWC."""

    def __init__(self, N_: int, H: int, W: int, dtype: str = "fp32", device=None):
        self.lib = N.load()
        self.device = torch.device(device if device is not None else "cuda")
        if self.device.type != "cuda":
            raise RuntimeError("aaa: the HIP path needs a ROCm GPU tensor device (no CPU fallback)")
        self.N, self.H, self.W, self.dtype = N_, H, W, dtype
        self.h, self.w = N.grid(H, W)
        self.H1, self.W1 = (H + 2 - 8) // 4 + 1, (W + 2 - 8) // 4 + 1
        self.desc = N.CnnDesc(N_, H, W, N.BF16 if dtype == "bf16" else N.F32)
        self.pk_bytes = self.lib.aaa_vision_cnn_packed_bytes(ctypes.byref(self.desc))
        self.ws_bytes = self.lib.aaa_vision_cnn_workspace_bytes(ctypes.byref(self.desc))
        if not self.pk_bytes or not self.ws_bytes:
            N.check(-1, "vision_cnn layout")

    def pack(self, cnn_flat):
        packed = torch.empty(self.pk_bytes, dtype=torch.uint8, device=self.device)
        N.check(self.lib.aaa_vision_cnn_pack(ctypes.byref(self.desc), N.ptr(cnn_flat), N.ptr(packed),
                                             N.stream_ptr(self.device)), "vision_cnn_pack")
        return packed

    def forward(self, cnn_flat, packed, frames, want_y1=False):
        """-> (y2 (N,h,w,64), y1 (N,H1,W1,32) or None, workspace)."""
        frames = _f32(frames, (self.N, self.H, self.W, 3))
        ws = torch.empty(self.ws_bytes, dtype=torch.uint8, device=self.device)
        y2 = torch.empty(self.N, self.h, self.w, 64, device=self.device)
        y1 = torch.empty(self.N, self.H1, self.W1, 32, device=self.device) if want_y1 else None
        N.check(self.lib.aaa_vision_cnn_fwd(ctypes.byref(self.desc), N.ptr(cnn_flat), N.ptr(packed), N.ptr(frames),
                                            N.ptr(y1), N.ptr(y2), N.ptr(ws), N.stream_ptr(self.device)),
                "vision_cnn_fwd")
        return y2, y1, ws

    def backward(self, packed, ws, dy2, want_dy1=False):
        """-> (flat grads of the 4 vision_cnn tensors (39,008), dy1 or None)."""
        dy2 = _f32(dy2, (self.N, self.h, self.w, 64))
        grads = torch.empty(32 * 3 * 64 + 32 + 64 * 32 * 16 + 64, device=self.device)
        dy1 = torch.empty(self.N, self.H1, self.W1, 32, device=self.device) if want_dy1 else None
        N.check(self.lib.aaa_vision_cnn_bwd(ctypes.byref(self.desc), N.ptr(packed), N.ptr(dy2), N.ptr(dy1),
                                            N.ptr(grads), N.ptr(ws), N.stream_ptr(self.device)), "vision_cnn_bwd")
        return grads, dy1


class ActorRunner:
    """One environment step of B <= 16 rows on the actor chain (aaa_actor_step:
    six launches sized for small B; fp32, zero-state policy core): the acting
    half of main_mp.py:49-59 / test_model.py:42-73.  The ConvLSTM state
    tensors ``h``/``c`` (B, h, w, 128) are read and overwritten in place, and
    every output goes to caller-preallocated tensors, so a step can be
    captured in a HIP graph and replayed."""

    def __init__(self, B: int, H: int, W: int, nq: int = 4, A: int = 18, device=None, frames_u8: bool = True):
        self.lib = N.load()
        self.device = torch.device(device if device is not None else "cuda")
        if self.device.type != "cuda":
            raise RuntimeError("aaa: the HIP path needs a ROCm GPU tensor device (no CPU fallback)")
        self.B, self.H, self.W, self.nq, self.A = B, H, W, nq, A
        self.frames_u8 = bool(frames_u8)
        self.cfg = N.Cfg(B, 1, H, W, nq, A, N.F32, N.FLAG_FRAMES_U8 if frames_u8 else 0)
        self.h, self.w = N.grid(H, W)
        self.P = self.h * self.w
        self.n_params, self.offsets, self.sizes = N.param_layout(self.cfg)
        self.ws_bytes = self.lib.aaa_actor_workspace_bytes(ctypes.byref(self.cfg))
        self.pk_bytes = self.lib.aaa_packed_bytes(ctypes.byref(self.cfg))
        if not self.ws_bytes or not self.pk_bytes:
            N.check(-1, "actor layout")

    def new_workspace(self):
        return torch.empty(self.ws_bytes, dtype=torch.uint8, device=self.device)

    def new_packed(self):
        return torch.empty(self.pk_bytes, dtype=torch.uint8, device=self.device)

    def state_shape(self):
        return (self.B, self.h, self.w, 128)

    def pack(self, flat_params, packed):
        assert flat_params.dtype == torch.float32 and flat_params.is_contiguous()
        assert flat_params.numel() == self.n_params, (flat_params.numel(), self.n_params)
        N.check(self.lib.aaa_pack_weights(ctypes.byref(self.cfg), N.ptr(flat_params), N.ptr(packed),
                                          N.stream_ptr(self.device)), "pack_weights")

    def step(self, flat_params, packed, basis, frames, workspace, h, c, logits, values, attn=None,
             prev_reward=None, prev_action=None, seed: int = 0, counter=None, actions=None, logp=None,
             dlogp=None, gates=None, h_out=None, c_out=None):
        """frames (B, H, W, 3) uint8 (or fp32 without frames_u8); h, c updated in
        place; logits/values (B, A), attn (B, h, w, nq) or None; actions (B,)
        int32 (None: no draw) with logp (B,) / dlogp (B, A) and the device draw
        ``counter`` (one-element int64, advanced per step) as aaa_sample_actions."""
        exp = (self.B, self.H, self.W, 3)
        dt = torch.uint8 if self.frames_u8 else torch.float32
        if tuple(frames.shape[-4:]) != exp or frames.numel() != self.B * self.H * self.W * 3 or \
                frames.dtype != dt or not frames.is_contiguous():
            raise ValueError(f"frames must be contiguous {dt} {exp}, got {tuple(frames.shape)} {frames.dtype}")
        for name, t in (("h", h), ("c", c)):
            if tuple(t.shape) != self.state_shape() or t.dtype != torch.float32 or not t.is_contiguous():
                raise ValueError(f"{name} must be contiguous fp32 {self.state_shape()}")
        io = N.ActorIO()
        for k, v in dict(params=flat_params, packed=packed, basis=basis, frames=frames, prev_reward=prev_reward,
                         prev_action=prev_action, h=h, c=c, logits=logits, values=values, attn=attn,
                         workspace=workspace, counter=counter, actions=actions, logp=logp,
                         dlogp_dlogits=dlogp, gates=gates, h_out=h_out, c_out=c_out).items():
            setattr(io, k, None if v is None else v.data_ptr())
        io.seed = int(seed) & (2**64 - 1)
        N.check(self.lib.aaa_actor_step(ctypes.byref(self.cfg), ctypes.byref(io), N.stream_ptr(self.device)),
                "actor_step")
