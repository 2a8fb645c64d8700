"""Single-component parity (SURVEY.md §8b's per-kernel C-ABI entries) against the
matching oracle piece, plus the index-range cases of the whole-batch GEMMs.

  * ConvLSTMCell.forward / aaa_convlstm_cell_fwd+bwd   vs ref_cpu.convlstm_cell (attention.py:110-126)
  * VisionNetwork.forward / aaa_vision_cnn_fwd+bwd     vs ref_cpu.vision_cnn + convlstm_cell (:152-181)
  * aaa_attn_fwd / aaa_attn_bwd                        vs ref_cpu.attention_readout (:319-348, 235-254)
  * conv1 at config 5's 5.38 M pixel rows (3200 frames of 168x168), forward and
    weight gradient, elementwise against fp64 F.conv2d -- the rows past
    3,728,457 where round 1's divider returned the wrong frame
  * every divisor the runtime builds for C2-C5 checked over the divider's
    whole domain (aaa_divisor_log + aaa_fastdiv_check)

fp32 at 1e-4 (norm-relative and elementwise, helpers.assert_close); bf16 at
2e-2 against the bf16-emulated oracle.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from helpers import assert_close, detinit, rel_err
from oracle import ref_cpu

import attention
from aaa_amd import _native as N
from aaa_amd.runtime import CnnRunner

pytestmark = pytest.mark.gpu
RTOL = 1e-4
PARAMS = detinit.deterministic_params(0, 18)
CELL_KEYS = [k for k in PARAMS if k.startswith("vision.vision_lstm.")]
CNN_KEYS = [k for k in PARAMS if k.startswith("vision.vision_cnn.")]


def _rnd(shape, seed, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.rand(shape, generator=g) * 2 - 1) * scale


def _load(module, prefix):
    detinit.load_into(module, {k[len(prefix):]: v for k, v in PARAMS.items() if k.startswith(prefix)})


def _tol(dt):
    return RTOL if dt == "fp32" else 2e-2


def _grads(module):
    return {n: p.grad.detach().cpu() for n, p in module.named_parameters()}


# ------------------------------------------------------------------ cell ----
@pytest.mark.parametrize("dt", ["fp32", "bf16"])
@pytest.mark.parametrize("B,a,b", [(2, 11, 11), (3, 7, 13), (1, 21, 21)])
def test_convlstm_cell_two_steps_vs_oracle(cuda, dt, B, a, b):
    """Two ConvLSTMCell steps from the zero state (prev_hidden carried, reference
    layout (B,128,a,b)), loss on both steps' (h, c), grads of the 12 params and
    of both inputs; non-square grids pin the orientation."""
    cell = attention.ConvLSTMCell(64, 128, 3)
    _load(cell, "vision.vision_lstm.")
    cell.conv_dtype = dt
    cell.to(cuda)
    xs = [_rnd((B, 64, a, b), 10 + t, 4.0) for t in range(2)]
    G = [_rnd((B, 128, a, b), 20 + k) for k in range(4)]
    xd = [x.to(cuda).requires_grad_(True) for x in xs]
    cell.reset()
    h1, c1 = cell(xd[0])
    assert tuple(cell.prev_hidden[0].shape) == (B, 128, a, b)
    assert tuple(cell.Wci.shape) == (1, 128, a, b) and float(cell.Wci.abs().max()) == 0.0
    h2, c2 = cell(xd[1])
    loss = sum((o * g.to(cuda)).sum() for o, g in zip((h1, c1, h2, c2), G))
    loss.backward()
    torch.cuda.synchronize()

    mode = "bf16" if dt == "bf16" else "fp32"
    P = ref_cpu.tensor_params({k: PARAMS[k] for k in CELL_KEYS})
    xr = [x.clone().requires_grad_(True) for x in xs]
    rh1, rc1, peep = ref_cpu.convlstm_cell(P, xr[0], None, mode, gate_store="fp16" if dt == "bf16" else "fp32")
    rh2, rc2, _ = ref_cpu.convlstm_cell(P, xr[1], (rh1, rc1), mode, peep, gate_store="fp16" if dt == "bf16" else "fp32")
    sum((o * g).sum() for o, g in zip((rh1, rc1, rh2, rc2), G)).backward()
    tol = _tol(dt)
    for name, o, r in (("h1", h1, rh1), ("c1", c1, rc1), ("h2", h2, rh2), ("c2", c2, rc2)):
        assert_close(o.detach().cpu().numpy(), r.detach().numpy(), tol, f"cell {name}")
    for t in range(2):
        assert_close(xd[t].grad.cpu().numpy(), xr[t].grad.numpy(), tol, f"cell dx{t}")
    g = _grads(cell)
    for k in CELL_KEYS:
        assert_close(g[k[len("vision.vision_lstm."):]].numpy(), P[k].grad.numpy(), tol, f"cell grad {k}")


def test_convlstm_cell_abi_state_grads(cuda):
    """The C entry with an explicit incoming state: dh0 / dc0 against autograd."""
    from aaa_amd.runtime import CellRunner
    B, h, w = 2, 11, 9
    r = CellRunner(B, h, w, "fp32", cuda)
    flat = torch.cat([torch.from_numpy(PARAMS[k]).reshape(-1) for k in CELL_KEYS]).to(cuda)
    packed = r.pack(flat)
    x, h0, c0 = _rnd((B, h, w, 64), 1, 3.0), _rnd((B, h, w, 128), 2), _rnd((B, h, w, 128), 3)
    dh1, dc1 = _rnd((B, h, w, 128), 4), _rnd((B, h, w, 128), 5)
    h1, c1, ws = r.forward(packed, x.to(cuda), h0.to(cuda), c0.to(cuda))
    dx, dh0, dc0, grads = r.backward(packed, ws, dh1.to(cuda), dc1.to(cuda))
    torch.cuda.synchronize()
    P = ref_cpu.tensor_params({k: PARAMS[k] for k in CELL_KEYS})
    perm = (0, 3, 2, 1)                      # NHWC <-> the reference's NCHW (Q3)
    xr, hr, cr = (t.permute(*perm).clone().requires_grad_(True) for t in (x, h0, c0))
    rh, rc, _ = ref_cpu.convlstm_cell(P, xr, (hr, cr))
    ((rh * dh1.permute(*perm)).sum() + (rc * dc1.permute(*perm)).sum()).backward()
    assert_close(h1.cpu().numpy(), rh.detach().permute(*perm).numpy(), RTOL, "h1")
    assert_close(c1.cpu().numpy(), rc.detach().permute(*perm).numpy(), RTOL, "c1")
    for name, o, ref in (("dx", dx, xr), ("dh0", dh0, hr), ("dc0", dc0, cr)):
        assert_close(o.cpu().numpy(), ref.grad.permute(*perm).numpy(), RTOL, name)
    off = 0
    for k in CELL_KEYS:
        n = PARAMS[k].size
        assert_close(grads[off:off + n].cpu().numpy(), P[k].grad.reshape(-1).numpy(), RTOL, f"grad {k}")
        off += n


# ---------------------------------------------------------------- vision ----
@pytest.mark.parametrize("dt", ["fp32", "bf16"])
@pytest.mark.parametrize("H,W", [(84, 84), (210, 160), (80, 80), (80, 100), (168, 168)])
def test_vision_network_vs_oracle(cuda, dt, H, W):
    """VisionNetwork.forward over 3 steps: O = the reference's O.transpose(1,3),
    prev_hidden in the reference's (B,128,w,h) layout, grads of all 16 vision
    params through a loss on every step's O.  80x80 / 80x100 give an odd conv1
    map (19 rows): the halo conv2 dgrad's py = 1 parity class is one row short
    there (one and two frames per tile)."""
    _vision_case(cuda, dt, H, W, 3, 2)


@pytest.mark.parametrize("conv", ["1", "2"])
@pytest.mark.parametrize("pipe", ["1", "2"])
@pytest.mark.parametrize("H,W", [(84, 84), (168, 168)])
def test_conv_wgrad_ring_vs_oracle(cuda, monkeypatch, conv, pipe, H, W):
    """bf16 conv1 / conv2 weight gradient on the LDS-DMA ring (AAA_CONV{1,2}_WGRAD_PIPE
    1) or the read-ahead ring (2): the 8x8/s4 gather of 2-tap x 4-channel pieces
    from the bordered RGBx image, the 4x4/s2/p2 gather; 32 frames so the pixel
    counts are whole numbers of K tiles."""
    monkeypatch.setenv(f"AAA_CONV{conv}_WGRAD_PIPE", pipe)
    _vision_case(cuda, "bf16", H, W, *((4, 8) if H == 84 else (4, 16)))


def _vision_case(cuda, dt, H, W, T, B):
    vis = attention.VisionNetwork()
    _load(vis, "vision.")
    vis.conv_dtype = dt
    vis.to(cuda)
    X = torch.from_numpy(detinit.frames_u8(1234, (T, B, H, W, 3)).astype(np.float32))
    hh, ww = ref_cpu.grid_of(H, W)
    G = [_rnd((B, hh, ww, 128), 40 + t) for t in range(T)]
    vis.reset()
    loss = 0
    outs = []
    for t in range(T):
        O = vis(X[t].to(cuda))
        outs.append(O)
        loss = loss + (O * G[t].to(cuda)).sum()
    loss.backward()
    torch.cuda.synchronize()
    mode = "bf16" if dt == "bf16" else "fp32"
    P = ref_cpu.tensor_params({k: PARAMS[k] for k in CNN_KEYS + CELL_KEYS})
    state, peep, rloss, routs = None, None, 0, []
    for t in range(T):
        hN, cN, peep = ref_cpu._vision_step(P, X[t], state, mode, peep, "fp16" if dt == "bf16" else "fp32")
        state = (hN, cN)
        routs.append(hN.transpose(1, 3))
        rloss = rloss + (routs[-1] * G[t]).sum()
    rloss.backward()
    tol = _tol(dt)
    if dt == "bf16":
        # O of the recurrent cell in bf16: elementwise within 2e-2 of the emulated
        # oracle plus the bf16 envelope -- |emulated - fp32 reference| of that
        # element, what the bf16 rounding itself moves it (a few saturating
        # elements drift past a flat 2e-2 after several steps at 21x21)
        P32 = ref_cpu.tensor_params({k: PARAMS[k] for k in CNN_KEYS + CELL_KEYS}, requires_grad=False)
        st32, pp32 = None, None
        with torch.no_grad():
            for t in range(T):
                h32, c32, pp32 = ref_cpu._vision_step(P32, X[t], st32, "fp32", pp32, "fp32")
                st32 = (h32, c32)
                x, r, r32 = (np.asarray(a, np.float64) for a in (outs[t].detach().cpu().numpy(),
                                                                  routs[t].detach().numpy(),
                                                                  h32.transpose(1, 3).numpy()))
                assert rel_err(x, r) <= tol, f"O[{t}] norm-relative"
                allow = tol * np.abs(r).max() + tol * np.abs(r) + np.abs(r - r32)
                bad = np.abs(x - r) > allow
                assert not bad.any(), (f"O[{t}]: {int(bad.sum())} elements beyond the bf16 envelope, worst excess "
                                       f"{float((np.abs(x - r) - allow).max()):.3e}")
    else:
        for t in range(T):
            assert_close(outs[t].detach().cpu().numpy(), routs[t].detach().numpy(), tol, f"O[{t}]")
    assert tuple(vis.vision_lstm.prev_hidden[0].shape) == (B, 128, ww, hh)
    assert_close(vis.vision_lstm.prev_hidden[1].detach().cpu().numpy(), state[1].detach().numpy(), tol, "c_T")
    g = _grads(vis)
    for k in CNN_KEYS + CELL_KEYS:
        assert_close(g[k[len("vision."):]].numpy(), P[k].grad.numpy(), tol, f"vision grad {k}")


def test_agent_state_is_reference_layout(cuda):
    """Agent's ConvLSTM state is exposed as the reference's (B,128,w,h) tensors
    (attention.py:125) and the zero peepholes exist after the first step
    (:132-141); a state written there in that layout is continued from."""
    T, B = 3, 2
    ag = attention.Agent(18, grid=(11, 11))
    detinit.load_into(ag, PARAMS)
    ag.to(cuda)
    X = torch.from_numpy(detinit.frames_u8(1234, (2 * T, B, 84, 84, 3)).astype(np.float32))
    ag.reset()
    with torch.no_grad():
        ag.unroll(X[:T].to(cuda))
    cell = ag.vision.vision_lstm
    P = ref_cpu.tensor_params(PARAMS, requires_grad=False)
    with torch.no_grad():
        _, _, _, (rh, rc) = ref_cpu.unroll(P, X[:T], return_state=True)
        rl, _, _ = ref_cpu.unroll(P, X[T:], state=(rh, rc))
    assert tuple(cell.prev_hidden[0].shape) == (B, 128, 11, 11) == tuple(rh.shape)
    assert_close(cell.prev_hidden[0].cpu().numpy(), rh.numpy(), RTOL, "h_T")
    assert_close(cell.prev_hidden[1].cpu().numpy(), rc.numpy(), RTOL, "c_T")
    assert tuple(cell.Wci.shape) == (1, 128, 11, 11) and float(cell.Wco.abs().max()) == 0.0
    ag.reset()
    cell.prev_hidden = (rh.to(cuda), rc.to(cuda))      # a caller-provided reference-layout state
    with torch.no_grad():
        lg, _, _ = ag.unroll(X[T:].to(cuda))
    assert_close(lg.cpu().numpy(), rl.numpy(), RTOL, "logits from a given state")


# ------------------------------------------------------------- attention ----
@pytest.mark.parametrize("nq,hw", [(4, (11, 11)), (8, (21, 21)), (4, (27, 20))])
@pytest.mark.parametrize("per_frame_q", [False, True])
def test_attention_readout_fwd_bwd_vs_oracle(cuda, nq, hw, per_frame_q):
    h, w = hw
    Fr = 6
    lib = N.load()
    O = _rnd((Fr, h, w, 128), 1, 2.0)
    S = ref_cpu.spatial_basis(h, w)
    Q = _rnd((Fr if per_frame_q else 1, nq, 72), 2, 0.5).expand(Fr, nq, 72).contiguous()
    pr, pa = _rnd((Fr,), 3), torch.arange(Fr, dtype=torch.float32) % 18
    Od, Sd, Qd, prd, pad = (t.contiguous().to(cuda) for t in (O, S, Q if per_frame_q else Q[0], pr, pa))
    attn = torch.empty(Fr, h, w, nq, device=cuda)
    ans = torch.empty(Fr, 256 * nq + 2, device=cuda)
    qs = nq * 72 if per_frame_q else 0
    N.check(lib.aaa_attn_fwd(Fr, h, w, nq, Od.data_ptr(), Sd.data_ptr(), Qd.data_ptr(), qs, prd.data_ptr(),
                             pad.data_ptr(), attn.data_ptr(), ans.data_ptr(), N.stream_ptr()), "attn_fwd")
    dans = _rnd((Fr, 256 * nq + 2), 4)
    dansd = dans.to(cuda)
    dO = torch.empty(Fr, h, w, 128, device=cuda)
    dQ = torch.empty(Fr, nq, 72, device=cuda)
    N.check(lib.aaa_attn_bwd(Fr, h, w, nq, Od.data_ptr(), Sd.data_ptr(), Qd.data_ptr(), qs, attn.data_ptr(),
                             dansd.data_ptr(), dO.data_ptr(), dQ.data_ptr(), N.stream_ptr()), "attn_bwd")
    torch.cuda.synchronize()
    Or, Qr = O.clone().requires_grad_(True), Q.clone().requires_grad_(True)
    A, answer = ref_cpu.attention_readout(Or, S, Qr, pr, pa)
    (answer * dans).sum().backward()
    assert_close(attn.cpu().numpy(), A.detach().numpy(), RTOL, "attention maps")
    assert_close(ans.cpu().numpy(), answer.detach().numpy(), RTOL, "answer")
    assert_close(dO.cpu().numpy(), Or.grad.numpy(), RTOL, "dO")
    assert_close(dQ.cpu().numpy(), Qr.grad.numpy(), RTOL, "dQ (per frame)")


# ------------------------------------------------- index-range (C5 rows) ----
@pytest.mark.parametrize("dt", ["fp32", "bf16"])
def test_conv1_at_config5_rows_vs_fp64(cuda, dt):
    """Config 5's per-GPU conv1: 64 x 50 = 3200 frames of 168x168 -> 5,379,200
    pixel rows.  Forward (conv1 and conv2) and the conv weight gradients of two
    64-frame windows (the only frames with a non-zero output gradient) against
    fp64 F.conv2d of the same frames (attention.py:156-169).  Round 1's divider
    put the last pixel of every frame past row 3,728,457 (frame 2217) into the
    wrong frame; window A (frames 2300-2363) lies past that row inside the first
    launch whatever the descriptor chunking (fp32: 2377 frames per launch,
    bf16: all 3200), window B is the batch's tail.  Measured with the round-1
    divider built in (AAA_LIB A/B): this test fails (profiles/r02/r1div_ab.log)."""
    Nf, H = 3200, 168
    wins = (slice(2300, 2364), slice(3136, 3200))
    r = CnnRunner(Nf, H, H, dt, cuda)
    flat = torch.cat([torch.from_numpy(PARAMS[k]).reshape(-1) for k in CNN_KEYS]).to(cuda)
    packed = r.pack(flat)
    gen = torch.Generator(device=cuda).manual_seed(5)
    X = torch.randint(0, 256, (Nf, H, H, 3), generator=gen, device=cuda, dtype=torch.uint8).float()
    y2, y1, ws = r.forward(flat, packed, X, want_y1=True)
    dy2 = torch.zeros(Nf, r.h, r.w, 64, device=cuda)
    G = [_rnd((64, r.h, r.w, 64), 6 + i) for i in range(len(wins))]
    for s, g in zip(wins, G):
        dy2[s] = g.to(cuda)
    grads, dy1 = r.backward(packed, ws, dy2, want_dy1=True)
    torch.cuda.synchronize()

    def rb(t):   # the bf16 path's operand rounding
        return t.to(torch.bfloat16).double() if dt == "bf16" else t.double()
    w0, b0, w1, b1 = (torch.from_numpy(PARAMS[k]).double().requires_grad_(True) for k in CNN_KEYS)
    tol = RTOL if dt == "fp32" else 1e-2
    loss = 0
    ry1s = []
    for i, (s, g) in enumerate(zip(wins, G)):
        x = X[s].cpu().double().transpose(1, 3)                          # attention.py:179
        ry1 = F.conv2d(rb(x), rb(w0), b0, stride=4, padding=1)
        ry1.retain_grad()
        ry2 = F.conv2d(rb(ry1), rb(w1), b1, stride=2, padding=2)
        loss = loss + (ry2 * g.double().permute(0, 3, 2, 1)).sum()
        ry1s.append(ry1)
        assert_close(y1[s].cpu().numpy(), ry1.detach().permute(0, 3, 2, 1).numpy(), tol, f"conv1 out, window {i}")
        assert_close(y2[s].cpu().numpy(), ry2.detach().permute(0, 3, 2, 1).numpy(), tol, f"conv2 out, window {i}")
    loss.backward()
    for i, (s, ry1) in enumerate(zip(wins, ry1s)):
        assert_close(dy1[s].cpu().numpy(), ry1.grad.permute(0, 3, 2, 1).numpy(), tol, f"conv1 output grad, window {i}")
    mask = torch.ones(Nf, dtype=torch.bool)
    for s in wins:
        mask[s] = False
    assert float(dy1[mask.to(cuda)].abs().max()) == 0.0
    off = 0
    for k, ref in zip(CNN_KEYS, (w0, b0, w1, b1)):
        n = PARAMS[k].size
        assert_close(grads[off:off + n].cpu().numpy(), ref.grad.reshape(-1).numpy(), tol, f"grad {k}")
        off += n


@pytest.mark.parametrize("cfg", ["c2", "c3", "c4", "c5"])
def test_every_runtime_divisor_exact(cuda, cfg):
    """Record every divisor the runtime builds for one full learner iteration of
    a bench config (aaa_divisor_log) and check each over the divider's whole
    domain 0 <= n < 2^31 against the exact quotient."""
    import bench
    from aaa_amd.learner import Learner
    c = bench.CONFIGS[cfg]
    N.divisor_log(0)
    N.divisor_log(1)
    lr = Learner(c["B"], c["T"], c["H"], c["W"], c["nq"], 18, c["dtype"], cuda)
    frames = torch.from_numpy(detinit.frames_u8(1, (c["T"], c["B"], c["H"], c["W"], 3)).astype(np.float32)).to(cuda)
    dl = torch.from_numpy(detinit.cotangent(2, (c["T"], c["B"], 18))).to(cuda)
    lr.step(frames, dl, dl)
    torch.cuda.synchronize()
    ds = N.divisor_log(0)
    assert len(ds) >= 8, ds
    bad = {d: N.fastdiv_check(d) for d in ds}
    assert not any(bad.values()), {d: n for d, n in bad.items() if n}
