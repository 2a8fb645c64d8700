"""Generate the golden fixtures by importing the REFERENCE itself.

Runs only in the build container, where /root/reference exists; it refuses to
run anywhere else.  The reference never travels: only the .npz outputs below
(inputs are regenerated from seeds by detinit) are committed.

Fixtures:
  G1  spatial basis S for (11,11), (21,21), (27,20)          attention.py:201-226
  G2  one step, B=2, 84x84: logits, values, attention map A, readout a
  G3  B=1, T=20, 84x84 fwd+bwd (config 1), raw 0..255 frames; G3n: frames/255
  G4  B=4, T=4 with prev_reward / prev_action given
  G5  REINFORCE finish_episode (main_mp.py:62-80) over a 12-step episode,
      driven through main_mp.Policy with gym stubbed out
  G6  210x160 frames with the default SpatialBasis(27,20), B=1, T=2 forward
  G7  bf16-emulated reference: every nn.Conv2d rounds its GEMM operands to
      bf16 (forward x,w; dgrad dy,w; wgrad x,dy), fp32 accumulate; B=2, T=4
  G9  stateful policy core: the reference with ``agent.prev_hidden`` set to
      zeros after reset(), so every step takes its else branch
      (attention.py:356-358: query from h_{t-1}, LSTMCell from (h, c));
      B=3, T=6 with prev_reward / prev_action, fwd+bwd

Weights: detinit.deterministic_params(seed=0).  Frames: detinit.frames_u8.
Loss for G3/G4/G7: sum(logits*Gl) + sum(values*Gv), Gl/Gv = detinit.cotangent.
Usage:  python tests/golden/gen_golden.py [G1 G2 ...]   (default: all)
"""
import importlib.util
import os
import sys
import types

sys.dont_write_bytecode = True
REF = "/root/reference"
if not os.path.isfile(os.path.join(REF, "attention.py")):
    sys.exit("gen_golden: /root/reference is absent; fixtures can only be generated "
             "in the build container")

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import helpers  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

detinit = helpers.detinit
torch.set_num_threads(8)


def _import_ref(name, fname):
    spec = importlib.util.spec_from_file_location(name, os.path.join(REF, fname))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


ref = _import_ref("ref_attention", "attention.py")


def new_agent(h=11, w=11, A=18):
    agent = ref.Agent(num_actions=A)
    detinit.load_into(agent, detinit.deterministic_params(0, A))
    if (h, w) != (27, 20):
        agent.spatial = ref.SpatialBasis(h, w)
    return agent


def frames(T, B, H=84, W=84, seed=1234):
    return torch.from_numpy(detinit.frames_u8(seed, (T, B, H, W, 3)).astype(np.float32))


def run(agent, X, prev_reward=None, prev_action=None, capture=False, stateful=False):
    agent.reset()
    if stateful:   # reach the reference's else branch (attention.py:356-358): a policy-core state exists
        agent.prev_hidden = torch.zeros(X.shape[1], agent.hidden_size)
    L, V, As, Rs = [], [], [], []
    orig_sm, orig_aa = ref.spatial_softmax, ref.apply_alpha
    if capture:
        def sm(A):
            out = orig_sm(A)
            As.append(out.detach().clone())
            return out

        def aa(A, Vv):
            out = orig_aa(A, Vv)
            Rs.append(out.detach().clone())
            return out
        ref.spatial_softmax, ref.apply_alpha = sm, aa
    try:
        for t in range(X.shape[0]):
            kw = {}
            if prev_reward is not None:
                kw["prev_reward"] = prev_reward[t]
            if prev_action is not None:
                kw["prev_action"] = prev_action[t]
            lg, vl = agent(X[t], **kw)
            L.append(lg), V.append(vl)
    finally:
        ref.spatial_softmax, ref.apply_alpha = orig_sm, orig_aa
    return torch.stack(L), torch.stack(V), As, Rs


def grads_fp(agent, out, prefix):
    for name, p in agent.named_parameters():
        g = p.grad if p.grad is not None else torch.zeros_like(p)
        helpers.store_fp(out, prefix, name, g.numpy())


def g1():
    out = {}
    for (h, w) in [(11, 11), (21, 21), (27, 20)]:
        out[f"S_{h}x{w}"] = ref.SpatialBasis(h, w).S.numpy()
    return out


def g2():
    agent = new_agent()
    X = frames(1, 2)
    lg, vl, As, Rs = run(agent, X, capture=True)
    return {"logits": lg.detach().numpy(), "values": vl.detach().numpy(),
            "attn": As[0].numpy(), "readout": Rs[0].numpy(), "T": 1, "B": 2}


def fwd_bwd(T, B, scale=1.0, with_prev=False, H=84, W=84, grid=(11, 11), stateful=False):
    agent = new_agent(*grid)
    X = frames(T, B, H, W) * scale
    pr = pa = None
    if with_prev:
        pr = torch.from_numpy(detinit.cotangent(77, (T, B)))
        pa = torch.from_numpy((detinit.frames_u8(78, (T, B)) % 18).astype(np.float32))
    lg, vl, As, _ = run(agent, X, pr, pa, capture=True, stateful=stateful)
    Gl = torch.from_numpy(detinit.cotangent(2, tuple(lg.shape)))
    Gv = torch.from_numpy(detinit.cotangent(3, tuple(vl.shape)))
    loss = (lg * Gl).sum() + (vl * Gv).sum()
    loss.backward()
    out = {"logits": lg.detach().numpy(), "values": vl.detach().numpy(),
           "attn": torch.stack(As).numpy(), "T": T, "B": B, "scale": scale}
    grads_fp(agent, out, "g_")
    return out


def g5():
    """REINFORCE through main_mp's own Policy / finish_episode (gym stubbed)."""
    sys.modules["gym"] = types.ModuleType("gym")
    saved = sys.modules.get("attention")
    sys.modules["attention"] = ref
    try:
        mm = _import_ref("ref_main_mp", "main_mp.py")
    finally:
        if saved is not None:
            sys.modules["attention"] = saved
        else:
            sys.modules.pop("attention", None)
    agent = new_agent()
    policy = mm.Policy(agent=agent)
    torch.manual_seed(543)
    T = 12
    obs = detinit.frames_u8(1234, (T, 84, 84, 3))
    rewards = (detinit.frames_u8(99, (T,)) % 3).astype(np.float64).tolist()
    logits = []
    orig_fwd = agent.forward

    def fwd(*a, **k):
        lg, vl = orig_fwd(*a, **k)
        logits.append(lg.detach().clone())
        return lg, vl
    agent.forward = fwd
    agent.reset()
    actions = []
    for t in range(T):
        actions.append(policy(obs[t], ts=t))
        policy.rewards.append(rewards[t])

    class _NoStep:
        def zero_grad(self):
            agent.zero_grad()

        def step(self):
            pass
    cfg = types.SimpleNamespace(gamma=0.99)
    mm.finish_episode(_NoStep(), policy, cfg)
    out = {"actions": np.array(actions, dtype=np.int64), "rewards": np.array(rewards),
           "logits": torch.stack(logits).numpy(), "T": T, "B": 1}
    grads_fp(agent, out, "g_")
    return out


def g6():
    agent = new_agent(27, 20)
    X = frames(2, 1, 210, 160)
    lg, vl, As, _ = run(agent, X, capture=True)
    return {"logits": lg.detach().numpy(), "values": vl.detach().numpy(),
            "attn": torch.stack(As).numpy(), "T": 2, "B": 1}


def _bf(t):
    return t.to(torch.bfloat16).to(t.dtype)


class _RoundedConv(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, stride, pad):
        xr, wr = _bf(x), _bf(w)
        ctx.save_for_backward(xr, wr)
        ctx.k = (stride, pad, x.shape, w.shape, b is not None)
        return F.conv2d(xr, wr, b, stride=stride, padding=pad)

    @staticmethod
    def backward(ctx, g):
        xr, wr = ctx.saved_tensors
        stride, pad, xs, ws, hb = ctx.k
        gr = _bf(g)
        return (torch.nn.grad.conv2d_input(xs, wr, gr, stride=stride, padding=pad),
                torch.nn.grad.conv2d_weight(xr, ws, gr, stride=stride, padding=pad),
                g.sum((0, 2, 3)) if hb else None, None, None)


def g7():
    orig = torch.nn.Conv2d.forward

    def fwd(self, x):
        return _RoundedConv.apply(x, self.weight, self.bias, self.stride, self.padding)
    torch.nn.Conv2d.forward = fwd
    try:
        return fwd_bwd(4, 2)
    finally:
        torch.nn.Conv2d.forward = orig


def main():
    jobs = {"G1": g1, "G2": g2, "G3": lambda: fwd_bwd(20, 1), "G3n": lambda: fwd_bwd(20, 1, 1 / 255.0),
            "G4": lambda: fwd_bwd(4, 4, with_prev=True), "G5": g5, "G6": g6, "G7": g7,
            "G9": lambda: fwd_bwd(6, 3, with_prev=True, stateful=True)}
    only = set(sys.argv[1:])
    for name, fn in jobs.items():
        if only and name not in only:
            continue
        out = fn()
        path = os.path.join(HERE, f"{name}.npz")
        np.savez_compressed(path, **{k: np.asarray(v) for k, v in out.items()})
        print(f"{name}: {len(out)} arrays -> {os.path.relpath(path)} "
              f"({os.path.getsize(path) // 1024} KiB)")


if __name__ == "__main__":
    main()
