"""main_mp.py's process structure on the drop-in Agent (tests/test_gpu_share.py runs it).

SURVEY.md §8(b): ``share_memory()``, ``parameters()`` and ``.to()`` must keep
working (main_mp.py:91-92,182).  Like main_mp.py:178-184 the parent builds
``attention.Agent(num_actions=18)`` on the CPU, calls ``agent.share_memory()``
and ``mp.spawn``s the workers; it never touches the GPU itself.  Each worker
follows train() (main_mp.py:83-92,100-116) and finish_episode()
(main_mp.py:62-80): Policy(agent) moved to the GPU, torch.optim.Adam over
policy.parameters(), agent.reset(), a 3-step episode of 210x160 uint8
observations through Policy.forward, the REINFORCE loss backward and the Adam
step.  Each worker checks its parameter gradients against the CPU oracle
(oracle/ref_cpu.py: the same episode's logits and REINFORCE loss with the
recorded actions, from the same weights) at 1e-4 norm-relative, and that
Adam moved its parameters.  The parent checks its shared CPU parameters are
untouched afterwards: as in the reference on a GPU, ``policy.to(device)``
gives each worker a private device copy ("the sharing silently
breaks"), so Hogwild updates never reach the shared tensors.

Prints one JSON line; exit status 1 on a failed check.
"""
import json
import os
import sys

import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import attention  # noqa: E402  (module level, as main_mp.py:8: registers aaa_amd, so spawned workers unpickle the Agent)

T_EP, H, W, A = 3, 210, 160, 18


def worker(rank, agent, q):
    import numpy as np
    from aaa_amd.policy import Policy
    from oracle import ref_cpu
    res = {"rank": rank}
    try:
        dev = torch.device("cuda:0")
        torch.manual_seed(10 + rank)
        w0 = {k: v.detach().clone() for k, v in agent.state_dict().items()}   # the shared CPU weights
        res["shared_in_worker"] = all(p.is_shared() for p in agent.parameters())
        policy = Policy(agent=agent)
        policy.to(dev)                                                  # main_mp.py:91
        optimizer = torch.optim.Adam(policy.parameters(), lr=1e-3)      # main_mp.py:92
        agent.reset()                                                   # main_mp.py:100
        rng = np.random.default_rng(100 + rank)
        obs = [rng.integers(0, 256, (H, W, 3), dtype=np.uint8) for _ in range(T_EP)]
        rewards = [0.0, 1.0, 0.0]
        actions = []
        for o, r in zip(obs, rewards):                                  # main_mp.py:108-116
            actions.append(int(policy(o)))
            policy.rewards.append(r)
        # finish_episode, main_mp.py:62-80
        eps = np.finfo(np.float32).eps.item()
        R, returns = 0, []
        for r in policy.rewards[::-1]:
            R = r + 0.99 * R
            returns.insert(0, R)
        returns = torch.tensor(returns)
        returns = (returns - returns.mean()) / (returns.std() + eps)
        policy_loss = [-lp * Rt for lp, Rt in zip(policy.saved_log_probs, returns)]
        optimizer.zero_grad()
        torch.cat(policy_loss).sum().backward()
        grads = {n: (p.grad.detach().cpu() if p.grad is not None else torch.zeros(p.shape))
                 for n, p in agent.named_parameters()}
        before = {n: p.detach().clone() for n, p in agent.named_parameters()}
        optimizer.step()
        torch.cuda.synchronize()
        del policy.rewards[:]
        del policy.saved_log_probs[:]
        # the oracle: the same episode from the same weights, the recorded actions
        P = ref_cpu.tensor_params({k: v.numpy() for k, v in w0.items()})
        X = torch.from_numpy(np.stack(obs)[:, None].astype(np.float32))
        lg, _, _ = ref_cpu.unroll(P, X, nq=4)
        ref_cpu.reinforce_loss(lg, actions, rewards).backward()
        worst, zero_ok = 0.0, True
        for n, g in grads.items():
            rg = P[n].grad if P[n].grad is not None else torch.zeros_like(P[n])
            if float(rg.norm()) == 0.0:
                zero_ok &= float(g.abs().max()) == 0.0
                continue
            worst = max(worst, float((g - rg).norm() / rg.norm()))
        moved = sum(int(not torch.equal(p.detach(), before[n])) for n, p in agent.named_parameters())
        on_gpu = all(p.is_cuda for p in agent.parameters())
        res.update({"actions": actions, "grad_worst_rel_vs_oracle": worst, "zero_grads_exact": zero_ok,
                    "params_moved_by_adam": moved, "params_on_gpu": on_gpu,
                    "ok": bool(worst <= 1e-4 and zero_ok and moved > 0 and on_gpu and res["shared_in_worker"])})
    except Exception as e:   # reported to the parent, which fails the run
        import traceback
        res.update({"ok": False, "error": repr(e), "trace": traceback.format_exc()[-3000:]})
    q.put(json.dumps(res))


def main():
    torch.manual_seed(0)
    agent = attention.Agent(num_actions=A)   # main_mp.py:180 (210x160 frames: the default 27x20 basis)
    agent.share_memory()                     # main_mp.py:182
    shared = all(p.is_shared() for p in agent.parameters())
    w0 = {k: v.detach().clone() for k, v in agent.state_dict().items()}
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    nprocs = int(os.environ.get("AAA_SHARE_PROCS", "2"))
    mp.spawn(worker, args=(agent, q), nprocs=nprocs, join=True)   # main_mp.py:184
    workers = sorted((json.loads(q.get()) for _ in range(nprocs)), key=lambda r: r["rank"])
    untouched = all(torch.equal(v, agent.state_dict()[k]) for k, v in w0.items())
    ok = shared and untouched and all(r["ok"] for r in workers)
    print(json.dumps({"shared_in_parent": shared, "parent_shared_params_untouched": untouched,
                      "workers": workers, "state_dict_keys": len(w0), "ok": ok}), flush=True)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
