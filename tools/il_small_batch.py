"""The IL loop's training step at the reference's own batch (il_exp.py:44:
n_batch = 32) and at 4096: cartpole, T = 35, up to 100 iterations with the stop
rule (il_env.py:153-188), then im_loss.backward() through the implicit
backward.  Prints one JSON line: per batch size the step time, the forward
(solve) and backward split, the iterations the solve ran and the number of
host polls, each from HIP events on the launch stream."""
import json
import os
import sys
import time
import warnings

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "differentiable-ilqr_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from dilqr import il  # noqa: E402
from dilqr.env_dx.cartpole import CartpoleDx  # noqa: E402


def measure(B, reps=5, dev=torch.device("cuda", 0)):
    env = il.IL_Env("cartpole", lqr_iter=100, mpc_T=35, device=dev)
    xi = torch.tensor(bench.make_problems(B, seed=2)[0], device=dev)
    params = torch.tensor((9.8, 3.0, 0.1, 1.0), device=dev, requires_grad=True)
    q, p = env.true_dx.get_true_obj()
    q, p = q.to(dev), p.to(dev)
    target = torch.zeros(35, B, 1, device=dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    fwd, bwd, tot, iters = [], [], [], []
    for r in range(reps + 1):
        params.grad = None
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ev[0].record()
        dx = CartpoleDx(params)
        m = il.MPC(5, 1, 35, u_lower=-100.0, u_upper=100.0, lqr_iter=100, verbose=0, exit_unconverged=False,
                   detach_unconverged=True, linesearch_decay=0.5, max_linesearch_iter=2, eps=1e-4)
        Q = torch.diag(q).unsqueeze(0).unsqueeze(0).repeat(35, B, 1, 1)
        P = p.unsqueeze(0).repeat(35, B, 1)
        _, uu, _ = m(xi, il.QuadCost(Q, P), dx)
        ev[1].record()
        loss = (target - uu).pow(2).mean()
        loss.backward()
        ev[2].record()
        torch.cuda.synchronize()
        if r:                                           # the first step loads code objects
            tot.append((time.perf_counter() - t0) * 1e3)
            fwd.append(ev[0].elapsed_time(ev[1]))
            bwd.append(ev[1].elapsed_time(ev[2]))
            sv = m.last_solve
            iters.append(sv.iterations if sv.stopped else sv.last_iteration + 1)
    med = lambda v: sorted(v)[len(v) // 2]  # noqa: E731
    return {"batch": B, "ms_per_step": med(tot), "forward_ms": med(fwd), "backward_ms": med(bwd),
            "iterations": iters, "path": "one-launch small-batch solve" if getattr(m.last_solve, "small", False) else "per-iteration launches"}


if __name__ == "__main__":
    # --both: each batch size on the one-launch small-batch solve AND on the
    # per-iteration launches (ops.SMALL_BATCH_MAX set to 0 for the latter), to
    # place SMALL_BATCH_MAX
    from dilqr import ops
    both = "--both" in sys.argv
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        sizes = [int(a) for a in sys.argv[1:] if not a.startswith("--")] or [32, 4096]
        out = []
        keep = ops.SMALL_BATCH_MAX
        for B in sizes:
            out.append(measure(B))
            if both and B <= keep:
                ops.SMALL_BATCH_MAX = 0
                out.append(measure(B))
                ops.SMALL_BATCH_MAX = keep
    print(json.dumps(out), flush=True)
