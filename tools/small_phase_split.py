"""The one-launch small-batch solve (dilqr_mpc_solve_small_f32) at the IL
loop's shape — cartpole, T = 35, B = 32, bounds +-100, decay 0.5, two passes,
100 iterations (eps = 0, the stop rule never fires) — timed with HIP events on
the launch stream.  With a library built with -DDILQR_PHASE_SKIP=1 (timing
only) every iteration ends after its sweep, so the difference between the two
builds is the line search's share (tools/ab.sh, AB_CMD).  Prints one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "differentiable-ilqr_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from dilqr import _native as N  # noqa: E402
from dilqr import ops  # noqa: E402
from dilqr.env_dx.cartpole import CartpoleDx  # noqa: E402

dev = torch.device("cuda", 0)
T, B, ITERS = 35, 32, 100
dx = CartpoleDx()
x0 = torch.tensor(bench.make_problems(B, seed=2)[0], device=dev)
q, p = dx.get_true_obj()
C = torch.diag(q).repeat(T, B, 1, 1).to(dev).contiguous()
c = p.repeat(T, B, 1).to(dev).contiguous()
th = ops.theta_of(dx, x0)
bd, _keep = N.make_bounds(-100.0, 100.0)
stream = torch.cuda.current_stream(dev)


sv = ops.MPCSolve(T, B, 5, 1, dev)


def run(_r):      # every call begins from x0 (best_cost_eps 1e-4, eps 0: all ITERS iterations run)
    sv.solve_small(dx.model_id, th, x0, C, c, bd, 0.5, 2, ITERS, 1e-4, 0.0, 10 ** 9)


run(0)
ms = bench._event_ms(stream, run, 5)
print(json.dumps({"solve_ms": round(ms, 4), "us_per_iteration": round(ms * 1e3 / ITERS, 2),
                  "iterations_run": int(sv.iterations) if hasattr(sv, "iterations") else None}), flush=True)
