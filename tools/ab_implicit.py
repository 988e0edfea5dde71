"""Config-4 cartpole implicit backward (B=65536, T=25, bounds +-10) kernel time
for A/B runs of library variants (tools/ab.sh with AB_CMD=tools/ab_implicit.py):
the solution of a 10-iteration solve, then HIP-event timing of the implicit
backward as bench.py times it.  Prints one JSON line."""
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
from dilqr.implicit import implicit_backward  # noqa: E402

dev = torch.device("cuda", 0)
T, n, m, B = bench.T_HORIZON, bench.N_STATE, bench.N_CTRL, bench.B_PER_GPU
x0n, q, p = bench.make_problems(B)
x0 = torch.tensor(x0n, device=dev)
C = torch.diag(torch.tensor(q)).repeat(T, B, 1, 1).to(dev).contiguous()
c = torch.tensor(p).repeat(T, B, 1).to(dev).contiguous()
theta = torch.tensor([9.8, 1.0, 0.1, 0.5], device=dev)
bd, _keep = N.make_bounds(-10.0, 10.0)
sv = ops.MPCSolve(T, B, n, m, dev, fixed_iters=10)
sv.solve_fixed(N.MODEL_CARTPOLE, theta, x0, C, c, bd, 0.5, 2, 1e-4)
x, u = sv.gather_best()
F, _f = ops.linearize(N.MODEL_CARTPOLE, theta, x, u)
K, _k, _ = ops.lqr_backward(C, c, F, n, m, x=x, u=u, u_lower=-10.0, u_upper=10.0)
g = torch.Generator(device=dev).manual_seed(1)
wx = torch.zeros(T, B, n, device=dev)
wu = torch.randn(T, B, m, device=dev, generator=g)
cart = CartpoleDx()
grads = implicit_backward(cart, wx, wu, C, c, None, None, x, u, K, -10.0, 10.0, None)
ms = bench.implicit_kernel_ms(cart, wx, wu, C, c, x, u, K, -10.0, 10.0, dev, reps=10)
chk = float(sum(t.double().abs().sum() for t in grads if torch.is_tensor(t)))
print(json.dumps({"implicit_ms": round(ms, 4), "grad_abs_sum": chk}), flush=True)
