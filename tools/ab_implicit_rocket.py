"""Config-3 shape rocket implicit backward (B=32768, T=30, unconstrained) kernel
time for A/B runs of library variants (tools/ab.sh with
AB_CMD=tools/ab_implicit_rocket.py): the solution of a 10-iteration solve,
then HIP-event timing of the implicit backward as bench.py times it.  Prints
one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "differentiable-ilqr_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from dilqr import ops  # noqa: E402
from dilqr.env_dx.rocket import RocketDx  # noqa: E402
from dilqr.implicit import implicit_backward  # noqa: E402

dev = torch.device("cuda", 0)
T, B, n, m = 30, 32768, 13, 3
rng = np.random.RandomState(0)
r = rng.uniform([0, -4, -2.5], [10, 4, 2.5], (B, 3))
v = rng.normal(0, 0.1, (B, 3))
q4 = np.array([1., 0, 0, 0]) + 0.05 * rng.normal(size=(B, 4))
q4 /= np.linalg.norm(q4, axis=1, keepdims=True)
w = rng.normal(0, 0.02, (B, 3))
x0 = torch.tensor(np.concatenate([r, v, q4, w], 1), dtype=torch.float32, device=dev)
dx = RocketDx()
q, p = dx.get_true_obj()
C = torch.diag(q).repeat(T, B, 1, 1).to(dev).contiguous()
c = p.repeat(T, B, 1).to(dev).contiguous()
theta = ops.theta_of(dx, x0)
x, u, _cost, _du, _sv = ops.mpc_solve(dx.model_id, theta, x0, C, c, T, lqr_iter=10, eps=0.0,
                                      linesearch_decay=0.2, max_linesearch_iter=5, not_improved_lim=10 ** 9)
F, _f = ops.linearize(dx.model_id, theta, x, u)
K, _k, _ = ops.lqr_backward(C, c, F, n, m, x=x, u=u)
g = torch.Generator(device=dev).manual_seed(1)
wx = torch.randn(T, B, n, device=dev, generator=g)
wu = torch.randn(T, B, m, device=dev, generator=g)
stream = torch.cuda.current_stream(dev)
grads = implicit_backward(dx, wx, wu, C, c, None, None, x, u, K, None, None, None)
ms = bench._event_ms(stream, lambda _r: implicit_backward(dx, wx, wu, C, c, None, None, x, u, K, None, None, None), 5)
chk = float(sum(t.double().abs().sum() for t in grads if torch.is_tensor(t)))
print(json.dumps({"implicit_rocket_ms": round(ms, 4), "grad_abs_sum": chk}), flush=True)
