"""Config 3 (rocket n=13 m=3 T=30 B=32768) kernel timings for A/B runs: the
fused MPC iteration (HIP events, iterations 1..5 of a solve), the standalone
sweep and the implicit backward.  Prints one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "differentiable-ilqr_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from dilqr import _native as N  # noqa: E402
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
sv = ops.MPCSolve(T, B, n, m, dev)
nb, _ = N.make_bounds(None, None)
s = N.stream(dev)
stream = torch.cuda.current_stream(dev)
sv.begin(N.MODEL_ROCKET, theta, x0)
sv.iterate(N.MODEL_ROCKET, theta, x0, C, c, nb, 0.2, 5, 0, 1e-4, 0.0, 10 ** 9)
it = {"i": 1}


def step(_r):
    N.call("dilqr_mpc_step_f32", N.MODEL_ROCKET, T, B, N.ptr(theta), N.ptr(x0), N.ptr(C), N.ptr(c), nb, 0.2, 5,
           it["i"], 1e-4, 0.0, 10 ** 9, sv.state, s)
    N.call("dilqr_mpc_stop_rule_f32", T, m, B, it["i"], sv.state, s)
    it["i"] += 1


iter_ms = bench._event_ms(stream, step, 5)
x, u = sv.gather_best()
cost = float(sv.best_cost.mean())
sweep = bench.sweep_roofline(n, m, T, B, dev, reps=3)
F, _f = ops.linearize(N.MODEL_ROCKET, theta, x, u)
K, _k, _ = ops.lqr_backward(C, c, F, n, m, x=x, u=u)
g = torch.Generator(device=dev).manual_seed(1)
wx = torch.zeros(T, B, n, device=dev)
wu = torch.randn(T, B, m, device=dev, generator=g)
ib = lambda _r: implicit_backward(dx, wx, wu, C, c, None, None, x, u, K, None, None, None)
ib(0)
ib_ms = bench._event_ms(stream, ib, 3)
print(json.dumps({"iter_step_ms": round(iter_ms, 4), "sweep_ms": round(sweep["avg_launch_ms"], 4),
                  "implicit_ms": round(ib_ms, 4), "mean_best_cost_it6": round(cost, 6)}), flush=True)
