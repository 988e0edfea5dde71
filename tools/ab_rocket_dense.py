"""Config 3 (rocket n=13 m=3 T=30 B=32768) MPC iteration time with every cost
a time-invariant diagonal one (the register-cost waves; the dense-cost
launches find nothing to do) and with every cost dense (diag(q) plus a small
symmetric off-diagonal coupling: the dense-cost launches do all the work).
HIP events around iterations 1..5 of a solve.  Prints one JSON line.
(the dense-cost launches' grid cap.)"""
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
theta = ops.theta_of(dx, x0)
nb, _ = N.make_bounds(None, None)
s = N.stream(dev)
stream = torch.cuda.current_stream(dev)
out = {}
for kind in ("diag", "dense"):
    Q = torch.diag(q).to(dev)
    if kind == "dense":
        E = 1e-3 * torch.ones(n + m, n + m, device=dev)
        Q = Q + E - torch.diag(torch.diag(E))
    C = Q.repeat(T, B, 1, 1).contiguous()
    c = p.repeat(T, B, 1).to(dev).contiguous()
    sv = ops.MPCSolve(T, B, n, m, dev)
    sv.begin(N.MODEL_ROCKET, theta, x0)
    sv.iterate(N.MODEL_ROCKET, theta, x0, C, c, nb, 0.2, 5, 0, 1e-4, 0.0, 10 ** 9)
    it = {"i": 1}

    def step(_r, C=C, c=c, sv=sv, it=it):
        N.call("dilqr_mpc_step_f32", N.MODEL_ROCKET, T, B, N.ptr(theta), N.ptr(x0), N.ptr(C), N.ptr(c), nb, 0.2, 5,
               it["i"], 1e-4, 0.0, 10 ** 9, sv.state, s)
        N.call("dilqr_mpc_stop_rule_f32", T, m, B, it["i"], sv.state, s)
        it["i"] += 1

    out[f"{kind}_iter_ms"] = round(bench._event_ms(stream, step, 5), 4)
    out[f"{kind}_cost"] = round(float(sv.best_cost.mean()), 5)
    del sv, C, c
    torch.cuda.empty_cache()
print(json.dumps(out), flush=True)
