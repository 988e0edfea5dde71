"""Config 3 (rocket): per iteration, the share of problems and of waves that
need more than one line-search pass (alpha < decay), and how often a problem's
accepted pass repeats the previous iteration's (a speculative write by the
previous winner's lane)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "differentiable-ilqr_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

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
C = torch.diag(q).repeat(T, B, 1, 1).to(dev).contiguous()
c = p.repeat(T, B, 1).to(dev).contiguous()
theta = ops.theta_of(dx, x0)
sv = ops.MPCSolve(T, B, n, m, dev)
nb, _ = N.make_bounds(None, None)
sv.begin(N.MODEL_ROCKET, theta, x0)
prev = None
for i in range(10):
    sv.iterate(N.MODEL_ROCKET, theta, x0, C, c, nb, 0.2, 5, i, 1e-4, 0.0, 10 ** 9)
    al = sv.alpha.clone()
    hist = {f"{x:g}": int((al == x).sum()) for x in (1.0, 0.2, 0.04, 0.008, 0.0016)}
    # lane-pair search (today): 32 problems per wave, rounds of 2 candidates
    w32 = al.view(-1, 32)
    r2 = float((w32 < 0.2 - 1e-7).any(1).float().mean())          # some problem needs candidates 3+
    r3 = float((w32 < 0.008 - 1e-9).any(1).float().mean())        # ... candidate 5
    # a 4-lanes-per-problem search: 16 problems per wave, one round of 4 candidates
    w16 = al.view(-1, 16)
    q2 = float((w16 < 0.008 - 1e-9).any(1).float().mean())
    # the quad search (k_mpc_search_quad): a wave rewrites (phase 2) when any
    # of its 16 problems accepted a pass other than 0
    ph2 = float((w16 < 1.0).any(1).float().mean())
    # a speculative write by the lane of each problem's previous winner: the
    # problems whose winner repeats, and the waves that would still rewrite
    if prev is not None:
        same = (al == prev)
        keep = float(same.float().mean())
        ph2p = float((~same).view(-1, 16).any(1).float().mean())
    else:
        keep, ph2p = float("nan"), float("nan")
    prev = al
    print(f"iter {i}: alpha hist {hist}; 32-problem waves needing round 2 {r2:.3f}, round 3 {r3:.3f}; "
          f"16-problem waves needing a 5th candidate {q2:.3f}, a phase-2 rewrite {ph2:.3f}; "
          f"winner repeats {keep:.4f}, rewrite with previous-winner speculation {ph2p:.3f}", flush=True)
