"""Config 4 (cartpole, bounds +-100) profiling driver: two fixed-iteration solves."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "differentiable-ilqr_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from dilqr import _native as N  # noqa: E402
from dilqr import ops  # noqa: E402

dev = torch.device("cuda", 0)
T, B = 25, 65536
lim = float(sys.argv[1]) if len(sys.argv) > 1 else 100.0
x0n, q, p = bench.make_problems(B)
x0 = torch.tensor(x0n, device=dev)
C = torch.diag(torch.tensor(q)).repeat(T, B, 1, 1).to(dev).contiguous()
c = torch.tensor(p).repeat(T, B, 1).to(dev).contiguous()
theta = torch.tensor([9.8, 1.0, 0.1, 0.5], device=dev)
sv = ops.MPCSolve(T, B, 5, 1, dev)
bd, keep = N.make_bounds(-lim, lim)
for _ in range(2):
    sv.begin(N.MODEL_CARTPOLE, theta, x0)
    for i in range(10):
        sv.iterate(N.MODEL_CARTPOLE, theta, x0, C, c, bd, 0.5, 2, i, 1e-4, 0.0, 10 ** 9)
torch.cuda.synchronize()
print("ok", float(sv.best_cost.mean()))
