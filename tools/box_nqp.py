"""Config 4 (cartpole T=25, 65536 problems, bounds +-LIM): pnqp iterations per
problem in the Riccati sweep at the current trajectory of iteration ITER of the
solve (the fused MPC kernel's sweep runs the same pnqp per step), and per wave
of 64 problems the maximum, which is what a wave pays.  n_qp[b] = sum over t of
(1 + pnqp iterations).

  python tools/box_nqp.py [LIM] [ITER]
"""
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
from dilqr import _native as N  # noqa: E402

LIM = float(sys.argv[1]) if len(sys.argv) > 1 else 100.0
ITER = int(sys.argv[2]) if len(sys.argv) > 2 else 5
dev = torch.device("cuda", 0)
T, B, n, m = bench.T_HORIZON, bench.B_PER_GPU, 5, 1
x0n, q, p = bench.make_problems(B)
x0 = torch.tensor(x0n, device=dev)
C = torch.diag(torch.tensor(q)).repeat(T, B, 1, 1).to(dev).contiguous()
c = torch.tensor(p).repeat(T, B, 1).to(dev).contiguous()
theta = torch.tensor([9.8, 1.0, 0.1, 0.5], device=dev)
x, u, _, _, _ = ops.mpc_solve(N.MODEL_CARTPOLE, theta, x0, C, c, T, u_lower=-LIM, u_upper=LIM, lqr_iter=ITER,
                              eps=0.0, linesearch_decay=0.5, max_linesearch_iter=2, not_improved_lim=10 ** 9)
F, _f = ops.linearize(N.MODEL_CARTPOLE, theta, x, u)
_, _, nqp = ops.lqr_backward(C, c, F, n, m, x=x, u=u, u_lower=-LIM, u_upper=LIM, want_nqp=True)
nq = nqp.cpu().numpy().astype(np.int64)
wave_max = nq.reshape(-1, 64).max(1)
slow = np.nonzero(nq > 2 * T)[0]
out = {"lim": LIM, "iteration": ITER, "n_qp_mean": float(nq.mean()), "n_qp_p99": float(np.percentile(nq, 99)),
       "n_qp_max": int(nq.max()), "problems_over_2T": int(len(slow)), "waves_with_one": int((wave_max > 2 * T).sum()),
       "hist": {int(k): int(v) for k, v in zip(*np.unique(np.minimum(nq, 200), return_counts=True))}}
if len(slow):
    b = int(slow[0])
    uu = u[:, b, 0].cpu().numpy()
    out["example"] = {"b": b, "n_qp": int(nq[b]), "u": [round(float(v), 3) for v in uu],
                      "finite": bool(np.isfinite(x[:, b].cpu().numpy()).all())}
print(json.dumps(out))
