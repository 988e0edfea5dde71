"""Where one headline solve's time goes (config 2: cartpole T=25, 65536 problems,
10 fixed iterations): HIP events around begin (u = 0 fill + rollout), iteration
0 (reads the caller's C, builds the packed copy), iterations 1..9 and the
stop-rule kernel after each, then whole solves through MPCSolve.iterate with no
events in between (`solve_iterate`: the number to compare variants by — the
events themselves add a few us per launch).  Prints one JSON line."""
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

dev = torch.device("cuda", 0)
T, n, m = bench.T_HORIZON, bench.N_STATE, bench.N_CTRL
B = int(sys.argv[1]) if len(sys.argv) > 1 else bench.B_PER_GPU
LIM = float(sys.argv[2]) if len(sys.argv) > 2 else None          # box +-LIM (config 4), default none
x0n, q, p = bench.make_problems(B)
x0 = torch.tensor(x0n, device=dev)
C = torch.diag(torch.tensor(q)).repeat(T, B, 1, 1).to(dev).contiguous()
c = torch.tensor(p).repeat(T, B, 1).to(dev).contiguous()
theta = torch.tensor([9.8, 1.0, 0.1, 0.5], device=dev)
sv = ops.MPCSolve(T, B, n, m, dev)
nb, _keep = N.make_bounds(None if LIM is None else -LIM, LIM)
s = N.stream(dev)
stream = torch.cuda.current_stream(dev)
ITERS, SOLVES = 10, 6


def ev():
    e = torch.cuda.Event(enable_timing=True)
    e.record(stream)
    return e


marks = []
for solve in range(SOLVES):
    e0 = ev()
    sv.begin(N.MODEL_CARTPOLE, theta, x0)
    e1 = ev()
    row = [e0, e1]
    for i in range(ITERS):
        N.call("dilqr_mpc_step_f32", N.MODEL_CARTPOLE, T, B, N.ptr(theta), N.ptr(x0), N.ptr(C), N.ptr(c), nb, 0.5, 2,
               i, 1e-4, 0.0, 10 ** 9, sv.state, s)
        row.append(ev())
        N.call("dilqr_mpc_stop_rule_f32", T, m, B, i, sv.state, s)
        row.append(ev())
    marks.append(row)
# the same solves as the bench runs them: no events between the launches
whole = []
for solve in range(SOLVES):
    e0 = ev()
    sv.begin(N.MODEL_CARTPOLE, theta, x0)
    for i in range(ITERS):
        sv.iterate(N.MODEL_CARTPOLE, theta, x0, C, c, nb, 0.5, 2, i, 1e-4, 0.0, 10 ** 9)
    whole.append((e0, ev()))
torch.cuda.synchronize()
res = {"begin": [], "iter0": [], "iterk": [], "stop_rule": [], "solve": []}
for row in marks[1:]:                       # the first solve warms up
    res["begin"].append(row[0].elapsed_time(row[1]))
    res["solve"].append(row[0].elapsed_time(row[-1]))
    for i in range(ITERS):
        a, b_, c_ = row[1 + 2 * i], row[2 + 2 * i], row[3 + 2 * i]
        res["iter0" if i == 0 else "iterk"].append(a.elapsed_time(b_))
        res["stop_rule"].append(b_.elapsed_time(c_))
out = {k: float(np.mean(v)) for k, v in res.items()}
out["per_iteration_of_solve"] = out["solve"] / ITERS
out["solve_iterate"] = float(np.mean([a.elapsed_time(b_) for a, b_ in whole[1:]]))
out["per_iteration_iterate"] = out["solve_iterate"] / ITERS
out["mean_best_cost"] = float(sv.best_cost.mean())
out["B"] = B
out["box"] = LIM
print(json.dumps(out))
