"""A/B timing of the dense time-varying cost path (bench.dense_cost_roofline:
the fused iteration on a dense SPD C_t,b distinct per (t, b), cartpole T = 25,
65 536 problems) beside the headline solve, for tools/ab.sh
(AB_CMD=tools/ab_dense_cost.py).  Prints one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "differentiable-ilqr_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda", 0)
B = bench.B_PER_GPU
x0n, q, p = bench.make_problems(B)
x0 = torch.tensor(x0n, device=dev)
theta = torch.tensor([9.8, 1.0, 0.1, 0.5], device=dev)
r = bench.dense_cost_roofline(dev, x0, theta, B)
print(json.dumps({"dense_iter_ms": round(r["avg_launch_ms"], 5), "dense_frac": round(r["frac"], 4)}))
