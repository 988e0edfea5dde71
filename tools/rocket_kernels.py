"""Config 3 kernel timings (rocket n=13 m=3 T=30 B=32768): standalone sweep, the
fused iteration, and a whole fixed-iteration MPC solve per iteration."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "differentiable-ilqr_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda", 0)
sw = bench.sweep_roofline(13, 3, 30, 32768, dev, reps=5)
sec = bench.secondary_configs(dev)["config3_rocket"]
print(json.dumps({"sweep_ms": sw["avg_launch_ms"], "iter_ms": sec["fused_iteration"]["avg_launch_ms"],
                  "mpc_ms_per_iter": sec["ms_per_iter"]}))
