"""Config 3 (rocket) profiling driver: two fixed-iteration solves and two sweeps."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "differentiable-ilqr_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda", 0)
bench.sweep_roofline(13, 3, 30, 32768, dev, reps=3)
out = bench.secondary_configs(dev)
print(out["config3_rocket"])
