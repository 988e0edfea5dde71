"""Standalone Riccati sweep times for A/B runs (tools/ab.sh with
AB_CMD=tools/ab_sweep.py): the north-star cartpole shape (n=5 m=1 T=25
B=65536) and the rocket one (n=13 m=3 T=30 B=32768), bench.sweep_roofline's
timing.  Prints one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "differentiable-ilqr_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda", 0)
cp = bench.sweep_roofline(5, 1, 25, 65536, dev, reps=10)
rk = bench.sweep_roofline(13, 3, 30, 32768, dev, reps=5)
print(json.dumps({"cartpole_sweep_ms": round(cp["avg_launch_ms"], 5), "rocket_sweep_ms": round(rk["avg_launch_ms"], 4)}),
      flush=True)
