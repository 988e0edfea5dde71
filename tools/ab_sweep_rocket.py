"""Rocket-shape standalone Riccati sweep (k_lqr_backward_group<13,3,UNC>, B=32768,
T=30, F from HBM) kernel time for A/B runs (tools/ab.sh with
AB_CMD=tools/ab_sweep_rocket.py), as bench.py's sweep_roofline times it."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "differentiable-ilqr_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda", 0)
r = bench.sweep_roofline(13, 3, 30, 32768, dev, reps=5)
print(json.dumps({"sweep_ms": round(r["avg_launch_ms"], 4), "frac": round(r["frac"], 4)}), flush=True)
