"""Rocket standalone Riccati sweep (k_lqr_backward_group<13,3,UNC>, F from HBM,
T = 30) timed at several batch sizes: per-problem time against the number of
wave rounds (4 problems per wave, 3 waves per SIMD, 1 024 SIMDs: 12 288
problems per round).  Prints one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "differentiable-ilqr_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda", 0)
out = {}
for B in (12288, 24576, 32768, 36864, 49152):
    r = bench.sweep_roofline(13, 3, 30, B, dev, reps=10)
    out[B] = {"ms": round(r["avg_launch_ms"], 4), "us_per_1k_problems": round(1e3 * r["avg_launch_ms"] / B * 1e3, 3),
              "rounds": round(B / 12288, 2), "frac": round(r["frac"], 3)}
    torch.cuda.empty_cache()
print(json.dumps(out))
