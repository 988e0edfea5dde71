"""Small-batch Riccati sweep mapping, timed: the standalone
cartpole sweep (n = 5, m = 1; F from HBM) at the IL loop's shape — T = 35,
n_batch 32..256, box +-100 and unconstrained — through whichever library is
in-tree.  tools/ab.sh with AB_CMD=tools/small_sweep_mapping.py times the lane
sweep (one lane per problem, the shipped build) against a build with
-DDILQR_GROUP_SWEEP_SMALL=4096 (tu_riccati.hip: the 16-lane group sweep, lane r
owns row r of Q, V exchanged through LDS).  HIP events around 200 launches on
torch's current stream.  Prints one JSON line: ms per sweep and us per horizon
step per (mode, B), plus checksums of K, k (the two mappings sum in different
orders, so the checksums agree to fp32 rounding, not bit for bit)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "differentiable-ilqr_amd"))
import torch  # noqa: E402

from dilqr import ops  # noqa: E402

dev = torch.device("cuda", 0)
T, n, m = 35, 5, 1
d = n + m
out = {}
for B in (32, 64, 256):
    g = torch.Generator(device="cpu").manual_seed(B)
    F = torch.zeros(T - 1, B, n, d)
    F[..., :n] = torch.eye(n) + 0.05 * torch.randn(T - 1, B, n, n, generator=g)
    F[..., n] = 0.1 * torch.randn(T - 1, B, n, generator=g)
    q = 0.1 + torch.rand(T, B, d, generator=g)
    C = torch.diag_embed(q)
    c = 0.1 * torch.randn(T, B, d, generator=g)
    x = torch.randn(T, B, n, generator=g)
    u = torch.randn(T, B, m, generator=g)
    F, C, c, x, u = (a.to(dev) for a in (F, C, c, x, u))
    for mode, lo, hi in (("box100", -100.0, 100.0), ("unc", None, None)):
        def run():
            return ops.lqr_backward(C, c, F, n, m, x=x, u=u, u_lower=lo, u_upper=hi)
        K, k, _ = run()
        for _ in range(20):
            run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 200
        e0.record()
        for _ in range(reps):
            run()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        out[f"{mode}_B{B}"] = {"ms": round(ms, 5), "us_per_step": round(1e3 * ms / T, 4),
                               "K_abs_sum": float(K.double().abs().sum()), "k_abs_sum": float(k.double().abs().sum())}
print(json.dumps(out))
