"""Where one fused MPC iteration's time goes, per wave (config 2: cartpole T=25,
65536 problems, 1024 waves): runs the headline solve on the DIAGNOSTIC build
(-DDILQR_STAMPS, libdilqr_stamps.so; the stamps cost a few % and never ship)
and reads the s_memtime stamps lane 0 of every wave wrote at the phase
boundaries of k_mpc_iterate: stop-rule prologue, sweep (linearise + Riccati +
old cost), line search, epilogue.  The clock is s_memtime / s_memrealtime
(100 MHz) over each wave.  Prints one JSON line.

  make -C differentiable-ilqr_amd stamps      # here, on the CPU
  python tools/phase_stamps.py [iteration]     # on the GPU box
  BOUNDS=100 python tools/phase_stamps.py       # config 4 (box +-100)
  python tools/phase_stamps.py solve           # the whole-solve launch (k_mpc_solve_fixed)
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("DILQR_LIB", os.path.join(ROOT, "differentiable-ilqr_amd", "dilqr", "libdilqr_stamps.so"))
sys.path.insert(0, os.path.join(ROOT, "differentiable-ilqr_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from dilqr import _native as N  # noqa: E402
from dilqr import ops  # noqa: E402

dev = torch.device("cuda", 0)
T, n, m = bench.T_HORIZON, bench.N_STATE, bench.N_CTRL
B = bench.B_PER_GPU
SOLVE = len(sys.argv) > 1 and sys.argv[1] == "solve"
STOP_AT = int(sys.argv[1]) if len(sys.argv) > 1 and not SOLVE else 5         # stamps of this iteration
x0n, q, p = bench.make_problems(B)
x0 = torch.tensor(x0n, device=dev)
C = torch.diag(torch.tensor(q)).repeat(T, B, 1, 1).to(dev).contiguous()
c = torch.tensor(p).repeat(T, B, 1).to(dev).contiguous()
theta = torch.tensor([9.8, 1.0, 0.1, 0.5], device=dev)
sv = ops.MPCSolve(T, B, n, m, dev)
LIM = float(os.environ.get("BOUNDS", "0"))
nb, _keep = N.make_bounds(-LIM, LIM) if LIM > 0 else N.make_bounds(None, None)
s = N.stream(dev)
W = B // 64
lib = N.lib()
lib.dilqr_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
lib.dilqr_debug_stamps.restype = ctypes.c_int

rows = []
if SOLVE:
    ITERS = 10
    sv = ops.MPCSolve(T, B, n, m, dev, fixed_iters=ITERS)
    for solve in range(4):
        sv.solve_fixed(N.MODEL_CARTPOLE, theta, x0, C, c, nb, 0.5, 2, 1e-4)
        torch.cuda.synchronize()
        buf = np.zeros(W * 8, dtype=np.uint64)
        assert lib.dilqr_debug_stamps(buf.ctypes.data, W * 8) == 0
        rows.append(buf.reshape(W, 8).astype(np.int64))
    out = {"kernel": "k_mpc_solve_fixed", "iterations": ITERS, "waves": W, "bounds": LIM or None}
    r = rows[-1]
    ghz = (r[:, 5] - r[:, 0]) / ((r[:, 7] - r[:, 6]) / 100e6) / 1e9
    out["clock_ghz_median"] = float(np.median(ghz))
    for name, a, b_, div in (("begin", 0, 1, 1), ("iteration0", 1, 3, 1), ("steady_iteration", 3, 4, ITERS - 2),
                             ("last_sweep", 4, 2, 1), ("last_line_search", 2, 5, 1), ("wave", 0, 5, 1)):
        cyc = np.concatenate([(x[:, b_] - x[:, a]) / div for x in rows[1:]])
        out[name + "_cycles"] = {"median": float(np.median(cyc)), "p10": float(np.percentile(cyc, 10)),
                                 "p90": float(np.percentile(cyc, 90)), "max": float(cyc.max())}
        out[name + "_us_median"] = float(np.median(cyc) / (out["clock_ghz_median"] * 1e3))
    out["kernel_span_us"] = float(np.median([(x[:, 7].max() - x[:, 6].min()) / 100.0 for x in rows[1:]]))
    out["wave_end_spread_us"] = float(np.median([(x[:, 7].max() - x[:, 7].min()) / 100.0 for x in rows[1:]]))
    out["wave_start_spread_us"] = float(np.median([(x[:, 6].max() - x[:, 6].min()) / 100.0 for x in rows[1:]]))
    # by XCD (workgroups go round-robin over the 8 XCDs: wave w on XCD w % 8):
    # wall time of each wave (100 MHz ticks) and its shader clock
    wall = np.stack([(x[:, 7] - x[:, 6]) / 100.0 for x in rows[1:]])           # [solves, W] us
    clk = np.stack([(x[:, 5] - x[:, 0]) / ((x[:, 7] - x[:, 6]) / 100e6) / 1e9 for x in rows[1:]])
    out["by_xcd"] = {str(k): {"wave_us_median": float(np.median(wall[:, k::8])),
                              "wave_us_max": float(wall[:, k::8].max()),
                              "clock_ghz_median": float(np.median(clk[:, k::8]))} for k in range(8)}
    # is a slow wave slow in every solve (place) or in one (data)?
    per_wave = wall.mean(0)
    out["wave_us_p50_p90_max_of_solve_means"] = [float(np.median(per_wave)), float(np.percentile(per_wave, 90)),
                                                 float(per_wave.max())]
    out["slowest_wave_rank_corr"] = float(np.corrcoef(wall[0], wall[-1])[0, 1])
    print(json.dumps(out))
    sys.exit(0)
for solve in range(4):
    sv.begin(N.MODEL_CARTPOLE, theta, x0)
    for i in range(STOP_AT + 1):
        N.call("dilqr_mpc_step_f32", N.MODEL_CARTPOLE, T, B, N.ptr(theta), N.ptr(x0), N.ptr(C), N.ptr(c), nb, 0.5, 2,
               i, 1e-4, 0.0, 10 ** 9, sv.state, s)
        if i == STOP_AT:
            torch.cuda.synchronize()
            buf = np.zeros(W * 8, dtype=np.uint64)
            assert lib.dilqr_debug_stamps(buf.ctypes.data, W * 8) == 0
            rows.append(buf.reshape(W, 8).astype(np.int64))
        N.call("dilqr_mpc_stop_rule_f32", T, m, B, i, sv.state, s)
    torch.cuda.synchronize()

out = {"iteration": STOP_AT, "waves": W, "bounds": LIM or None}
r = rows[-1]
ghz = (r[:, 4] - r[:, 0]) / ((r[:, 7] - r[:, 6]) / 100e6) / 1e9
out["clock_ghz_median"] = float(np.median(ghz))
for name, a, b_ in (("prologue", 0, 1), ("sweep", 1, 2), ("line_search", 2, 3), ("epilogue", 3, 4), ("wave", 0, 4)):
    cyc = np.concatenate([x[:, b_] - x[:, a] for x in rows[1:]])
    out[name + "_cycles"] = {"median": float(np.median(cyc)), "p10": float(np.percentile(cyc, 10)),
                             "p90": float(np.percentile(cyc, 90)), "max": float(cyc.max())}
    out[name + "_us_median"] = float(np.median(cyc) / (out["clock_ghz_median"] * 1e3))
span = [(x[:, 7].max() - x[:, 6].min()) / 100.0 for x in rows[1:]]           # us, 100 MHz ticks
start_spread = [(x[:, 6].max() - x[:, 6].min()) / 100.0 for x in rows[1:]]
out["kernel_span_us"] = float(np.median(span))
end_spread = [(x[:, 7].max() - x[:, 7].min()) / 100.0 for x in rows[1:]]
out["wave_end_spread_us"] = float(np.median(end_spread))
out["wave_start_spread_us"] = float(np.median(start_spread))
out["per_step_cycles"] = {"sweep": out["sweep_cycles"]["median"] / T, "line_search": out["line_search_cycles"]["median"] / T}
print(json.dumps(out))
