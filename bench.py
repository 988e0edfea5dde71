#!/usr/bin/env python3
"""Headline benchmark: iLQR iterations/s on cartpole T=25, 65536 problems per GPU.

BASELINE.json metric: "iLQR iters/sec (whole node), batch=65536 cartpole T=25 at
1/2/4/8 MI355X" (configs[1]; configs[4] = the same at 8 GPUs, sharded).

A step = one whole mpc_explicit.MPC.forward solve (mpc_explicit.py:228-299) over
the rank's 65536 problems from u = 0: the initial rollout and lqr_iter = 10
iLQR iterations (rollout-linearise-Riccati-line search + best-iterate
bookkeeping each), the MPC default.  eps = 0 and not_improved_lim = inf keep
every iteration live (the reference's own fixed-iteration protocol,
BASELINE.md), so each solve is ONE dilqr_mpc_solve_fixed_f32 call: begin and
all ten iterations in one launch (each lane iterates its own problem), plus
the best_du finish launch.  value = problems x iterations / s.

Multi-GPU: one process per GPU (torchrun); problems shard as contiguous slices
of the one generated set; no collective in the data path (weak scaling).  The
barrier + synchronize bracket the timed region; the time is the MAX over ranks.

Prints ONE JSON line on rank 0 with `roofline` (the whole-solve launch, HIP
events on its stream) and `cpu_baseline` (the reference's CPU PyTorch op
structure restated in fp32 torch, oracle/torch_cpu.py, on the host cores).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "differentiable-ilqr_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

T_HORIZON = 25
B_PER_GPU = 65536
N_STATE, N_CTRL = 5, 1
D = N_STATE + N_CTRL
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec

# Algorithmic bytes, fp32.
#  Fused MPC iteration, per problem: the stage cost AS THE TIMED PATH READS IT
#  (iter_cost_floats), x_init, the current trajectory in, the new one out,
#  cost and du_norm.  SURVEY.md's 5,428 B/problem counts the caller's C, c at
#  every step; the kernel reads the solve's packed copy instead, and for the
#  reference's own cost (diag(q), p repeated over t) only its 2d floats once.
PACKED_FLOATS = D * (D + 1) // 2 + D                                   # 27 at d=6


def iter_cost_floats(flags, T=T_HORIZON, d=D):
    """Cost floats one iteration (>= 1) reads per problem, by the iteration-0
    flags (dilqr.h dilqr_mpc_state: bit0 symmetric, bit1 diagonal, bit2 time-invariant)."""
    pk = d * (d + 1) // 2 + d
    f = np.asarray(flags).astype(np.int64)
    out = np.full(f.shape, T * (d * d + d), np.float64)                    # asymmetric: the caller's C, c
    if d <= 8:                                                              # packed copies: one-lane models
        out[(f & 1) != 0] = T * pk                                          # packed symmetric
        out[(f & 5) == 5] = pk                                              # ... time-invariant: one record
        out[(f & 3) == 3] = T * 2 * d                                       # diagonal: diag(C_t), c_t
    out[(f & 7) == 7] = 2 * d                                               # time-invariant diagonal: registers
    return out


def iter_bytes_per_problem(cost_floats, T=T_HORIZON, n=N_STATE, d=D):
    return 4 * (cost_floats + n + 2 * T * d + 2)


def solve_bytes_per_problem(flags, iters, T=T_HORIZON, n=N_STATE, m=N_CTRL, d=D):
    """Algorithmic bytes of one fixed-count solve (dilqr_mpc_solve_fixed_f32), per
    problem: begin (x_init in, slot 0 out), iteration 0 (the caller's C, c in, the
    packed copy out: one record for a time-invariant cost), iterations 1..iters-1
    (the cost as iter_cost_floats reads it), each iteration x_init, the current
    trajectory in, the new one out, its du rows, cost and du_norm; the finish
    (two du rows in, best_du and full_du_norm out)."""
    pk = d * (d + 1) // 2 + d
    f = np.asarray(flags).astype(np.int64)
    packed_out = np.where((f & 4) != 0, pk, T * pk)
    per_iter = n + 2 * T * d + T * m + 2
    floats = ((n + T * d)
              + (T * (d * d + d) + packed_out + per_iter)
              + (iters - 1) * (iter_cost_floats(f, T, d) + per_iter)
              + (2 * T * m + 2))
    return 4 * floats
#  Riccati sweep, per problem: C, c_back, F in; K, k out
SWEEP_BYTES_PER_PROBLEM = 4 * (T_HORIZON * D * D + T_HORIZON * D + (T_HORIZON - 1) * N_STATE * D
                               + T_HORIZON * N_CTRL * N_STATE + T_HORIZON * N_CTRL)                  # 7,680


def make_problems(B_total, seed=0):
    """x,dx ~ U(-.5,.5), th ~ U(-pi,pi), dth ~ U(-1,1)."""
    rng = np.random.RandomState(seed)
    th = rng.uniform(-np.pi, np.pi, B_total)
    x0 = np.stack([rng.uniform(-.5, .5, B_total), rng.uniform(-.5, .5, B_total), np.cos(th), np.sin(th),
                   rng.uniform(-1, 1, B_total)], 1).astype(np.float32)
    q = np.array([0.1, 0.1, 1., 1., 0.1, 0.001], np.float32)       # cartpole get_true_obj
    p = np.array([0., 0., -1., 0., 0., 0.], np.float32)
    return x0, q, p


def shard_rows(B_total, world, rank):
    per = B_total // world
    return rank * per, (rank + 1) * per


def cpu_baseline(budget_s=25.0):
    """The reference's CPU PyTorch path as a restatement with its op structure
    (oracle/torch_cpu.py, fp32; pinned to the reference's fp32 goldens by
    tests/test_torch_cpu.py), on this host's cores, chunked like the reference
    must be (its line search's diag(alphas) is B x B): per-iteration time =
    (t(6 iters) - t(1)) / 5, best of 3, best chunk."""
    from oracle import torch_cpu as tc
    r = tc.time_config2(make_problems, T=T_HORIZON, budget_s=budget_s)
    return {"value": r["value"], "unit": "problem-iters/s", "cores": r["threads"], "kind": "port",
            "dtype": "f32", "cpu_model": tc.cpu_model(), "host_cpus": os.cpu_count(), "chunk": r["chunk"],
            "by_chunk": r["by_chunk"],
            "sample": f"oracle/torch_cpu.py (the reference's op structure in fp32 torch, {r['threads']} host "
                      f"threads), cartpole T=25 unconstrained, chunks {list(r['by_chunk'])} x (1, 6) iterations, "
                      f"best of 3, {r['elapsed_s']:.1f}s"}


def rank_records(tdist, dev, elapsed, lo, hi, props=None):
    """Each rank's own record, all-gathered after the timed region (never inside
    it; the data path has no collective): the process group's world size, the
    device's name, PCI location and UUID, the rank's shard rows and its own
    elapsed time.  Returned on every rank: {world_size, backend, distinct_devices,
    elapsed_min_s, elapsed_max_s, spread, per_rank: [...]}."""
    p = (props or torch.cuda.get_device_properties)(dev)
    rec = {"rank": tdist.get_rank(), "local_rank": int(os.environ.get("LOCAL_RANK", "0")), "device": str(dev),
           "name": p.name, "gcn_arch": p.gcnArchName,
           "pci": f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}", "uuid": str(p.uuid),
           "rows": [int(lo), int(hi)], "elapsed_s": float(elapsed), "host": os.uname().nodename}
    recs = [None] * tdist.get_world_size()
    tdist.all_gather_object(recs, rec)
    recs.sort(key=lambda r: r["rank"])
    el = [r["elapsed_s"] for r in recs]
    return {"world_size": tdist.get_world_size(), "backend": tdist.get_backend(),
            "distinct_devices": len({(r["host"], r["uuid"]) for r in recs}),
            "rows_cover": all(a["rows"][1] == b["rows"][0] for a, b in zip(recs, recs[1:])),
            "elapsed_min_s": min(el), "elapsed_max_s": max(el),
            "spread": (max(el) - min(el)) / max(el) if max(el) > 0 else 0.0, "per_rank": recs}


def _timed_solves(sv, model_id, theta, x0, C, c, bounds, decay, max_ls, lqr_iter, solves, warmup_solves):
    """Whole fixed-iteration solves (eps=0, not_improved_lim=inf) -> (problem-iters/s, ms/iteration)."""
    from dilqr import _native as N

    def solve():
        if sv.fixed_iters == lqr_iter:                  # the stop rule cannot fire: fixed-count solve
            sv.solve_fixed(model_id, theta, x0, C, c, bounds, decay, max_ls, 1e-4)
            return
        sv.begin(model_id, theta, x0)
        for i in range(lqr_iter):
            sv.iterate(model_id, theta, x0, C, c, bounds, decay, max_ls, i, 1e-4, 0.0, 10 ** 9)
    for _ in range(warmup_solves):
        solve()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(solves):
        solve()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    assert bool(torch.isfinite(sv.best_cost).all()), "non-finite costs"
    del N
    return sv.B * lqr_iter * solves / dt, dt * 1e3 / (lqr_iter * solves)


def _event_ms(stream, fn, reps, warm_ms=20.0, prep=None):
    """Average time of fn(r), r = 0..reps-1, launched back to back between ONE
    pair of HIP events on `stream` (an event pair around every launch adds
    several us of its own to a 40-us kernel; rocprof's kernel durations agree
    with this figure, profiles/).  A stateful fn (an MPC iteration) passes
    `prep`, which re-establishes its starting state (begin + iteration 0, launches
    only) after the warm-up calls, so the timed calls see the states they would
    have seen without them."""
    # first call alone: its duration sizes the warm-up below
    torch.cuda.synchronize()
    t = time.perf_counter()
    fn(0)
    torch.cuda.synchronize()
    est_ms = (time.perf_counter() - t) * 1e3
    warm = int(min(400, max(2, warm_ms / max(est_ms, 1e-3))))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    # the stream sleeps while the host queues every launch, so the event pair
    # times the kernels back to back, not the host's launch rate (a ctypes
    # launch takes tens of us of Python, comparable to one 36-us iteration);
    # then ~warm_ms of untimed calls before the first event, since the clocks
    # fall back while one wave spins and ramp again over tens of ms of load
    # (profiles/r06/bench_warmup_sweep.txt)
    torch.cuda._sleep(int(min(100.0, 2.0 + 0.05 * (warm + reps)) * 2e6))
    for r in range(warm):
        if prep is not None and r % max(reps, 1) == 0:
            prep()                  # warm calls repeat the timed sequence (iterations 1..reps)
        fn(r % max(reps, 1))
    if prep is not None:
        prep()
    e0.record(stream)
    for r in range(reps):
        fn(r)
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def riccati_workload(n, m, T, B, dev, seed=0):
    """SURVEY.md §8(d) Riccati-kernel roofline workload: C = L L^T + 0.1 I (SPD,
    distinct per (t,b)), c_back ~ N(0,1), F = [I + 0.05 N | 0.1 N]."""
    d = n + m
    g = torch.Generator(device=dev).manual_seed(seed)
    L = torch.randn(T, B, d, d, device=dev, generator=g) * (0.5 / d ** 0.5)
    C = (L @ L.transpose(-1, -2) + 0.1 * torch.eye(d, device=dev)).contiguous()
    del L
    cb = torch.randn(T, B, d, device=dev, generator=g)
    F = torch.cat([torch.eye(n, device=dev) + 0.05 * torch.randn(T - 1, B, n, n, device=dev, generator=g),
                   0.1 * torch.randn(T - 1, B, n, m, device=dev, generator=g)], -1).contiguous()
    return C, cb, F


def sweep_roofline(n, m, T, B, dev, reps=5):
    """Standalone Riccati sweep (F from HBM) on the synthetic workload."""
    from dilqr import _native as N
    C, cb, F = riccati_workload(n, m, T, B, dev)
    K = torch.empty(T, B, m, n, device=dev)
    k = torch.empty(T, B, m, device=dev)
    nb = N.Bounds(N.BOUNDS_NONE, 0.0, 0.0, None, None)
    s = N.stream(dev)
    call = lambda r: N.call("dilqr_lqr_backward_f32", n, m, T, B, N.ptr(C), N.ptr(cb), None, None, N.ptr(F), nb,
                            None, 0, N.ptr(K), N.ptr(k), None, None, s)
    call(0)
    ms = _event_ms(torch.cuda.current_stream(dev), call, reps)
    d = n + m
    nbytes = 4 * (T * d * d + T * d + (T - 1) * n * d + T * m * n + T * m) * B
    gbs = nbytes / (ms * 1e-3) / 1e9
    return {"shape": [n, m, T, B], "avg_launch_ms": ms, "algorithmic_bytes_per_launch": nbytes,
            "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS}


def dense_cost_roofline(dev, x0, theta, B, reps=10):
    """The same fused iteration on a cost that really streams: a dense SPD C_t,b
    distinct per (t, b) (bitwise symmetric, so the packed-symmetric path: 27
    floats per step), iterations 1..reps timed with HIP events on the launch
    stream.  Bytes per problem: 4*(T*27 + n + 2*T*d + 2) = 3,928."""
    from dilqr import _native as N
    from dilqr import ops
    T = T_HORIZON
    g = torch.Generator(device=dev).manual_seed(5)
    L = torch.randn(T, B, D, D, device=dev, generator=g) * (0.3 / D ** 0.5)
    A = L @ L.transpose(-1, -2)
    del L
    q = torch.tensor([0.1, 0.1, 1., 1., 0.1, 0.001], device=dev)
    C = (0.5 * (A + A.transpose(-1, -2)) + torch.diag(q)).contiguous()   # bitwise symmetric
    del A
    c = (torch.tensor([0., 0., -1., 0., 0., 0.], device=dev) + 0.01 * torch.randn(T, B, D, device=dev, generator=g))
    c = c.contiguous()
    sv = ops.MPCSolve(T, B, N_STATE, N_CTRL, dev)
    nb, _ = N.make_bounds(None, None)
    s = N.stream(dev)
    stream = torch.cuda.current_stream(dev)
    def prep():
        sv.begin(N.MODEL_CARTPOLE, theta, x0)
        sv.iterate(N.MODEL_CARTPOLE, theta, x0, C, c, nb, 0.5, 2, 0, 1e-4, 0.0, 10 ** 9)
    prep()
    ms = _event_ms(stream, lambda r: N.call("dilqr_mpc_step_f32", N.MODEL_CARTPOLE, T, B, N.ptr(theta), N.ptr(x0),
                                            N.ptr(C), N.ptr(c), nb, 0.5, 2, r + 1, 1e-4, 0.0, 10 ** 9, sv.state, s),
                   reps, prep=prep)
    cf = iter_cost_floats(sv.cost_sym.cpu().numpy())
    nbytes = float(iter_bytes_per_problem(cf).sum())
    gbs = nbytes / (ms * 1e-3) / 1e9
    del sv, C, c
    return {"kernel": "k_mpc_iterate<Cartpole,UNC,LDS gains> (packed symmetric cost, 27 floats per step)",
            "workload": "dense SPD C_t,b distinct per (t,b), cartpole T=25, 65536 problems",
            "bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS,
            "algorithmic_bytes_per_launch": nbytes, "avg_launch_ms": ms,
            "problem_iters_per_s": B / (ms * 1e-3)}


FP32_PEAK_TFLOPS = 157.3      # MI355X_MICROARCH.md: peak FP32 (vector)
PMC_COMMIT = [None]


# VALU issue ceilings (tools/microbench/valu_issue.hip, profiles/r02/valu_issue.log,
# re-measured in profiles/r05/valu_issue.log): independent v_fma_f32 wave-instructions
# per second per SIMD with 1, 2 and 4 waves resident per SIMD
VALU_ISSUE_PER_SIMD = {1: 320000 / 0.817e-3, 2: 640000 / 1.300e-3, 4: 1280000 / 2.384e-3}
N_SIMD = 1024                 # 256 CUs x 4 SIMDs


def issue_roofline(pmc_entry, n_waves, ms):
    """The issue roofline of a launch: VALU wave-instructions per SIMD per second
    (PMC SQ_INSTS_VALU per wave x waves per SIMD / the launch time) against the
    microbenchmark's independent-FMA issue rate at the same residency (1 wave
    per SIMD for the one-lane-per-problem solve) and the saturated rate."""
    vi = pmc_entry.get("valu_instr_per_wave")
    if not vi:
        return None
    wps = n_waves / N_SIMD
    achieved = vi * wps / (ms * 1e-3)
    res = min(VALU_ISSUE_PER_SIMD, key=lambda k: abs(k - max(wps, 1.0)))
    peak = VALU_ISSUE_PER_SIMD[res]
    return {"unit": "VALU wave-instr/s per SIMD", "valu_instr_per_wave": vi, "waves_per_simd": wps,
            "achieved": achieved, "peak": peak, "peak_residency_waves": res, "frac": achieved / peak,
            "peak_saturated": VALU_ISSUE_PER_SIMD[4], "frac_of_saturated": achieved / VALU_ISSUE_PER_SIMD[4],
            "source": "PMC valu_instr_per_wave (profiles/pmc_traffic.json) x waves / avg launch time; peaks from "
                      "tools/microbench/valu_issue.hip"}


def load_pmc():
    """profiles/pmc_traffic.json -> {kernel signature: counters} (tools/pmc_summary.py)."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        t = json.load(open(path))
    except (OSError, ValueError):
        return {}
    PMC_COMMIT[0] = t.get("measured_at_commit")
    return t.get("kernels", {})


def with_pmc(entry, sig):
    """Attach the PMC figures of kernel `sig` (HBM-side bytes -> traffic, issue
    fractions) to a roofline entry.  A tuple of signatures: the launches of one
    step together (traffic summed, counters per kernel)."""
    pmc = load_pmc()
    if isinstance(sig, tuple):
        ks = [pmc.get(s_) for s_ in sig]
        if all(ks):
            entry["traffic"] = sum(k.get("hbm_bytes_per_launch", 0.0) for k in ks)
            entry["pmc"] = {s_: {f: v for f, v in k.items() if f not in ("hbm_bytes_per_launch", "measured_at")}
                            for s_, k in zip(sig, ks)}
            entry["pmc_measured_at"] = ks[0].get("measured_at", PMC_COMMIT[0])
        return entry
    k = pmc.get(sig)
    if k:
        entry["traffic"] = k.get("hbm_bytes_per_launch")
        entry["pmc"] = {f: v for f, v in k.items() if f not in ("hbm_bytes_per_launch", "measured_at")}
        entry["pmc_measured_at"] = k.get("measured_at", PMC_COMMIT[0])
    return entry


def implicit_flops_per_problem(model, T):
    """Counted algorithmic flops of the implicit backward per problem
    (tools/implicit_flops.py -> profiles/implicit_flops.json)."""
    path = os.path.join(ROOT, "profiles", "implicit_flops.json")
    per_step = json.load(open(path))["models"][model]["per_step"]
    return per_step * T


def implicit_kernel_ms(dx, wx, wu, C, c, x, u, K, lo, hi, dev, reps=5):
    """Average duration of dilqr_implicit_backward_f32 launched back to back on
    preallocated buffers (the autograd wrapper's allocations kept out)."""
    from dilqr import _native as N
    from dilqr import ops
    T, B, n = x.shape
    m = u.shape[2]
    d = n + m
    th = ops.theta_of(dx, x)
    bounds, keep = N.make_bounds(lo, hi)
    ws = torch.empty(T * B * N.lib().dilqr_implicit_ws_floats(dx.model_id), device=dev)
    dC = torch.empty(T, B, d, d, device=dev)
    dc = torch.empty(T, B, d, device=dev)
    dth = torch.empty(B, th.shape[0], device=dev)
    s = N.stream(dev)
    args = [N.ptr(a.contiguous()) for a in (C, c, x, u, K, wx, wu)]
    call = lambda _r: N.call("dilqr_implicit_backward_f32", dx.model_id, T, B, N.ptr(th), *args, bounds,  # noqa
                             N.ptr(ws), N.ptr(dC), N.ptr(dc), N.ptr(dth), s)
    call(0)
    ms = _event_ms(torch.cuda.current_stream(dev), call, reps)
    del keep
    return ms


def implicit_boundary_bytes(n, m, T, B):
    """Bytes the implicit backward must move per launch: C, c, x, u, K (the
    gains of the no-op forward), dl/dx, dl/du in; dC, dc out (dtheta, B*p floats,
    and theta are negligible).  Its private workspace (the modified Riccati
    gains B -> C and the rollout y C -> D) is not counted."""
    d = n + m
    return 4 * T * B * (d * d + d + n + m + m * n + n + m + d * d + d)


def implicit_roofline(kernel, flops, nbytes, ms, B, T, bounds, pmc_sig):
    """Both rooflines of an implicit backward launch: fp32 vector flops and HBM
    (boundary bytes), with the PMC counters of the same instantiation; `bound`
    names the limiter the counters show (waitcnt stall vs VALU busy)."""
    tf = flops / (ms * 1e-3) / 1e12
    gbs = nbytes / (ms * 1e-3) / 1e9
    e = with_pmc({"kernel": kernel, "avg_ms": ms, "problems_per_s": B / (ms * 1e-3), "batch": B, "T": T,
                  "bounds": bounds, "unit": "GB/s", "achieved": gbs, "peak": HBM_PEAK_GBS,
                  "frac": gbs / HBM_PEAK_GBS, "algorithmic_bytes_per_launch": nbytes,
                  "bytes_model": "boundary bytes: C, c, x, u, K, dl/dx, dl/du in; dC, dc out",
                  "flops": {"flops_per_launch": flops, "achieved": tf, "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                            "frac": tf / FP32_PEAK_TFLOPS,
                            "source": "profiles/implicit_flops.json (counted per problem, tools/implicit_flops.py)"}},
                 pmc_sig)
    pm = e.get("pmc", {})
    if "valu_busy" in pm and "waitcnt_stall" in pm:
        e["bound"] = "hbm" if pm["waitcnt_stall"] > pm["valu_busy"] else "valu"
        e["limiter"] = (f"PMC: waitcnt stall {pm['waitcnt_stall']:.2f} vs VALU busy {pm['valu_busy']:.2f} of wave "
                        f"cycles")
    else:
        e["bound"] = "hbm"
    if e.get("traffic"):
        e["traffic_over_boundary"] = e["traffic"] / nbytes
    return e


def rocket_problems(B, dev):
    """near-hover initial states, get_true_obj cost."""
    rng = np.random.RandomState(0)
    r = rng.uniform([0, -4, -2.5], [10, 4, 2.5], (B, 3))
    v = rng.normal(0, 0.1, (B, 3))
    q4 = np.array([1., 0, 0, 0]) + 0.05 * rng.normal(size=(B, 4))
    q4 /= np.linalg.norm(q4, axis=1, keepdims=True)
    w = rng.normal(0, 0.02, (B, 3))
    x0 = torch.tensor(np.concatenate([r, v, q4, w], 1), dtype=torch.float32, device=dev)
    from dilqr.env_dx.rocket import RocketDx
    dx = RocketDx()
    q, p = dx.get_true_obj()
    T = 30
    C = torch.diag(q).repeat(T, B, 1, 1).to(dev).contiguous()
    c = p.repeat(T, B, 1).to(dev).contiguous()
    return dx, x0, C, c


def steady_iteration_ms(sv, model_id, theta, x0, C, c, bounds, decay, max_ls, dev, reps=10):
    """Average duration of the fused MPC iteration kernel in steady state:
    begin + iteration 0, then iterations 1..reps launched back to back
    (dilqr_mpc_step_f32, no stop-rule launches between them: eps = 0 and
    not_improved_lim = inf) between one pair of HIP events on the launch stream."""
    from dilqr import _native as N
    s = N.stream(dev)

    def prep():
        sv.begin(model_id, theta, x0)
        sv.iterate(model_id, theta, x0, C, c, bounds, decay, max_ls, 0, 1e-4, 0.0, 10 ** 9)
    prep()
    return _event_ms(torch.cuda.current_stream(dev), lambda r: N.call(
        "dilqr_mpc_step_f32", model_id, sv.T, sv.B, N.ptr(theta), N.ptr(x0), N.ptr(C), N.ptr(c), bounds,
        float(decay), int(max_ls), r + 1, 1e-4, 0.0, 10 ** 9, sv.state, s), reps, prep=prep)


def secondary_configs(dev):
    """BASELINE.json configs 3 and 4 on one GPU (information lines beside the headline)."""
    from dilqr import _native as N
    from dilqr import ops
    from dilqr.implicit import implicit_backward
    from dilqr.env_dx.cartpole import CartpoleDx
    out = {}
    stream = torch.cuda.current_stream(dev)
    # ---- config 3: rocket n=13 m=3 T=30 B=32768, unconstrained, decay 0.2, max_ls 5, lqr_iter 10
    T, B, n, m = 30, 32768, 13, 3
    dx, x0, C, c = rocket_problems(B, dev)
    theta = ops.theta_of(dx, x0)
    sv = ops.MPCSolve(T, B, n, m, dev, fixed_iters=10)
    nb, _ = N.make_bounds(None, None)
    val, ms_it = _timed_solves(sv, N.MODEL_ROCKET, theta, x0, C, c, nb, 0.2, 5, 10, 2, 1)
    # the launches the timed solves run per iteration, steady state: the group
    # sweep (8 lanes per problem) and the line search (one candidate per lane)
    it_ms = steady_iteration_ms(ops.MPCSolve(T, B, n, m, dev), N.MODEL_ROCKET, theta, x0, C, c, nb, 0.2, 5, dev)
    d = n + m
    # bytes of one steady iteration as the kernels move them (counted the way
    # iter_cost_floats counts cartpole): the cost as the register-cost kernels
    # read it (a time-invariant diagonal one: 2d floats), x_init, the current
    # trajectory in and the new one out, cost and du_norm, plus the gain
    # records (K_t, k_t: m*n + m floats per step) the group sweep hands the
    # lane-pair search through HBM (written once, read once)
    cf = iter_cost_floats(sv.cost_sym.cpu().numpy(), T=T, d=d)
    it_bytes = float((iter_bytes_per_problem(cf, T=T, n=n, d=d) + 4 * 2 * T * (m * n + m)).sum())
    boundary = float(iter_bytes_per_problem(cf, T=T, n=n, d=d).sum())            # 4,028 B/problem
    survey_bytes = 4 * (T * d * d + T * d + n + 2 * T * d + 2) * B             # 36,540 B/problem, SURVEY §8(d)
    gbs = it_bytes / (it_ms * 1e-3) / 1e9
    out["config3_rocket"] = {
        "value": val, "unit": "problem-iters/s", "ms_per_iter": ms_it, "batch": B, "T": T,
        "fused_iteration": with_pmc(
            {"kernel": "k_mpc_sweep_g8<Rocket,UNC,register cost> + k_mpc_search_quad<Rocket,NONE,register cost> "
                       "(+ the dense-cost instantiations on a small grid, which leave at once): one MPC iteration of "
                       "the timed solves, steady state",
             "bound": "hbm", "avg_launch_ms": it_ms, "algorithmic_bytes_per_launch": it_bytes,
             "bytes_model": "cost as read (time-invariant diagonal: 2d floats in registers) + x_init + tau in/out "
                            "+ cost, du_norm + gain records through HBM (2 T (mn+m) floats)",
             "survey_bytes_per_launch": survey_bytes,
             "survey_bytes_note": "SURVEY.md §8(d) 36,540 B/problem counts the caller's C at every step, which the "
                                  "steady kernels never read (not a roofline figure)",
             "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS,
             "boundary_bytes_per_launch": boundary,
             "boundary_bytes_model": "what crosses the iteration's boundary: the register cost (2d), x_init, tau in "
                                     "and out, cost and du_norm per problem (no gain records)",
             "frac_on_boundary_bytes": boundary / (it_ms * 1e-3) / 1e9 / HBM_PEAK_GBS},
            ("k_mpc_sweep_g8<Rocket, 0, true>", "k_mpc_sweep_g8<Rocket, 0, false>",
             "k_mpc_search_quad<Rocket, 0, true>", "k_mpc_search_quad<Rocket, 0, false>")),
        "riccati_sweep": sweep_roofline(n, m, T, B, dev)}
    # rocket implicit backward (16-lane groups) at the solution of the timed solves
    x, u = sv.gather_best()
    F, _f = ops.linearize(N.MODEL_ROCKET, theta, x, u)
    K, _k, _ = ops.lqr_backward(C, c, F, n, m, x=x, u=u)
    g = torch.Generator(device=dev).manual_seed(1)
    wx = torch.zeros(T, B, n, device=dev)
    wu = torch.randn(T, B, m, device=dev, generator=g)                 # loss = sum(u * w), SURVEY §8(d)
    implicit_backward(dx, wx, wu, C, c, None, None, x, u, K, None, None, None)      # the autograd path runs
    ms = implicit_kernel_ms(dx, wx, wu, C, c, x, u, K, None, None, dev)
    out["config3_rocket"]["implicit_backward"] = implicit_roofline(
        "k_implicit_backward_group<Rocket> (dC, dc, dtheta)", implicit_flops_per_problem("rocket", T) * B,
        implicit_boundary_bytes(n, m, T, B), ms, B, T, "none", "k_implicit_backward_group<Rocket, RocketD2, 0, 7>")
    del sv, C, c, x0, x, u, F, K, wx, wu
    # ---- config 4: cartpole T=25 B=65536 with bounds (+-100 reference value, +-10 stress) + implicit backward
    T, B, n, m = 25, 65536, 5, 1
    x0n, qn, pn = make_problems(B)
    x0 = torch.tensor(x0n, device=dev)
    C = torch.diag(torch.tensor(qn)).repeat(T, B, 1, 1).to(dev).contiguous()
    c = torch.tensor(pn).repeat(T, B, 1).to(dev).contiguous()
    theta = torch.tensor([9.8, 1.0, 0.1, 0.5], device=dev)
    sv = ops.MPCSolve(T, B, n, m, dev, fixed_iters=10)
    for lim in (100.0, 10.0):
        bd, keep = N.make_bounds(-lim, lim)
        val, ms_it = _timed_solves(sv, N.MODEL_CARTPOLE, theta, x0, C, c, bd, 0.5, 2, 10, 3, 1)
        active = float(((sv.gather_best()[1].abs() - lim).abs() < 1e-6).float().mean())
        # the timed solves' launch (k_mpc_solve_fixed<Cartpole,BOX> + finish), event-timed
        s_ms = _event_ms(stream, lambda r: sv.solve_fixed(N.MODEL_CARTPOLE, theta, x0, C, c, bd, 0.5, 2, 1e-4), 5)
        sb = float(solve_bytes_per_problem(sv.cost_sym.cpu().numpy(), 10).sum())
        sv2 = ops.MPCSolve(T, B, n, m, dev)
        k_ms = steady_iteration_ms(sv2, N.MODEL_CARTPOLE, theta, x0, C, c, bd, 0.5, 2, dev)
        kb = float(iter_bytes_per_problem(iter_cost_floats(sv2.cost_sym.cpu().numpy())).sum())
        del sv2
        out[f"config4_cartpole_box{int(lim)}"] = {
            "value": val, "unit": "problem-iters/s", "ms_per_iter": ms_it, "batch": B, "T": T,
            "active_control_frac": active,
            "solve_launch": with_pmc(
                {"kernel": "k_mpc_solve_fixed<Cartpole,BOX,LDS gains> + k_mpc_fixed_finish (the timed solves)",
                 "bound": "hbm", "avg_launch_ms": s_ms, "algorithmic_bytes_per_launch": sb,
                 "achieved": sb / (s_ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                 "frac": sb / (s_ms * 1e-3) / 1e9 / HBM_PEAK_GBS},
                "k_mpc_solve_fixed<Cartpole, 1, true>" if lim == 100.0 else "-"),
            "steady_iteration": with_pmc(
                {"kernel": "k_mpc_iterate<Cartpole,BOX,LDS gains,steady> (the stop-rule path's per-iteration launch)",
                 "bound": "hbm", "avg_launch_ms": k_ms, "algorithmic_bytes_per_launch": kb,
                 "achieved": kb / (k_ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                 "frac": kb / (k_ms * 1e-3) / 1e9 / HBM_PEAK_GBS},
                "k_mpc_iterate<Cartpole, 1, true, false>" if lim == 100.0 else "-")}
    x, u = sv.gather_best()
    F, _f = ops.linearize(N.MODEL_CARTPOLE, theta, x, u)
    K, _k, _ = ops.lqr_backward(C, c, F, n, m, x=x, u=u, u_lower=-10.0, u_upper=10.0)
    g = torch.Generator(device=dev).manual_seed(1)
    wx = torch.zeros(T, B, n, device=dev)
    wu = torch.randn(T, B, m, device=dev, generator=g)                 # loss = sum(u * w), SURVEY §8(d)
    cart = CartpoleDx()
    implicit_backward(cart, wx, wu, C, c, None, None, x, u, K, -10.0, 10.0, None)
    ms = implicit_kernel_ms(cart, wx, wu, C, c, x, u, K, -10.0, 10.0, dev)
    out["config4_implicit_backward"] = implicit_roofline(
        "k_implicit_backward<Cartpole> (dC, dc, dtheta)", implicit_flops_per_problem("cartpole", T) * B,
        implicit_boundary_bytes(n, m, T, B), ms, B, T, "+-10", "k_implicit_backward<Cartpole>")
    del sv, C, c
    # ---- one empc training step of the IL loop (il_exp.py:297-352):
    # MPC forward (lqr_iter 100, eps 1e-4, bounds +-100, T=35) + im_loss backward into the
    # dynamics parameters, cartpole, 4096 problems from config-2 initial states
    # at 4096 problems and at the reference's own n_batch = 32 (il_exp.py:44; one
    # workgroup: the whole stop-rule loop in one launch, dilqr_mpc_solve_small_f32)
    from dilqr import il
    import warnings
    env = il.IL_Env("cartpole", lqr_iter=100, mpc_T=35, device=dev)
    qi, pi_ = env.true_dx.get_true_obj()
    qi, pi_ = qi.to(dev), pi_.to(dev)
    for Bi, key in ((4096, "il_empc_step_cartpole"), (32, "il_empc_step_cartpole_b32")):
        xi = torch.tensor(make_problems(Bi, seed=2)[0], device=dev)
        params = torch.tensor((9.8, 3.0, 0.1, 1.0), device=dev, requires_grad=True)
        target = torch.zeros(35, Bi, 1, device=dev)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        fwd, bwd = [], []

        def il_step(rec=False):
            params.grad = None
            if rec:
                ev[0].record()
            _, uu = env.mpc(CartpoleDx(params), xi, qi, pi_)
            if rec:
                ev[1].record()
            loss = (target - uu).pow(2).mean()
            loss.backward()
            if rec:
                ev[2].record()
                torch.cuda.synchronize()
                fwd.append(ev[0].elapsed_time(ev[1]))
                bwd.append(ev[1].elapsed_time(ev[2]))
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            il_step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(3):
                il_step()
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) * 1e3 / 3
            il_step(rec=True)
        out[key] = {"ms_per_step": ms, "batch": Bi, "T": 35, "lqr_iter_max": 100,
                    "forward_ms": fwd[0], "backward_ms": bwd[0],
                    "forward_path": ("one launch (dilqr_mpc_solve_small_f32)" if Bi <= 256
                                     else "two launches per iteration, host poll every 8"),
                    "what": "MPC forward to the stop rule + implicit backward into theta"}
    return out


def profile_set(name, dev):
    """--kernels-only --profile-set NAME: a few launches of one family of
    kernels for rocprofv3 (PMC passes per family, tools/profile_pmc.sh)."""
    from dilqr import _native as N
    from dilqr import ops
    from dilqr.implicit import implicit_backward
    out = {}
    if name == "rocket":                          # k_mpc_sweep_g8 + k_mpc_search_lane<Rocket>, config 3
        T, B = 30, 32768
        dx, x0, C, c = rocket_problems(B, dev)
        theta = ops.theta_of(dx, x0)
        nb, _ = N.make_bounds(None, None)
        out["rocket_iter_ms"] = steady_iteration_ms(ops.MPCSolve(T, B, 13, 3, dev), N.MODEL_ROCKET, theta, x0, C, c,
                                                    nb, 0.2, 5, dev, reps=4)
    elif name == "box":                           # k_mpc_iterate<Cartpole,BOX,...>, config 4 +-100
        T, B = T_HORIZON, B_PER_GPU
        x0n, qn, pn = make_problems(B)
        x0 = torch.tensor(x0n, device=dev)
        C = torch.diag(torch.tensor(qn)).repeat(T, B, 1, 1).to(dev).contiguous()
        c = torch.tensor(pn).repeat(T, B, 1).to(dev).contiguous()
        theta = torch.tensor([9.8, 1.0, 0.1, 0.5], device=dev)
        bd, _ = N.make_bounds(-100.0, 100.0)
        out["box_iter_ms"] = steady_iteration_ms(ops.MPCSolve(T, B, 5, 1, dev), N.MODEL_CARTPOLE, theta, x0, C, c,
                                                 bd, 0.5, 2, dev, reps=4)
        sv = ops.MPCSolve(T, B, 5, 1, dev, fixed_iters=10)             # the timed solves' launch
        out["box_solve_ms"] = _event_ms(torch.cuda.current_stream(dev), lambda r: sv.solve_fixed(
            N.MODEL_CARTPOLE, theta, x0, C, c, bd, 0.5, 2, 1e-4), 3)
    elif name == "implicit":                      # both implicit backward kernels (config 4 and 3 shapes)
        from dilqr.env_dx.cartpole import CartpoleDx
        for model, T, B, lim in (("cartpole", 25, 65536, 10.0), ("rocket", 30, 32768, None)):
            if model == "cartpole":
                dx = CartpoleDx()
                x0 = torch.tensor(make_problems(B)[0], device=dev)
                q, p = dx.get_true_obj()
                C = torch.diag(q).repeat(T, B, 1, 1).to(dev).contiguous()
                c = p.repeat(T, B, 1).to(dev).contiguous()
                decay, mls = 0.5, 2
            else:
                dx, x0, C, c = rocket_problems(B, dev)
                decay, mls = 0.2, 5
            n, m = dx.n_state, dx.n_ctrl
            theta = ops.theta_of(dx, x0)
            lo, hi = (-lim, lim) if lim else (None, None)
            # the unfused kernels: this set must not re-measure the solve instantiations
            # the box / headline sets attach to their bench lines (other shapes)
            ws = ops.mpc_solve_unfused(dx.model_id, theta, x0, C, c, T, u_lower=lo, u_upper=hi, lqr_iter=5, eps=0.0,
                                       linesearch_decay=decay, max_linesearch_iter=mls, not_improved_lim=10 ** 9)
            x, u = ws.best_x, ws.best_u
            F, _f = ops.linearize(dx.model_id, theta, x, u)
            K, _k, _ = ops.lqr_backward(C, c, F, n, m, x=x, u=u, u_lower=lo, u_upper=hi)
            wx = torch.zeros(T, B, n, device=dev)
            wu = torch.randn(T, B, m, device=dev, generator=torch.Generator(device=dev).manual_seed(1))
            implicit_backward(dx, wx, wu, C, c, None, None, x, u, K, lo, hi, None)
            out[f"{model}_implicit_ms"] = implicit_kernel_ms(dx, wx, wu, C, c, x, u, K, lo, hi, dev, reps=3)
    else:
        raise ValueError(f"unknown profile set {name}")
    torch.cuda.synchronize(dev)
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # defaults: 200 warmup solves (~75 ms) before the timed ones.  The GPU's
    # clocks ramp over tens of milliseconds of load; 5 warmup solves (1.9 ms)
    # timed a cold GPU: 1.70-1.72e9 against 1.87-1.88e9 once warm, on one box
    # (profiles/r06/bench_warmup_sweep.txt)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--lqr-iter", type=int, default=10)
    ap.add_argument("--batch", type=int, default=B_PER_GPU, help="problems per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-secondary", action="store_true", help="skip the config 3/4 information lines")
    ap.add_argument("--kernels-only", action="store_true",
                    help="profiling mode: a few launches of the fused iteration and the sweep, no JSON line")
    ap.add_argument("--dump", default=None,
                    help="directory: each rank saves its shard's best trajectories after the timed solves "
                         "(tests/test_dist.py compares them with a whole-batch solve)")
    ap.add_argument("--profile-set", default="headline", choices=("headline", "rocket", "box", "implicit"),
                    help="with --kernels-only: which kernel family to launch (PMC passes per family)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # under torchrun (RANK set) the process group is initialised even for one
    # rank, so the RCCL path (init, barriers, the timing all-reduce) runs
    # as it does at N > 1 (tests/test_dist.py drives it on one GPU)
    dist = world > 1 or "RANK" in os.environ
    # BENCH_DIST_BACKEND=gloo rehearses the N>1 path with several ranks on one GPU
    # (the timing all-reduce then runs on the host); the driver's runs use RCCL
    backend = os.environ.get("BENCH_DIST_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    dev_index = local_rank if backend == "nccl" else local_rank % max(ndev, 1)
    if dist:
        import torch.distributed as tdist
        torch.cuda.set_device(dev_index)
        if backend == "nccl":
            tdist.init_process_group("nccl", device_id=torch.device("cuda", dev_index))
        else:
            tdist.init_process_group(backend)
    dev = torch.device("cuda", dev_index)

    from dilqr import _native as N
    from dilqr import ops

    if args.kernels_only and args.profile_set != "headline":
        profile_set(args.profile_set, dev)
        return

    B = args.batch
    B_total = B * world
    x0_all, q, p = make_problems(B_total)
    lo, hi = shard_rows(B_total, world, rank)
    x0 = torch.tensor(x0_all[lo:hi], device=dev)
    C = torch.diag(torch.tensor(q)).repeat(T_HORIZON, B, 1, 1).to(dev).contiguous()     # materialised per (t,b)
    c = torch.tensor(p).repeat(T_HORIZON, B, 1).to(dev).contiguous()
    theta = torch.tensor([9.8, 1.0, 0.1, 0.5], device=dev)
    # eps = 0 and not_improved_lim = 1e9: the stop rule cannot fire, so the
    # solve is a fixed-count one (ops.mpc_solve takes the same path): begin and
    # every iteration in one launch, best_du formed by the finish launch
    sv = ops.MPCSolve(T_HORIZON, B, N_STATE, N_CTRL, dev, fixed_iters=args.lqr_iter)
    bounds, _ = N.make_bounds(None, None)
    stream = torch.cuda.current_stream(dev)
    s = N.stream(dev)

    def step():                 # one MPC.forward solve of lqr_iter iterations
        sv.solve_fixed(N.MODEL_CARTPOLE, theta, x0, C, c, bounds, 0.5, 2, 1e-4)

    if args.kernels_only:
        args.steps, args.warmup, args.no_cpu_baseline, args.no_secondary = 0, 2, True, True
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if dist:
        tdist.barrier()
    torch.cuda.synchronize(dev)
    # HIP events on the launch stream bracket the same K solves: the roofline's
    # per-launch duration of the dominant kernel is measured over the timed
    # region itself (one step = k_mpc_solve_fixed + k_mpc_fixed_finish)
    ev_t0, ev_t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev_t0.record(stream)
    for _ in range(args.steps):
        step()
    ev_t1.record(stream)
    torch.cuda.synchronize(dev)
    if dist:
        tdist.barrier()
    elapsed = time.perf_counter() - t0
    timed_solve_ms = ev_t0.elapsed_time(ev_t1) / args.steps if args.steps else None
    ranks = None
    if dist:
        own = elapsed
        tt = torch.tensor([elapsed], device=dev if backend == "nccl" else "cpu", dtype=torch.float64)
        tdist.all_reduce(tt, op=tdist.ReduceOp.MAX)
        elapsed = float(tt.item())
        # outside the timed region: what each rank ran on, so the line proves
        # that N ranks solved on N distinct devices (rank_record)
        ranks = rank_records(tdist, dev, own, lo, hi)
        assert ranks["world_size"] == world, "WORLD_SIZE disagrees with the process group"
    assert args.kernels_only or bool(torch.isfinite(sv.best_cost).all()), "non-finite costs"
    if args.dump:
        # the last timed solve of this rank's shard (rows [lo, hi) of the global batch)
        xb, ub = sv.gather_best()
        os.makedirs(args.dump, exist_ok=True)
        torch.save({"rows": (lo, hi), "x": xb.cpu(), "u": ub.cpu(), "cost": sv.best_cost.cpu()},
                   os.path.join(args.dump, f"shard{rank}.pt"))

    # ---- roofline of the dominant kernel: the whole-solve launch
    # (k_mpc_solve_fixed + its finish, one dilqr_mpc_solve_fixed_f32 call = one
    # step), reps solves back to back between one pair of HIP events on ITS
    # stream (the current stream, where ops launch it)
    reps = 10
    # the same solves timed again by the secondary lines' event helper (a
    # cross-check of the timed-region figure)
    solve_ms_separate = _event_ms(stream, lambda r: step(), reps)
    solve_ms = timed_solve_ms if timed_solve_ms is not None else solve_ms_separate
    solve_bytes = float(solve_bytes_per_problem(sv.cost_sym.cpu().numpy(), args.lqr_iter).sum())
    # ---- the per-iteration kernel of the stop-rule path (k_mpc_iterate<...,
    # FIRST=false>): iterations 1..reps of a solve launched back to back.  No
    # stop-rule launches in between: with eps = 0 and not_improved_lim = inf the
    # rule cannot fire.
    def prep_iter():
        sv.begin(N.MODEL_CARTPOLE, theta, x0)
        sv.iterate(N.MODEL_CARTPOLE, theta, x0, C, c, bounds, 0.5, 2, 0, 1e-4, 0.0, 10 ** 9)
    prep_iter()
    iter_ms = _event_ms(stream, lambda r: N.call(
        "dilqr_mpc_step_f32", N.MODEL_CARTPOLE, T_HORIZON, B, N.ptr(theta), N.ptr(x0), N.ptr(C), N.ptr(c), bounds,
        0.5, 2, r + 1, 1e-4, 0.0, 10 ** 9, sv.state, s), reps, prep=prep_iter)
    cost_floats = iter_cost_floats(sv.cost_sym.cpu().numpy())
    iter_bytes = float(iter_bytes_per_problem(cost_floats).sum())
    cost_path = ("time-invariant diagonal cost held in registers (2d floats per problem)"
                 if (cost_floats == 2 * D).all() else f"mixed cost paths, {cost_floats.mean():.0f} cost floats/problem")
    xa, ua = sv.gather_best()

    # standalone Riccati sweep (the north-star's >=50% HBM target kernel)
    F, _f = ops.linearize(N.MODEL_CARTPOLE, theta, xa, ua)
    K = torch.empty(T_HORIZON, B, N_CTRL, N_STATE, device=dev)
    k = torch.empty(T_HORIZON, B, N_CTRL, device=dev)
    cb = torch.randn(T_HORIZON, B, D, device=dev)
    nb = N.Bounds(N.BOUNDS_NONE, 0.0, 0.0, None, None)
    sweep = lambda r: N.call(  # noqa: E731
        "dilqr_lqr_backward_f32", N_STATE, N_CTRL, T_HORIZON, B, N.ptr(C), N.ptr(cb), None, None, N.ptr(F), nb, None,
        0, N.ptr(K), N.ptr(k), None, None, s)
    sweep(0)            # the first launch from this unit's code object loads it (~ms): keep it out of the timing
    sweep_ms = _event_ms(stream, sweep, reps)
    sweep_bytes = SWEEP_BYTES_PER_PROBLEM * B

    # PMC figures of the same kernel at this shape (tools/profile_pmc.sh over
    # `bench.py --kernels-only`, summarised by tools/pmc_summary.py): HBM-side
    # bytes per launch with the gfx950 FETCH_SIZE correction, and the issue
    # breakdown (what bounds the kernel: VALU issue, not HBM)
    pmc = load_pmc()
    head_pmc = pmc.get("k_mpc_solve_fixed<Cartpole, 0, true>", {})
    fin_pmc = pmc.get("k_mpc_fixed_finish", {})
    traffic = None
    if "hbm_bytes_per_launch" in head_pmc and "hbm_bytes_per_launch" in fin_pmc:
        traffic = (head_pmc["hbm_bytes_per_launch"] + fin_pmc["hbm_bytes_per_launch"]) * B / B_PER_GPU
    it_pmc = pmc.get("k_mpc_iterate<Cartpole, 0, true, false>", {})
    it_traffic = it_pmc.get("hbm_bytes_per_launch")
    it_traffic = None if it_traffic is None else it_traffic * B / B_PER_GPU
    dense = None if args.kernels_only or world > 1 else dense_cost_roofline(dev, x0, theta, B)

    if rank == 0 and args.kernels_only:
        print(json.dumps({"solve_ms": solve_ms, "iter_ms": iter_ms, "sweep_ms": sweep_ms}), flush=True)
    elif rank == 0:
        value = B_total * args.lqr_iter * args.steps / elapsed
        achieved = solve_bytes / (solve_ms * 1e-3) / 1e9
        it_achieved = iter_bytes / (iter_ms * 1e-3) / 1e9
        sweep_gbs = sweep_bytes / (sweep_ms * 1e-3) / 1e9
        line = {
            "metric": "iLQR iters/sec (whole node), batch=65536 cartpole T=25 at 1/2/4/8 MI355X",
            "value": value,
            "unit": "problem-iters/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps,
            "ms_per_iteration": elapsed * 1e3 / (args.steps * args.lqr_iter),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (SURVEY.md §8(d) config 2 x_init, seed 0; cartpole get_true_obj cost materialised "
                    "per (t,b))",
            "config": {"workload": "cartpole n=5 m=1 T=25, unconstrained iLQR, 65536 problems per GPU, "
                                   f"step = one whole-batch MPC solve of lqr_iter={args.lqr_iter} from u=0",
                       "batch_per_gpu": B, "global_batch": B_total, "T": T_HORIZON, "lqr_iter": args.lqr_iter,
                       "parallelism": f"batch-sharded x{world} (no collective)",
                       "batch_iters_per_s": world * args.lqr_iter * args.steps / elapsed},
            "roofline": {"kernel": "k_mpc_solve_fixed<Cartpole,UNC,LDS gains> + k_mpc_fixed_finish (one whole "
                                   "fixed-count solve: begin + iteration 0 reading the caller's C + "
                                   f"{args.lqr_iter - 1} steady iterations; " + cost_path + ")",
                         "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "traffic_measured_at": head_pmc.get("measured_at", PMC_COMMIT[0]),
                         "algorithmic_bytes_per_launch": solve_bytes, "avg_launch_ms": solve_ms,
                         "avg_launch_ms_source": "HIP events on the launch stream around the timed solves",
                         "avg_launch_ms_separate": solve_ms_separate,
                         "limiter": {"what": "VALU issue at one wave per SIMD (B=65536 = 1024 waves); not HBM",
                                     **{k: v for k, v in head_pmc.items()
                                        if k not in ("hbm_bytes_per_launch", "measured_at")}},
                         "issue": issue_roofline(head_pmc, (B + 63) // 64, solve_ms)},
            "roofline_steady_iteration": {
                "kernel": "k_mpc_iterate<Cartpole,UNC,LDS gains,steady> (the stop-rule path's per-iteration launch; "
                          + cost_path + ")",
                "bound": "hbm", "achieved": it_achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": it_achieved / HBM_PEAK_GBS, "traffic": it_traffic, "algorithmic_bytes_per_launch": iter_bytes,
                "avg_launch_ms": iter_ms,
                "pmc": {k: v for k, v in it_pmc.items() if k not in ("hbm_bytes_per_launch", "measured_at")},
                "pmc_measured_at": it_pmc.get("measured_at")},
            "roofline_dense_cost": dense,
            "riccati_roofline": {"kernel": "k_lqr_backward<5,1,UNC> (standalone sweep, F from HBM)",
                                 "bound": "hbm", "achieved": sweep_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                 "frac": sweep_gbs / HBM_PEAK_GBS, "algorithmic_bytes_per_launch": sweep_bytes,
                                 "avg_launch_ms": sweep_ms},
        }
        if ranks is not None:
            line["ranks"] = ranks
        if world == 1 and not args.no_secondary:
            line["secondary"] = secondary_configs(dev)
        if world == 1 and not args.no_cpu_baseline:
            cb = cpu_baseline()
            line["cpu_baseline"] = cb
            # no published number exists for this metric; the
            # ratio is to the reference-structured CPU path timed above on this
            # box's host cores (a baseline, not a target)
            line["vs_baseline"] = value / cb["value"]
            line["vs_baseline_basis"] = (f"cpu_baseline: the reference's CPU PyTorch op structure in fp32 on "
                                         f"{cb['cores']} host threads ({cb['cpu_model']}), best chunk {cb['chunk']}")
        print(json.dumps(line), flush=True)
    if dist:
        tdist.barrier()
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
